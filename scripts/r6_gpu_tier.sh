# The round-end GPU checks on the current tree: pytest -m gpu and smoke().
set -e
OUT=gpurun_out/${TAG:-r6aj}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
tail -2 $OUT/smoke.txt
