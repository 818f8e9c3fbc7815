set -e
OUT=gpurun_out/${TAG:-r6m}
mkdir -p $OUT
SO=$(python -c "import flex_gpu_scheduler_amd._xsched as m; print(m.__file__)")
timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 1024 --waves 12 --tag n1024 --seed 0 --hz 2000
timeout -k 10 300 python scripts/alloc_callers.py $OUT/n1024.samples "$SO" xs-sched > $OUT/alloc_sched.txt
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/n1024.samples --exe "$SO" --lines "find_nodes_that_fit" --top 40 > $OUT/lines_fnf.txt 2>&1 || true
rm -f $OUT/n1024.samples
