set -o pipefail
mkdir -p gpurun_out/r3o
for i in 1 2 3; do
  for e in 1 0; do
    XSCHED_MALLOC_TUNE=$e timeout -k 10 240 python bench.py --no-scenarios --no-open-loop > gpurun_out/r3o/ab_tune${e}_$i.json 2> gpurun_out/r3o/ab_tune${e}_$i.err || exit $?
    echo "tune=$e run=$i $(python -c "import json;d=json.load(open('gpurun_out/r3o/ab_tune${e}_$i.json'));print(d['value'],d['config']['p99_gang_admit_ms'])")"
  done
done
