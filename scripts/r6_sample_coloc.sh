# Headline bench waves under the sampler, gang co-location None vs Preferred,
# then bench.py A/B without the GPU probe (torch/HIP not initialised).
set -e
OUT=gpurun_out/r6d
mkdir -p $OUT
SO=$(python -c "import flex_gpu_scheduler_amd._xsched as m; print(m.__file__)")
for m in None Preferred; do
  timeout -k 10 200 python scripts/sample_bench_waves.py $OUT --waves 160 --colocation $m --tag w_$m --seed 0
  timeout -k 10 200 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/w_$m.samples --exe "$SO" --top 60 > $OUT/w_${m}_report.txt 2>&1
  rm -f $OUT/w_$m.samples
done
for m in None Preferred None Preferred; do
  timeout -k 10 200 python bench.py --no-gpu-probe --no-open-loop --no-service-mode --no-scenarios --no-placement --nodes1024-waves 0 --gang-colocation $m > $OUT/bench_noprobe_$m.json 2>> $OUT/bench.err
  python -c "import json; d=json.load(open('$OUT/bench_noprobe_$m.json')); print('noprobe $m', d['value'])"
done
