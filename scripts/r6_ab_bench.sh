# bench.py A/B of gangColocation None vs Preferred (no GPU probe, no extras).
set -e
OUT=gpurun_out/${TAG:-r6e}
mkdir -p $OUT
for i in 1 2; do
  for m in None Preferred; do
    timeout -k 10 200 python bench.py --no-gpu-probe --no-open-loop --no-service-mode --no-scenarios --no-placement --nodes1024-waves ${N1024:-0} --gang-colocation $m > $OUT/bench_${m}_$i.json 2>> $OUT/bench.err
    python -c "import json; d=json.load(open('$OUT/bench_${m}_$i.json')); c=d['config']; print('$m', $i, d['value'], c.get('nodes1024_pods_per_s'), c['p99_gang_admit_ms'])"
  done
done
