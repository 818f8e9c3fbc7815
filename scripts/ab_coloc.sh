set -e
mkdir -p gpurun_out
for i in 1 2; do
  for m in None Preferred; do
    timeout -k 10 200 python bench.py --no-open-loop --no-service-mode --no-scenarios --no-placement --nodes1024-waves 0 --gang-colocation $m > gpurun_out/r6b_ab_${m}_$i.json 2>> gpurun_out/r6b_ab.err
    python -c "import json,sys; d=json.load(open('gpurun_out/r6b_ab_${m}_$i.json')); print('$m', $i, d['value'], d['config']['headline'][:80])"
  done
done
