# Two full default bench.py runs back to back (run-to-run spread on one box).
set -e
OUT=gpurun_out/${TAG:-r6ap}
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 1000 python bench.py > $OUT/bench$i.json 2> $OUT/bench$i.err
  python -c "import json; d=json.loads(open('$OUT/bench$i.json').read().strip().splitlines()[-1]); print(d['config']['headline'])"
done
