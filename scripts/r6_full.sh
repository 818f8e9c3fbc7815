# Full default bench (the driver's command) then the colocation A/B.
set -e
OUT=gpurun_out/${TAG:-r6f}
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench1.json 2> $OUT/bench1.err
python -c "import json; d=json.load(open('$OUT/bench1.json')); print(d['value'], d['config']['headline'])"
TAG=${TAG:-r6f}_ab bash scripts/r6_ab_bench.sh
