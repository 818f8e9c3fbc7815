#!/usr/bin/env bash
# A/B of one environment knob on the headline bench (bench.py, open loop and
# scenarios off), alternating runs: bash scripts/ab_env.sh TAG VAR VALUE_A VALUE_B [RUNS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; var=$2; a=$3; b=$4; runs=${5:-3}
OUT=gpurun_out/$tag
mkdir -p "$OUT"
for i in $(seq "$runs"); do
  for v in "$a" "$b"; do
    env "$var=$v" timeout -k 10 240 python bench.py --no-scenarios --no-open-loop > "$OUT/ab_${var}_${v}_$i.json" 2> "$OUT/ab_${var}_${v}_$i.err" || exit 1
    echo "$var=$v run=$i $(python -c "import json;d=json.load(open('$OUT/ab_${var}_${v}_$i.json'));print(d['value'],d['config']['p99_gang_admit_ms'])")" | tee -a "$OUT/ab_${var}.txt"
  done
done
