#!/usr/bin/env bash
# 1-GPU headline bench at 64 nodes (default config, 3 runs) and at 1,024
# nodes, each under its own time limit. Usage: bash scripts/bench_r2.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
tag=${1:-r2}
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-scenarios > "$OUT/${tag}_bench64_$i.json" 2> "$OUT/${tag}_bench64_$i.err" || exit $?
done
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --nodes 1024 --no-scenarios > "$OUT/${tag}_bench1024.json" 2> "$OUT/${tag}_bench1024.err" || exit $?
python - "$OUT" "$tag" <<'PY'
import json, sys, glob
out, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{out}/{tag}_bench*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["config"]["p99_gang_admit_ms"])
PY
