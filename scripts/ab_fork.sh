#!/usr/bin/env bash
# A/B of the Parallelizer's fork threshold (XSCHED_MIN_PARALLEL_NS): the
# 1,024-node bench and the 5,000-node scheduler_perf matrix per setting.
# Usage: bash scripts/ab_fork.sh <tag> <ns> [<ns> ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
tag=$1; shift
for ns in "$@"; do
  for i in 1 2; do
    XSCHED_MIN_PARALLEL_NS=$ns timeout -k 10 200 python bench.py --steps 10 --warmup 3 --nodes 1024 --no-scenarios \
      > "$OUT/${tag}_fork${ns}_bench1024_$i.json" 2> "$OUT/${tag}_fork${ns}_bench1024_$i.err" || exit $?
  done
  XSCHED_MIN_PARALLEL_NS=$ns timeout -k 10 300 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 5000 --pods 5000 --cpus l3 \
    > "$OUT/${tag}_fork${ns}_sched_perf_5000.jsonl" 2>&1 || exit $?
done
python - "$OUT" "$tag" <<'PY'
import json, sys, glob
out, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{out}/{tag}_fork*_bench1024_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["config"]["p99_gang_admit_ms"])
for f in sorted(glob.glob(f"{out}/{tag}_fork*_sched_perf_5000.jsonl")):
    rows = [json.loads(l) for l in open(f) if l.startswith("{")]
    print(f.split("/")[-1], " ".join(f"{r['workload']}={r['pods_per_s']:.0f}" for r in rows))
PY
