#!/usr/bin/env bash
# Round-2 closing box session: GPU tier, smoke(), default bench, and the
# scheduler_perf PreemptionBasic rows at 500 / 5,000 nodes. Each GPU step has
# its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
tag=${1:-r2z}
mkdir -p "$OUT"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/${tag}_pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${tag}_smoke.log" 2>&1 || exit $?
timeout -k 10 240 python bench.py > "$OUT/${tag}_bench1.json" 2> "$OUT/${tag}_bench1.err" || exit $?
timeout -k 10 300 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 500 --pods 1000 --cpus l3 \
  --only PreemptionBasic Unschedulable > "$OUT/${tag}_sched_perf_500.jsonl" 2>&1 || exit $?
timeout -k 10 600 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 5000 --pods 5000 --cpus l3 \
  --only PreemptionBasic Unschedulable > "$OUT/${tag}_sched_perf_5000.jsonl" 2>&1 || exit $?
tail -1 "$OUT/${tag}_pytest_gpu.log"; tail -1 "$OUT/${tag}_smoke.log" | cut -c1-200
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['config']['p99_gang_admit_ms'])" "$OUT/${tag}_bench1.json"
cat "$OUT/${tag}_sched_perf_500.jsonl" "$OUT/${tag}_sched_perf_5000.jsonl" | cut -c1-200
