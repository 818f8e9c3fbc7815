#!/usr/bin/env bash
# One MI355X box session. Usage: bash scripts/gpu_session.sh TAG step [step ...]
# steps: pytest smoke bench bench3 nodes1024 ab1024 abbin1024 sample1024 timeline1024 pmc sched500 sched5000 remote sample_pre sample_sched
#        sample_bench rocprof
# Every GPU step runs under its own time limit; the script stops at the first
# failure (no retries). A heartbeat line every 60 s keeps long steps visible.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
OUT=gpurun_out/$tag
mkdir -p "$OUT"
( while sleep 60; do echo "[$tag] heartbeat $(date +%T)"; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
for step in "$@"; do
  echo "[$tag] $step $(date +%T)"
  case $step in
    pytest) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
              > "$OUT/pytest_gpu.txt" 2>&1 ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 ;;
    bench) timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench1.json" \
             2> "$OUT/bench1.err" ;;
    bench3) for i in 1 2 3; do
              timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-scenarios --no-placement \
                --no-service-mode > "$OUT/bench64_$i.json" 2> "$OUT/bench64_$i.err" || exit $?
            done ;;
    bench_r3shape)
      # The round-3 measurement shape (20 timed single-wave steps) next to the
      # default 16-wave steps, same tree and box.
      for i in 1 2; do
        timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --waves-per-step 1 --no-scenarios --no-placement \
          --no-service-mode --no-open-loop > "$OUT/bench_r3shape_$i.json" 2> "$OUT/bench_r3shape_$i.err" || exit $?
      done ;;
    benchab)
      # A/B of an env toggle (AB_VAR, AB_VALUES) on the default 64-node bench
      # (open-loop capacity included), alternating 2x.
      var=${AB_VAR:-XSCHED_PARSE_POOL}
      for i in 1 2; do
        for v in ${AB_VALUES:-0 1}; do
          env "$var=$v" timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-scenarios --no-placement \
            --no-service-mode > "$OUT/benchab_${var}_${v}_$i.json" 2> "$OUT/benchab_${var}_${v}_$i.err" || exit $?
        done
      done ;;
    treeab)
      # A/B of two trees on one box: ./abtree (an older commit, built in
      # place) against this tree, default 64-node bench and 1,024 nodes.
      for i in 1 2 3; do
        for t in abtree .; do
          which=$( [ "$t" = . ] && echo cur || echo old )
          (cd "$t" && timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-scenarios --no-placement \
            --no-service-mode) > "$OUT/treeab_${which}_64_$i.json" 2> "$OUT/treeab_${which}_64_$i.err" || exit $?
          (cd "$t" && timeout -k 10 300 python3 bench.py --nodes 1024 --steps 4 --warmup 1 --no-scenarios --no-placement \
            --no-service-mode --no-open-loop) > "$OUT/treeab_${which}_1024_$i.json" 2> "$OUT/treeab_${which}_1024_$i.err" || exit $?
        done
      done ;;
    tune)
      # Probe variant sweep (unroll x cache policy x workgroups/CU) per mode at
      # the default 2 GiB working set.
      timeout -k 10 400 python3 -c "import json; from flex_gpu_scheduler_amd.ops.hip_probe import probe; p = probe(); print(json.dumps([p.tune(mode=m, iters=10) for m in ('read', 'write', 'copy', 'triad')]))" \
        > "$OUT/tune.json" 2> "$OUT/tune.err" ;;
    treeab1024ol)
      # A/B of two trees on one box (./abtree, an older commit built in place,
      # against this tree): the 1,024-node bench with its open-loop search.
      for i in 1 2; do
        for t in abtree .; do
          which=$( [ "$t" = . ] && echo cur || echo old )
          (cd "$t" && timeout -k 10 400 python3 bench.py --nodes 1024 --steps 4 --warmup 1 --no-scenarios \
            --no-placement --no-service-mode --nodes1024-waves 0) > "$OUT/treeab1024ol_${which}_$i.json" \
            2> "$OUT/treeab1024ol_${which}_$i.err" || exit $?
        done
      done ;;
    nodes1024_3) for i in 1 2 3; do
                   timeout -k 10 400 python3 bench.py --nodes 1024 --steps 4 --warmup 1 --no-scenarios --no-placement \
                     --no-service-mode > "$OUT/bench_nodes_1024_$i.json" 2> "$OUT/bench_nodes_1024_$i.err" || exit $?
                 done ;;
    nodes1024) timeout -k 10 400 python3 bench.py --nodes 1024 --steps 4 --warmup 1 --no-scenarios --no-placement \
                 --no-service-mode > "$OUT/bench_nodes_1024.json" 2> "$OUT/bench_nodes_1024.err" ;;
    pmc) OUTDIR="$OUT" bash scripts/pmc_round.sh ;;
    probe_timing) OUTDIR="$OUT" bash scripts/probe_timing.sh ;;
    sched500) timeout -k 10 400 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 500 --pods 1000 \
                --cpus l3 > "$OUT/sched_perf_500.jsonl" 2>&1 ;;
    sched5000) timeout -k 10 700 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 5000 --pods 5000 \
                --cpus l3 > "$OUT/sched_perf_5000.jsonl" 2>&1 ;;
    schedperf_capacity)
      timeout -k 10 600 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 5000 --pods 5000 --cpus l3 \
        --only SchedulingBasic CapacityScheduling-Admission > "$OUT/sched_perf_capacity_5000.jsonl" 2>&1 &&
      timeout -k 10 600 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 5000 --pods 1000 --cpus l3 \
        --only PreemptionBasic CapacityScheduling-Reclaim >> "$OUT/sched_perf_capacity_5000.jsonl" 2>&1 ;;
    remote) timeout -k 10 600 python -u -m flex_gpu_scheduler_amd.tools.remote_bench --matrix > "$OUT/remote_bench.jsonl" \
              2>&1 ;;
    sample_pre|sample_sched)
      # Wall-clock thread sampler of the native stress driver
      # (abbin/xsched_stress_prof = build_ext.build_prof output; symbolized
      # here with tools/sample_report.py against the same binary).
      wl=PreemptionBasic; pods=2000
      [ "$step" = sample_sched ] && { wl=SchedulingBasic; pods=5000; }
      python -m flex_gpu_scheduler_amd.tools.stress "/tmp/s_$wl" --workload "$wl" --nodes 5000 --pods "$pods" &&
      cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))") &&
      XSCHED_SAMPLE_HZ=2000 XSCHED_SAMPLE="$OUT/$wl.samples" timeout -k 5 300 taskset -c "$cpus" \
        abbin/xsched_stress_prof "/tmp/s_$wl" 1 > "$OUT/$wl.sample_run.txt" 2>&1 ;;
    sample_bench)
      # The headline bench waves (64 nodes, 40 waves) under the sampler.
      python -m flex_gpu_scheduler_amd.tools.stress /tmp/s_bench --nodes 64 &&
      cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))") &&
      XSCHED_SAMPLE_HZ=2000 XSCHED_SAMPLE="$OUT/bench.samples" timeout -k 5 300 taskset -c "$cpus" \
        abbin/xsched_stress_prof /tmp/s_bench 40 > "$OUT/bench.sample_run.txt" 2>&1 ;;
    ab1024)
      # A/B of an env toggle (AB_VAR, default XSCHED_GANG_WINDOW) on the
      # 1,024-node bench waves in the native stress driver (abbin/xsched_stress),
      # pinned to one idle L3 domain, alternating 3x.
      var=${AB_VAR:-XSCHED_GANG_WINDOW}
      python -m flex_gpu_scheduler_amd.tools.stress /tmp/s_1024 --nodes 1024 &&
      cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))") &&
      for i in 1 2 3; do
        for v in ${AB_VALUES:-0 1}; do
          echo "$var=$v $(env "$var=$v" timeout -k 5 200 taskset -c "$cpus" abbin/xsched_stress /tmp/s_1024 6 | tail -1)" \
            >> "$OUT/ab1024.txt" || exit 1
        done
      done ;;
    abbin1024)
      # A/B of two stress binaries (abbin/xsched_stress_base vs abbin/xsched_stress)
      # on the 1,024-node bench waves, same CPU domain, alternating 3x.
      python -m flex_gpu_scheduler_amd.tools.stress /tmp/s_1024 --nodes 1024 &&
      cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))") &&
      for i in 1 2 3; do
        for b in xsched_stress_base xsched_stress; do
          echo "$b $(timeout -k 5 200 taskset -c "$cpus" abbin/$b /tmp/s_1024 6 | tail -1)" >> "$OUT/abbin1024.txt" || exit 1
        done
      done ;;
    abbin64)
      # The same binary A/B on the 64-node headline waves (40 waves).
      python -m flex_gpu_scheduler_amd.tools.stress /tmp/s_bench --nodes 64 &&
      cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))") &&
      for i in 1 2 3; do
        for b in xsched_stress_base xsched_stress; do
          echo "$b $(timeout -k 5 200 taskset -c "$cpus" abbin/$b /tmp/s_bench 40 | tail -1)" >> "$OUT/abbin64.txt" || exit 1
        done
      done ;;
    sample64)
      python -m flex_gpu_scheduler_amd.tools.stress /tmp/s_bench --nodes 64 &&
      cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))") &&
      XSCHED_SAMPLE_HZ=4000 XSCHED_SAMPLE="$OUT/n64.samples" timeout -k 5 200 taskset -c "$cpus" \
        abbin/xsched_stress /tmp/s_bench 160 > "$OUT/n64.sample_run.txt" 2>&1 &&
      python -m flex_gpu_scheduler_amd.tools.sample_report "$OUT/n64.samples" --exe abbin/xsched_stress --top 40 \
        > "$OUT/n64_samples.txt" 2>&1 && rm -f "$OUT/n64.samples" ;;
    sample1024)
      python -m flex_gpu_scheduler_amd.tools.stress /tmp/s_1024 --nodes 1024 &&
      cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))") &&
      XSCHED_SAMPLE_HZ=2000 XSCHED_SAMPLE="$OUT/n1024.samples" timeout -k 5 200 taskset -c "$cpus" \
        abbin/xsched_stress /tmp/s_1024 6 > "$OUT/n1024.sample_run.txt" 2>&1 &&
      python -m flex_gpu_scheduler_amd.tools.sample_report "$OUT/n1024.samples" --exe abbin/xsched_stress --top 40 \
        > "$OUT/n1024_samples.txt" 2>&1 && rm -f "$OUT/n1024.samples" ;;
    timeline64)
      # The 64-node headline waves under the timestamped sampler (samples kept
      # for window reports; symbolize against abbin/xsched_stress).
      python -m flex_gpu_scheduler_amd.tools.stress /tmp/s_bench --nodes 64 &&
      cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))") &&
      XSCHED_SAMPLE_HZ=4000 XSCHED_SAMPLE="$OUT/t64.samples" timeout -k 5 200 taskset -c "$cpus" \
        abbin/xsched_stress /tmp/s_bench 40 > "$OUT/t64.sample_run.txt" 2>&1 &&
      python -m flex_gpu_scheduler_amd.tools.sample_report "$OUT/t64.samples" --exe abbin/xsched_stress --timeline 2 \
        --roles xs-sched,xs-informer,xsched_stress,xs-bind > "$OUT/t64_timeline.txt" 2>&1 &&
      python -m flex_gpu_scheduler_amd.tools.sample_report "$OUT/t64.samples" --exe abbin/xsched_stress --top 60 \
        > "$OUT/t64_samples.txt" 2>&1 ;;
    timeline1024)
      # The 1,024-node waves under the timestamped sampler: per 5-ms bin and
      # thread role, the busy share and the top own-code frame (wave start-up,
      # scheduling, deletion drain).
      python -m flex_gpu_scheduler_amd.tools.stress /tmp/s_1024 --nodes 1024 &&
      cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))") &&
      XSCHED_SAMPLE_HZ=4000 XSCHED_SAMPLE="$OUT/t1024.samples" timeout -k 5 200 taskset -c "$cpus" \
        abbin/xsched_stress /tmp/s_1024 4 > "$OUT/t1024.sample_run.txt" 2>&1 &&
      python -m flex_gpu_scheduler_amd.tools.sample_report "$OUT/t1024.samples" --exe abbin/xsched_stress --timeline 5 \
        --roles xs-sched,xs-informer,xsched_stress,xs-bind > "$OUT/t1024_timeline.txt" 2>&1 &&
      python -m flex_gpu_scheduler_amd.tools.sample_report "$OUT/t1024.samples" --exe abbin/xsched_stress --top 40 \
        > "$OUT/t1024_samples.txt" 2>&1 ;;
    rocprof)
      # Kernel trace + per-kernel stats of one short bench run (the probe,
      # health, MFMA and placement kernels on the GPU path).
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_bench" -o bench -- \
        python3 bench.py --steps 5 --warmup 1 --no-open-loop --no-scenarios --no-service-mode \
        > "$OUT/rocprof_bench.log" 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "[$tag] $step rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
echo "[$tag] done"
