# rocprofv3 kernel trace + stats of a short bench.py run (the GPU probes and
# the placement check are the bench's GPU work); rocpd db under gpurun_out/.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6ar_rocprof_bench
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6ar_rocprof_bench -o bench -- python3 $R/bench.py --steps 5 --warmup 1 --no-open-loop --no-scenarios --no-service-mode > $R/gpurun_out/r6ar_rocprof_bench/bench.log 2>&1
tail -c 200 $R/gpurun_out/r6ar_rocprof_bench/bench.log
