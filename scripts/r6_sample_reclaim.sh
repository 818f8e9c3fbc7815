# PreemptionBasic vs CapacityScheduling-Reclaim at 5,000 nodes, plain and
# under the sampler (scheduling-thread profile of each).
set -e
OUT=gpurun_out/${TAG:-r6an}
mkdir -p $OUT
SO=$(python -c "import flex_gpu_scheduler_amd._xsched as m; print(m.__file__)")
timeout -k 10 600 python -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 5000 --pods 1000 --cpus l3 --only PreemptionBasic CapacityScheduling-Reclaim
for w in PreemptionBasic CapacityScheduling-Reclaim; do
  timeout -k 10 600 python scripts/sample_sched_perf.py $OUT $w --nodes 5000 --pods 1000
  timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/$w.samples --exe "$SO" --top 50 > $OUT/$w.report.txt 2>&1
  timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/$w.samples --exe "$SO" --timeline 100 --roles xs-sched,xs-filter,xs-informer,xs-bind,python > $OUT/$w.timeline.txt 2>&1 || true
  rm -f $OUT/$w.samples
done
