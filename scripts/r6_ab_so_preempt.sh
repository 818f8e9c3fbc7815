# A/B of two extension builds (ab_old/, ab_new/) on the scheduler_perf
# preemption rows at 5,000 nodes, alternated.
set -e
SO=flex_gpu_scheduler_amd/_xsched.cpython-310-x86_64-linux-gnu.so
for i in 1 2; do
  for v in old new; do
    cp ab_$v/_xsched.cpython-310-x86_64-linux-gnu.so $SO
    timeout -k 10 600 python -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 5000 --pods 1000 --cpus l3 --only PreemptionBasic CapacityScheduling-Reclaim | sed "s/^/$v /" | cut -c1-170
  done
done
cp ab_new/_xsched.cpython-310-x86_64-linux-gnu.so $SO
