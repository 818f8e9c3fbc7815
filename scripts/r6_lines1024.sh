# Sampler at 1,024 nodes with the -g1 extension (dbg/, same code): per-line
# hot spots and allocation callers of the scheduling thread.
set -e
OUT=gpurun_out/${TAG:-r6n}
mkdir -p $OUT
SO=$(python -c "import flex_gpu_scheduler_amd._xsched as m; print(m.__file__)")
cp dbg/$(basename "$SO") "$SO"
timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 1024 --waves 12 --tag n1024 --seed 0 --hz 2000
timeout -k 10 300 python scripts/alloc_callers.py $OUT/n1024.samples "$SO" xs-sched > $OUT/alloc_sched.txt
for f in find_nodes_that_fit run_score schedule_cycle "Coscheduling::permit" "Coscheduling::pre_filter" "FlexGPU::reserve" "SchedulerCache::assume_pod" "TopologyMatch::score_many" "place_memory" "WaitingPods::add" "TopologyMatch::filter_impl"; do
  echo "=== $f" >> $OUT/lines.txt
  timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/n1024.samples --exe "$SO" --lines "$f" --top 25 >> $OUT/lines.txt 2>&1 || true
  echo "=== callers of $f" >> $OUT/lines.txt
  timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/n1024.samples --exe "$SO" --callers "$f" --top 15 >> $OUT/lines.txt 2>&1 || true
done
rm -f $OUT/n1024.samples
