# Sampler at 1,024 nodes with the -g1 extension (dbg/, same code): per-line
# hot spots of the informer's delete path.
set -e
OUT=gpurun_out/${TAG:-r6al}
mkdir -p $OUT
SO=$(python -c "import flex_gpu_scheduler_amd._xsched as m; print(m.__file__)")
cp dbg/$(basename "$SO") "$SO"
timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 1024 --waves 12 --tag n1024 --seed 0 --hz 2000
for f in handle_pod_deletes take_pods remove_pods remove_pod_locked "NodeInfo::remove_pod" "SchedulerCache::writable" informer_loop "Informers::group_remove" "move_all_to_active_or_backoff"; do
  echo "=== $f" >> $OUT/lines.txt
  timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/n1024.samples --exe "$SO" --lines "$f" --top 20 >> $OUT/lines.txt 2>&1 || true
done
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/n1024.samples --exe "$SO" --top 60 > $OUT/report.txt 2>&1 || true
rm -f $OUT/n1024.samples
