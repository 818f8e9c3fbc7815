# A saturated open-loop trial under the sampler, with a per-thread timeline
# (which stage of the pipeline is busy when the backlog grows).
set -e
OUT=gpurun_out/${TAG:-r6w}
mkdir -p $OUT
SO=$(python -c "import flex_gpu_scheduler_amd._xsched as m; print(m.__file__)")
timeout -k 10 300 python scripts/sample_openloop.py $OUT --seed 0 --waves 16 --detail --sample-last --hz 2000 --sequence ${SEQ:-102371,117000,117000}
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/openloop.samples --exe "$SO" --timeline 20 --roles xs-sched,xs-informer,python,xs-bind,xs-reaper > $OUT/ol_timeline.txt 2>&1
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/openloop.samples --exe "$SO" --top 50 > $OUT/ol_report.txt 2>&1
rm -f $OUT/openloop.samples
# The headline burst waves (64 nodes) under the sampler, for comparison.
timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 64 --waves 16 --tag burst64 --seed 0 --hz 4000
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/burst64.samples --exe "$SO" --top 70 > $OUT/burst64_report.txt 2>&1
rm -f $OUT/burst64.samples
