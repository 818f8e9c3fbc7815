# The scheduling loop's profile in a steady open-loop trial just under the
# capacity edge (no backlog): where the per-attempt time goes.
set -e
OUT=gpurun_out/${TAG:-r6z}
mkdir -p $OUT
SO=$(python -c "import flex_gpu_scheduler_amd._xsched as m; print(m.__file__)")
timeout -k 10 300 python scripts/sample_openloop.py $OUT --seed 0 --waves 16 --detail --sample-last --hz 4000 --sequence ${SEQ:-102371,106000}
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/openloop.samples --exe "$SO" --top 70 > $OUT/ol_steady_report.txt 2>&1
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/openloop.samples --exe "$SO" --timeline 50 --roles xs-sched,xs-informer,python,xs-bind > $OUT/ol_steady_timeline.txt 2>&1
rm -f $OUT/openloop.samples
