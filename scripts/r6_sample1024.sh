# 1,024-node headline waves under the sampler (Preferred), report on the box.
set -e
OUT=gpurun_out/${TAG:-r6g}
mkdir -p $OUT
SO=$(python -c "import flex_gpu_scheduler_amd._xsched as m; print(m.__file__)")
timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 1024 --waves 12 --colocation ${COLOC:-Preferred} --tag n1024 --seed 0 --hz 2000
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/n1024.samples --exe "$SO" --top 70 > $OUT/n1024_report.txt 2>&1
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/n1024.samples --exe "$SO" --timeline 5 --roles xs-sched,xs-bind,xs-informer,python > $OUT/n1024_timeline.txt 2>&1 || true
rm -f $OUT/n1024.samples
