# Sampler on a 109.4k trial: fresh vs right after an overloaded 130k trial.
set -e
OUT=gpurun_out/${TAG:-r6j}
mkdir -p $OUT/a $OUT/b
SO=$(python -c "import flex_gpu_scheduler_amd._xsched as m; print(m.__file__)")
timeout -k 10 300 python scripts/sample_openloop.py $OUT/a --seed 0 --waves 16 --sequence 102371,109400 --sample-last | tee $OUT/a/seq.txt
timeout -k 10 300 python scripts/sample_openloop.py $OUT/b --seed 0 --waves 16 --sequence 102371,130000,109400 --sample-last | tee $OUT/b/seq.txt
for d in a b; do
  timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.sample_report $OUT/$d/openloop.samples --exe "$SO" --top 50 > $OUT/$d/report.txt 2>&1
  rm -f $OUT/$d/openloop.samples
done
