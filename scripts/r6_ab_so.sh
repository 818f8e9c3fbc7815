# A/B of two builds of the extension (ab_old/, ab_new/), alternated on one box:
# burst waves (64 nodes) and open-loop trials near the capacity edge.
set -e
OUT=gpurun_out/${TAG:-r6ab}
mkdir -p $OUT
SO=flex_gpu_scheduler_amd/_xsched.cpython-310-x86_64-linux-gnu.so
for i in 1 2; do
  for v in old new; do
    cp ab_$v/_xsched.cpython-310-x86_64-linux-gnu.so $SO
    echo "$v burst $(timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 64 --waves 32 --tag b_${v}_$i --seed 0 --hz 20)"
    rm -f $OUT/b_${v}_$i.samples
    timeout -k 10 300 python scripts/sample_openloop.py $OUT/ol_${v}_$i --seed 0 --waves 16 --detail --sequence ${SEQ:-102371,112000,117000,122000} | sed "s/^/$v ol /" | cut -c1-170
  done
done
cp ab_new/_xsched.cpython-310-x86_64-linux-gnu.so $SO
