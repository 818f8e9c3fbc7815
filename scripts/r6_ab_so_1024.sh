# A/B of two builds of the extension (ab_old/, ab_new/), alternated on one box:
# burst waves (64 nodes) and 1,024-node waves.
set -e
OUT=gpurun_out/${TAG:-r6ak}
mkdir -p $OUT
python -c "f=open('/proc/cpuinfo').read(); print('cpu flags:', {k: (k in f) for k in ('avx2','bmi2','fma','avx512f')})"
SO=flex_gpu_scheduler_amd/_xsched.cpython-310-x86_64-linux-gnu.so
for i in 1 2; do
  for v in old new; do
    cp ab_$v/_xsched.cpython-310-x86_64-linux-gnu.so $SO
    echo "$v burst $(timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 64 --waves 32 --tag b_${v}_$i --seed 0 --hz 20)"
    echo "$v n1024 $(timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 1024 --waves 12 --tag n_${v}_$i --seed 0 --hz 20)"
    rm -f $OUT/*.samples
  done
done
cp ab_old/_xsched.cpython-310-x86_64-linux-gnu.so $SO
