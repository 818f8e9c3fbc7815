# 1,024-node waves under fork thresholds (XSCHED_MIN_PARALLEL_NS), alternated.
set -e
OUT=gpurun_out/${TAG:-r6p}
mkdir -p $OUT
for i in 1 2; do
  for v in ${VALUES:-default 120000 250000 1000000000}; do
    if [ $v = default ]; then unset XSCHED_MIN_PARALLEL_NS; else export XSCHED_MIN_PARALLEL_NS=$v; fi
    echo "$v $(timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 1024 --waves 12 --tag w_${v}_$i --seed 0 --hz 50)"
    rm -f $OUT/w_${v}_$i.samples
  done
done
