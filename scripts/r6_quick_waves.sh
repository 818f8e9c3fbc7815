# Quick sanity of the current build: burst waves (64 nodes) and 1,024-node waves.
set -e
OUT=gpurun_out/${TAG:-r6av}
mkdir -p $OUT
echo "burst $(timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 64 --waves 48 --tag b --seed 0 --hz 20)"
echo "n1024 $(timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 1024 --waves 12 --tag n --seed 0 --hz 20)"
rm -f $OUT/*.samples
