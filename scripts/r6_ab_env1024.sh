# 1,024-node waves under alternating environments. VARIANTS: "name|VAR=v VAR2=v;name2|..."
set -e
OUT=gpurun_out/${TAG:-r6s}
mkdir -p $OUT
IFS=';' read -ra VS <<< "$VARIANTS"
for i in 1 2; do
  for v in "${VS[@]}"; do
    name=${v%%|*}; envs=${v#*|}
    echo "$name $(env $envs timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 1024 --waves 12 --tag w_${name}_$i --seed 0 --hz 50)"
    rm -f $OUT/w_${name}_$i.samples
  done
done
