# CPU placement and binder count: burst waves (64 nodes) and open-loop trials
# near the edge, each variant twice, alternating. VARIANTS: "name|pin|optionsJSON;..."
set -e
OUT=gpurun_out/${TAG:-r6aa}
mkdir -p $OUT
IFS=';' read -ra VS <<< "$VARIANTS"
for i in 1 2; do
  for v in "${VS[@]}"; do
    IFS='|' read -r name pin opts <<< "$v"
    echo "$name burst $(timeout -k 10 300 python scripts/sample_bench_waves.py $OUT --nodes 64 --waves 32 --tag b_${name}_$i --seed 0 --hz 20 --pin $pin --options "$opts")"
    rm -f $OUT/b_${name}_$i.samples
    timeout -k 10 300 python scripts/sample_openloop.py $OUT/ol_${name}_$i --seed 0 --waves 16 --detail --pin $pin --options "$opts" --sequence ${SEQ:-102371,112000,117000} | sed "s/^/$name ol /" | cut -c1-200
  done
done
