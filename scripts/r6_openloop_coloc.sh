# Open-loop trials (no overload first) with gangColocation None vs Preferred.
set -e
OUT=gpurun_out/${TAG:-r6l}
mkdir -p $OUT
for i in 1 2; do
  for m in None Preferred; do
    echo "== $m $i"
    timeout -k 10 300 python scripts/sample_openloop.py $OUT --seed 0 --waves 16 --colocation $m --sequence 102371,109400,116000,122000 | tee $OUT/seq_${m}_$i.txt
  done
done
