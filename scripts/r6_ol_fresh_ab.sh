# After an overloaded trial, a fresh shard in the same process: without and
# with a settle (old shard dropped, 1 s wait, malloc_trim) before the new one.
set -e
OUT=gpurun_out/${TAG:-r6ag}
mkdir -p $OUT
for i in 1 2; do
  for st in 0 1; do
    timeout -k 10 300 python scripts/sample_openloop.py $OUT/s${st}_$i --seed 0 --waves 16 --fresh-after 1 --settle $st --sequence 102371,131000,109600,109600 | sed "s/^/settle=$st /" | cut -c1-150
  done
done
