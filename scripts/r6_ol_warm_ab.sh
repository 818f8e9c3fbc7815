# Is the first open-loop trial on a fresh (burst-warmed) shard slower than a
# later one? A: the trial straight after the burst warm-up, B: after a 60k
# open-loop trial. Each in its own process (a fresh shard), alternated.
set -e
OUT=gpurun_out/${TAG:-r6af}
mkdir -p $OUT
for i in 1 2 3; do
  echo "A $(timeout -k 10 300 python scripts/sample_openloop.py $OUT/a$i --seed 0 --waves 16 --sequence 109600 | cut -c1-150)"
  echo "B $(timeout -k 10 300 python scripts/sample_openloop.py $OUT/b$i --seed 0 --waves 16 --sequence 60000,109600 | tail -1 | cut -c1-150)"
done
