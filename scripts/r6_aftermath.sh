# Is the open-loop trial after an overloaded one slower because of the
# overload (aftermath) or is the rate simply above capacity?
set -e
OUT=gpurun_out/${TAG:-r6i}
mkdir -p $OUT
run() { echo "== $*"; timeout -k 10 300 python scripts/sample_openloop.py $OUT --seed 0 --waves 16 "$@"; }
run --sequence 102371,109400,109400 | tee $OUT/seq_no_overload.txt
run --sequence 102371,130000,109400,109400 | tee $OUT/seq_overload.txt
run --sequence 102371,130000,109400,109400 --fresh-after 1 | tee $OUT/seq_overload_fresh_shard.txt
run --sequence 102371,116000,116000 | tee $OUT/seq_no_overload_116.txt
