# Open-loop trials near the cliff with per-type p99s, generator lags and the
# 5-ms timeline (in flight, held, attempts, unschedulable, parks).
set -e
OUT=gpurun_out/${TAG:-r6v}
mkdir -p $OUT
timeout -k 10 300 python scripts/sample_openloop.py $OUT --seed 0 --waves 16 --detail --sequence ${SEQ:-102371,112000,112000,117000,117000}
