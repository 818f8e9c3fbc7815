# Open-loop capacity: GPU-free child (default) vs the rank's own process, twice.
set -e
OUT=gpurun_out/${TAG:-r6h}
mkdir -p $OUT
for i in 1 2; do
  for mode in child inproc; do
    flag=""; [ $mode = inproc ] && flag="--open-loop-in-process"
    timeout -k 10 400 python bench.py $flag --no-service-mode --no-scenarios --no-placement --nodes1024-waves 0 > $OUT/ol_${mode}_$i.json 2>> $OUT/ol.err
    python -c "
import json; d=json.load(open('$OUT/ol_${mode}_$i.json')); c=d['config']; ol=c['gang_admit_open_loop']
print('$mode', $i, d['value'], c['open_loop_capacity_pods_per_s'], ol['load_90']['all_gangs']['p99_create_to_bound_ms'], c.get('deny_mode_open_loop_p99_create_to_bound_ms'), c.get('deny_mode_denied_gang_fraction'))
print('  ', [(t['offered_pods_per_s'], t['served'], t['p99_create_to_bound_ms']) for t in ol['capacity_search'][-6:]])"
  done
done
