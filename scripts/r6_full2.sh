# One full default bench.py run (the driver's N=1 command) with its stderr progress.
set -e
mkdir -p gpurun_out/${TAG:-r6ae}
timeout -k 10 1000 python bench.py > gpurun_out/${TAG:-r6ae}/bench1.json 2> gpurun_out/${TAG:-r6ae}/bench1.err
tail -c 300 gpurun_out/${TAG:-r6ae}/bench1.json
