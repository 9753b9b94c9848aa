set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/strip_scaling.py --all-ranks > gpurun_out/r02_strips72.log 2>&1 || { cat gpurun_out/r02_strips72.log; exit 1; }
cat gpurun_out/r02_strips72.log
