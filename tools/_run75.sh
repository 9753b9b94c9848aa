set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/strip_scaling.py --ranks 1 2 4 8 --inflight 1 2 3 > gpurun_out/r02_strips75.log 2>&1 || { cat gpurun_out/r02_strips75.log; exit 1; }
cat gpurun_out/r02_strips75.log
