set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/strip_scaling.py --ranks 1 8 16 64 135 > gpurun_out/r02_strips73a.log 2>&1 || { cat gpurun_out/r02_strips73a.log; exit 1; }
cat gpurun_out/r02_strips73a.log
RT_TILE_ORDER=1 timeout -k 10 300 python tools/strip_scaling.py --ranks 1 8 16 64 135 > gpurun_out/r02_strips73b.log 2>&1 || { cat gpurun_out/r02_strips73b.log; exit 1; }
cat gpurun_out/r02_strips73b.log
