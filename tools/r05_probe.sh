#!/bin/bash
# r05 GPU probe: variant benches, tile costs and the strip bound of the default build (logs in gpurun_out/r05)
mkdir -p gpurun_out/r05
timeout -k 10 400 python tools/variants.py run base c10 c12 -- --steps 50 > gpurun_out/r05/variants.log 2>&1 || exit 1
timeout -k 10 200 python tools/tile_costs.py gpu sphere1m 5 gpurun_out/r05/tile_costs.npy > gpurun_out/r05/tile_costs.log 2>&1 || exit 1
timeout -k 10 300 python tools/strip_scaling.py --ranks 1 2 4 8 --steps 30 --all-ranks > gpurun_out/r05/strips.log 2>&1 || exit 1
