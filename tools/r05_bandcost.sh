#!/bin/bash
set -e
O=gpurun_out/r05bc
mkdir -p $O
RT_HEAVY_GROUP=4 timeout -k 10 300 python tools/band_tile_costs.py sphere1m 8 > $O/g4.log 2>&1
RT_HEAVY_GROUP=0 timeout -k 10 300 python tools/band_tile_costs.py sphere1m 8 > $O/g0.log 2>&1
grep N= $O/g4.log $O/g0.log
