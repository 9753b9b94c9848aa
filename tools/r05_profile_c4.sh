#!/bin/bash
# r05 C4 measurement: the bench line, rocprofv3 kernel trace + PMC passes, tile costs, strip bound,
# and the RT_COUNT build's work counts (logs in gpurun_out/r05c4)
set -u
OUT=gpurun_out/r05c4
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $OUT/bench.json.log 2>&1 || exit 1
bash tools/profile_gpu.sh r05 || exit 2
timeout -k 10 200 python tools/tile_costs.py gpu sphere1m 5 $OUT/tile_costs.npy > $OUT/tile_costs.log 2>&1 || exit 3
timeout -k 10 300 python tools/strip_scaling.py --ranks 1 2 4 8 --steps 30 --all-ranks > $OUT/strips.log 2>&1 || exit 4
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 300 python tools/count_gpu_work.py sphere1m seg > $OUT/work_counts.log 2>&1 || exit 5
