#!/bin/bash
# r05: work counts (C4, C5) on the current kernels, then C5's kernel split under rocprofv3
set -e
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 300 python tools/count_gpu_work.py sphere1m seg > $O/count_c4.log 2>&1
tail -1 $O/count_c4.log
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 400 python tools/count_gpu_work.py sphere1m_refl seg > $O/count_c5.log 2>&1
tail -1 $O/count_c5.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c5 -o c5 -- python bench.py --config sphere1m_refl --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/c5_bench.log 2>&1
f=$(find $O/c5 -name "*kernel_stats.csv" | head -1)
cut -d, -f1-5 "$f" | head -14
