#!/bin/bash
# r05: C5 kernel trace at HEAD (rocprofv3 --kernel-trace --stats, csv)
set -e
O=gpurun_out/r05c5t
mkdir -p $O
export TMPDIR=/tmp
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config sphere1m_refl --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/trace.log 2>&1
f=$(find $O/trace -name "run_kernel_stats.csv" | head -1)
cut -d, -f1-5 "$f" | head -8
