#!/bin/bash
# r05, VERDICT r04 item 6: the C5 frame engine -- bench line, kernel trace and PMC passes
# (a heartbeat line every 30 s: a C5 frame takes seconds and the bench prints only at its end)
set -e
O=gpurun_out/r05c5
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 > $O/bench.json.log 2>&1
tail -1 $O/bench.json.log | cut -c1-300
bash tools/profile_gpu.sh r05c5 --config sphere1m_refl
