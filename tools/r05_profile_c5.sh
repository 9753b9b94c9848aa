#!/bin/bash
# r05, VERDICT r04 item 6: the C5 frame engine -- bench line, kernel trace and PMC passes
set -e
O=gpurun_out/r05c5
mkdir -p $O
timeout -k 10 400 python bench.py --config sphere1m_refl > $O/bench.json.log 2>&1
tail -1 $O/bench.json.log | cut -c1-300
bash tools/profile_gpu.sh r05c5 --config sphere1m_refl
