#!/bin/bash
# r05: strips at N = 1 / 8 (every rank) by frames in flight
set -e
O=gpurun_out/r05if2
mkdir -p $O
timeout -k 10 600 python tools/strip_scaling.py --ranks 1 8 --steps 30 --all-ranks --inflight 1 2 3 4 > $O/strips_inflight.log 2>&1
grep bound $O/strips_inflight.log
