#!/bin/bash
# r05: the GPU suite and the C5 bench line at the default chunk (2^27 slots)
set -e
O=gpurun_out/r05chunk3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 > $O/bench_c5.json.log 2>&1
grep -h '^{' $O/bench_c5.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C5', d['value'], d['ms_per_step'], d.get('max_abs_dpixel'), d['cpu_baseline'].get('value'))"
