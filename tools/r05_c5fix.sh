#!/bin/bash
# r05: kernels read KParams in place (no per-lane scratch copy): GPU suite, C5 and C4 bench lines
set -e
O=gpurun_out/r05c5b
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 > $O/bench_c5.json.log 2>&1
grep -h '^{' $O/bench_c5.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C5', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_c4.json.log 2>&1
grep -h '^{' $O/bench_c4.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C4', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
