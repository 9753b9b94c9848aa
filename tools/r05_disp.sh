#!/bin/bash
# r05: parallax mapping from a one-channel copy of the displacement map (RT_DISP_CHANNEL=1, default) or
# the RGBA texture; the GPU suite first
set -e
O=gpurun_out/r05disp
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name channel
  RT_DISP_CHANNEL=$2 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('max_abs_dpixel'))"
}
run ch1 1
run ch0 0
run ch1b 1
