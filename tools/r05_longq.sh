#!/bin/bash
# r05: refl_trace_long_kernel's batches from a ticket (default) or a fixed grid stride; parity first
set -e
O=gpurun_out/r05q
mkdir -p $O
RT_LIB_PATH=_variants/librt_lq1.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_frames.py -k deferral > $O/pytest_deferral.log 2>&1
tail -1 $O/pytest_deferral.log
RT_LIB_PATH=_variants/librt_lq1.so timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "c5" > $O/pytest_c5.log 2>&1
tail -1 $O/pytest_c5.log
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name lib defer
  RT_LIB_PATH=$2 RT_REFL_DEFER=$3 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
L=_variants/librt_lq1.so
run q1_d32 $L 32
run q0_d32 raytracercpp_amd/librt_mi355x.so 32
run q1_d24 $L 24
run q1_d16 $L 16
run q1_d32b $L 32
