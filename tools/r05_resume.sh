#!/bin/bash
# r05: deferred reflection queries continued (RT_REFL_RESUME=1, default) or restarted; parity first
set -e
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_frames.py -k deferral > $O/pytest_deferral.log 2>&1
tail -1 $O/pytest_deferral.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "c5" > $O/pytest_c5.log 2>&1
tail -1 $O/pytest_c5.log
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name lib defer resume
  RT_LIB_PATH=$2 RT_REFL_DEFER=$3 RT_REFL_RESUME=$4 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
L=raytracercpp_amd/librt_mi355x.so
run res_d32 $L 32 1
run nores_d32 $L 32 0
run res_d16 $L 16 1
run res_d24 $L 24 1
run ol2_d32 _variants/librt_ol2.so 32 1
run ol3_d32 _variants/librt_ol3.so 32 1
run res_d32b $L 32 1
