#!/bin/bash
# r05: wave-adaptive deferral (W_LONG_FEW lanes left past W_LONG_MIN iterations: stop them too)
set -e
O=gpurun_out/r05few
mkdir -p $O
RT_LIB_PATH=_variants/librt_f8m8.so timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_frames.py tests/test_gpu_parity.py -k "deferral or c5" > $O/pytest_f8m8.log 2>&1
tail -1 $O/pytest_f8m8.log
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name lib
  RT_LIB_PATH=$2 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
run base raytracercpp_amd/librt_mi355x.so
run f8m12 _variants/librt_f8m12.so
run f16m12 _variants/librt_f16m12.so
run f8m8 _variants/librt_f8m8.so
run f4m16 _variants/librt_f4m16.so
