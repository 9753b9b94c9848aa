#!/bin/bash
# r05: waves per SIMD of refl_trace_kernel (RT_OCC_REFL_TRACE, build-time)
set -e
O=gpurun_out/r05occ
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name lib
  RT_LIB_PATH=$2 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
run o4 raytracercpp_amd/librt_mi355x.so
run o3 _variants/librt_ot3.so
run o5 _variants/librt_ot5.so
run o4b raytracercpp_amd/librt_mi355x.so
