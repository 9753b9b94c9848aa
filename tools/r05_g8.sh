#!/bin/bash
# r05: lane groups of 8 for the deferred reflection queries at 2^27-slot chunks
set -e
O=gpurun_out/r05g8
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name lib defer
  RT_LIB_PATH=$2 RT_REFL_DEFER=$3 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
run g4_d32 raytracercpp_amd/librt_mi355x.so 32
run g8_d32 _variants/librt_g8.so 32
run g8_d24 _variants/librt_g8.so 24
run g4_d32b raytracercpp_amd/librt_mi355x.so 32
