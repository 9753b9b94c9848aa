#!/bin/bash
# r05: C5 by the lane group of the deferred reflection queries (RT_REFL_LONG_G, build-time) and the
# deferral threshold (RT_REFL_DEFER)
set -e
O=gpurun_out/r05g
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name lib defer
  RT_LIB_PATH=$2 RT_REFL_DEFER=$3 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
L=raytracercpp_amd/librt_mi355x.so
run g4_d48 $L 48
run g1_d48 _variants/librt_lg1.so 48
run g2_d48 _variants/librt_lg2.so 48
run g8_d48 _variants/librt_lg8.so 48
run g4_d24 $L 24
run g4_d16 $L 16
run g8_d16 _variants/librt_lg8.so 16
run g4_d32 $L 32
run g4_d48b $L 48
