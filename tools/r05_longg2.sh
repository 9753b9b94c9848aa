#!/bin/bash
# r05: second pass of tools/r05_longg.sh around the best points
set -e
O=gpurun_out/r05g2
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name lib defer
  RT_LIB_PATH=$2 RT_REFL_DEFER=$3 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
L=raytracercpp_amd/librt_mi355x.so
run g4_d32 $L 32
run g8_d32 _variants/librt_lg8.so 32
run g8_d24 _variants/librt_lg8.so 24
run g4_d40 $L 40
run g8_d40 _variants/librt_lg8.so 40
run g4_d28 $L 28
run g4_d32b $L 32
run g8_d32b _variants/librt_lg8.so 32
