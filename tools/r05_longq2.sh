#!/bin/bash
# r05: the GPU suite on the ticketed long kernel (default), then C5 around it (group 8, thresholds)
set -e
O=gpurun_out/r05q2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name lib defer
  RT_LIB_PATH=$2 RT_REFL_DEFER=$3 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
L=raytracercpp_amd/librt_mi355x.so
run g4_d32 $L 32
run g8_d32 _variants/librt_g8q.so 32
run g4_d40 $L 40
run g4_d48 $L 48
run g8_d48 _variants/librt_g8q.so 48
run g4_d32b $L 32
