#!/bin/bash
# r05: C5 variants (default / shadow pass's octree fallback in line / reflection kernels at 5 waves per SIMD)
set -e
O=gpurun_out/r05c5v
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
for v in default shinl occ5 default; do
  if [ $v = default ]; then L=raytracercpp_amd/librt_mi355x.so; else L=_variants/librt_$v.so; fi
  RT_LIB_PATH=$L timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$v.json.log 2>&1
  grep -h '^{' $O/bench_$v.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
