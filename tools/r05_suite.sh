#!/bin/bash
# r05: the GPU suite, then C4 (default) and C5 bench lines with their parity checks
set -e
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_c4.log 2>&1
grep -h '^{' $O/bench_c4.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('c4', d['value'], d['ms_per_step'], d.get('roofline',{}).get('achieved'), d.get('check'))"
timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_c5.log 2>&1
grep -h '^{' $O/bench_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('c5', d['value'], d['ms_per_step'], d.get('check'))"
# lanes per sample in the main reflection trace kernel (build-time RT_REFL_G)
run() {   # name lib defer
  RT_LIB_PATH=$2 RT_REFL_DEFER=$3 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
if [ -f _variants/librt_rg2.so ]; then
  RT_LIB_PATH=_variants/librt_rg2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_frames.py -k deferral > $O/pytest_rg2.log 2>&1
  tail -1 $O/pytest_rg2.log
  run rg2_d32 _variants/librt_rg2.so 32
  run rg2_d64 _variants/librt_rg2.so 64
  run rg4_d32 _variants/librt_rg4.so 32
  run rg4_d64 _variants/librt_rg4.so 64
  run rg1_d32 raytracercpp_amd/librt_mi355x.so 32
fi
