#!/bin/bash
# r05 (end of round): profiles of HEAD -- $1 = c4: bench line, kernel trace, PMC passes, tile costs,
# strips, RT_COUNT work counts; $1 = c5: bench line, kernel trace, PMC passes
set -e
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
O=gpurun_out/r05h_$1
mkdir -p $O
if [ "$1" = c4 ]; then
  timeout -k 10 300 python bench.py > $O/bench_c4.json.log 2>&1
  grep -h '^{' $O/bench_c4.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C4', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
  bash tools/profile_gpu.sh r05c4h
  timeout -k 10 300 python tools/tile_costs.py gpu sphere1m 5 $O/tile_costs.npy > $O/tile_costs.log 2>&1
  timeout -k 10 300 python tools/strip_scaling.py --ranks 1 2 4 8 --steps 30 --all-ranks > $O/strips.log 2>&1
  grep bound $O/strips.log
  RT_LIB_PATH=_variants/librt_count.so timeout -k 10 300 python tools/count_gpu_work.py sphere1m seg > $O/work_counts.log 2>&1
else
  timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 > $O/bench_c5.json.log 2>&1
  grep -h '^{' $O/bench_c5.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C5', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
  bash tools/profile_gpu.sh r05c5h --config sphere1m_refl
  RT_LIB_PATH=_variants/librt_count.so timeout -k 10 400 python tools/count_gpu_work.py sphere1m_refl seg > $O/work_counts_c5.log 2>&1
fi
