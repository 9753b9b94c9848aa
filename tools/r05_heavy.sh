#!/bin/bash
# r05: the split tiles (ray_trace_heavy_kernel on a side stream): parity, bench by group / split,
# strips and tile costs
set -e
O=gpurun_out/r05h2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_frames.py > $O/pytest_frames.log 2>&1
tail -1 $O/pytest_frames.log
for v in "4 0.5" "0 0.5" "4 0.25" "2 0.5" "4 1.0" "4 0.5"; do
  set -- $v
  RT_HEAVY_GROUP=$1 RT_HEAVY_SPLIT=$2 timeout -k 10 240 python bench.py > $O/bench_g$1_s$2.log 2>&1
  grep -h '^{' $O/bench_g$1_s$2.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('G=$1 split=$2', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
done
for v in "4 0.5" "0 0.5" "4 0.25"; do
  set -- $v
  RT_HEAVY_GROUP=$1 RT_HEAVY_SPLIT=$2 timeout -k 10 300 python tools/strip_scaling.py --ranks 1 2 4 8 --steps 30 --all-ranks > $O/strips_g$1_s$2.log 2>&1
  echo "G=$1 split=$2"; grep bound $O/strips_g$1_s$2.log
done
RT_HEAVY_GROUP=4 timeout -k 10 240 python tools/tile_costs.py gpu sphere1m 5 $O/tc_g4.npy > $O/tile_costs_g4.log 2>&1
head -4 $O/tile_costs_g4.log
