#!/bin/bash
# r05: split tiles traced inside the plain kernel (trace_split_part): parity, bench and strips by knob
set -e
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_frames.py > $O/pytest_frames.log 2>&1
tail -1 $O/pytest_frames.log
for v in "0 0.5" "4 0.5" "4 0.25" "0 0.5" "4 0.5"; do
  set -- $v
  RT_HEAVY_GROUP=$1 RT_HEAVY_SPLIT=$2 timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_g$1_s$2.log 2>&1
  grep -h '^{' $O/bench_g$1_s$2.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('G=$1 split=$2', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
done
for v in "0 0.5" "4 0.5" "4 0.25"; do
  set -- $v
  RT_HEAVY_GROUP=$1 RT_HEAVY_SPLIT=$2 timeout -k 10 300 python tools/strip_scaling.py --ranks 1 2 4 8 --steps 30 --all-ranks > $O/strips_g$1_s$2.log 2>&1
  echo "G=$1 split=$2"; grep bound $O/strips_g$1_s$2.log
done
