#!/bin/bash
# r05: the quick wide BVH resident for the frames after a geometry change -- the GPU suite, the first
# frame after set_object_transform (kernel and wall time, same image as after rt_finish_accel), C4 bench
set -e
O=gpurun_out/r05q2
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python tools/first_frame.py sphere1m 4 > $O/first_frame_quick.log 2>&1
RT_WBVH_QUICK_FIRST=0 timeout -k 10 300 python tools/first_frame.py sphere1m 2 > $O/first_frame_octree.log 2>&1
grep -h '^{' $O/first_frame_quick.log $O/first_frame_octree.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['set_object_transform_ms'], d['first_frame_kernel_ms'], d['first_frame_wall_ms'], d['wide_frame_kernel_ms'], d['same_image'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c4.json.log 2>&1
grep -h '^{' $O/bench_c4.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C4', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'), d.get('first_call_s'), d.get('build_ms'))"
