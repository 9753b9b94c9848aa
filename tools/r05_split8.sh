#!/bin/bash
# r05: the quick tree (GPU suite, first frame) and the split tiles with 8 lanes per pixel (4 x 2 pixel
# parts, the RT_SPLIT_G=8 variant) against the default 4: frames parity, C4 bench, strips
set -e
O=gpurun_out/r05s8
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
    d = json.loads(l); print('first frame', d['set_object_transform_ms'], d['first_frame_kernel_ms'], d['first_frame_wall_ms'], d['wide_frame_kernel_ms'], d['same_image'])"
RT_LIB_PATH=_variants/librt_split8.so timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_frames.py -k "heavy" > $O/pytest_split8.log 2>&1
tail -1 $O/pytest_split8.log
for v in default split8 default split8; do
  if [ $v = default ]; then L=raytracercpp_amd/librt_mi355x.so; else L=_variants/librt_$v.so; fi
  RT_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_$v.log 2>&1
  grep -h '^{' $O/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
done
for v in default split8; do
  if [ $v = default ]; then L=raytracercpp_amd/librt_mi355x.so; else L=_variants/librt_$v.so; fi
  RT_LIB_PATH=$L timeout -k 10 300 python tools/strip_scaling.py --ranks 1 2 4 8 --steps 30 --all-ranks > $O/strips_$v.log 2>&1
  echo $v; grep bound $O/strips_$v.log
done
