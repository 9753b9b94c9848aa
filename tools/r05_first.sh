#!/bin/bash
# r05: the first frame after a geometry change on the octree specialisation:
# parity of the octree-path frames, first-frame kernel time by occupancy variant
set -e
O=gpurun_out/r05ff
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread -k "octree or frame_modes or async or transform or golden or exact" > $O/pytest_oct.log 2>&1
tail -1 $O/pytest_oct.log
for v in default oct4 oct6; do
  if [ $v = default ]; then L=raytracercpp_amd/librt_mi355x.so; else L=_variants/librt_$v.so; fi
  RT_LIB_PATH=$L timeout -k 10 300 python tools/first_frame.py sphere1m 3 > $O/first_$v.log 2>&1
  echo $v; grep '^{' $O/first_$v.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(' ', d['first_frame_kernel_ms'], d['first_frame_wall_ms'], d['wide_frame_kernel_ms'], d['same_image'])"
done
