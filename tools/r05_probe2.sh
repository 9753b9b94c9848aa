#!/bin/bash
# r05 GPU probe 2: camera QS variants' tile costs and strip bounds; hair1m and robot benches
mkdir -p gpurun_out/r05
for v in c10 c12; do
  RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 200 python tools/tile_costs.py gpu sphere1m 5 gpurun_out/r05/tile_costs_$v.npy > gpurun_out/r05/tile_costs_$v.log 2>&1 || exit 1
  RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 300 python tools/strip_scaling.py --ranks 1 8 --steps 30 --all-ranks > gpurun_out/r05/strips_$v.log 2>&1 || exit 1
done
for v in base c12; do
  RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 300 python bench.py --config hair1m --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r05/bench_hair1m_$v.log 2>&1 || exit 1
  RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 300 python bench.py --config robot1080 --no-cpu-baseline --steps 50 > gpurun_out/r05/bench_robot_$v.log 2>&1 || exit 1
done
