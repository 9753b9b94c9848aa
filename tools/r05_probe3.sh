#!/bin/bash
# r05 GPU probe 3: the full GPU suite on the default build, then camera QS 2^-10 on hair1m / robot
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/pytest_gpu.log 2>&1 || exit 1
for v in base c10; do
  RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 300 python bench.py --config hair1m --no-cpu-baseline --no-check --steps 20 --warmup 5 > gpurun_out/r05/bench3_hair1m_$v.log 2>&1 || exit 1
  RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 300 python bench.py --config robot1080 --no-cpu-baseline --no-check --steps 50 > gpurun_out/r05/bench3_robot_$v.log 2>&1 || exit 1
  RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-check --steps 50 > gpurun_out/r05/bench3_c4_$v.log 2>&1 || exit 1
done
