set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest22.log 2>&1
timeout -k 10 100 python tools/phase_split.py "primary+shadow" "primary only" > gpurun_out/r02_phase22.log 2>&1
RT_TILE_ORDER=0 timeout -k 10 100 python tools/phase_split.py "primary+shadow" >> gpurun_out/r02_phase22.log 2>&1
RT_LIB_PATH=_variants/librt_tt.so timeout -k 10 200 python tools/tile_times.py > gpurun_out/r02_tiles22.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench22.log 2>&1
