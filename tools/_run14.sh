set -u
timeout -k 10 200 python tools/phase_split.py "primary+shadow" "primary only" > gpurun_out/r02_phase14.log 2>&1
RT_LIB_PATH=_variants/librt_tt.so timeout -k 10 200 python tools/tile_times.py > gpurun_out/r02_tiles14.log 2>&1
