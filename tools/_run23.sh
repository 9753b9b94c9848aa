set -u
RT_LIB_PATH=_variants/librt_tt.so timeout -k 10 200 python tools/tile_timeline.py > gpurun_out/r02_timeline23.log 2>&1
RT_TILE_ORDER=0 RT_LIB_PATH=_variants/librt_tt.so timeout -k 10 200 python tools/tile_timeline.py > gpurun_out/r02_timeline23b.log 2>&1
