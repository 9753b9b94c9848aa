set -u
timeout -k 10 300 python tools/variants.py run ifif -- --steps 20 --warmup 5 > gpurun_out/r02_var17.log 2>&1
RT_LIB_PATH=_variants/librt_ifif_tt.so timeout -k 10 200 python tools/tile_times.py > gpurun_out/r02_tiles17.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench17.log 2>&1
