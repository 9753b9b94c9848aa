set -u
timeout -k 10 500 python tools/variants.py run s12 s12o6 -- --steps 20 --warmup 5 > gpurun_out/r02_var28.log 2>&1
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench28.log 2>&1
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_s12ws.so timeout -k 10 200 python tools/wave_stats.py > gpurun_out/r02_waves28a.log 2>&1
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_s12o6ws.so timeout -k 10 200 python tools/wave_stats.py > gpurun_out/r02_waves28b.log 2>&1
