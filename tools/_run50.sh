set -u
timeout -k 10 500 python tools/variants.py run nopf pf512 pf2k pf8k nopf pf512 pf2k pf8k -- --steps 20 --warmup 5 > gpurun_out/r02_var50.log 2>&1
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_ws.so timeout -k 10 200 python tools/wave_stats.py > gpurun_out/r02_ws50.log 2>&1
