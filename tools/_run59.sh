set -u
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_ph.so timeout -k 10 200 python tools/phase_time.py > gpurun_out/r02_phase59.log 2>&1
