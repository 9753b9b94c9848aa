set -u
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_ph.so timeout -k 10 200 python tools/phase_time.py > gpurun_out/r02_phase56.log 2>&1
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 200 python tools/count_gpu_work.py sphere1m seg > gpurun_out/r02_count56.log 2>&1
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 300 python tools/count_gpu_work.py sphere1m_refl seg >> gpurun_out/r02_count56.log 2>&1
