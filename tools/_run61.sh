set -u
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 200 python tools/count_gpu_work.py sphere1m seg > gpurun_out/r02_count61.log 2>&1 || exit 1
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 300 python tools/count_gpu_work.py sphere1m_refl seg >> gpurun_out/r02_count61.log 2>&1 || exit 2
bash tools/profile_gpu.sh r02 > gpurun_out/r02_prof61.log 2>&1 || exit 3
