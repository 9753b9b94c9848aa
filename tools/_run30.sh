set -u
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 200 python tools/count_gpu_work.py sphere1m > gpurun_out/r02_count30.log 2>&1
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 200 python tools/count_gpu_work.py sphere1m_refl seg > gpurun_out/r02_count30_c5.log 2>&1
bash tools/profile_gpu.sh r02 > gpurun_out/prof_r02.log 2>&1
