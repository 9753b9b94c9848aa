set -u
timeout -k 10 300 python tools/variants.py run base occ4 base occ4 -- --steps 20 --warmup 5 > gpurun_out/r02_var37.log 2>&1
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 200 python tools/count_gpu_work.py sphere1m seg > gpurun_out/r02_count37.log 2>&1
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 300 python tools/count_gpu_work.py sphere1m_refl seg >> gpurun_out/r02_count37.log 2>&1
