set -u
RT_LIB_PATH=_variants/librt_count.so timeout -k 10 200 python tools/count_gpu_work.py sphere1m seg > gpurun_out/r02_count38.log 2>&1
timeout -k 10 300 python tools/phase_split.py "primary+shadow" "primary only" "all rays miss (sphere behind the camera)" > gpurun_out/r02_phase38.log 2>&1
