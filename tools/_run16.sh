set -u
timeout -k 10 200 python tools/phase_split.py "primary+shadow" "primary only" "primary only, barycentric shading" "all rays miss (sphere behind the camera)" > gpurun_out/r02_phase16.log 2>&1
