set -u
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench34.log 2>&1
RT_SPLIT=0 timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r02_bench34.log 2>&1
timeout -k 10 300 python tools/variants.py run sh16 sh32 sh64 -- --steps 20 --warmup 5 > gpurun_out/r02_var34.log 2>&1
RT_SPLIT=0 timeout -k 10 300 python tools/variants.py run sh16 sh32 sh64 -- --steps 20 --warmup 5 >> gpurun_out/r02_var34.log 2>&1
