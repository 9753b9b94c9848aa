set -u
timeout -k 10 500 python tools/variants.py run b2 b4 b8 noslab -- --steps 20 --warmup 5 > gpurun_out/r02_var25.log 2>&1
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench25.log 2>&1
