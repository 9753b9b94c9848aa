set -u
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench29.log 2>&1
timeout -k 10 500 python tools/variants.py run noslab s10 -- --steps 20 --warmup 5 > gpurun_out/r02_var29.log 2>&1
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r02_bench29.log 2>&1
