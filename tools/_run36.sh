set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest36.log 2>&1
for i in 1 2; do
RT_PLAIN=0 timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r02_bench36.log 2>&1
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r02_bench36.log 2>&1
done
