set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest33.log 2>&1
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench33.log 2>&1
RT_SPLIT=0 timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r02_bench33.log 2>&1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof33 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_prof33.log 2>&1
