set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest76.log 2>&1 || { tail -30 gpurun_out/r02_pytest76.log; exit 1; }
tail -2 gpurun_out/r02_pytest76.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench76a.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --inflight 1 > gpurun_out/r02_bench76b.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02_bench76c.log 2>&1 || exit 4
grep -h '^{' gpurun_out/r02_bench76*.log
