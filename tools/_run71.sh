set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest71.log 2>&1 || { tail -30 gpurun_out/r02_pytest71.log; exit 1; }
tail -3 gpurun_out/r02_pytest71.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02_bench71.log 2>&1 || exit 2
cat gpurun_out/r02_bench71.log
