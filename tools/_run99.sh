set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_pytest99.log 2>&1 || { tail -30 gpurun_out/r02_pytest99.log; exit 1; }
tail -1 gpurun_out/r02_pytest99.log
timeout -k 10 300 python bench.py > gpurun_out/r02_bench99.log 2>&1 || exit 2
grep -h '^{' gpurun_out/r02_bench99.log
timeout -k 10 200 python tools/strip_scaling.py --ranks 1 2 4 8 --inflight 2 > gpurun_out/r02_strips99.log 2>&1 || exit 3
grep -h 'bound' gpurun_out/r02_strips99.log
