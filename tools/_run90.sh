set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_pytest90.log 2>&1 || { tail -30 gpurun_out/r02_pytest90.log; exit 1; }
tail -1 gpurun_out/r02_pytest90.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/r02_bench90.log 2>&1 || exit 2
grep -h '^{' gpurun_out/r02_bench90.log | cut -c 1-200
grep -h '^{' gpurun_out/r02_bench90.log | grep -o '"max_abs_dpixel.*'
timeout -k 10 200 python tools/strip_scaling.py --ranks 1 8 --inflight 2 > gpurun_out/r02_strips90.log 2>&1 || exit 3
grep -h '"rank": 0' gpurun_out/r02_strips90.log | cut -c 1-90
