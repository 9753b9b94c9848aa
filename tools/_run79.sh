set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest79.log 2>&1 || { tail -30 gpurun_out/r02_pytest79.log; exit 1; }
tail -2 gpurun_out/r02_pytest79.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/r02_bench79a.log 2>&1 || exit 2
RT_FUSED_SSAA=0 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench79b.log 2>&1 || exit 3
grep -h '^{' gpurun_out/r02_bench79*.log | cut -c 1-330
grep -h '^{' gpurun_out/r02_bench79a.log | grep -o '"max_abs_dpixel.*'
timeout -k 10 300 python tools/strip_scaling.py --ranks 1 8 --inflight 1 2 > gpurun_out/r02_strips79.log 2>&1 || exit 4
cat gpurun_out/r02_strips79.log
