set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_pytest87.log 2>&1 || { tail -30 gpurun_out/r02_pytest87.log; exit 1; }
tail -1 gpurun_out/r02_pytest87.log
timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c5_87.log 2>&1 || exit 4
grep -h '^{' gpurun_out/r02_c5_87.log | cut -c 1-300
