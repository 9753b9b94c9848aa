set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_pytest97.log 2>&1 || { tail -30 gpurun_out/r02_pytest97.log; exit 1; }
tail -1 gpurun_out/r02_pytest97.log
timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 > gpurun_out/r02_c5_97.log 2>&1 || exit 4
grep -h '^{' gpurun_out/r02_c5_97.log | cut -c 1-250
grep -h '^{' gpurun_out/r02_c5_97.log | grep -o '"cpu_baseline.*'
