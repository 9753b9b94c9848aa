set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest86.log 2>&1 || { tail -30 gpurun_out/r02_pytest86.log; exit 1; }
tail -1 gpurun_out/r02_pytest86.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke86.log 2>&1 || { tail -5 gpurun_out/r02_smoke86.log; exit 2; }
tail -1 gpurun_out/r02_smoke86.log | cut -c 1-200
timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c5_86.log 2>&1 || exit 4
grep -h '^{' gpurun_out/r02_c5_86.log | cut -c 1-300
timeout -k 10 300 python tools/strip_scaling.py --ranks 1 2 4 8 --inflight 1 2 3 > gpurun_out/r02_strips86.log 2>&1 || exit 3
grep bound gpurun_out/r02_strips86.log
