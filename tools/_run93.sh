set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_pytest93.log 2>&1 || { tail -30 gpurun_out/r02_pytest93.log; exit 1; }
tail -1 gpurun_out/r02_pytest93.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke93.log 2>&1 || { tail -5 gpurun_out/r02_smoke93.log; exit 2; }
tail -1 gpurun_out/r02_smoke93.log | cut -c 1-120
timeout -k 10 300 python bench.py > gpurun_out/r02_bench93.log 2>&1 || exit 3
grep -h '^{' gpurun_out/r02_bench93.log
