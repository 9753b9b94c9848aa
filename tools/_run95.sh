set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_pytest95.log 2>&1 || { tail -30 gpurun_out/r02_pytest95.log; exit 1; }
tail -1 gpurun_out/r02_pytest95.log
grep -c . gpurun_out/r02_pytest95.log
