set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest70.log 2>&1 || exit 1
timeout -k 10 500 python tools/variants.py run head new head new -- --steps 20 --warmup 5 > gpurun_out/r02_var70.log 2>&1
