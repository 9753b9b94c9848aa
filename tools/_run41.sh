set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest41.log 2>&1 || exit 1
timeout -k 10 400 python tools/variants.py run base new occ6 base new occ6 -- --steps 20 --warmup 5 > gpurun_out/r02_var41.log 2>&1
