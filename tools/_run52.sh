set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest52.log 2>&1 || exit 1
timeout -k 10 600 python tools/variants.py run rowm b16x8 b32x8 b8x8 b32x16 rowm b16x8 b32x8 b8x8 b32x16 -- --steps 20 --warmup 5 > gpurun_out/r02_var52.log 2>&1
