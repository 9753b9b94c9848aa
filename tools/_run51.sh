set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest51.log 2>&1 || exit 1
timeout -k 10 600 python tools/variants.py run g1 g2 g4 g4d640 g4d2560 g1 g2 g4 g4d640 g4d2560 -- --steps 20 --warmup 5 > gpurun_out/r02_var51.log 2>&1
