set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest66.log 2>&1 || exit 1
timeout -k 10 500 python tools/variants.py run nopair pair nopair pair -- --steps 20 --warmup 5 > gpurun_out/r02_var66.log 2>&1
timeout -k 10 500 python tools/variants.py run nopair pair -- --config sphere1m_refl --steps 2 --warmup 1 >> gpurun_out/r02_var66.log 2>&1
