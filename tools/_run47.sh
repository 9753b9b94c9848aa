set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest47.log 2>&1 || exit 1
timeout -k 10 400 python tools/variants.py run nopf pf nopf pf -- --steps 20 --warmup 5 > gpurun_out/r02_var47.log 2>&1
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_ph.so timeout -k 10 200 python tools/phase_time.py > gpurun_out/r02_phase47.log 2>&1
