set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest81.log 2>&1 || { tail -30 gpurun_out/r02_pytest81.log; exit 1; }
tail -2 gpurun_out/r02_pytest81.log
timeout -k 10 400 python tools/variants.py run w4 w8 w4 w8 -- --steps 50 --warmup 5 > gpurun_out/r02_var81.log 2>&1 || exit 2
RT_W_SAH_CT=2 timeout -k 10 400 python tools/variants.py run w4 -- --steps 50 --warmup 5 >> gpurun_out/r02_var81.log 2>&1 || exit 2
RT_W_SAH_CT=3 timeout -k 10 400 python tools/variants.py run w4 -- --steps 50 --warmup 5 >> gpurun_out/r02_var81.log 2>&1 || exit 2
cat gpurun_out/r02_var81.log
RT_LIB_PATH=_variants/librt_w8.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest81w8.log 2>&1 || { tail -30 gpurun_out/r02_pytest81w8.log; exit 3; }
tail -2 gpurun_out/r02_pytest81w8.log
