set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest82.log 2>&1 || { tail -30 gpurun_out/r02_pytest82.log; exit 1; }
tail -2 gpurun_out/r02_pytest82.log
timeout -k 10 400 python tools/variants.py run w4 w8 w4 w8 -- --steps 50 --warmup 5 > gpurun_out/r02_var82.log 2>&1 || exit 2
RT_W_SAH_CT=2 timeout -k 10 400 python tools/variants.py run w4 -- --steps 50 --warmup 5 >> gpurun_out/r02_var82.log 2>&1 || exit 2
RT_W_SAH_CT=3 timeout -k 10 400 python tools/variants.py run w4 -- --steps 50 --warmup 5 >> gpurun_out/r02_var82.log 2>&1 || exit 2
cat gpurun_out/r02_var82.log
timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c5_82a.log 2>&1 || exit 4
RT_REFL_FUSE=0 timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c5_82b.log 2>&1 || exit 5
RT_REFL_CHUNK_LOG2=23 timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c5_82c.log 2>&1 || exit 6
grep -h '^{' gpurun_out/r02_c5_82*.log | cut -c 1-300
RT_LIB_PATH=_variants/librt_w8.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest82w8.log 2>&1 || { tail -30 gpurun_out/r02_pytest82w8.log; exit 3; }
tail -2 gpurun_out/r02_pytest82w8.log
