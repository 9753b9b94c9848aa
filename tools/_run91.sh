set -u
mkdir -p gpurun_out
timeout -k 10 500 python tools/variants.py run w4 cur w4 cur -- --steps 50 --warmup 5 > gpurun_out/r02_var91.log 2>&1 || exit 2
cat gpurun_out/r02_var91.log
