set -u
mkdir -p gpurun_out
timeout -k 10 500 python tools/variants.py run w4 bq8 sh16 w4 bq8 sh16 -- --steps 50 --warmup 5 > gpurun_out/r02_var88.log 2>&1 || exit 2
cat gpurun_out/r02_var88.log
