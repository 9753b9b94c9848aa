set -u
mkdir -p gpurun_out
timeout -k 10 500 python tools/variants.py run base loop3 nosb base loop3 nosb -- --steps 50 --warmup 10 > gpurun_out/r02_var94.log 2>&1 || exit 2
cat gpurun_out/r02_var94.log
