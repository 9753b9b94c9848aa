set -u
timeout -k 10 500 python tools/variants.py run occ4 occ3 occ4nb occ4 occ3 occ4nb -- --steps 20 --warmup 5 > gpurun_out/r02_var64.log 2>&1
