set -u
timeout -k 10 500 python tools/variants.py run new occ4 occ6 new occ4 occ6 -- --steps 20 --warmup 5 > gpurun_out/r02_var63.log 2>&1
