set -u
timeout -k 10 600 python tools/variants.py run bq quads b8 quads8 bq quads b8 quads8 -- --steps 20 --warmup 5 > gpurun_out/r02_var58.log 2>&1
