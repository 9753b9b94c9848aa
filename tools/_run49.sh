set -u
timeout -k 10 400 python tools/variants.py run nopf nost nostpf nopf nost nostpf -- --steps 20 --warmup 5 > gpurun_out/r02_var49.log 2>&1
