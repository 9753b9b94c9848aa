set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest8.log 2>&1
timeout -k 10 200 python tools/phase_split.py "primary+shadow" "primary only" > gpurun_out/r02_phase8.log 2>&1
RT_WIDE_LEAN=0 timeout -k 10 100 python tools/phase_split.py "primary+shadow" "primary only" > gpurun_out/r02_phase8_full.log 2>&1
timeout -k 10 300 python tools/variants.py run occ3 occ4 occ6 -- --steps 20 --warmup 5 > gpurun_out/r02_var8.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_bench8.log 2>&1
