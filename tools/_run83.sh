set -u
mkdir -p gpurun_out
timeout -k 10 500 python tools/variants.py run w4 occ5 occ3 bq2 w4 occ5 -- --steps 50 --warmup 5 > gpurun_out/r02_var83.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --inflight 3 --no-cpu-baseline > gpurun_out/r02_bench83q3.log 2>&1 || exit 3
cat gpurun_out/r02_var83.log
grep -h '^{' gpurun_out/r02_bench83q3.log | cut -c 1-250
RT_REFL_CHUNK_LOG2=24 timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c5_83a.log 2>&1 || exit 5
RT_REFL_CHUNK_LOG2=25 timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c5_83b.log 2>&1 || exit 6
grep -h '^{' gpurun_out/r02_c5_83*.log | cut -c 1-300
