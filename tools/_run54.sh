set -u
bash tools/profile_gpu.sh r02 > gpurun_out/r02_prof54.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r02_bench_c4.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --config sphere1m_refl --steps 3 --warmup 1 > gpurun_out/r02_bench_c5.log 2>&1 || exit 3
