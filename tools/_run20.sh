set -u
export TMPDIR=/tmp
RT_WIDE_BUDGET=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof20a -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_prof20a.log 2>&1
RT_WIDE_BUDGET=64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof20b -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_prof20b.log 2>&1
