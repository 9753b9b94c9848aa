set -u
export TMPDIR=/tmp
RT_WIDE_LEAN=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof21a -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_prof21a.log 2>&1
RT_WIDE_BUDGET=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof21b -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_prof21b.log 2>&1
