set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03e.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/pytest_r03e.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r03e.json.log 2>&1 || exit 3
tail -1 gpurun_out/bench_r03e.json.log | cut -c1-1200
mkdir -p gpurun_out/prof_r03e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03e/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r03e/trace.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_r03e/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r03e/pmc_fetch.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_r03e/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r03e/pmc_write.log 2>&1 || exit 6
echo done
