set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_gpu.sh r02c > gpurun_out/r02_prof84.log 2>&1 || { tail -20 gpurun_out/r02_prof84.log; exit 1; }
python tools/profile_summary.py gpurun_out/prof_r02c gpurun_out/sum_r02c > /dev/null || exit 2
mkdir -p gpurun_out/c5prof84
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof84/trace -o run -- python3 bench.py --config sphere1m_refl --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c5prof84/bench.log 2>&1 || { tail gpurun_out/c5prof84/bench.log; exit 3; }
f=$(find gpurun_out/c5prof84/trace -name "run_kernel_stats.csv" | head -1)
cp $f gpurun_out/c5prof84/kernel_stats.csv
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/r02_bench84.log 2>&1 || exit 4
grep -h '^{' gpurun_out/r02_bench84.log
timeout -k 10 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/nccl_check.py > gpurun_out/r02_nccl84.log 2>&1 || { tail -20 gpurun_out/r02_nccl84.log; exit 5; }
tail -1 gpurun_out/r02_nccl84.log
grep -h '^{' gpurun_out/prof_r02c/trace.log | cut -c 1-300
