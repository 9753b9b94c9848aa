set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_gpu.sh r02d > gpurun_out/r02_prof100.log 2>&1 || { tail -20 gpurun_out/r02_prof100.log; exit 1; }
python tools/profile_summary.py gpurun_out/prof_r02d gpurun_out/sum_r02d > /dev/null || exit 2
grep -h '^{' gpurun_out/prof_r02d/trace.log | grep -o '"kernel_ms": [0-9.]*'
