set -u
bash tools/profile_gpu.sh r02b > gpurun_out/r02_prof77.log 2>&1 || { tail -20 gpurun_out/r02_prof77.log; exit 1; }
python tools/profile_summary.py gpurun_out/prof_r02b gpurun_out/sum_r02b
