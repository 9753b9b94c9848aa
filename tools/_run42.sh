set -u
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/r02_counters_avail.txt 2>&1 || true
