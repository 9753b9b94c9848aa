set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest15.log 2>&1
timeout -k 10 200 python tools/phase_split.py "primary+shadow" "primary only" > gpurun_out/r02_phase15.log 2>&1
