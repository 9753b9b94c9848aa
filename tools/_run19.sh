set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest19.log 2>&1
for b in 0 32 48 64 96 128; do echo "budget $b"; RT_WIDE_BUDGET=$b timeout -k 10 100 python tools/phase_split.py "primary+shadow" ; done > gpurun_out/r02_budget19.log 2>&1
