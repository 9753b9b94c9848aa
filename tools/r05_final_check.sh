#!/bin/bash
# r05 end of round: the GPU suite, smoke(), and the default bench line on the final build
set -e
O=gpurun_out/r05end
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json.log 2>&1
grep -h '^{' $O/bench.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C4', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'), d['roofline'].get('frac'), d['cpu_baseline'].get('value'))"
