#!/bin/bash
# r05: the C5 parity tests and the renderer's device memory at the default chunk (2^27 slots)
set -e
O=gpurun_out/r05chunk2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_frames.py tests/test_gpu_parity.py tests/test_progressive.py -k "deferral or c5 or reflection or progressive" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
timeout -k 10 300 python tools/c5_memory.py > $O/memory.log 2>&1
tail -1 $O/memory.log
