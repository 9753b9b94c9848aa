import os
import sys

import pytest

# Renderers made by the tests build the wide BVH before their first frame (synchronous
# acceleration structures), so single-frame parity tests run on the default
# certified path; test_async_accel_frames covers the background build (first frames on the octree).
os.environ.setdefault("RT_ASYNC_ACCEL", "0")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librt_mi355x.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running")
