"""bench.py plumbing on CPU: the self-launch of N ranks (torch.distributed.run child process when
WORLD_SIZE is unset), the strip gather and re-assembly over gloo with the dpixel check, and a
roofline object a reader can recompute from the fields it carries."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("n,balance", [(1, True), (2, True), (3, True), (2, False)])
def test_bench_self_launch_dry_run(n, balance):
    """The N-rank self-launch, the flat all-gather with rank 0's in-step re-assembly, and (N > 1) the
    cost-balanced band lists from all-reduced band costs: the frame equals the pattern."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1"]
                       + ([] if balance else ["--no-balance"]), cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == n and line["config"]["world_size"] == n
    assert line["config"]["bands"] == ("cost-balanced lists" if balance and n > 1 else "interleaved b % N")
    assert line["dry_run"] is True and line["max_abs_dpixel"] == 0


def test_roofline_recomputable():
    sys.path.insert(0, ROOT)
    import bench
    rl = bench.roofline("sphere1m", 1, 1.55, 2.7, 1.38, 3840 * 2160)
    assert rl is not None and rl["bound"] == "l1_l2_gather" and rl["peak"] == bench.PEAK_L2_GBS
    b = sum(rl["units_per_frame"][k] * rl["bytes_per_unit"][k] for k in rl["units_per_frame"])
    assert b == rl["bytes_per_launch"]
    assert abs(b / (rl["kernel_ms"] * 1e-3) / 1e9 - rl["achieved"]) < 0.1
    assert abs(rl["achieved"] / rl["peak"] - rl["frac"]) < 1e-4
    assert rl["kernel_ms"] == 1.55 and rl["overlapped_launch_ms"] == 2.7   # priced on the non-overlapped launch
    rl8 = bench.roofline("sphere1m", 8, None, 0.7, 0.3, 3840 * 2160)
    assert rl8["kernel_ms"] == 0.3   # N > 1: no sync leg, the step interval
    assert abs(rl8["bytes_per_launch"] * 8 - b) <= 8   # each rank reads its share of the frame
