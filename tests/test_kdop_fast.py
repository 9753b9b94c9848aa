"""The certificate's fast path (wbvh.hpp kdop_certifies: quotients through an approximate
reciprocal, decided only when the comparison is won by more than 2^-19 of the magnitudes) must
decide exactly as the correctly rounded k-DOP test (kdop_certifies_exact, bvh.h:79-105).
tests/c/kdop_fast.cpp builds the header on the host with a reciprocal hook up to 4 ulps off (the
device's v_rcp_f32 is within 1) and checks 2M random k-DOPs / rays, half of them with t within a
few ulps of t_near (the close calls the fast path must hand to the exact one), plus skipped
planes, denominators below 2^-100 and tiny directions.  CPU only."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fast_certificate_decides_as_the_exact_one(tmp_path):
    exe = str(tmp_path / "kdop_fast")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O2", "-ffp-contract=off", "-fno-fast-math", "-x", "hip",
                        "--offload-arch=gfx950", "-o", exe, os.path.join(ROOT, "tests", "c", "kdop_fast.cpp")],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0 and out.stdout.startswith("ok "), out.stdout + out.stderr
