"""What the sound wide query rests on, checked directly.

1. The rounding lemma (wbvh.hpp wbvh_closest, wq_h0),
checked directly on Moller-Trumbore's float arithmetic (mt_record = triangle.cpp:25-91): over 10^7
accepted hits of random triangles (slivers and obtuse ones included) and rays with |cos(n, d)| from
1e-10 to 1, the reported point lies within R of its triangle and within eta of its plane (case (a)),
and the origin within H0 of the plane (case (b)), with the exact constants of wbvh.hpp, evaluated in
long double by tests/c/wq_lemma.cpp, and with the float functions the kernels run (wq_reach, wq_split,
wq_eta, wq_h0 on float bounds of the exact quantities).
2. The metadata the proof reads: the checkers report a tree's conditioning bytes and a frame's risk
words that are not sound (tests/c/wbvh_mutation.cpp).  CPU only."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reported_points_within_the_query_bounds(tmp_path):
    exe = str(tmp_path / "wq_lemma")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O2", "-ffp-contract=off", "-fno-fast-math", "-x", "hip",
                        "--offload-arch=gfx950", "-o", exe, os.path.join(ROOT, "tests", "c", "wq_lemma.cpp")],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = subprocess.run([exe, "10000000"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0 and out.stdout.startswith("ok "), out.stdout + out.stderr
    f = out.stdout.split()
    assert int(f[1]) >= 10_000_000
    # every Q = q sin(alpha) decade from 1 to 1e-9 and below holds acceptances
    decades = [int(x) for x in f[f.index("Q-decades") + 1:f.index("float-bounds")]]
    assert len(decades) == 10 and min(decades) > 1000, decades
    # the float functions the kernels evaluate hold on the same hits (ratios <= 1; the exit status
    # already fails on a violation)
    ratios = [float(x) for x in f[f.index("float-bounds") + 1:]]
    assert len(ratios) == 4 and max(ratios) <= 1.0 and min(ratios) > 0.0, ratios
    print(out.stdout)


def test_metadata_checkers_report_corrupted_bytes(tmp_path):
    """check_wbvh's conditioning checks (smin, s2, sth, lmax, rho on every root-to-leaf path) and
    check_risk_words (keys and at-risk boxes) report 0 violations on a built tree and report every
    byte moved to the unsafe side (tests/c/wbvh_mutation.cpp, linked against librt_mi355x.so)."""
    lib = os.path.join(ROOT, "raytracercpp_amd")
    exe = str(tmp_path / "wbvh_mutation")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O2", "-ffp-contract=off", "-fno-fast-math", "-x", "hip",
                        "--offload-arch=gfx950", "-o", exe, os.path.join(ROOT, "tests", "c", "wbvh_mutation.cpp"),
                        "-L" + lib, "-lrt_mi355x", "-Wl,-rpath," + lib],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0 and out.stdout.startswith("ok "), out.stdout + out.stderr
    assert int(out.stdout.split()[1]) >= 40
