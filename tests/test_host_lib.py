"""Host-side checks that need no GPU: the C-ABI library loads and exports exactly the
symbols include/rt_mi355x.h and rt_mi355x_diag.h declare (no compute calls), settings defaults mirror
RenderSettings, host math / OBJ loading against the committed fixtures, and the
strip layout used for multi-GPU rendering."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from raytracercpp_amd import _lib, scenes, strips
from raytracercpp_amd.scene import RenderSettings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rt_mi355x.h")
DIAG_HEADER = os.path.join(ROOT, "include", "rt_mi355x_diag.h")   # the diagnostic entry points


def declared_functions(headers=(HEADER, DIAG_HEADER)):
    out = set()
    for h in headers:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        out |= set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text))
    return out


def test_diagnostics_apart_from_the_renderer_surface():
    """rt_mi355x.h holds the Renderer surface; the diagnostics live in rt_mi355x_diag.h only."""
    main, diag = declared_functions((HEADER,)), declared_functions((DIAG_HEADER,))
    assert {"rt_tile_costs", "rt_debug_read", "rt_wide_query", "rt_risk_words", "rt_wbvh_query", "rt_wbvh_query_ex",
            "rt_octree_digest", "rt_ocone_check", "rt_ocone_read", "rt_risk_cap_check"} == diag
    assert not (main & diag)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    declared = declared_functions()
    assert len(declared) > 30
    for name in declared:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (rt_[a-z0-9_]+)$", out, flags=re.M))
    assert declared == exported, (declared ^ exported)
    assert set(_lib.SIGNATURES) == declared


def test_default_settings_mirror_rendersettings():
    c = _lib.RtSettings()
    _lib.lib().rt_default_settings(ctypes.byref(c))
    ref = RenderSettings()   # rendererSettings.h:30-102 defaults
    for name, _ in _lib.RtSettings._fields_:
        if hasattr(ref, name):
            assert pytest.approx(getattr(c, name)) == getattr(ref, name), name
    assert c.image_width == 1024 and c.max_recursion_depth == 5 and c.bvh_leaf_object_count == 40


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from raytracercpp_amd.renderer import Renderer
    with pytest.raises(RuntimeError):
        Renderer(0)


def test_obj_loader_matches_fixture_triangles():
    """cube / robot through the product loader == the reference loader's triangles in the fixtures."""
    from golden_cases import Case
    for name in ("c2_cube", "robot"):
        c = Case(name)
        sc2, _ = (scenes.cube1080 if name == "c2_cube" else scenes.robot1080)(width=320, height=180)
        assert np.array_equal(sc2.tri.view(np.uint32), c.scene.tri.view(np.uint32))
        assert np.array_equal(sc2.tri_mat, c.scene.tri_mat)
        assert np.array_equal(sc2.materials[:, :15].view(np.uint32), c.scene.materials[:, :15].view(np.uint32))


def test_generated_workloads_are_deterministic():
    a, _ = scenes.bumpy70k(width=8, height=8)
    b, _ = scenes.bumpy70k(width=8, height=8)
    assert a.triangle_hash() == b.triangle_hash()
    import json
    counts = json.load(open(os.path.join(ROOT, "profiles", "work_counts.json")))
    assert counts["bumpy70k"]["triangle_sha256"] == a.triangle_hash()


def test_det_sincos_accuracy():
    x = np.linspace(-20, 20, 100001)
    s, c = scenes.det_sincos(x)
    assert np.max(np.abs(s - np.sin(x))) < 1e-14 and np.max(np.abs(c - np.cos(x))) < 1e-14


@pytest.mark.parametrize("h,band,n", [(1080, 8, 1), (1080, 8, 2), (1080, 8, 8), (1080, 7, 3), (90, 16, 8), (5, 8, 4)])
def test_strip_layout_partitions_every_row_once(h, band, n):
    seen = np.concatenate([strips.rank_rows(h, band, r, n) for r in range(n)])
    seen = seen[seen >= 0]
    assert np.array_equal(np.sort(seen), np.arange(h))
    assert all(len(strips.rank_rows(h, band, r, n)) == strips.local_rows(h, band, n) for r in range(n))


def test_strip_assemble_roundtrip():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 2**32, size=(37, 11), dtype=np.uint64).astype(np.uint32)
    for n, band in ((1, 4), (3, 4), (5, 2)):
        parts = []
        for r in range(n):
            g = strips.rank_rows(37, band, r, n)
            p = np.zeros((len(g), 11), np.uint32)
            p[g >= 0] = img[g[g >= 0]]
            parts.append(p)
        assert np.array_equal(strips.assemble(parts, 37, band), img)


def test_trace_ray_rejects_mismatched_rays():
    """Renderer.trace_ray / trace_rays refuse origin and direction arrays of different lengths
    before the C call (rt_trace_ray copies n rays from each buffer)."""
    import pytest as _pt
    from raytracercpp_amd.renderer import Renderer
    o = np.zeros((4, 3), np.float32)
    d = np.zeros((3, 3), np.float32)
    for f in (Renderer.trace_ray, Renderer.trace_rays):
        with _pt.raises(ValueError):
            f(None, o, d)
