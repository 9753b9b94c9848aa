"""The quick wide BVH (wbvh.hpp build_wbvh_quick): the octree's own hierarchy as the
wide BVH, resident for the frames right after a geometry change while the SAH tree builds.  The same
host checks as the SAH tree's (tests/test_wbvh.py, through rt_wbvh_query with RT_WBVH_QUICK=1, which
makes the library's build_wbvh build the quick tree): check_wbvh finds 0 violations of the boxes,
slabs, cones and conditioning bytes on every root-to-leaf path, and every certified answer is the
oracle's BVH::intersect record (bvh.h:212-287), grazing rays and the camera / light risk words
included.  CPU only."""
import numpy as np
import pytest

import test_wbvh as tw
from raytracercpp_amd import _lib, scenes


@pytest.fixture(autouse=True)
def quick(monkeypatch):
    monkeypatch.setenv("RT_WBVH_QUICK", "1")


@pytest.mark.parametrize("scene_name", ["robot", "voxels", "grazing", "soup", "bumpy_camera", "bumpy_shadow"])
def test_quick_certified_queries_match_oracle(scene_name):
    tw.test_certified_queries_match_oracle(scene_name)


def test_quick_structure_on_degenerate_inputs():
    """Pile-ups at the octree's maximum depth (500 copies of one triangle: leaves far above 8
    triangles, nested runs), degenerate triangles, a single triangle, one 40-triangle leaf."""
    tw.test_structure_on_degenerate_inputs()


@pytest.mark.parametrize("seed,sin_lo,sin_hi", [(99, 1e-7, 1e-3), (5, 1e-9, 1e-5)])
def test_quick_grazing_plane(seed, sin_lo, sin_hi):
    tw.test_grazing_plane_certified_answers_match_oracle(seed, sin_lo, sin_hi)


def test_quick_grazing_sphere_and_slivers():
    tw.test_grazing_sphere_certified_answers_match_oracle()
    tw.test_grazing_sliver_soup_certified_answers_match_oracle()


@pytest.mark.parametrize("h", [0.0, 1e-7])
def test_quick_risk_words_camera_plane(h):
    tw.test_risk_bits_camera_grazing_plane(h)


def test_quick_risk_words_light_terminator():
    tw.test_risk_bits_light_sphere_terminator()


def test_quick_tree_shape():
    """The quick tree of the 1M-triangle sphere: every leaf child holds at most 8 triangles, the
    octree's depth (12) at most doubles (groups and runs), and the host probe's query sees it
    (violations 0 through the SAH tree's checker)."""
    sc, st = scenes.sphere1m(width=64, height=36)
    o = np.zeros((1, 3), np.float32)
    d = np.array([[0, 0, -1]], np.float32)
    *_, stats, ms = _lib.wbvh_query(sc.tri, o, d, st.bvh_max_depth, st.bvh_leaf_object_count)
    assert stats["violations"] == 0
    assert stats["max_leaf"] <= 8
    assert 0 < stats["depth"] <= 2 * (st.bvh_max_depth + 1)
    print(f"quick tree of sphere1m: {stats['nodes']} nodes, {stats['leaves']} leaves, depth {stats['depth']}, "
          f"build {ms[1]:.1f} ms (octree {ms[0]:.1f} ms)")
