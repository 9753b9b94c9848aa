"""The parallel host octree build (the renderer's) against the reference's one-insert-at-a-time
algorithm restated (rt_octree_digest builder 1) and against the oracle's tree: identical
flattened nodes, triangle records, slot map and statistics.  CPU only (no GPU call)."""
import dataclasses

import numpy as np
import pytest

from oracle.bindings import Oracle
from raytracercpp_amd import _lib, scenes
from raytracercpp_amd.scene import RenderSettings

STAT_KEYS = ("inner", "leaves", "empty_leaves", "max_leaf", "max_depth", "nodes")


def soup(seed, n, dup=0.2):
    """Random triangles with duplicated and degenerate ones (coincident centroids, zero area)."""
    rng = np.random.default_rng(seed)
    t = rng.uniform(-1, 1, (n, 9)).astype(np.float32)
    k = int(n * dup)
    t[rng.integers(0, n, k)] = t[rng.integers(0, n, k)]
    t[:k // 2, 3:6] = t[:k // 2, 0:3]          # degenerate: a == b
    t[k // 2:k, :] = np.round(t[k // 2:k, :], 1)   # many equal coordinates / centroids on cell planes
    return t


CASES = [
    ("robot", lambda: scenes.robot1080()[0].tri, 12, 40),
    ("robot_d6_l8", lambda: scenes.robot1080()[0].tri, 6, 8),
    ("bumpy70k", lambda: scenes.bumpy70k()[0].tri, 12, 40),
    ("soup_d12_l4", lambda: soup(1, 20000), 12, 4),
    ("soup_d3_l1", lambda: soup(2, 5000), 3, 1),
    ("soup_d0", lambda: soup(3, 1000), 0, 40),        # max_depth 0: the root never splits
    ("soup_leaf0", lambda: soup(4, 3000), 5, 0),      # every non-empty node above max depth splits
    ("soup_leafneg", lambda: soup(5, 3000), 12, -1),  # (size_t)(long)-1: never splits
    ("single", lambda: soup(6, 1, 0), 12, 40),
]


@pytest.mark.parametrize("name,make,depth,leaf", CASES, ids=[c[0] for c in CASES])
def test_parallel_build_equals_insertion_order_build(name, make, depth, leaf, monkeypatch):
    tri = make()
    ref = _lib.octree_digest(tri, depth, leaf, builder=1)
    for threads in ("1", "3", "8"):
        monkeypatch.setenv("RT_BUILD_THREADS", threads)
        got = _lib.octree_digest(tri, depth, leaf, builder=0)
        assert got[0] == ref[0], f"digest differs at {threads} threads"
        assert got[1] == ref[1]


@pytest.mark.parametrize("name,make,depth,leaf", CASES[:5], ids=[c[0] for c in CASES[:5]])
def test_build_statistics_match_oracle_tree(name, make, depth, leaf):
    tri = make()
    _, st, _ = _lib.octree_digest(tri, depth, leaf, builder=0)
    base, _ = scenes.robot1080(width=64, height=36)
    sc = dataclasses.replace(base, tri=np.ascontiguousarray(tri, np.float32), tri_mat=np.zeros(len(tri), np.int32),
                             tri_uv=None)
    o = Oracle(sc, RenderSettings(bvh_max_depth=depth, bvh_leaf_object_count=leaf)).bvh_stats()
    for k in STAT_KEYS:
        assert st[k] == o[k], k


def test_sphere1m_parallel_build_equals_insertion_order_build():
    sc, st = scenes.sphere1m()
    ref = _lib.octree_digest(sc.tri, 12, 40, builder=1)
    got = _lib.octree_digest(sc.tri, 12, 40, builder=0)
    assert got[0] == ref[0] and got[1] == ref[1]
