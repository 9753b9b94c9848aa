"""Loads the golden fixtures written by tests/golden/make_golden.py (reference outputs)."""
from __future__ import annotations

import json
import os

import numpy as np

from raytracercpp_amd import scenes
from raytracercpp_amd.scene import RenderSettings, SceneData, bits_to_f32

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def case_names():
    return [k for k in manifest() if not k.startswith("_")]


def _settings(d) -> RenderSettings:
    st = RenderSettings()
    for k, v in d.items():
        cur = getattr(st, k)
        setattr(st, k, bool(v) if isinstance(cur, bool) else type(cur)(v))
    return st


def _scene(z, prefix, meta) -> SceneData:
    if prefix + "tri" in z:
        tri = z[prefix + "tri"]
        uv = z[prefix + "tri_uv"] if prefix + "tri_uv" in z else None
    else:
        g = meta["generator"]
        assert g["kind"] == "uv_sphere"
        tri, uv = scenes.uv_sphere_triangles(g["nu"], g["nv"], bump=g["bump"], texcoords=g["texcoords"])
        tri = scenes.transform_triangles(bits_to_f32(g["xform"]), tri)
    textures = {}
    sky = None
    for key in z.files:
        if key.startswith(prefix + "tex"):
            textures[int(key[len(prefix) + 3:])] = z[key]
    if prefix + "sky0" in z:
        sky = [z[f"{prefix}sky{i}"] for i in range(6)]
    sc = SceneData(tri=tri, tri_mat=z[prefix + "tri_mat"], tri_uv=uv, shape_kind=z[prefix + "shape_kind"],
                   shape=z[prefix + "shape"], shape_mat=z[prefix + "shape_mat"], materials=z[prefix + "materials"],
                   cam_pos=z[prefix + "cam_pos"], proj_inv=z[prefix + "proj_inv"],
                   cam_to_world=z[prefix + "cam_to_world"], light=z[prefix + "light"], textures=textures,
                   skybox=sky, proj=z[prefix + "proj"] if prefix + "proj" in z else None,
                   world_to_cam=z[prefix + "world_to_cam"] if prefix + "world_to_cam" in z else None)
    if prefix + "cam_lens" in z:
        fov, aspect = (float(x) for x in z[prefix + "cam_lens"])
        sc.cam_fov = fov
        sc.cam_aspect = None if np.isnan(aspect) else aspect
    assert sc.triangle_hash() == meta["tri_sha256"], "rebuilt triangles differ from the fixture's"
    return sc


class Case:
    def __init__(self, name):
        self.name = name
        self.meta = manifest()[name]
        self.z = np.load(os.path.join(GOLDEN, name + ".npz"))
        self.scene = _scene(self.z, "in_", self.meta)
        self.settings = _settings(self.meta["settings"])

    def expected(self):
        z = self.z
        out = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
        return out

    def row_samples(self):
        """[(scene, settings, {row: {argb, hit_id, hit_t, rgba}})]"""
        res = []
        for j, bm in enumerate(self.meta["row_samples"]):
            sc = _scene(self.z, f"big{j}_", bm)
            st = _settings(bm["settings"])
            rows = {r: {k: self.z[f"big{j}_row{r}_{k}"] for k in ("argb", "hit_id", "hit_t", "rgba")}
                    for r in bm["rows"]}
            res.append((sc, st, rows))
        return res
