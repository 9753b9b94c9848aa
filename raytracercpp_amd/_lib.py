"""ctypes binding of librt_mi355x.so (include/rt_mi355x.h).

The product path is this HIP library; there is no CPU fallback.  Loading fails
loudly when the in-tree .so is missing (build it with ``__graft_entry__.build()``
or ``make -C raytracercpp_amd/csrc``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librt_mi355x.so")
# development only (tools/variants.py): benchmark an alternative build of the same library
if os.environ.get("RT_LIB_PATH"):
    LIB_PATH = os.environ["RT_LIB_PATH"]

RT_OK = 0
ERRORS = {-1: "RT_EINVAL", -2: "RT_EHIP", -3: "RT_ENOMEM", -4: "RT_ESTATE", -5: "RT_EUNSUPPORTED", -6: "RT_EIO"}

_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)
_i64p = C.POINTER(C.c_int64)


class RtSettings(C.Structure):
    _fields_ = [
        ("image_width", C.c_int32), ("image_height", C.c_int32),
        ("enable_ssaa", C.c_int32), ("ssaa_factor", C.c_int32),
        ("enable_clipping", C.c_int32), ("hybrid_rasterization_tracing", C.c_int32),
        ("shading_method", C.c_int32), ("compute_shadows", C.c_int32), ("max_recursion_depth", C.c_int32),
        ("enable_bvh", C.c_int32), ("bvh_max_depth", C.c_int32), ("bvh_leaf_object_count", C.c_int32),
        ("enable_ssao", C.c_int32), ("ssao_sample_count", C.c_int32),
        ("ssao_radius", C.c_float), ("ssao_amount", C.c_float),
        ("enable_ambient", C.c_int32), ("enable_diffuse", C.c_int32), ("enable_specular", C.c_int32),
        ("enable_emissive", C.c_int32), ("rough_reflections_sample_count", C.c_int32),
        ("enable_ao_mapping", C.c_int32), ("enable_diffuse_mapping", C.c_int32),
        ("enable_normal_mapping", C.c_int32), ("enable_displacement_mapping", C.c_int32),
        ("displacement_mapping_strength", C.c_float), ("parallax_mapping_steps", C.c_int32),
        ("enable_roughness_mapping", C.c_int32), ("enable_skysphere", C.c_int32), ("enable_skybox", C.c_int32),
        ("rng_seed", C.c_uint32),
    ]


class RtStats(C.Structure):
    _fields_ = [
        ("primary_rays", C.c_int64), ("shadow_rays", C.c_int64), ("reflection_rays", C.c_int64),
        ("kernel_ms", C.c_float), ("post_ms", C.c_float), ("build_ms", C.c_float),
        ("octree_inner", C.c_int64), ("octree_leaves", C.c_int64), ("octree_empty_leaves", C.c_int64),
        ("octree_max_leaf", C.c_int64), ("octree_max_depth", C.c_int64),
        ("gpu_nodes", C.c_int64), ("gpu_tris", C.c_int64),
        ("render_width", C.c_int32), ("render_height", C.c_int32), ("seg_scale", C.c_float),
        ("work", C.c_int64 * 4), ("work_wide", C.c_int64 * 4), ("uncertified", C.c_int64 * 6),
        ("wave_steps", C.c_int64 * 6), ("build_split_ms", C.c_float * 4), ("host_builds", C.c_int64),
        ("wide_tree", C.c_int32),
    ]

    def as_dict(self):
        def conv(n, t):
            v = getattr(self, n)
            if t is C.c_float:
                return float(v)
            if isinstance(v, C.Array):
                return [float(x) if n == "build_split_ms" else int(x) for x in v]
            return int(v)
        return {n: conv(n, t) for n, t in self._fields_}


# every exported symbol and its ctypes signature (restype, argtypes); tests check
# that the .so exports exactly what include/rt_mi355x.h declares.
_H = C.c_void_p
SIGNATURES = {
    "rt_default_settings": (None, [C.POINTER(RtSettings)]),
    "rt_create": (_H, [C.c_int]),
    "rt_destroy": (None, [_H]),
    "rt_last_error": (C.c_char_p, []),
    "rt_get_settings": (C.c_int, [_H, C.POINTER(RtSettings)]),
    "rt_set_settings": (C.c_int, [_H, C.POINTER(RtSettings)]),
    "rt_change_render_size": (C.c_int, [_H, C.c_int32, C.c_int32]),
    "rt_set_exact": (C.c_int, [_H, C.c_int]),
    "rt_finish_accel": (C.c_int, [_H]),
    "rt_set_devices": (C.c_int, [_H, _i32p, C.c_int32]),
    "rt_set_triangles": (C.c_int, [_H, _f32p, _i32p, _f32p, C.c_int64]),
    "rt_add_sphere": (C.c_int, [_H, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int32]),
    "rt_add_plane": (C.c_int, [_H] + [C.c_float] * 6 + [C.c_int32]),
    "rt_clear_geometry": (C.c_int, [_H]),
    "rt_set_materials": (C.c_int, [_H, _f32p, C.c_int32]),
    "rt_get_material_count": (C.c_int, [_H, _i32p]),
    "rt_change_camera_fov": (C.c_int, [_H, C.c_float]),
    "rt_change_camera_aspect_ratio": (C.c_int, [_H, C.c_float]),
    "rt_set_light_position": (C.c_int, [_H, C.c_float, C.c_float, C.c_float]),
    "rt_set_camera_transform": (C.c_int, [_H, _f32p]),
    "rt_apply_transformation_to_camera": (C.c_int, [_H, _f32p]),
    "rt_set_camera_matrices": (C.c_int, [_H, _f32p, _f32p, _f32p]),
    "rt_set_camera_projection": (C.c_int, [_H, _f32p, _f32p]),
    "rt_set_camera_lens": (C.c_int, [_H, C.c_float, C.c_float]),
    "rt_get_ssao_buffers": (C.c_int, [_H, _f32p, _f32p, _i32p]),
    "rt_get_camera_matrices": (C.c_int, [_H, _f32p, _f32p, _f32p]),
    "rt_set_object_transform": (C.c_int, [_H, _f32p]),
    "rt_reset_previous_transform": (C.c_int, [_H]),
    "rt_set_texture": (C.c_int, [_H, C.c_int32, C.c_int32, C.c_int32, _f32p]),
    "rt_set_skybox": (C.c_int, [_H, _i32p, _i32p, C.POINTER(_f32p)]),
    "rt_reconstruct_bvh_new": (C.c_int, [_H]),
    "rt_destroy_bvh": (C.c_int, [_H]),
    "rt_ray_trace": (C.c_int, [_H]),
    "rt_raster_trace": (C.c_int, [_H]),
    "rt_post_process": (C.c_int, [_H]),
    "rt_get_image": (C.c_int, [_H, _u32p, _i32p, _i32p]),
    "rt_render": (C.c_int, [_H, _f32p]),
    "rt_lock_image": (C.c_int, [_H]),
    "rt_unlock_image": (C.c_int, [_H]),
    "rt_request_aux": (C.c_int, [_H, C.c_int32, C.c_int32, C.c_int32]),
    "rt_get_internal": (C.c_int, [_H, _u32p, _f32p, _i32p, _f32p, _u8p]),
    "rt_get_stats": (C.c_int, [_H, C.POINTER(RtStats)]),
    "rt_local_rows": (C.c_int, [_H, C.c_int32, C.c_int32, C.c_int32, _i32p]),
    "rt_render_bands_device": (C.c_int, [_H, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "rt_render_band_list_device": (C.c_int, [_H, C.c_int32, _i32p, C.c_int32, C.c_void_p, C.c_void_p]),
    "rt_band_costs": (C.c_int, [_H, C.c_void_p, C.POINTER(C.c_double), C.c_int32]),
    "rt_trace_rays": (C.c_int, [_H, _f32p, _f32p, C.c_int64, _i32p, _f32p, _f32p, _f32p, _u8p]),
    "rt_trace_ray": (C.c_int, [_H, _f32p, _f32p, C.c_int64, C.c_int32, _f32p, _i32p, _f32p, _u8p, _u8p]),
    "rt_wide_query": (C.c_int, [_H, _f32p, _f32p, C.c_int64, C.c_int32, _f32p, _f32p, _i32p, _i32p, _f32p, _f32p, _f32p,
                                _u8p]),
    "rt_risk_words": (C.c_int, [_H, C.c_int32, C.POINTER(C.c_uint64), C.c_int64, _i64p, _i64p]),
    "rt_kernel_times": (C.c_int, [_H, _f32p, C.c_int32]),
    "rt_band_counters": (C.c_int, [_H, _i64p, _i64p]),
    "rt_make_transform": (None, [C.c_int32, C.c_float, C.c_float, C.c_float, _f32p]),
    "rt_compose": (None, [_f32p, _f32p, _f32p]),
    "rt_inverse": (None, [_f32p, _f32p]),
    "rt_perspective": (None, [C.c_float, C.c_float, C.c_float, C.c_float, _f32p]),
    "rt_transform_points": (None, [_f32p, _f32p, C.c_int64, _f32p]),
    "rt_obj_open": (_H, [C.c_char_p, _f32p, C.c_int32]),
    "rt_obj_counts": (C.c_int, [_H, _i64p, _i32p, _i32p]),
    "rt_obj_fetch": (C.c_int, [_H, _f32p, _i32p, _f32p, _f32p]),
    "rt_obj_close": (None, [_H]),
    "rt_octree_digest": (C.c_int, [_f32p, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_uint64), _i64p,
                                   _f32p]),
    "rt_debug_read": (C.c_int, [_H, C.POINTER(C.c_uint64), C.c_int64]),
    "rt_tile_costs": (C.c_int, [_H, C.POINTER(C.c_uint32), C.c_int64, _i32p, _i32p]),
    "rt_wbvh_query": (C.c_int, [_f32p, C.c_int64, C.c_int32, C.c_int32, _f32p, _f32p, C.c_int64, _i32p, _i32p, _f32p,
                                _f32p, _f32p, _i64p, _f32p]),
    "rt_wbvh_query_ex": (C.c_int, [_f32p, C.c_int64, C.c_int32, C.c_int32, _f32p, _f32p, C.c_int64, _f32p, _f32p,
                                   C.c_int32, _f32p, _f32p, _i32p, _i32p, _f32p, _f32p, _f32p, _i64p, _f32p, _i32p,
                                   C.c_int32, _i64p]),
    "rt_ocone_check": (C.c_int, [_f32p, C.c_int64, C.c_int32, C.c_int32, C.c_int32, _f32p, _f32p, C.c_int64, _i32p,
                                 _i64p, C.POINTER(C.c_uint32), _i32p, _f32p, C.POINTER(C.c_uint32)]),
    "rt_ocone_read": (C.c_int, [_H, C.POINTER(C.c_uint32), C.c_int64, _i32p, _f32p]),
    "rt_risk_cap_check": (C.c_int, [_f32p, C.c_int64, C.c_int32, C.c_int32, _f32p, _f32p, C.c_int64, C.c_float, _i32p,
                                    _i64p]),
}

_lib = None


def lib():
    """The loaded librt_mi355x.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: the HIP library must be built "
                               "(python -c 'import __graft_entry__ as g; g.build()')")
        # torch bundles its own libamdhip64.so.7 (same soname as ROCm's): load it first
        # so that a process using both (device buffers, RCCL) runs ONE HIP runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class RtError(RuntimeError):
    def __init__(self, code, where):
        msg = lib().rt_last_error()
        super().__init__(f"{where}: {ERRORS.get(code, code)}: {msg.decode() if msg else ''}")
        self.code = code


def check(rc, where):
    if rc != RT_OK:
        raise RtError(rc, where)
    return rc


def ptr(a, t):
    if a is None:
        return C.cast(None, t)
    return a.ctypes.data_as(t)


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


# ---- mat.cpp helpers -----------------------------------------------------------
_KINDS = {"translation": 0, "rx": 1, "ry": 2, "rz": 3, "scale": 4, "identity": 5}


def make_transform(kind, x=0.0, y=0.0, z=0.0):
    out = np.zeros(16, np.float32)
    lib().rt_make_transform(_KINDS[kind], x, y, z, ptr(out, _f32p))
    return out


def compose(a, b):
    a, b = f32(a), f32(b)
    out = np.zeros(16, np.float32)
    lib().rt_compose(ptr(a, _f32p), ptr(b, _f32p), ptr(out, _f32p))
    return out


def inverse(m):
    m = f32(m)
    out = np.zeros(16, np.float32)
    lib().rt_inverse(ptr(m, _f32p), ptr(out, _f32p))
    return out


def perspective(fov, aspect, znear=0.1, zfar=1000.0):
    out = np.zeros(16, np.float32)
    lib().rt_perspective(fov, aspect, znear, zfar, ptr(out, _f32p))
    return out


def camera_matrices(fov, aspect, znear=0.1, zfar=1000.0):
    """Camera::set_aspect_ratio (camera.cpp:5-11): (Perspective, Perspective.inverse())."""
    p = perspective(fov, aspect, znear, zfar)
    return p, inverse(p)


def transform_points(m, pts):
    m = f32(m)
    pts = f32(pts).reshape(-1, 3)
    out = np.zeros_like(pts)
    lib().rt_transform_points(ptr(m, _f32p), ptr(pts, _f32p), pts.shape[0], ptr(out, _f32p))
    return out


def load_obj(path, xform, mat_offset=0):
    """read_meshio_data + create_triangles -> (tri9, mat, uv6 or None, mats16)."""
    xform = f32(xform)
    L = lib()
    h = L.rt_obj_open(path.encode(), ptr(xform, _f32p), mat_offset)
    if not h:
        raise RuntimeError(f"rt_obj_open({path}): {L.rt_last_error().decode()}")
    try:
        n = C.c_int64()
        nm = C.c_int32()
        has_uv = C.c_int32()
        check(L.rt_obj_counts(h, C.byref(n), C.byref(nm), C.byref(has_uv)), "rt_obj_counts")
        tri = np.zeros((n.value, 9), np.float32)
        mat = np.zeros(n.value, np.int32)
        uv = np.zeros((n.value, 6), np.float32) if has_uv.value else None
        mats = np.zeros((nm.value, 16), np.float32)
        check(L.rt_obj_fetch(h, ptr(tri, _f32p), ptr(mat, _i32p), ptr(uv, _f32p), ptr(mats, _f32p)), "rt_obj_fetch")
        return tri, mat, uv, mats
    finally:
        L.rt_obj_close(h)


def wbvh_query(tri9, orig, dirs, max_depth=12, leaf=40, cam=None, light=None, shadow_rays=False, rays_out=False,
               ray_nodes=None, ocone_dim=0, oc_stats=None):
    """rt_wbvh_query(_ex): the wide-BVH certified closest hit on the host (no GPU).  Returns
    (status, id, t, u, v, stats dict, (octree ms, wide-BVH ms)); status 0 certified miss,
    1 certified hit, 2 not certified.  cam / light: the frame's grazing-risk points (rays from cam
    read the camera's bits); shadow_rays: orig / dirs are hit points and normals, traced as
    is_shadowed's rays towards light.  rays_out: (o, d) of the queried rays are appended."""
    tri9 = f32(tri9).reshape(-1, 9)
    o = f32(orig).reshape(-1, 3)
    d = f32(dirs).reshape(-1, 3)
    n = o.shape[0]
    st = np.zeros(n, np.int32)
    ids = np.zeros(n, np.int32)
    t, u, v = (np.zeros(n, np.float32) for _ in range(3))
    stats = np.zeros(8, np.int64)
    ms = np.zeros(2, np.float32)
    oo = np.zeros((n, 3), np.float32)
    do = np.zeros((n, 3), np.float32)
    c = None if cam is None else f32(cam).reshape(3)
    li = None if light is None else f32(light).reshape(3)
    check(lib().rt_wbvh_query_ex(ptr(tri9, _f32p), tri9.shape[0], max_depth, leaf, ptr(o, _f32p), ptr(d, _f32p), n,
                                 None if c is None else ptr(c, _f32p), None if li is None else ptr(li, _f32p),
                                 1 if shadow_rays else 0, ptr(oo, _f32p), ptr(do, _f32p),
                                 ptr(st, _i32p), ptr(ids, _i32p), ptr(t, _f32p), ptr(u, _f32p), ptr(v, _f32p),
                                 ptr(stats, _i64p), ptr(ms, _f32p),
                                 None if ray_nodes is None else ptr(ray_nodes, _i32p), int(ocone_dim),
                                 None if oc_stats is None else ptr(oc_stats, _i64p)), "rt_wbvh_query")
    keys = ("nodes", "leaves", "max_leaf", "depth", "node_visits", "tri_tests", "violations", "sah_x1000")
    out = (st, ids, t, u, v, dict(zip(keys, map(int, stats))), (float(ms[0]), float(ms[1])))
    return out + (oo, do) if rays_out else out


def ocone_check(tri9, orig, dirs, max_depth=12, leaf=40, ocone_dim=64, grid=None, want_cells=False):
    """rt_ocone_check: (skip flags, dict[, cells]) -- the origin cones' brute-force soundness check (no
    GPU).  grid: (cells uint32 [n, 2], dims, lo_ih) to check instead of building one (Renderer.ocone_read);
    want_cells: also return the built grid's words."""
    tri9 = f32(tri9).reshape(-1, 9)
    o = f32(orig).reshape(-1, 3)
    d = f32(dirs).reshape(-1, 3)
    skip = np.zeros(o.shape[0], np.int32)
    out = np.zeros(6, np.int64)
    _u32p = C.POINTER(C.c_uint32)
    cells = dims = lo_ih = None
    if grid is not None:
        cells = np.ascontiguousarray(grid[0], np.uint32)
        dims = np.ascontiguousarray(grid[1], np.int32)
        lo_ih = f32(grid[2])
    built = None
    if want_cells:
        # the grid's size: the renderer's frame (ocone_dim + 2 cells at most per axis)
        built = np.zeros(((ocone_dim + 2) ** 3, 2), np.uint32)
    check(lib().rt_ocone_check(ptr(tri9, _f32p), tri9.shape[0], max_depth, leaf, ocone_dim, ptr(o, _f32p),
                               ptr(d, _f32p), o.shape[0], ptr(skip, _i32p), ptr(out, _i64p),
                               None if cells is None else ptr(cells, _u32p), None if dims is None else ptr(dims, _i32p),
                               None if lo_ih is None else ptr(lo_ih, _f32p), None if built is None else ptr(built, _u32p)),
          "rt_ocone_check")
    keys = ("violations", "skipping", "grazing_tests", "cells", "empty_cells", "noskip_cells")
    res = (skip, dict(zip(keys, map(int, out))))
    return res + (built,) if want_cells else res


def risk_cap_check(tri9, cam, dirs, max_depth=12, leaf=40, cap_override=-1.0):
    """rt_risk_cap_check: (skip flags, dict) -- the camera risk cap's brute-force soundness check (no GPU)."""
    tri9 = f32(tri9).reshape(-1, 9)
    c = f32(cam).reshape(3)
    d = f32(dirs).reshape(-1, 3)
    skip = np.zeros(d.shape[0], np.int32)
    out = np.zeros(4, np.int64)
    check(lib().rt_risk_cap_check(ptr(tri9, _f32p), tri9.shape[0], max_depth, leaf, ptr(c, _f32p), ptr(d, _f32p),
                                  d.shape[0], float(cap_override), ptr(skip, _i32p), ptr(out, _i64p)), "rt_risk_cap_check")
    return skip, {"violations": int(out[0]), "skipping": int(out[1]), "grazing_tests": int(out[2]),
                  "cap": float(out[3]) * 1e-9 if out[3] >= 0 else None}


def octree_digest(tri9, max_depth=12, leaf=40, builder=0):
    """rt_octree_digest: (digest, stats dict, build ms) of the flattened host octree (no GPU)."""
    tri9 = f32(tri9).reshape(-1, 9)
    dg = C.c_uint64()
    st = np.zeros(7, np.int64)
    ms = C.c_float()
    check(lib().rt_octree_digest(ptr(tri9, _f32p), tri9.shape[0], max_depth, leaf, builder, C.byref(dg),
                                 ptr(st, _i64p), C.byref(ms)), "rt_octree_digest")
    keys = ("inner", "leaves", "empty_leaves", "max_leaf", "max_depth", "nodes", "levels")
    return int(dg.value), dict(zip(keys, map(int, st))), float(ms.value)
