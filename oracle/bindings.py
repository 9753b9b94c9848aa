"""ctypes bindings to the oracle -- TEST INFRASTRUCTURE ONLY.

* ``Oracle``  : liboracle.so, the C restatement of the reference hot path (oracle.c).
* ``RefHarness`` : oracle/_ref/libref_harness.so, the reference's own Qt-free
  translation units + a restated per-pixel driver (ref_harness.cpp).  Only exists
  where /root/reference was present at build time (never on the GPU box unless
  the built .so travelled with the snapshot).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_harness.so")

NTEX = 6
_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)
_i64p = C.POINTER(C.c_int64)


class OrcScene(C.Structure):
    _fields_ = [
        ("ntri", C.c_int64), ("tri", _f32p), ("tri_mat", _i32p), ("tri_uv", _f32p),
        ("nshape", C.c_int32), ("shape_kind", _i32p), ("shape", _f32p), ("shape_mat", _i32p),
        ("nmat", C.c_int32), ("mat", _f32p),
        ("cam_pos", C.c_float * 3), ("proj_inv", C.c_float * 16), ("cam_to_world", C.c_float * 16),
        ("light", C.c_float * 3),
        ("tex_w", C.c_int32 * NTEX), ("tex_h", C.c_int32 * NTEX), ("tex", _f32p * NTEX),
        ("sky_w", C.c_int32 * 6), ("sky_h", C.c_int32 * 6), ("sky", _f32p * 6),
        ("proj", C.c_float * 16), ("world_to_cam", C.c_float * 16),
        ("cam_fov", C.c_float), ("cam_aspect", C.c_float),
    ]


class OrcSettings(C.Structure):
    _fields_ = [
        ("image_width", C.c_int32), ("image_height", C.c_int32),
        ("enable_ssaa", C.c_int32), ("ssaa_factor", C.c_int32),
        ("shading_method", C.c_int32), ("compute_shadows", C.c_int32),
        ("max_recursion_depth", C.c_int32),
        ("enable_bvh", C.c_int32), ("bvh_max_depth", C.c_int32), ("bvh_leaf_object_count", C.c_int32),
        ("enable_ambient", C.c_int32), ("enable_diffuse", C.c_int32), ("enable_specular", C.c_int32),
        ("enable_emissive", C.c_int32), ("rough_reflections_sample_count", C.c_int32),
        ("enable_ao_mapping", C.c_int32), ("enable_diffuse_mapping", C.c_int32),
        ("enable_normal_mapping", C.c_int32), ("enable_displacement_mapping", C.c_int32),
        ("displacement_mapping_strength", C.c_float), ("parallax_mapping_steps", C.c_int32),
        ("enable_roughness_mapping", C.c_int32), ("enable_skysphere", C.c_int32),
        ("enable_skybox", C.c_int32), ("rng_seed", C.c_uint32), ("enable_clipping", C.c_int32),
        ("enable_ssao", C.c_int32), ("ssao_sample_count", C.c_int32),
        ("ssao_radius", C.c_float), ("ssao_amount", C.c_float),
    ]


class OrcOutputs(C.Structure):
    _fields_ = [("argb", _u32p), ("rgba", _f32p), ("hit_id", _i32p), ("hit_t", _f32p), ("shadow", _u8p),
                ("zbuf", _f32p), ("nbuf", _f32p)]


class OrcCounters(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "primary_rays", "shadow_rays", "reflection_rays",
        "vol_tests_primary", "tri_tests_primary", "vol_tests_shadow", "tri_tests_shadow",
        "vol_tests_refl", "tri_tests_refl", "child_tests_primary", "child_tests_shadow")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


def _ptr(a, t):
    if a is None:
        return C.cast(None, t)
    return a.ctypes.data_as(t)


class _Pinned:
    """Keeps numpy arrays alive while a C struct points at them."""

    def __init__(self):
        self.keep = []

    def arr(self, a, dtype):
        if a is None:
            return None
        a = np.ascontiguousarray(a, dtype=dtype)
        self.keep.append(a)
        return a


def make_orc_scene(scene, pin: _Pinned, settings=None) -> OrcScene:
    s = OrcScene()
    if settings is not None:
        s.cam_fov, s.cam_aspect = scene.lens(settings)
    tri = pin.arr(scene.tri.reshape(-1, 9), np.float32)
    s.ntri = tri.shape[0]
    s.tri = _ptr(tri, _f32p)
    s.tri_mat = _ptr(pin.arr(scene.tri_mat, np.int32), _i32p)
    s.tri_uv = _ptr(pin.arr(scene.tri_uv, np.float32), _f32p)
    s.nshape = int(len(scene.shape_kind))
    s.shape_kind = _ptr(pin.arr(scene.shape_kind, np.int32), _i32p)
    s.shape = _ptr(pin.arr(scene.shape.reshape(-1, 6) if len(scene.shape_kind) else np.zeros((1, 6)), np.float32), _f32p)
    s.shape_mat = _ptr(pin.arr(scene.shape_mat, np.int32), _i32p)
    mats = pin.arr(scene.materials.reshape(-1, 16), np.float32)
    s.nmat = mats.shape[0]
    s.mat = _ptr(mats, _f32p)
    s.cam_pos[:] = [float(x) for x in np.asarray(scene.cam_pos, np.float32)]
    s.proj_inv[:] = [float(x) for x in np.asarray(scene.proj_inv, np.float32)]
    s.cam_to_world[:] = [float(x) for x in np.asarray(scene.cam_to_world, np.float32)]
    s.light[:] = [float(x) for x in np.asarray(scene.light, np.float32)]
    if getattr(scene, "proj", None) is not None:
        s.proj[:] = [float(x) for x in np.asarray(scene.proj, np.float32)]
    if getattr(scene, "world_to_cam", None) is not None:
        s.world_to_cam[:] = [float(x) for x in np.asarray(scene.world_to_cam, np.float32)]
    for slot in range(NTEX):
        img = scene.textures.get(slot) if scene.textures else None
        if img is not None:
            a = pin.arr(img, np.float32)
            s.tex_h[slot], s.tex_w[slot] = a.shape[0], a.shape[1]
            s.tex[slot] = _ptr(a, _f32p)
    if scene.skybox is not None:
        for i, f in enumerate(scene.skybox):
            a = pin.arr(f, np.float32)
            s.sky_h[i], s.sky_w[i] = a.shape[0], a.shape[1]
            s.sky[i] = _ptr(a, _f32p)
    return s


def make_orc_settings(st) -> OrcSettings:
    o = OrcSettings()
    for name, typ in OrcSettings._fields_:
        v = getattr(st, name)
        setattr(o, name, float(v) if typ is C.c_float else int(v))
    return o


class RenderResult:
    def __init__(self, w, h):
        n = w * h
        self.width, self.height = w, h
        self.argb = np.zeros(n, np.uint32)
        self.rgba = np.zeros((n, 4), np.float32)
        self.hit_id = np.zeros(n, np.int32)
        self.hit_t = np.zeros(n, np.float32)
        self.shadow = np.zeros(n, np.uint8)
        self.zbuf = np.zeros(n, np.float32)
        self.nbuf = np.zeros((n, 3), np.float32)
        self.counters = {}
        self.seconds = 0.0

    def outputs(self):
        o = OrcOutputs()
        o.argb = _ptr(self.argb, _u32p)
        o.rgba = _ptr(self.rgba, _f32p)
        o.hit_id = _ptr(self.hit_id, _i32p)
        o.hit_t = _ptr(self.hit_t, _f32p)
        o.shadow = _ptr(self.shadow, _u8p)
        o.zbuf = _ptr(self.zbuf, _f32p)
        o.nbuf = _ptr(self.nbuf, _f32p)
        return o


class Oracle:
    """C restatement (oracle.c).  One instance = one built scene (octree built in the ctor)."""

    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            if not os.path.exists(ORACLE_SO):
                raise RuntimeError(f"{ORACLE_SO} missing: run `make -C oracle`")
            L = C.CDLL(ORACLE_SO)
            L.orc_create.restype = C.c_void_p
            L.orc_create.argtypes = [C.POINTER(OrcScene), C.POINTER(OrcSettings)]
            L.orc_destroy.argtypes = [C.c_void_p]
            L.orc_render_rows.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(OrcOutputs),
                                          C.POINTER(OrcCounters), C.c_int]
            L.orc_render_row_set.argtypes = [C.c_void_p, _i32p, C.c_int, C.POINTER(OrcOutputs),
                                             C.POINTER(OrcCounters), C.c_int]
            L.orc_raster.argtypes = [C.c_void_p, C.POINTER(OrcOutputs), C.POINTER(OrcCounters), C.c_int]
            L.orc_downscale_argb.argtypes = [_u32p, C.c_int, C.c_int, C.c_int, _u32p]
            L.orc_bvh_query.argtypes = [C.c_void_p, _f32p, _f32p, C.c_int64, _i32p, _f32p, _f32p, _f32p, _u8p, _i64p]
            L.orc_bvh_stats.argtypes = [C.c_void_p, _i64p]
            L.orc_trace_rays_shaded.argtypes = [C.c_void_p, _f32p, _f32p, C.c_int64, C.c_int, _f32p, _i32p, _f32p,
                                                _u8p, _u8p, C.POINTER(OrcCounters)]
            L.orc_bvh_node.argtypes = [C.c_void_p, C.c_int, _f32p, _f32p, _i32p, _i32p, _i32p]
            L.orc_heap_order.argtypes = [_f32p, C.c_int, _i32p]
            L.orc_ssao.argtypes = [C.c_void_p, _f32p, _f32p, _u32p, _i32p, C.c_int]
            cls._lib = L
        return cls._lib

    def __init__(self, scene, settings):
        L = self.lib()
        self._pin = _Pinned()
        self._sc = make_orc_scene(scene, self._pin, settings)
        self._st = make_orc_settings(settings)
        self.settings = settings
        self._h = L.orc_create(C.byref(self._sc), C.byref(self._st))

    def close(self):
        if self._h:
            self.lib().orc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render_rows(self, row_begin=0, row_count=None, nthreads=0) -> RenderResult:
        rw, rh = self.settings.render_size()
        if row_count is None:
            row_count = rh - row_begin
        res = RenderResult(rw, row_count)
        cnt = OrcCounters()
        out = res.outputs()
        t0 = time.perf_counter()
        rc = self.lib().orc_render_rows(self._h, row_begin, row_count, C.byref(out), C.byref(cnt), nthreads)
        res.seconds = time.perf_counter() - t0
        if rc != 0:
            raise RuntimeError("orc_render_rows failed")
        res.counters = cnt.as_dict()
        return res

    def render_row_set(self, rows, nthreads=0) -> RenderResult:
        """render_rows on an arbitrary list of internal rows (output row i = rows[i]), with the
        threads spread over the rows' pixels (a few rows of an expensive frame)."""
        rows = np.ascontiguousarray(rows, np.int32)
        rw, _ = self.settings.render_size()
        res = RenderResult(rw, len(rows))
        cnt = OrcCounters()
        out = res.outputs()
        t0 = time.perf_counter()
        rc = self.lib().orc_render_row_set(self._h, _ptr(rows, _i32p), len(rows), C.byref(out), C.byref(cnt), nthreads)
        res.seconds = time.perf_counter() - t0
        if rc != 0:
            raise RuntimeError("orc_render_row_set failed")
        res.counters = cnt.as_dict()
        return res

    def raster(self, nthreads=0) -> RenderResult:
        """Renderer::raster_trace restated (sequential triangle order), the whole render."""
        rw, rh = self.settings.render_size()
        res = RenderResult(rw, rh)
        cnt = OrcCounters()
        out = res.outputs()
        t0 = time.perf_counter()
        rc = self.lib().orc_raster(self._h, C.byref(out), C.byref(cnt), nthreads)
        res.seconds = time.perf_counter() - t0
        if rc != 0:
            raise RuntimeError("orc_raster failed")
        res.counters = cnt.as_dict()
        return res

    def ssao(self, res: RenderResult, nthreads=0):
        """post_process_ssao_SIMD on a full internal frame (res from render_rows() or raster()):
        returns (argb after the SSAO blur, per-pixel occlusion counts)."""
        argb = res.argb.copy()
        ao = np.zeros(res.argb.shape[0], np.int32)
        rc = self.lib().orc_ssao(self._h, _ptr(res.zbuf, _f32p), _ptr(res.nbuf, _f32p), _ptr(argb, _u32p),
                                 _ptr(ao, _i32p), nthreads)
        if rc != 0:
            raise RuntimeError("orc_ssao failed")
        return argb, ao

    def bvh_query(self, orig, dirs):
        orig = np.ascontiguousarray(orig, np.float32)
        dirs = np.ascontiguousarray(dirs, np.float32)
        n = orig.shape[0]
        ids = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        u = np.zeros(n, np.float32)
        v = np.zeros(n, np.float32)
        ret = np.zeros(n, np.uint8)
        counts = np.zeros(3, np.int64)
        self.lib().orc_bvh_query(self._h, _ptr(orig, _f32p), _ptr(dirs, _f32p), n, _ptr(ids, _i32p), _ptr(t, _f32p),
                                 _ptr(u, _f32p), _ptr(v, _f32p), _ptr(ret, _u8p), _ptr(counts, _i64p))
        return ids, t, u, v, ret, counts

    def trace_ray(self, orig, dirs, depth=0):
        """Renderer::trace_ray (shaded), fresh HitInfo per ray -> (rgba, src, t, found, shadowed, counters)."""
        orig = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        n = orig.shape[0]
        rgba = np.zeros((n, 4), np.float32)
        src = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        found = np.zeros(n, np.uint8)
        shadowed = np.zeros(n, np.uint8)
        cnt = OrcCounters()
        self.lib().orc_trace_rays_shaded(self._h, _ptr(orig, _f32p), _ptr(dirs, _f32p), n, int(depth),
                                         _ptr(rgba, _f32p), _ptr(src, _i32p), _ptr(t, _f32p), _ptr(found, _u8p),
                                         _ptr(shadowed, _u8p), C.byref(cnt))
        return rgba, src, t, found, shadowed, cnt.as_dict()

    def bvh_stats(self):
        st = np.zeros(6, np.int64)
        self.lib().orc_bvh_stats(self._h, _ptr(st, _i64p))
        return dict(zip(("inner", "leaves", "empty_leaves", "max_leaf", "max_depth", "nodes"), map(int, st)))

    @classmethod
    def downscale(cls, argb, w, h, factor):
        a = np.ascontiguousarray(argb, np.uint32)
        out = np.zeros((w // factor) * (h // factor), np.uint32)
        rc = cls.lib().orc_downscale_argb(_ptr(a, _u32p), w, h, factor, _ptr(out, _u32p))
        if rc != 0:
            raise ValueError("size not divisible by factor")
        return out

    @classmethod
    def heap_order(cls, keys):
        k = np.ascontiguousarray(keys, np.float32)
        out = np.zeros(len(k), np.int32)
        cls.lib().orc_heap_order(_ptr(k, _f32p), len(k), _ptr(out, _i32p))
        return out


class RefHarness:
    """oracle/_ref/libref_harness.so (reference TUs).  Raises if not built."""

    _lib = None
    SO = REF_SO

    @classmethod
    def available(cls):
        return os.path.exists(cls.SO)

    @classmethod
    def lib(cls):
        if cls._lib is None:
            if not os.path.exists(cls.SO):
                raise RuntimeError(f"{cls.SO} missing: run `make -C oracle ref` where /root/reference exists")
            L = C.CDLL(cls.SO)
            L.ref_camera_matrices.argtypes = [C.c_float, C.c_float, C.c_float, C.c_float, _f32p, _f32p]
            L.ref_make_transform.argtypes = [C.c_int, C.c_float, C.c_float, C.c_float, _f32p]
            L.ref_compose.argtypes = [_f32p, _f32p, _f32p]
            L.ref_inverse.argtypes = [_f32p, _f32p]
            L.ref_transform_points.argtypes = [_f32p, _f32p, C.c_int64, _f32p]
            L.ref_load_obj.restype = C.c_int64
            L.ref_load_obj.argtypes = [C.c_char_p, _f32p, C.c_int, _f32p, _i32p, _f32p, C.c_int64, _i32p, _f32p,
                                       C.c_int32, _i32p]
            L.ref_last_render_seconds.restype = C.c_double
            L.ref_last_render_seconds.argtypes = []
            L.ref_specular_threshold.restype = C.c_float
            L.ref_specular_threshold.argtypes = [C.c_float] * 4
            L.ref_triangle_intersect.argtypes = [_f32p, _f32p, _f32p, _f32p]
            L.ref_bvh_query.argtypes = [_f32p, C.c_int64, C.c_int, C.c_int, _f32p, _f32p, C.c_int64, _i32p, _f32p,
                                        _f32p, _f32p, _u8p]
            L.ref_render_rows.argtypes = [C.POINTER(OrcScene), C.POINTER(OrcSettings), C.c_int, C.c_int,
                                          C.POINTER(OrcOutputs), C.POINTER(OrcCounters)]
            L.ref_raster.argtypes = [C.POINTER(OrcScene), C.POINTER(OrcSettings), C.POINTER(OrcOutputs),
                                     C.POINTER(OrcCounters)]
            L.ref_downscale_argb.argtypes = [_u32p, C.c_int, C.c_int, C.c_int, _u32p]
            L.ref_heap_order.argtypes = [_f32p, C.c_int, _i32p]
            L.ref_ssao.argtypes = [C.POINTER(OrcScene), C.POINTER(OrcSettings), _f32p, _f32p, _u32p, _i32p]
            L.ref_set_rng_sequential.argtypes = [C.c_int, C.c_uint32]
            L.ref_set_threads.argtypes = [C.c_int]
            cls._lib = L
        return cls._lib

    @classmethod
    def set_threads(cls, n):
        """OpenMP team size of the harness's row loops (omp_set_num_threads)."""
        cls.lib().ref_set_threads(int(n))

    @classmethod
    def set_rng_sequential(cls, on, seed=0):
        """The reference's own XorShiftGenerator stream at OMP_NUM_THREADS=1 (one thread, row
        order) instead of the path-keyed one; see ref_harness.cpp g_seq."""
        cls.lib().ref_set_rng_sequential(1 if on else 0, int(seed) & 0xFFFFFFFF)

    # --- transforms (mat.cpp) -------------------------------------------------
    @classmethod
    def camera_matrices(cls, fov, aspect, znear=0.1, zfar=1000.0):
        p = np.zeros(16, np.float32)
        pi = np.zeros(16, np.float32)
        cls.lib().ref_camera_matrices(fov, aspect, znear, zfar, _ptr(p, _f32p), _ptr(pi, _f32p))
        return p, pi

    @classmethod
    def transform(cls, kind, x=0.0, y=0.0, z=0.0):
        kinds = {"translation": 0, "rx": 1, "ry": 2, "rz": 3, "scale": 4, "identity": 5}
        out = np.zeros(16, np.float32)
        cls.lib().ref_make_transform(kinds[kind], x, y, z, _ptr(out, _f32p))
        return out

    @classmethod
    def compose(cls, a, b):
        a = np.ascontiguousarray(a, np.float32)
        b = np.ascontiguousarray(b, np.float32)
        out = np.zeros(16, np.float32)
        cls.lib().ref_compose(_ptr(a, _f32p), _ptr(b, _f32p), _ptr(out, _f32p))
        return out

    @classmethod
    def inverse(cls, a):
        a = np.ascontiguousarray(a, np.float32)
        out = np.zeros(16, np.float32)
        cls.lib().ref_inverse(_ptr(a, _f32p), _ptr(out, _f32p))
        return out

    @classmethod
    def transform_points(cls, m, pts):
        m = np.ascontiguousarray(m, np.float32)
        pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 3)
        out = np.zeros_like(pts)
        cls.lib().ref_transform_points(_ptr(m, _f32p), _ptr(pts, _f32p), pts.shape[0], _ptr(out, _f32p))
        return out

    @classmethod
    def load_obj(cls, path, xform, mat_offset=0, cap=4_000_000):
        xform = np.ascontiguousarray(xform, np.float32)
        tri = np.zeros((cap, 9), np.float32)
        mat = np.zeros(cap, np.int32)
        uv = np.zeros((cap, 6), np.float32)
        has_uv = C.c_int32(0)
        mats = np.zeros((64, 16), np.float32)
        nmat = C.c_int32(0)
        n = cls.lib().ref_load_obj(path.encode(), _ptr(xform, _f32p), mat_offset, _ptr(tri, _f32p), _ptr(mat, _i32p),
                                   _ptr(uv, _f32p), cap, C.byref(has_uv), _ptr(mats, _f32p), 64, C.byref(nmat))
        if n < 0:
            raise RuntimeError("ref_load_obj failed")
        return tri[:n].copy(), mat[:n].copy(), (uv[:n].copy() if has_uv.value else None), mats[:nmat.value].copy()

    @classmethod
    def specular_threshold(cls, spec, ns):
        return float(cls.lib().ref_specular_threshold(float(spec[0]), float(spec[1]), float(spec[2]), float(ns)))

    @classmethod
    def bvh_query(cls, tri, max_depth, leaf, orig, dirs):
        tri = np.ascontiguousarray(tri, np.float32).reshape(-1, 9)
        orig = np.ascontiguousarray(orig, np.float32)
        dirs = np.ascontiguousarray(dirs, np.float32)
        n = orig.shape[0]
        ids = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        u = np.zeros(n, np.float32)
        v = np.zeros(n, np.float32)
        ret = np.zeros(n, np.uint8)
        cls.lib().ref_bvh_query(_ptr(tri, _f32p), tri.shape[0], max_depth, leaf, _ptr(orig, _f32p), _ptr(dirs, _f32p),
                                n, _ptr(ids, _i32p), _ptr(t, _f32p), _ptr(u, _f32p), _ptr(v, _f32p), _ptr(ret, _u8p))
        return ids, t, u, v, ret

    @classmethod
    def render_rows(cls, scene, settings, row_begin=0, row_count=None) -> RenderResult:
        pin = _Pinned()
        sc = make_orc_scene(scene, pin, settings)
        st = make_orc_settings(settings)
        rw, rh = settings.render_size()
        if row_count is None:
            row_count = rh - row_begin
        res = RenderResult(rw, row_count)
        out = res.outputs()
        cnt = OrcCounters()
        t0 = time.perf_counter()
        rc = cls.lib().ref_render_rows(C.byref(sc), C.byref(st), row_begin, row_count, C.byref(out), C.byref(cnt))
        res.wall_seconds = time.perf_counter() - t0         # includes the reference's octree build
        res.seconds = cls.lib().ref_last_render_seconds()   # the pixel loop only
        if rc != 0:
            raise RuntimeError("ref_render_rows failed")
        res.counters = cnt.as_dict()
        return res

    @classmethod
    def raster(cls, scene, settings) -> RenderResult:
        """raster_trace on the reference's vec4 / Triangle4 / Transform / Triangle code."""
        pin = _Pinned()
        sc = make_orc_scene(scene, pin, settings)
        st = make_orc_settings(settings)
        rw, rh = settings.render_size()
        res = RenderResult(rw, rh)
        out = res.outputs()
        cnt = OrcCounters()
        if cls.lib().ref_raster(C.byref(sc), C.byref(st), C.byref(out), C.byref(cnt)) != 0:
            raise RuntimeError("ref_raster failed")
        res.counters = cnt.as_dict()
        return res

    @classmethod
    def render_row_sample(cls, scene, settings, row_begin, row_count, row_stride) -> RenderResult:
        """Internal rows row_begin + i * row_stride (i < row_count), for CPU timing samples."""
        pin = _Pinned()
        sc = make_orc_scene(scene, pin, settings)
        st = make_orc_settings(settings)
        rw, _ = settings.render_size()
        res = RenderResult(rw, row_count)
        out = res.outputs()
        cnt = OrcCounters()
        rc = cls.lib().ref_render_row_sample(C.byref(sc), C.byref(st), row_begin, row_count, row_stride,
                                             C.byref(out), C.byref(cnt))
        if rc != 0:
            raise RuntimeError("ref_render_row_sample failed")
        res.seconds = cls.lib().ref_last_render_seconds()
        res.counters = cnt.as_dict()
        return res

    @classmethod
    def ssao(cls, scene, settings, res: RenderResult):
        """post_process_ssao_SIMD (renderer.cpp:1229-1434) on the reference's SIMD helpers."""
        pin = _Pinned()
        sc = make_orc_scene(scene, pin, settings)
        st = make_orc_settings(settings)
        argb = res.argb.copy()
        ao = np.zeros(res.argb.shape[0], np.int32)
        if cls.lib().ref_ssao(C.byref(sc), C.byref(st), _ptr(res.zbuf, _f32p), _ptr(res.nbuf, _f32p),
                              _ptr(argb, _u32p), _ptr(ao, _i32p)) != 0:
            raise RuntimeError("ref_ssao failed")
        return argb, ao

    @classmethod
    def heap_order(cls, keys):
        k = np.ascontiguousarray(keys, np.float32)
        out = np.zeros(len(k), np.int32)
        cls.lib().ref_heap_order(_ptr(k, _f32p), len(k), _ptr(out, _i32p))
        return out

    @classmethod
    def downscale(cls, argb, w, h, factor):
        a = np.ascontiguousarray(argb, np.uint32)
        out = np.zeros((w // factor) * (h // factor), np.uint32)
        rc = cls.lib().ref_downscale_argb(_ptr(a, _u32p), w, h, factor, _ptr(out, _u32p))
        if rc != 0:
            raise ValueError("size not divisible by factor")
        return out


class RefHarnessShipped(RefHarness):
    """oracle/_ref/libref_harness_v3.so: the same reference TUs and harness built with the reference's
    shipped optimisation flags as far as they are portable (tp2/CMakeLists.txt:105-117: -O3 with
    -march=native -mfma; here -march=x86-64-v3 -mfma, GCC's default contraction): a CPU-baseline timing
    only, never a parity checker (contracted FMAs change a few pixels)."""

    _lib = None
    SO = os.path.join(os.path.dirname(REF_SO), "libref_harness_v3.so")
