"""Python mirror of the reference's ``Renderer`` (tp2/projets/renderer/renderer.h:20-355)
and of ``render(Renderer&)`` (tp2/projets/utils/mainUtils.cpp:6-21), backed by the
HIP library through its C ABI (include/rt_mi355x.h).  Method names, argument
meaning and call order follow the reference; errors raise :class:`RtError`
instead of asserting or invoking undefined behaviour.
"""
from __future__ import annotations

import ctypes as C
import time
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import RtSettings, RtStats, check, f32, ptr
from .scene import RenderSettings, SceneData, SHAPE_SPHERE, TEX_AO, TEX_DIFFUSE, TEX_NORMAL, TEX_DISPLACEMENT, \
    TEX_ROUGHNESS, TEX_SKYSPHERE

_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)


def _to_c(st: RenderSettings) -> RtSettings:
    c = RtSettings()
    _lib.lib().rt_default_settings(C.byref(c))
    for name, typ in RtSettings._fields_:
        if hasattr(st, name):
            v = getattr(st, name)
            setattr(c, name, float(v) if typ is C.c_float else int(v))
    return c


def _from_c(c: RtSettings) -> RenderSettings:
    st = RenderSettings()
    for name, typ in RtSettings._fields_:
        if hasattr(st, name):
            v = getattr(c, name)
            cur = getattr(st, name)
            setattr(st, name, bool(v) if isinstance(cur, bool) else (float(v) if typ is C.c_float else int(v)))
    return st


class Renderer:
    """One renderer on one GPU (HIP device ordinal ``device``)."""

    def __init__(self, device: int = 0, settings: Optional[RenderSettings] = None):
        L = _lib.lib()
        self._h = L.rt_create(int(device))
        if not self._h:
            raise RuntimeError(f"rt_create({device}): {L.rt_last_error().decode()}")
        self.device = device
        if settings is not None:
            self.set_render_settings(settings)

    # -- lifetime -------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().rt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _call(self, name, *args):
        return check(getattr(_lib.lib(), name)(self._h, *args), name)

    # -- settings (renderer.h:46, 118) ----------------------------------------------
    def render_settings(self) -> RenderSettings:
        c = RtSettings()
        self._call("rt_get_settings", C.byref(c))
        return _from_c(c)

    def set_render_settings(self, st: RenderSettings):
        c = _to_c(st)
        self._call("rt_set_settings", C.byref(c))

    def change_render_size(self, width: int, height: int):
        self._call("rt_change_render_size", int(width), int(height))

    def set_devices(self, ids):
        """rt_set_devices: render() uses every device in ids (ids[0] = this renderer's device),
        bands gathered to ids[0] with RCCL; an empty list returns to one device."""
        a = np.ascontiguousarray(list(ids), np.int32)
        self._call("rt_set_devices", ptr(a, _i32p) if len(a) else None, len(a))

    def finish_accel(self):
        """rt_finish_accel: wait for the background build of the leaf cones / slabs and the wide
        BVH (frames before it take the exact octree path)."""
        self._call("rt_finish_accel")

    def set_exact(self, on: bool = True):
        """Exact mode: every query walks the octree over the whole line, as
        the reference does, instead of the certified wide BVH."""
        self._call("rt_set_exact", 1 if on else 0)

    # -- geometry (renderer.h:57-62) ------------------------------------------------
    def set_triangles(self, tri9, mat, uv6=None):
        tri9 = f32(tri9).reshape(-1, 9)
        mat = np.ascontiguousarray(mat, np.int32)
        uv = None if uv6 is None else f32(uv6).reshape(-1, 6)
        self._call("rt_set_triangles", ptr(tri9, _f32p), ptr(mat, _i32p), ptr(uv, _f32p), tri9.shape[0])

    def add_sphere(self, center: Sequence[float], radius: float, mat_index: int = 0):
        self._call("rt_add_sphere", float(center[0]), float(center[1]), float(center[2]), float(radius), int(mat_index))

    def add_plane(self, point: Sequence[float], normal: Sequence[float], mat_index: int = 0):
        self._call("rt_add_plane", *[float(x) for x in point], *[float(x) for x in normal], int(mat_index))

    def clear_geometry(self):
        self._call("rt_clear_geometry")

    def set_materials(self, mats16):
        m = f32(mats16).reshape(-1, 16)
        self._call("rt_set_materials", ptr(m, _f32p), m.shape[0])

    def get_material_count(self) -> int:
        n = C.c_int32()
        self._call("rt_get_material_count", C.byref(n))
        return n.value

    # -- camera / light (renderer.h:72-75, 96-98) -----------------------------------
    def change_camera_fov(self, fov: float):
        self._call("rt_change_camera_fov", float(fov))

    def change_camera_aspect_ratio(self, aspect: float):
        self._call("rt_change_camera_aspect_ratio", float(aspect))

    def set_light_position(self, p: Sequence[float]):
        self._call("rt_set_light_position", float(p[0]), float(p[1]), float(p[2]))

    def set_camera_transform(self, m):
        m = f32(m)
        self._call("rt_set_camera_transform", ptr(m, _f32p))

    def apply_transformation_to_camera(self, m):
        m = f32(m)
        self._call("rt_apply_transformation_to_camera", ptr(m, _f32p))

    def set_camera_matrices(self, pos, proj_inv, cam_to_world):
        pos, pi, cw = f32(pos), f32(proj_inv), f32(cam_to_world)
        self._call("rt_set_camera_matrices", ptr(pos, _f32p), ptr(pi, _f32p), ptr(cw, _f32p))

    def set_camera_projection(self, proj, world_to_cam):
        """Camera::_perspective_proj_mat / _world_to_camera_mat, used by raster_trace."""
        pr, wc = f32(proj), f32(world_to_cam)
        self._call("rt_set_camera_projection", ptr(pr, _f32p), ptr(wc, _f32p))

    def set_camera_lens(self, fov: float, aspect: float):
        """Camera::_fov / _aspect_ratio without touching the matrices (read by SSAO)."""
        self._call("rt_set_camera_lens", float(fov), float(aspect))

    def get_camera_matrices(self):
        pos, pi, cw = np.zeros(3, np.float32), np.zeros(16, np.float32), np.zeros(16, np.float32)
        self._call("rt_get_camera_matrices", ptr(pos, _f32p), ptr(pi, _f32p), ptr(cw, _f32p))
        return pos, pi, cw

    def set_object_transform(self, m):
        m = f32(m)
        self._call("rt_set_object_transform", ptr(m, _f32p))

    def reset_previous_transform(self):
        self._call("rt_reset_previous_transform")

    # -- textures (renderer.h:77-90) ------------------------------------------------
    def _set_tex(self, slot, img):
        if img is None:
            self._call("rt_set_texture", slot, 0, 0, ptr(None, _f32p))
            return
        a = f32(img)
        h, w = a.shape[0], a.shape[1]
        self._call("rt_set_texture", slot, w, h, ptr(a, _f32p))

    def set_ao_map(self, img): self._set_tex(TEX_AO, img)
    def set_diffuse_map(self, img): self._set_tex(TEX_DIFFUSE, img)
    def set_normal_map(self, img): self._set_tex(TEX_NORMAL, img)
    def set_displacement_map(self, img): self._set_tex(TEX_DISPLACEMENT, img)
    def set_roughness_map(self, img): self._set_tex(TEX_ROUGHNESS, img)
    def set_skysphere(self, img): self._set_tex(TEX_SKYSPHERE, img)
    def clear_ao_map(self): self._set_tex(TEX_AO, None)
    def clear_diffuse_map(self): self._set_tex(TEX_DIFFUSE, None)
    def clear_normal_map(self): self._set_tex(TEX_NORMAL, None)
    def clear_displacement_map(self): self._set_tex(TEX_DISPLACEMENT, None)
    def clear_roughness_map(self): self._set_tex(TEX_ROUGHNESS, None)

    def set_skybox(self, faces):
        """faces: right, left, top, bottom, back, front (skybox.h:12-16), each (h, w, 4) float32."""
        arrs = [f32(f) for f in faces]
        w = (C.c_int32 * 6)(*[a.shape[1] for a in arrs])
        h = (C.c_int32 * 6)(*[a.shape[0] for a in arrs])
        p = (_f32p * 6)(*[ptr(a, _f32p) for a in arrs])
        self._keep_sky = arrs
        self._call("rt_set_skybox", w, h, p)

    # -- BVH (renderer.h:104-109) ---------------------------------------------------
    def reconstruct_bvh_new(self):
        self._call("rt_reconstruct_bvh_new")

    def destroy_bvh(self):
        self._call("rt_destroy_bvh")

    # -- rendering (renderer.h:149-154) ---------------------------------------------
    def ray_trace(self):
        self._call("rt_ray_trace")

    def raster_trace(self):
        """Renderer::raster_trace (renderer.cpp:869-1006): the hybrid raster + trace path."""
        self._call("rt_raster_trace")

    def post_process(self):
        self._call("rt_post_process")

    def get_image(self, out=None) -> np.ndarray:
        """Renderer::get_image: the current ARGB32 image as (h, w) uint32 (row 0 = bottom).
        Safe from a display thread while another thread renders (progressive readback): the
        size query and the copy run under the image lock.  ``out``: a (h, w) uint32 array to
        fill (a display that keeps its image buffer, as a QImage); a new one when it does not
        match the image's size."""
        w, h = C.c_int32(), C.c_int32()
        self.lock_image()
        try:
            self._call("rt_get_image", ptr(None, _u32p), C.byref(w), C.byref(h))
            if out is None or out.shape != (h.value, w.value) or out.dtype != np.uint32 or not out.flags.c_contiguous:
                out = np.empty((h.value, w.value), np.uint32)
            self._call("rt_get_image", ptr(out, _u32p), C.byref(w), C.byref(h))
        finally:
            self.unlock_image()
        return out

    def lock_image(self):
        """Renderer::lock_image_mutex (renderer.h:41)."""
        self._call("rt_lock_image")

    def unlock_image(self):
        """Renderer::unlock_image_mutex (renderer.h:42)."""
        self._call("rt_unlock_image")

    def request_aux(self, rgba=False, hit=False, shadow=False):
        self._call("rt_request_aux", int(rgba), int(hit), int(shadow))

    def get_internal(self, argb=True, rgba=False, hit=False, shadow=False):
        st = self.stats()
        n = st["render_width"] * st["render_height"]
        out = {}
        a = np.zeros(n, np.uint32) if argb else None
        r = np.zeros((n, 4), np.float32) if rgba else None
        hid = np.zeros(n, np.int32) if hit else None
        ht = np.zeros(n, np.float32) if hit else None
        sh = np.zeros(n, np.uint8) if shadow else None
        self._call("rt_get_internal", ptr(a, _u32p), ptr(r, _f32p), ptr(hid, _i32p), ptr(ht, _f32p), ptr(sh, _u8p))
        for k, v in (("argb", a), ("rgba", r), ("hit_id", hid), ("hit_t", ht), ("shadow", sh)):
            if v is not None:
                out[k] = v
        return out

    def get_ssao_buffers(self, ao=True):
        """(z, normals (n, 3), occlusion counts or None) of the last frame / SSAO pass."""
        st = self.stats()
        n = st["render_width"] * st["render_height"]
        z = np.zeros(n, np.float32)
        n4 = np.zeros((n, 4), np.float32)
        a = np.zeros(n, np.int32) if ao else None
        self._call("rt_get_ssao_buffers", ptr(z, _f32p), ptr(n4, _f32p), ptr(a, _i32p))
        return z, np.ascontiguousarray(n4[:, :3]), a

    def tile_costs(self):
        """The last frame's per-tile shader cycles, shape (tiles_y, tiles_x) (rt_tile_costs)."""
        tx, ty = C.c_int32(0), C.c_int32(0)
        self._call("rt_tile_costs", None, 0, C.byref(tx), C.byref(ty))
        out = np.zeros(tx.value * ty.value, np.uint32)
        self._call("rt_tile_costs", out.ctypes.data_as(C.POINTER(C.c_uint32)), out.size, C.byref(tx), C.byref(ty))
        return out.reshape(ty.value, tx.value)

    def ocone_read(self):
        """The resident origin-cone grid (rt_ocone_read): (cells uint32 [n, 2], dims int32 [3], lo_ih float32 [4])."""
        dims = np.zeros(3, np.int32)
        lo_ih = np.zeros(4, np.float32)
        i32 = C.POINTER(C.c_int32)
        f32p = C.POINTER(C.c_float)
        self._call("rt_ocone_read", None, 0, dims.ctypes.data_as(i32), lo_ih.ctypes.data_as(f32p))
        cells = np.zeros((int(np.prod(dims.astype(np.int64))), 2), np.uint32)
        self._call("rt_ocone_read", cells.ctypes.data_as(C.POINTER(C.c_uint32)), cells.size, dims.ctypes.data_as(i32),
                   lo_ih.ctypes.data_as(f32p))
        return cells, dims, lo_ih

    def debug_read(self, n):
        """Diagnostic builds: the last frame's per-wave records (rt_debug_read)."""
        out = np.zeros(n, np.uint64)
        self._call("rt_debug_read", out.ctypes.data_as(C.POINTER(C.c_uint64)), n)
        return out

    def stats(self) -> dict:
        s = RtStats()
        self._call("rt_get_stats", C.byref(s))
        return s.as_dict()

    # -- image strips (multi-GPU) ---------------------------------------------------
    def local_rows(self, band_rows, rank, nranks) -> int:
        n = C.c_int32()
        self._call("rt_local_rows", int(band_rows), int(rank), int(nranks), C.byref(n))
        return n.value

    def render_bands_device(self, band_rows, rank, nranks, d_out_ptr: int, stream_ptr: int = 0):
        self._call("rt_render_bands_device", int(band_rows), int(rank), int(nranks), C.c_void_p(d_out_ptr),
                   C.c_void_p(stream_ptr))

    def render_band_list_device(self, band_rows, bands, d_out_ptr: int, stream_ptr: int = 0):
        """rt_render_band_list_device: the listed output bands into consecutive local bands of d_out
        (cost-balanced strips, strips.assign_bands)."""
        b = np.ascontiguousarray(bands, np.int32)
        self._call("rt_render_band_list_device", int(band_rows), ptr(b, _i32p), int(b.size), C.c_void_p(d_out_ptr),
                   C.c_void_p(stream_ptr))

    def band_costs(self, nbands: int, stream_ptr: int = 0, out=None) -> np.ndarray:
        """rt_band_costs: the cost (tile shader cycles) of each output band of the last band launch on the
        stream; the bands it did not render stay as in ``out`` (zeros by default)."""
        c = np.zeros(nbands, np.float64) if out is None else np.ascontiguousarray(out, np.float64)
        self._call("rt_band_costs", C.c_void_p(stream_ptr), c.ctypes.data_as(C.POINTER(C.c_double)), int(nbands))
        return c

    def trace_rays(self, orig, dirs):
        """BVH::intersect for a batch of rays -> (tri_id, t, u, v, ret)."""
        o = f32(orig).reshape(-1, 3)
        d = f32(dirs).reshape(-1, 3)
        if d.shape != o.shape:
            raise ValueError(f"trace_rays: {o.shape[0]} origins but {d.shape[0]} directions")
        n = o.shape[0]
        ids = np.zeros(n, np.int32)
        t, u, v = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
        ret = np.zeros(n, np.uint8)
        self._call("rt_trace_rays", ptr(o, _f32p), ptr(d, _f32p), n, ptr(ids, _i32p), ptr(t, _f32p), ptr(u, _f32p),
                   ptr(v, _f32p), ptr(ret, _u8p))
        return ids, t, u, v, ret

    def wide_query(self, orig, dirs, kind=1):
        """rt_wide_query: the frames' wide-BVH query on the GPU with its status -> dict(o, d, status,
        id, t, u, v, shadowed); kind 0 plain rays, 1 camera rays, 2 (hit point, normal) pairs as
        is_shadowed's rays towards the light."""
        o = f32(orig).reshape(-1, 3)
        d = f32(dirs).reshape(-1, 3)
        if d.shape != o.shape:
            raise ValueError(f"wide_query: {o.shape[0]} origins but {d.shape[0]} directions")
        n = o.shape[0]
        out = dict(o=np.zeros((n, 3), np.float32), d=np.zeros((n, 3), np.float32), status=np.zeros(n, np.int32),
                   id=np.zeros(n, np.int32), t=np.zeros(n, np.float32), u=np.zeros(n, np.float32),
                   v=np.zeros(n, np.float32), shadowed=np.zeros(n, np.uint8))
        self._call("rt_wide_query", ptr(o, _f32p), ptr(d, _f32p), n, int(kind), ptr(out["o"], _f32p),
                   ptr(out["d"], _f32p), ptr(out["status"], _i32p), ptr(out["id"], _i32p), ptr(out["t"], _f32p),
                   ptr(out["u"], _f32p), ptr(out["v"], _f32p), ptr(out["shadowed"], _u8p))
        return out

    def risk_words(self, src=0):
        """rt_risk_words: the current camera / light risk words, src 0 the GPU's, 1 the host walk's
        -> (words, violations of check_risk_words)."""
        n, bad = C.c_int64(), C.c_int64()
        self._call("rt_risk_words", int(src), None, 0, C.byref(n), None)
        out = np.zeros(n.value, np.uint64)
        self._call("rt_risk_words", int(src), out.ctypes.data_as(C.POINTER(C.c_uint64)), out.size, C.byref(n),
                   C.byref(bad))
        return out, bad.value

    def trace_ray(self, orig, dirs, current_recursion_depth=0):
        """Renderer::trace_ray (shaded) for a batch of rays, each with a fresh HitInfo
        -> (rgba [n,4], hit_src, t, intersection_found, shadowed)."""
        o = f32(orig).reshape(-1, 3)
        d = f32(dirs).reshape(-1, 3)
        if d.shape != o.shape:
            raise ValueError(f"trace_ray: {o.shape[0]} origins but {d.shape[0]} directions")
        n = o.shape[0]
        rgba = np.zeros((n, 4), np.float32)
        src = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        found = np.zeros(n, np.uint8)
        shadowed = np.zeros(n, np.uint8)
        self._call("rt_trace_ray", ptr(o, _f32p), ptr(d, _f32p), n, int(current_recursion_depth), ptr(rgba, _f32p),
                   ptr(src, _i32p), ptr(t, _f32p), ptr(found, _u8p), ptr(shadowed, _u8p))
        return rgba, src, t, found, shadowed

    def kernel_times(self, n):
        ms = np.zeros(n, np.float32)
        self._call("rt_kernel_times", ptr(ms, _f32p), int(n))
        return ms

    def band_counters(self):
        a, b = C.c_int64(), C.c_int64()
        self._call("rt_band_counters", C.byref(a), C.byref(b))
        return a.value, b.value

    # -- convenience ----------------------------------------------------------------
    def load_scene(self, sc: SceneData, st: RenderSettings):
        """Settings, camera, light, materials, geometry and textures of a SceneData."""
        self.set_render_settings(st)
        self.change_render_size(st.image_width, st.image_height)
        self.set_camera_matrices(sc.cam_pos, sc.proj_inv, sc.cam_to_world)
        if sc.proj is not None and sc.world_to_cam is not None:
            self.set_camera_projection(sc.proj, sc.world_to_cam)
        self.set_camera_lens(*sc.lens(st))
        self.set_light_position(sc.light)
        self.set_materials(sc.materials)
        self.clear_geometry()
        for k in range(len(sc.shape_kind)):
            s = sc.shape[k]
            if sc.shape_kind[k] == SHAPE_SPHERE:
                self.add_sphere(s[:3], s[3], int(sc.shape_mat[k]))
            else:
                self.add_plane(s[:3], s[3:6], int(sc.shape_mat[k]))
        self.set_triangles(sc.tri, sc.tri_mat, sc.tri_uv)
        for slot in range(6):
            self._set_tex(slot, sc.textures.get(slot) if sc.textures else None)
        if sc.skybox is not None:
            self.set_skybox(sc.skybox)


def render(renderer: Renderer) -> float:
    """render(Renderer&) (utils/mainUtils.cpp:6-21): ray_trace + post_process; returns ms."""
    ms = C.c_float()
    check(_lib.lib().rt_render(renderer._h, C.byref(ms)), "rt_render")
    return float(ms.value)
