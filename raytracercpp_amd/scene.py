"""Scene description shared by the product renderer, the parity tests and bench.py.

A :class:`SceneData` is plain arrays: world-space triangles (as
``MeshIOUtils::create_triangles`` leaves them, tp2/projets/utils/meshIOUtils.cpp:4-30),
analytic shapes (``Renderer::add_analytic_shape``, renderer.cpp:146), the material
table (``Material``, tp2/src/materials.h:14-38), camera matrices
(``Camera``, tp2/projets/scene/camera.h:9-33), the point light and textures.

:class:`RenderSettings` mirrors ``RenderSettings`` field for field
(tp2/projets/renderer/rendererSettings.h:6-105), plus ``rng_seed`` for the
counter-based rough-reflection RNG.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

# RenderSettings::ShadingMethod (rendererSettings.h:8-25)
RT_SHADING = 0
ABS_NORMALS_SHADING = 1
PASTEL_NORMALS_SHADING = 2
BARYCENTRIC_COORDINATES_SHADING = 3
VISUALIZE_AO = 4

# texture slots (renderer.h:77-84)
TEX_AO, TEX_DIFFUSE, TEX_NORMAL, TEX_DISPLACEMENT, TEX_ROUGHNESS, TEX_SKYSPHERE = range(6)

# material record layout (16 float32)
MAT_AMBIENT, MAT_DIFFUSE, MAT_SPECULAR, MAT_EMISSION = 0, 3, 6, 9
MAT_REFLECTION, MAT_ROUGHNESS, MAT_NS, MAT_SPEC_THRESHOLD = 12, 13, 14, 15
MAT_STRIDE = 16

SHAPE_SPHERE = 0
SHAPE_PLANE = 1


@dataclass
class RenderSettings:
    """rendererSettings.h:6-105 (defaults identical)."""

    image_width: int = 1024
    image_height: int = 1024
    enable_ssaa: bool = False
    ssaa_factor: int = 2
    shading_method: int = RT_SHADING
    compute_shadows: bool = False
    max_recursion_depth: int = 5
    enable_bvh: bool = True
    bvh_max_depth: int = 12
    bvh_leaf_object_count: int = 40
    enable_ambient: bool = True
    enable_diffuse: bool = True
    enable_specular: bool = True
    enable_emissive: bool = True
    rough_reflections_sample_count: int = 3
    enable_ao_mapping: bool = False
    enable_diffuse_mapping: bool = False
    enable_normal_mapping: bool = False
    enable_displacement_mapping: bool = False
    displacement_mapping_strength: float = 0.02
    parallax_mapping_steps: int = 32
    enable_roughness_mapping: bool = False
    enable_skysphere: bool = False
    enable_skybox: bool = False
    rng_seed: int = 0x5EED1234
    enable_clipping: bool = True                 # raster_trace frustum clipping
    hybrid_rasterization_tracing: bool = False   # render(): raster_trace instead of ray_trace
    enable_ssao: bool = False                    # post_process: SSAO before the SSAA downscale
    ssao_sample_count: int = 64
    ssao_radius: float = 0.5
    ssao_amount: float = 1.0

    def render_size(self):
        """Renderer::get_render_width_height (renderer.cpp:116-120)."""
        if self.enable_ssaa:
            return self.image_width * self.ssaa_factor, self.image_height * self.ssaa_factor
        return self.image_width, self.image_height

    def copy(self, **kw) -> "RenderSettings":
        return dataclasses.replace(self, **kw)


def material(diffuse=(0.0, 0.0, 0.0), specular=(0.0, 0.0, 0.0), emission=(0.0, 0.0, 0.0),
             ambient=(1.0, 1.0, 1.0), reflection=0.0, roughness=0.0, ns=0.0, specular_threshold=0.0):
    """One Material record (materials.h:18-37); default ctor gives ambient_coeff = 1."""
    m = np.zeros(MAT_STRIDE, dtype=np.float32)
    m[MAT_AMBIENT:MAT_AMBIENT + 3] = ambient
    m[MAT_DIFFUSE:MAT_DIFFUSE + 3] = diffuse
    m[MAT_SPECULAR:MAT_SPECULAR + 3] = specular
    m[MAT_EMISSION:MAT_EMISSION + 3] = emission
    m[MAT_REFLECTION] = reflection
    m[MAT_ROUGHNESS] = roughness
    m[MAT_NS] = ns
    m[MAT_SPEC_THRESHOLD] = specular_threshold
    return m


@dataclass
class SceneData:
    tri: np.ndarray                       # (n, 9) float32
    tri_mat: np.ndarray                   # (n,) int32
    tri_uv: Optional[np.ndarray]          # (n, 6) float32 or None
    shape_kind: np.ndarray                # (k,) int32
    shape: np.ndarray                     # (k, 6) float32
    shape_mat: np.ndarray                 # (k,) int32
    materials: np.ndarray                 # (m, 16) float32
    cam_pos: np.ndarray                   # (3,) float32
    proj_inv: np.ndarray                  # (16,) float32 row-major
    cam_to_world: np.ndarray              # (16,) float32 row-major
    light: np.ndarray                     # (3,) float32
    textures: Dict[int, np.ndarray] = field(default_factory=dict)   # slot -> (h, w, 4) float32
    skybox: Optional[List[np.ndarray]] = None                        # 6 faces (h, w, 4) float32
    proj: Optional[np.ndarray] = None           # (16,) Camera::_perspective_proj_mat (raster_trace)
    world_to_cam: Optional[np.ndarray] = None   # (16,) Camera::_world_to_camera_mat (raster_trace)
    cam_fov: float = 80.0                       # Camera::_fov (SSAO, renderer.cpp:1245, 1379)
    cam_aspect: Optional[float] = None          # Camera::_aspect_ratio; None: render_w / render_h

    def lens(self, st: "RenderSettings"):
        """(Camera::_fov, Camera::_aspect_ratio) as float32; the aspect defaults to
        set_aspect_ratio(render_w / render_h) (renderer.cpp:93, 260)."""
        if self.cam_aspect is not None:
            return float(np.float32(self.cam_fov)), float(np.float32(self.cam_aspect))
        rw, rh = st.render_size()
        return float(np.float32(self.cam_fov)), float(np.float32(rw) / np.float32(rh))

    @property
    def ntri(self) -> int:
        return int(self.tri.shape[0])

    def triangle_hash(self) -> str:
        import hashlib
        h = hashlib.sha256()
        h.update(np.ascontiguousarray(self.tri, dtype=np.float32).tobytes())
        h.update(np.ascontiguousarray(self.tri_mat, dtype=np.int32).tobytes())
        if self.tri_uv is not None:
            h.update(np.ascontiguousarray(self.tri_uv, dtype=np.float32).tobytes())
        return h.hexdigest()


def empty_shapes():
    return (np.zeros(0, np.int32), np.zeros((0, 6), np.float32), np.zeros(0, np.int32))


def bits_to_f32(bits) -> np.ndarray:
    return np.asarray(bits, dtype=np.uint32).view(np.float32).copy()


def f32_to_bits(a) -> List[int]:
    return [int(x) for x in np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).ravel()]
