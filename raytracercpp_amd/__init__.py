"""MI355X-native primary-ray + shadow-ray renderer (drop-in for TomClabault/RayTracerCPP's
ray-trace hot path).  The compute path is librt_mi355x.so (HIP, gfx950); see DESIGN.md."""
from .scene import RenderSettings, SceneData, material  # noqa: F401
from . import scenes  # noqa: F401


def Renderer(*args, **kwargs):
    from .renderer import Renderer as _R
    return _R(*args, **kwargs)


def render(renderer):
    from .renderer import render as _r
    return _r(renderer)
