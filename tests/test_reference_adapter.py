"""The reference-side binding (include/reference_adapter/gpu_renderer.h) compiled
against the reference's own Qt-free headers in /root/reference (triangle.h, materials.h,
camera.h, mat.h, rendererSettings.h) and this repository's C ABI, and linked with the reference's
own compiled Triangle / vector / colour / matrix translation units (oracle/_ref, `make -C oracle
ref`).  The program tests/c/adapter_golden builds the scene from reference types and renders it
through GpuRenderer.  Compiled here (CPU test, where /root/reference exists); the built program
travels to the GPU box, which renders reference golden cases through it."""
import os
import subprocess

import numpy as np
import pytest

from golden_cases import Case
from test_c_api import read_image, write_scene

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/tp2"
SRC = os.path.join(ROOT, "tests", "c", "adapter_golden.cpp")
EXE = os.path.join(ROOT, "tests", "c", "adapter_golden")
LIBDIR = os.path.join(ROOT, "raytracercpp_amd")
REF_OBJ = os.path.join(ROOT, "oracle", "_ref", "obj")


def build_adapter_program(out=EXE):
    """g++ -Wall -Wextra -Werror on the adapter (its own code) with the reference's headers; the
    reference's TUs (Triangle, Point / Vector, Color, Transform, Camera) from oracle/_ref."""
    objs = [os.path.join(REF_OBJ, p) for p in ("projets/triangle.o", "projets/ray.o", "src/vec.o", "src/mat.o",
                                               "src/color.o", "projets/scene/camera.o")]
    incs = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "include", "reference_adapter")]
    for d in ("src", "projets", "projets/scene", "projets/renderer"):
        incs += ["-isystem", os.path.join(REF, d)]   # the reference's headers: its own warnings are not ours
    cmd = (["g++", "-std=gnu++17", "-Wall", "-Wextra", "-Werror", "-O1"] + incs + [SRC] + objs +
           ["-o", out, "-L", LIBDIR, "-lrt_mi355x", "-Wl,-rpath," + LIBDIR, "-L/opt/rocm/lib",
            "-Wl,-rpath-link,/opt/rocm/lib", "-lm"])
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="/root/reference absent (the GPU box uses the built program)")
def test_adapter_compiles_against_reference_headers(tmp_path):
    exe = build_adapter_program(str(tmp_path / "adapter_golden"))
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr   # argument check only: no GPU call


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["robot", "ssaa3_cube", "c3_bumpy70k", "raster_robot"])
def test_adapter_renders_golden(tmp_path, name):
    """The reference's types through GpuRenderer give the reference's final image (the
    reference-generated golden of tests/golden)."""
    if not os.path.exists(EXE):
        pytest.fail("tests/c/adapter_golden not built: __graft_entry__.build() compiles it where /root/reference "
                    "exists, and the built program travels to the GPU box")
    c = Case(name)
    scene = str(tmp_path / "scene.bin")
    out = str(tmp_path / "image.bin")
    write_scene(scene, c.scene, c.settings)
    r = subprocess.run([EXE, scene, out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    img = read_image(out)
    exp = c.expected()
    want = exp["final"] if c.settings.enable_ssaa else exp["argb"]
    assert img.shape == (c.settings.image_height, c.settings.image_width)
    assert np.array_equal(img.ravel(), want.ravel()), f"{int((img.ravel() != want.ravel()).sum())} pixels differ"
