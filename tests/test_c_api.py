"""The C ABI from C: tests/c/render_golden.c is compiled against include/rt_mi355x.h alone and
renders reference golden cases through rt_render + rt_get_image, on one device and through
rt_set_devices (the single-process multi-device path: interleaved bands gathered to ids[0]).
The compile check runs on CPU; the renders need the GPU."""
import os
import struct
import subprocess

import numpy as np
import pytest

from golden_cases import Case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "render_golden.c")
EXE = os.path.join(ROOT, "tests", "c", "render_golden")
LIBDIR = os.path.join(ROOT, "raytracercpp_amd")


def build_c_program(out=EXE):
    """gcc, C99, warnings as errors, the public header and the in-tree library only."""
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", "-I", os.path.join(ROOT, "include"), SRC,
           "-o", out, "-L", LIBDIR, "-lrt_mi355x", "-Wl,-rpath," + LIBDIR, "-L/opt/rocm/lib",
           "-Wl,-rpath-link,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


def write_scene(path, sc, st):
    """The scene file render_golden.c reads (its header comment)."""
    from raytracercpp_amd.renderer import _to_c
    import ctypes as C
    cs = _to_c(st)
    fov, aspect = sc.lens(st)
    f32 = lambda a, n: np.ascontiguousarray(a, np.float32).reshape(-1)[:n].tobytes()
    has_proj = sc.proj is not None and sc.world_to_cam is not None
    with open(path, "wb") as f:
        f.write(b"RTSC" + struct.pack("<i", C.sizeof(cs)) + bytes(cs))
        f.write(f32(sc.cam_pos, 3) + f32(sc.proj_inv, 16) + f32(sc.cam_to_world, 16))
        f.write(struct.pack("<i", int(has_proj)))
        f.write(f32(sc.proj, 16) if has_proj else bytes(64))
        f.write(f32(sc.world_to_cam, 16) if has_proj else bytes(64))
        f.write(struct.pack("<ff", fov, aspect) + f32(sc.light, 3))
        m = np.ascontiguousarray(sc.materials, np.float32).reshape(-1, 16)
        f.write(struct.pack("<i", m.shape[0]) + m.tobytes())
        t = np.ascontiguousarray(sc.tri, np.float32).reshape(-1, 9)
        f.write(struct.pack("<q", t.shape[0]) + t.tobytes() + np.ascontiguousarray(sc.tri_mat, np.int32).tobytes())
        f.write(struct.pack("<i", int(sc.tri_uv is not None)))
        if sc.tri_uv is not None:
            f.write(np.ascontiguousarray(sc.tri_uv, np.float32).tobytes())


def read_image(path):
    with open(path, "rb") as f:
        w, h = struct.unpack("<ii", f.read(8))
        return np.frombuffer(f.read(), np.uint32).reshape(h, w)


def test_c_program_compiles(tmp_path):
    exe = build_c_program(str(tmp_path / "render_golden"))
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr   # argument check only: no GPU call


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["robot", "ssaa3_cube", "raster_robot", "c4_sphere1m"])
@pytest.mark.parametrize("devices", [[], [0]])
def test_c_program_renders_golden(tmp_path, name, devices):
    """rt_render + rt_get_image from C give the reference's final image; with rt_set_devices([0])
    the frame goes through the band / gather path (bands of 8 rows re-assembled on device 0)."""
    exe = EXE if os.path.exists(EXE) else build_c_program(str(tmp_path / "render_golden"))
    c = Case(name)
    scene = str(tmp_path / "scene.bin")
    out = str(tmp_path / "image.bin")
    write_scene(scene, c.scene, c.settings)
    r = subprocess.run([exe, scene, out] + [str(d) for d in devices], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    img = read_image(out)
    exp = c.expected()
    want = exp["final"] if c.settings.enable_ssaa else exp["argb"]
    assert img.shape == (c.settings.image_height, c.settings.image_width)
    assert np.array_equal(img.ravel(), want.ravel()), f"{int((img.ravel() != want.ravel()).sum())} pixels differ"
