"""The C side of the cgo shim.

cgo compiles its preamble and calls as C, so examples/cornell_c99.c — the Go
cornellBox (main.go:278-320) lowered one C constructor call per Go constructor, then
(*Camera).Render (camera.go:156) as rt_scene_create + rt_render + rt_format_ppm — is
built here as strict C99 against include/rt_abi.h and librt_amd.so.  The Go side
itself cannot be compiled (no Go toolchain in the image); these tests pin everything
below it: the header is valid C, the library links from C, the C-built scene is the
harness's scene, and (GPU) its render is the harness's render bit for bit.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "go_raytracer_amd")
SRC = os.path.join(REPO, "examples", "cornell_c99.c")


@pytest.fixture(scope="module")
def client(rt, tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("no C compiler")
    exe = str(tmp_path_factory.mktemp("cclient") / "cornell_c99")
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(REPO, "include"), SRC, "-L", LIBDIR, "-lrt_amd",
                    "-Wl,-rpath," + LIBDIR, "-o", exe], check=True)
    return exe


def _run(exe, *args):
    p = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_c99_client_builds_the_harness_scene(rt, client):
    info = _run(client, "info")
    t, cam, w, l = rt.demo_scene("cornell")
    with rt.Scene(t, w, l) as sc:
        ref = sc.info()
    assert info["abi"] == rt.lib().rt_abi_version()
    for k in ("n_quads", "n_world_prims", "n_lights", "n_materials", "n_textures",
              "n_bvh_nodes", "features"):
        assert info[k] == ref[k], k


@pytest.mark.gpu
def test_c99_client_render_is_the_harness_render(rt, gpu, client, tmp_path):
    out = tmp_path / "img.f32"
    st = _run(client, "render", 96, 16, 7, out)
    img = np.fromfile(out, dtype=np.float32).reshape(st["height"], st["width"], 3)
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width, cam.SamplesPerPixel = 96, 16
    with rt.Scene(t, w, l) as sc:
        ref, rst = sc.render(cam, seed=7)
    assert np.array_equal(img, ref, equal_nan=True)
    assert st["segments"] == rst["segments"]
    ppm = tmp_path / "img.ppm"
    _run(client, "ppm", 96, 16, 7, ppm)
    assert ppm.read_bytes() == rt.format_ppm(ref)
