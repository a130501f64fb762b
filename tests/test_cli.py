"""rtbench, the main.go command line (main.go:414-478) over the C ABI.

CPU tests pin the flag handling the reference gets from Go's flag package
(unknown flag / bad value -> usage + exit 2, -h -> exit 0) and main.go's
defaultScene behaviour (the output file is created and left empty).  The GPU
test checks that the CLI's image is byte-identical to the Python harness's
render of the same scene, seed and overrides (same library, same kernels)."""
import json
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "go_raytracer_amd", "rtbench")

pytestmark = pytest.mark.skipif(not os.path.exists(CLI), reason="rtbench not built (make -C go_raytracer_amd/csrc)")


def run(*args, cwd=None, timeout=120):
    return subprocess.run([CLI, *args], capture_output=True, text=True, cwd=cwd, timeout=timeout)


def test_help_lists_the_reference_flags():
    r = run("-h")
    assert r.returncode == 0
    for f in ("-N int", "-S int", "-o string", "-cpuprofile string"):
        assert f in r.stderr
    assert '(default "image.ppm")' in r.stderr


@pytest.mark.parametrize("args", [["-x"], ["-S", "six"], ["-N"], ["-seed", "-1"], ["---S=1"],
                                  ["-progress=maybe"]])
def test_bad_flags_exit_2(args):
    r = run(*args)
    assert r.returncode == 2, r
    assert "Usage of" in r.stderr


@pytest.mark.parametrize("scene", [[], ["-S", "-1"], ["-S=0"], ["-S", "9"], ["--S", "42"]])
def test_default_scene_writes_an_empty_file(tmp_path, scene):
    out = tmp_path / "image.ppm"
    r = run(*scene, "-o", str(out))
    assert r.returncode == 0, r.stderr
    assert out.exists() and out.stat().st_size == 0


def test_default_output_name(tmp_path):
    r = run(cwd=tmp_path)
    assert r.returncode == 0
    assert (tmp_path / "image.ppm").exists()


def test_flag_parsing_stops_at_first_non_flag(tmp_path):
    # "-S 6" after a positional argument is not parsed (Go's flag.Parse): default scene
    out = tmp_path / "a.ppm"
    r = run("-o", str(out), "positional", "-S", "6")
    assert r.returncode == 0 and out.stat().st_size == 0


def test_unwritable_output_fails(tmp_path):
    r = run("-o", str(tmp_path / "no" / "such" / "dir.ppm"))
    assert r.returncode == 1
    assert "Error creating output file" in r.stderr


def test_render_without_device_fails_loudly(rt, tmp_path):
    if rt.device_count() > 0:
        pytest.skip("a HIP device is visible")
    r = run("-S", "6", "-width", "8", "-spp", "1", "-o", str(tmp_path / "c.ppm"))
    assert r.returncode == 1
    assert "no HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("scene,name", [(6, "cornell"), (1, "book1")])
def test_cli_image_matches_harness(rt, gpu, tmp_path, scene, name):
    out, prof = tmp_path / "img.ppm", tmp_path / "prof.json"
    r = run("-S", str(scene), "-width", "40", "-spp", "9", "-depth", "6", "-seed", "5",
            "-o", str(out), "-cpuprofile", str(prof), "-progress", "-stats")
    assert r.returncode == 0, r.stderr
    assert "100.0%" in r.stderr
    t, cam, w, l = rt.demo_scene(name)
    cam.Width, cam.SamplesPerPixel, cam.MaxDepth = 40, 9, 6
    with rt.Scene(t, w, l) as sc:
        img, st = sc.render(cam, seed=5, progress_slices=20)
    assert out.read_bytes() == rt.format_ppm(img)
    js = json.loads(prof.read_text())
    assert js["scene"] == name and js["samples"] == st["samples"] == 40 * img.shape[0] * 9
    assert np.isfinite(js["samples_per_s"])


@pytest.mark.gpu
@pytest.mark.parametrize("scene,slices", [(1, 1024), (1, 7), (4, 1024), (6, 1024)])
def test_cli_short_progress_slices_terminate(rt, gpu, tmp_path, scene, slices):
    """the r5i session's book1 render at 40 px, 9 spp with progress slices
    never finished its last slice (the build then carried an in-shading chunk pool, removed in
    8001c64).  Slices shorter than one chunk batch (3,120 chunks over 1,024 launches), with the
    drain split on, in a child process with a time limit: every launch must end.  The image
    is the one of a single launch (exact pixel sums)."""
    out1, out2 = tmp_path / "a.ppm", tmp_path / "b.ppm"
    common = ["-S", str(scene), "-width", "40", "-spp", "9", "-depth", "6", "-seed", "5"]
    r = run(*common, "-o", str(out1), "-slices", str(slices), "-progress", timeout=60)
    assert r.returncode == 0, r.stderr
    assert "100.0%" in r.stderr
    r = run(*common, "-o", str(out2), timeout=60)
    assert r.returncode == 0, r.stderr
    assert out1.read_bytes() == out2.read_bytes()
