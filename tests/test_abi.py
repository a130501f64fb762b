"""The C ABI library loads and exports every symbol include/rt_abi.h declares;
ctypes struct layouts match the C compiler's (no compute calls: CPU-only)."""
import ctypes as C
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(REPO, "include", "rt_abi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*(rt_[a-z0-9_]+)\s*\(",
                       src, flags=re.M)
    return sorted(set(names))


def test_every_declared_symbol_is_exported(rt):
    names = declared_functions()
    assert len(names) >= 40
    L = C.CDLL(rt._lib.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_bindings_cover_header(rt):
    assert set(declared_functions()) == set(rt._lib.SIGNATURES), \
        set(declared_functions()) ^ set(rt._lib.SIGNATURES)


def test_abi_version(rt):
    # 2: rt_render_multi, rt_stats.overflow_samples; 3: rt_tune_set (no environment reads),
    # rt_scene_info.tuned, rt_stats.tuned / chunk_records; 4: rt_tune_get, rt_tune_set refuses
    # values that are not a number in the knob's range
    assert rt.lib().rt_abi_version() == 4


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no C compiler")
def test_struct_layouts_match_c(rt, tmp_path):
    from go_raytracer_amd import _lib
    structs = {"rt_camera": _lib.RtCamera, "rt_camera_derived": _lib.RtCameraDerived,
               "rt_scene_info": _lib.RtSceneInfo, "rt_render_opts": _lib.RtRenderOpts,
               "rt_stats": _lib.RtStats, "rt_tree_view": _lib.RtTreeView,
               "rt_obj_image": _lib.RtObjImage, "rt_obj_options": _lib.RtObjOptions,
               "rt_obj_info": _lib.RtObjInfo}
    prog = ['#include <stdio.h>', '#include "rt_abi.h"', "int main(void){"]
    for n in structs:
        prog.append(f'printf("{n} %zu\\n", sizeof({n}));')
    prog.append("return 0;}")
    c = tmp_path / "sz.c"
    c.write_text("\n".join(prog))
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(c), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    for line in out.strip().splitlines():
        n, sz = line.split()
        assert C.sizeof(structs[n]) == int(sz), (n, C.sizeof(structs[n]), sz)


def test_errors_are_codes_not_aborts(rt):
    t = rt.Tree()
    with pytest.raises(rt.RtError) as e:
        t.sphere((0, 0, 0), 1, 99)  # bad material handle
    assert e.value.code == -1
    assert "rt_new_sphere" in rt.lib().rt_last_error().decode()
    with pytest.raises(rt.RtError):
        t.bvh(t.list())  # BuildBVH of an empty list dereferences nil in the reference


def test_device_count_never_aborts(rt):
    assert rt.device_count() >= 0


def test_progress_without_render(rt):
    t, cam, w, l = rt.demo_scene("cornell")
    with rt.Scene(t, w, l) as sc:
        assert sc.progress() == (0, 0)


def test_render_multi_argument_errors(rt):
    """rt_render_multi validates its arguments before touching a device."""
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width, cam.SamplesPerPixel = 8, 1
    with rt.Scene(t, w, l) as sc:
        with pytest.raises(rt.RtError):
            sc.render_multi(cam, [])


def _all_knobs_off_default(rt):
    """A non-default value for every knob the library knows (rt_tune_list)."""
    odd = {"RT_BVH_BUILDER": "host", "RT_WAVE_TIMES": "/nonexistent/wt.bin", "RT_BIG_SPHERE_R": "1e30",
           "RT_BVH_CT": "3.5", "RT_BVH_CI": "0.25", "RT_THREADS": "3"}
    return {k: odd.get(k, "0" if k not in ("RT_TREE", "RT_BVH8", "RT_FEATURES_ALL", "RT_TIMING")
                       else "1") for k in rt.tune_knobs()}


def _scene_state(rt, name):
    t, cam, w, l = rt.demo_scene(name)
    with rt.Scene(t, w, l) as sc:
        info = sc.info()
        nodes, refs, root, bounds = sc.export_bvh()
        return info, nodes.tobytes(), refs.tobytes(), root, sc.export_bvh8()[0].size


@pytest.mark.parametrize("name", ["cornell", "book2", "book1"])
def test_environment_does_not_configure_the_library(rt, name, monkeypatch):
    """the library reads no RT_* environment variable.  With every knob
    set to a non-default value in the environment, a scene's info, BVH and kernel features
    are those of a clean environment, and it reports no tuning (rt_scene_info.tuned = 0)."""
    base = _scene_state(rt, name)
    assert base[0]["tuned"] == 0
    knobs = _all_knobs_off_default(rt)
    assert len(knobs) >= 30
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("RT_BVH_BUILDER", "device")  # would fail without a GPU if it were read
    assert _scene_state(rt, name) == base


def test_tuning_is_explicit_and_reported(rt, tune):
    """Knobs change behaviour only through rt_tune_set, and the scene reports them."""
    assert rt.tune_knobs()["RT_BOX_LEAVES"] is True  # changes image bits
    assert rt.tune_knobs()["RT_STEP_BUDGET"] is False  # moves work only
    with pytest.raises(rt.RtError):
        rt.tune("RT_NOT_A_KNOB", 1)
    t, cam, w, l = rt.demo_scene("book1")  # its perlin orbs are built but never placed
    with rt.Scene(t, w, l) as sc:
        feats = sc.info()["features"]
    tune("RT_FEATURES_ALL", 1)
    tune("RT_TIMING", 0)
    t, cam, w, l = rt.demo_scene("book1")
    with rt.Scene(t, w, l) as sc:
        info = sc.info()
    assert info["tuned"] == 2 and info["features"] != feats
    rt.untune()
    with rt.tuning(RT_BVH_LEAF=2):
        t, cam, w, l = rt.demo_scene("book1")
        with rt.Scene(t, w, l) as sc:
            assert sc.info()["tuned"] == 1
    t, cam, w, l = rt.demo_scene("book1")
    with rt.Scene(t, w, l) as sc:
        assert sc.info()["tuned"] == 0


@pytest.mark.parametrize("name,value", [
    ("RT_STEP_BUDGET", "0"), ("RT_STEP_BUDGET", "-3"), ("RT_STEP_BUDGET", "abc"),
    ("RT_STEP_BUDGET", "5x"), ("RT_STEP_BUDGET", ""), ("RT_SHADE_MIN", "0"), ("RT_TAIL_K", "0"),
    ("RT_CHUNK_NEED", "1e3"), ("RT_PARTS_LOG2", "7"), ("RT_BVH_CT", "nan"), ("RT_QBVH", "2"),
    ("RT_BVH_BUILDER", "gpu"), ("RT_GRAB_MIN", "99999999999999999999"), ("RT_SWEEP", "backwards"),
])
def test_tune_set_refuses_bad_values(rt, tune, name, value):
    """a scheduling knob out of range (a step budget of 0 would leave every traversal
    without steps and the fused loop spinning) is refused with RT_ERR_INVALID, before any render,
    and the knob keeps its previous value."""
    tune(name, {"RT_BVH_BUILDER": "host", "RT_BVH_CT": "2.5", "RT_SWEEP": "reverse"}.get(name, "1"))
    before = rt.tune_get(name)
    with pytest.raises(rt.RtError, match="rt_tune_set"):
        rt.tune(name, value)
    assert rt.tune_get(name) == before


def test_tune_get_and_tuning_restores(rt, tune):
    """rt_tune_get reads a knob back; rt.tuning puts back the values knobs had on entry."""
    assert rt.tune_get("RT_GRAB_MIN") is None
    with pytest.raises(rt.RtError):
        rt.tune_get("RT_NOT_A_KNOB")
    tune("RT_GRAB_MIN", 64)
    assert rt.tune_get("RT_GRAB_MIN") == "64"
    assert int(rt.lib().rt_tune_get(b"RT_GRAB_MIN", None, 0)) == 3
    with rt.tuning(RT_GRAB_MIN=8, RT_SPLIT_MIN=0):
        assert rt.tune_get("RT_GRAB_MIN") == "8" and rt.tune_get("RT_SPLIT_MIN") == "0"
    assert rt.tune_get("RT_GRAB_MIN") == "64" and rt.tune_get("RT_SPLIT_MIN") is None
    with pytest.raises(rt.RtError):
        with rt.tuning(RT_SPLIT_MIN=1, RT_STEP_BUDGET=0):
            pass
    assert rt.tune_get("RT_SPLIT_MIN") is None and rt.tune_get("RT_STEP_BUDGET") is None
