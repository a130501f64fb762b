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
    assert rt.lib().rt_abi_version() == 2  # 2: rt_render_multi, rt_stats.overflow_samples


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
