"""OBJ/MTL loader: the C loader (csrc/host_obj.cpp) against
the Python restatement of objLoader.go / mtlLoader.go (oracle/objload.py) —
bit-identical triangles, same materials, same light list — plus hand-derived
expectations that pin the restatement itself (the reference ships no OBJ
fixture or loader test).  CPU only: nothing renders here."""
import ctypes as C
import math
import os
import struct

import numpy as np
import pytest

from oracle import objload

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "obj")

NODE = np.dtype([("kind", "<i4"), ("mat", "<i4"), ("a", "<i4"), ("b", "<i4"), ("p", "<f8", 10)])
TRI = np.dtype([("v", "<f8", 9), ("n", "<f8", 9), ("uv", "<f8", 6), ("flags", "<i4"),
                ("mat", "<i4")])
MAT = np.dtype([("kind", "<i4"), ("tex", "<i4"), ("albedo", "<f8", 3), ("fuzz", "<f8"),
                ("ior", "<f8")])
TEX = np.dtype([("kind", "<i4"), ("a", "<i4"), ("b", "<i4"), ("variant", "<i4"),
                ("color", "<f8", 3), ("scale", "<f8")])
IMG = np.dtype([("w", "<i4"), ("h", "<i4"), ("rgb", "<u8")])


def _arr(ptr, n, dt):
    if n == 0:
        return np.zeros(0, dt)
    buf = (C.c_char * (n * dt.itemsize)).from_address(ptr)
    return np.frombuffer(bytes(buf), dtype=dt)


def tree_triangles(tree, model, lights):
    """(triangles, light indices) from the C tree: the BVH's children in order."""
    v = tree.view()
    nodes = _arr(v.nodes, v.n_nodes, NODE)
    kids = _arr(v.children, v.n_children, np.dtype("<i4"))
    tris = _arr(v.tris, v.n_tris, TRI)
    mats = _arr(v.materials, v.n_materials, MAT)
    texs = _arr(v.textures, v.n_textures, TEX)
    imgs = _arr(v.images, v.n_images, IMG)

    def image(i):
        im = imgs[i]
        data = bytes((C.c_char * int(im["w"] * im["h"] * 3)).from_address(int(im["rgb"])))
        return (int(im["w"]), int(im["h"]), data)

    def desc(mid):
        m = mats[mid]
        k = int(m["kind"])
        if k == 1:
            return ("metal", tuple(float(x) for x in m["albedo"]), float(m["fuzz"]))
        if k == 2:
            return ("dielectric", float(m["ior"]))
        t = texs[m["tex"]]
        name = {0: "lambertian", 3: "light", 4: "isotropic"}[k]
        if int(t["kind"]) == 2:
            return (name + "_image", image(int(t["a"])))
        return (name, tuple(float(x) for x in t["color"]))

    bvh = nodes[model]
    assert bvh["kind"] == 1  # BuildBVH (objLoader.go:512)
    ids = kids[bvh["a"]:bvh["a"] + bvh["b"]]
    out = []
    for nid in ids:
        nd = nodes[nid]
        assert nd["kind"] == 4
        tr = tris[nd["a"]]
        fl = lambda a: [float(x) for x in a]  # noqa: E731
        out.append((fl(tr["v"]), fl(tr["n"]) if tr["flags"] & 1 else None,
                    fl(tr["uv"]) if tr["flags"] & 2 else None, desc(int(tr["mat"]))))
    ln = nodes[lights]
    assert ln["kind"] == 0
    lids = list(kids[ln["a"]:ln["a"] + ln["b"]])
    pos = {int(n): i for i, n in enumerate(ids)}
    return out, [pos[int(n)] for n in lids]


def bits(x):
    return None if x is None else [struct.pack("<d", float(c)) for c in x]


def oracle_desc(d, images):
    if d[0].endswith("_image"):
        return (d[0], images[d[1]])
    return d


def same(c_tris, c_lights, ref, images):
    assert len(c_tris) == len(ref.tris)
    for i, (a, b) in enumerate(zip(c_tris, ref.tris)):
        assert bits(a[0]) == bits(b[0]), (i, a[0], b[0])
        assert bits(a[1]) == bits(b[1]), (i, a[1], b[1])
        assert bits(a[2]) == bits(b[2]), (i, a[2], b[2])
        da, db = a[3], oracle_desc(b[3], images)
        assert da[0] == db[0], (i, da, db)
        assert repr(da) == repr(db), (i, da, db)
    assert c_lights == ref.lights


@pytest.fixture
def mixed(tmp_path):
    """The mixed fixture with its texture map written next to it (map paths are
    opened as written, relative to the working directory: imageLoader.go:30)."""
    tex = tmp_path / "tex.ppm"
    rgb = bytes([255, 0, 0, 0, 255, 0, 0, 0, 255, 255, 255, 255, 10, 20, 30, 40, 50, 60])
    tex.write_bytes(b"P6\n3 2\n255\n" + rgb)
    obj = open(os.path.join(FIX, "mixed.obj"), "rb").read()
    mtl = open(os.path.join(FIX, "mixed.mtl"), "rb").read().replace(b"@TEX@", str(tex).encode())
    (tmp_path / "mixed.obj").write_bytes(obj)
    (tmp_path / "mixed.mtl").write_bytes(mtl)
    return tmp_path, obj, mtl, {str(tex): (3, 2, rgb)}


OPTION_SETS = [
    {},
    {"ScaleFactor": 5.0, "Position": (0.0, 1.8, 0.0)},
    {"FlipYZ": True, "FlipFaces": True},
    {"Center": False, "Position": (9.0, 9.0, 9.0)},
    {"IgnoreNormals": True, "FindWindows": True},
    {"IgnoreMtl": True},
]


@pytest.mark.parametrize("opts", OPTION_SETS, ids=lambda o: ",".join(o) or "defaults")
def test_loader_matches_restatement(rt, mixed, opts):
    d, obj, mtl, images = mixed
    t = rt.Tree()
    o = rt.LoadObjOptions(Debug=False, **opts)
    model, lights = t.LoadObjWithOptions(str(d / "mixed.obj"), o)
    c_tris, c_lights = tree_triangles(t, model, lights)
    kw = dict(scale=o.ScaleFactor, flip_yz=o.FlipYZ, ignore_normals=o.IgnoreNormals,
              center=o.Center, flip_faces=o.FlipFaces, position=o.Position,
              ignore_mtl=o.IgnoreMtl, find_windows=o.FindWindows)
    ref = objload.load_obj(obj, mtl, **kw)
    same(c_tris, c_lights, ref, images)
    info = t.last_obj_info
    assert (info.n_vertices, info.n_normals, info.n_texcoords, info.n_triangles) == \
        (ref.n_vertices, ref.n_normals, ref.n_texcoords, len(ref.tris))
    assert info.n_lights == len(ref.lights)
    assert info.n_materials == ref.n_materials


def test_memory_form_matches_file_form(rt, mixed):
    d, obj, mtl, images = mixed
    t1, t2 = rt.Tree(), rt.Tree()
    o = rt.LoadObjOptions(Debug=False)
    a = tree_triangles(t1, *t1.LoadObjWithOptions(str(d / "mixed.obj"), o))
    b = tree_triangles(t2, *t2.LoadObjWithOptions(None, o, mtl_text=mtl, obj_text=obj))
    assert repr(a) == repr(b)


def test_hand_derived_expectations(rt, mixed):
    """Pins the restatement: values worked out by hand from objLoader.go."""
    d, obj, mtl, images = mixed
    t = rt.Tree()
    model, lights = t.LoadObjWithOptions(str(d / "mixed.obj"), rt.LoadObjOptions(Debug=False))
    tris, lidx = tree_triangles(t, model, lights)
    # bounds of the 39 vertices: x [-3, 5], y [-3, 5], z [-3.5, 3.5] -> centre (1, 1, 0)
    info = t.last_obj_info
    assert list(info.center) == [1.0, 1.0, 0.0]
    # first face "f 1/1/1 2/2/1 3/3/2 4/4/2": fan (1,2,3), (1,3,4), centred
    assert tris[0][0] == [-1.0, -1.0, 0.0, 1.0, -1.0, 0.0, 1.0, 1.0, 0.0]
    assert tris[1][0] == [-1.0, -1.0, 0.0, 1.0, 1.0, 0.0, -1.0, 1.0, 0.0]
    assert tris[0][2] == [0, 0, 1, 0, 1, 1] and tris[1][2] == [0, 0, 1, 1, 0, 1]
    s = 1 / math.sqrt(2)
    assert tris[0][1] == [0, 0, 1, 0, 0, 1, 0, s, s]  # vn normalised by x * (1/len)
    assert tris[0][3] == ("lambertian", (0.73, 0.73, 0.73))
    # pentagon: 3 fan triangles, normals only, gold metal: fuzz (1 - 250/1000)^2
    assert [x[2] for x in tris[2:5]] == [None] * 3 and all(x[1] for x in tris[2:5])
    assert tris[2][3] == ("metal", (1.0, 0.843, 0.0), 0.5625)
    # "f -1 -2 -3" -> vertices 39, 38, 37 (relative to the total count); "f 0 2 99" -> 1, 2, 39
    assert tris[5][0][:3] == [-0.5, 1.0, 3.0] and tris[5][3] == ("dielectric", 1.45)
    assert tris[6][0][:3] == [-1.0, -1.0, 0.0] and tris[6][0][6:] == [-0.5, 1.0, 3.0]
    # unknown material -> the default Lambertian(0.8); uv but no normals
    assert tris[7][3] == ("lambertian", (0.8, 0.8, 0.8)) and tris[7][1] is None
    # "f 4//3 ..." where vn 3 is defined just before: normal (1,0,0); lamp is a light
    assert tris[8][1] == [1, 0, 0] * 3 and tris[8][3] == ("light", (15.0, 14.0, 13.0))
    assert tris[9][3] == ("isotropic", (0.5, 0.6, 0.7))       # Tf -> d = 0.5
    assert tris[10][3] == ("metal", (0.05, 0.05, 0.06), 0.3)  # illum 3
    blend = 1.0 - (((0.06 + 0.05) + 0.04) / 0.2)  # spec summed x+y+z
    assert tris[11][3][0] == "metal" and tris[11][3][2] == 0.0  # Ns >= 1000 -> roughness 0
    assert tris[11][3][1][0] == (1.0 - blend) * 0.06 + blend * 0.05
    assert tris[12][3] == ("lambertian_image", images[next(iter(images))])
    assert tris[13][3] == ("lambertian_image", images[next(iter(images))])  # map_Ka fallback
    assert tris[14][3] == ("lambertian", (0.9, 0.9, 0.9))     # illum 9 -> diffuse
    assert tris[15][3][0] == "light_image"
    assert len(tris) == 16 and lidx == [8, 15]


PARSE_CASES = [  # strconv.ParseFloat(s, 64): (value, ok)
    ("1", 1.0, True), ("-2.5e3", -2500.0, True), ("+.5", 0.5, True), ("5.", 5.0, True),
    ("inf", math.inf, True), ("+Inf", math.inf, True), ("-infinity", -math.inf, True),
    ("infin", 0.0, False), ("nan", math.nan, True), ("NaN", math.nan, True),
    ("+nan", 0.0, False), ("1e400", math.inf, False), ("-1e400", -math.inf, False),
    ("1e-400", 0.0, True), ("0x1p-2", 0.25, True), ("0x1", 0.0, False), ("0x", 0.0, False),
    ("1_000", 1000.0, True), ("_1", 0.0, False), ("1__0", 0.0, False), ("1_", 0.0, False),
    (".", 0.0, False), ("e5", 0.0, False), ("1e", 0.0, False), ("1e+", 0.0, False),
    ("1.2.3", 0.0, False), ("1e5x", 0.0, False), ("0.1", 0.1, True),
    ("4.9406564584124654e-324", 5e-324, True), ("1.7976931348623157e308", 1.7976931348623157e308,
                                                 True),
]


@pytest.mark.parametrize("s,val,ok", PARSE_CASES)
def test_restated_parse_float(s, val, ok):
    v, k = objload.parse_float(s)
    assert k == ok
    assert (math.isnan(v) and math.isnan(val)) or v == val


def test_c_parse_float_through_vertex_lines(rt):
    """The C parser accepts exactly the vertex lines Go's ParseFloat accepts."""
    lines = [f"v {s} 0 0" for s, _, _ in PARSE_CASES] + ["f 1 2 3"]
    text = "\n".join(lines).encode()
    t = rt.Tree()
    o = rt.LoadObjOptions(Debug=False, Center=False)
    model, lights = t.LoadObjWithOptions(None, o, obj_text=text)
    info = t.last_obj_info
    accepted = [(s, v) for s, v, ok in PARSE_CASES if ok]
    assert info.n_vertices == len(accepted)
    tris, _ = tree_triangles(t, model, lights)
    first3 = [x for x in tris[0][0][0::3]]
    for got, (s, want) in zip(first3, accepted[:3]):
        assert got == want, s


@pytest.mark.parametrize("s,val,ok", [("12", 12, True), ("-3", -3, True), ("+4", 4, True),
                                      ("1.0", 0, False), ("", 0, False), ("+", 0, False),
                                      ("9223372036854775808", 2 ** 63 - 1, False),
                                      ("1_0", 0, False)])
def test_restated_atoi(s, val, ok):
    assert objload.atoi(s) == (val, ok)


def test_crlf_and_unicode_space(rt):
    obj = "v 0 0 0\r\nv 1 0 0\r\n v 0 1 0 \r\nf 1 2 3\r\n".encode()
    t = rt.Tree()
    model, lights = t.LoadObjWithOptions(None, rt.LoadObjOptions(Debug=False, Center=False),
                                         obj_text=obj)
    tris, _ = tree_triangles(t, model, lights)
    assert tris[0][0] == [0, 0, 0, 1, 0, 0, 0, 1, 0]
    ref = objload.load_obj(obj, center=False)
    assert bits(ref.tris[0][0]) == bits(tris[0][0])


def test_fatal_cases_are_error_codes(rt, tmp_path):
    t = rt.Tree()
    o = rt.LoadObjOptions(Debug=False)
    with pytest.raises(rt.RtError) as e:  # log.Fatalf("Could not open file ...")
        t.LoadObjWithOptions(str(tmp_path / "missing.obj"), o)
    assert e.value.code == -5
    with pytest.raises(rt.RtError) as e:  # log.Fatalf("No triangles found in OBJ file")
        t.LoadObjWithOptions(None, o, obj_text=b"v 0 0 0\nv 1 0 0\n")
    assert "No triangles" in str(e.value)
    long_line = b"v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n# " + b"x" * 70000 + b"\n"
    with pytest.raises(rt.RtError) as e:  # scanner.Err() -> log.Fatalf (objLoader.go:472-474)
        t.LoadObjWithOptions(None, o, obj_text=long_line)
    assert "too long" in str(e.value)
    with pytest.raises(ValueError):
        objload.load_obj(long_line)
    # an MTL naming an image that cannot be opened is fatal (imageLoader.go:31-33)
    obj = b"mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl a\nf 1 2 3\n"
    with pytest.raises(rt.RtError) as e:
        t.LoadObjWithOptions(None, o, obj_text=obj,
                             mtl_text=b"newmtl a\nmap_Kd /nonexistent/x.ppm\n")
    assert e.value.code == -5


def test_missing_mtl_file_is_a_warning(rt, tmp_path):
    (tmp_path / "a.obj").write_bytes(b"mtllib nope.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\n"
                                     b"usemtl x\nf 1 2 3\n")
    t = rt.Tree()
    model, lights = t.LoadObjWithOptions(str(tmp_path / "a.obj"), rt.LoadObjOptions(Debug=False))
    tris, lidx = tree_triangles(t, model, lights)
    assert tris[0][3] == ("lambertian", (0.8, 0.8, 0.8)) and lidx == []


def test_loaded_model_flattens(rt, mixed):
    """A loaded model goes through rt_scene_create like any Hittable (host only)."""
    d, obj, mtl, images = mixed
    t = rt.Tree()
    model, lights = t.LoadObjWithOptions(str(d / "mixed.obj"), rt.LoadObjOptions(Debug=False))
    world = t.list(t.rotate_y(model, 180))
    with rt.Scene(t, world, lights) as sc:
        i = sc.info()
    assert i["n_triangles"] >= 16 and i["n_lights"] == 2


def test_c_parse_float_is_correctly_rounded(rt):
    """The loader's fast path (Clinger: mantissa <= 2^53, |exp10| <= 22) and its
    strtod fallback both return the correctly rounded double, like Go's ParseFloat:
    compared bit for bit with Python's float() on random decimal strings."""
    rng = np.random.default_rng(5)
    toks = []
    for _ in range(3000):
        nd = int(rng.integers(1, 20))
        digits = "".join(str(int(d)) for d in rng.integers(0, 10, nd))
        dot = int(rng.integers(0, nd + 1))
        s = digits[:dot] + "." + digits[dot:] if rng.random() < 0.8 else digits
        if s in (".", ""):
            s = "0"
        if rng.random() < 0.3:
            s += "e" + str(int(rng.integers(-30, 30)))
        if rng.random() < 0.5:
            s = "-" + s
        toks.append(s)
    n = len(toks) // 3
    text = "".join(f"v {a} {b} {c}\n" for a, b, c in zip(toks[0::3], toks[1::3], toks[2::3]))
    text += "".join(f"f {i} {i + 1} {i + 2}\n" for i in range(1, n - 1, 3))
    t = rt.Tree()
    model, lights = t.LoadObjWithOptions(None, rt.LoadObjOptions(Debug=False, Center=False),
                                         obj_text=text.encode())
    tris, _ = tree_triangles(t, model, lights)
    got = [x for tr in tris for x in tr[0]]
    want = [float(x) for x in toks[:len(got)]]
    assert len(got) >= 2900
    assert [struct.pack("<d", x) for x in got] == [struct.pack("<d", x) for x in want]
