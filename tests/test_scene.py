"""Host-side scene pipeline: flattening (transforms baked, media multiplicity,
light table), the device BVH's structural invariants, and error behaviour.
CPU-only: no device memory is touched."""
import numpy as np
import pytest

from tests import scenes


def info(rt, name):
    t, cam, w, l = rt.demo_scene(name)
    with rt.Scene(t, w, l) as sc:
        return sc.info()


def test_cornell_flattening(rt):
    i = info(rt, "cornell")
    # 5 walls + light + 2 boxes x 6 quads in the world, + the light copy for sampling
    assert i["n_world_prims"] == 18 and i["n_quads"] == 19 and i["n_lights"] == 1
    assert i["n_media"] == 0


def test_book2_flattening(rt):
    i = info(rt, "book2")
    # ground boxes as 6 quads each: the book2 kernel set has no box leaves (rt_device.h)
    assert i["n_world_prims"] == 2400 + 1 + 1006  # boxes, light, spheres (1000 rotated)
    assert not i["features"] & rt.RT_FT_BOX
    assert i["n_media"] == 2 and i["medium_draws"] == 2  # flat world list: no duplication
    assert i["n_images"] == 1 and i["n_perlins"] == 1


def test_book1_scene_content(rt):
    i = info(rt, "book1")
    # ground + 3 big + sun + random small spheres (perlin orbs are never added, main.go:52-60)
    assert 300 < i["n_world_prims"] < 484 + 5
    assert i["n_lights"] == 1


def test_medium_multiplicity_from_span1_leaf(rt):
    """bvh.go:44-46 duplicates span-1 leaves: a medium there is tested twice."""
    t, cam, w, l = scenes.dup_medium(rt)
    with rt.Scene(t, w, l) as sc:
        i = sc.info()
    assert i["n_media"] == 1 and i["medium_draws"] == 2


def test_scene_is_pure_function_of_seed(rt):
    def fingerprint(seed):
        t, cam, w, l = rt.demo_scene("book1", seed=seed)
        with rt.Scene(t, w, l) as sc:
            nodes, refs, root, bounds = sc.export_bvh()
        return bounds.tobytes()
    assert fingerprint(1) == fingerprint(1)
    assert fingerprint(1) != fingerprint(2)


def bvh_invariants(sc):
    """Every world prim is in exactly one leaf and every box contains what is below
    it (the exported BVH2; the BVH4 shares its leaves and boxes)."""
    nodes, refs, root, bounds = sc.export_bvh()
    i = sc.info()
    n = len(refs)
    assert n == i["n_world_prims"]
    seen = np.zeros(n, np.int32)
    stack = [(root, np.full(3, -np.inf, np.float32), np.full(3, np.inf, np.float32))]
    while stack:  # iterative: device-built trees of big meshes are deep
        code, lo, hi = stack.pop()
        if code & 0x80000000:
            first, cnt = (code >> 4) & 0x7FFFFFF, (code & 15) + 1
            seen[first:first + cnt] += 1
            b = bounds[first:first + cnt]
            assert (b[:, :3] >= lo - 1e-6).all() and (b[:, 3:] <= hi + 1e-6).all()
            continue
        nd = nodes[code]
        c0 = int(nd[3:4].view(np.uint32)[0])
        c1 = int(nd[7:8].view(np.uint32)[0])
        for c, (blo, bhi) in ((c0, (nd[0:3], nd[4:7])), (c1, (nd[8:11], nd[12:15]))):
            assert (blo >= lo - 1e-6).all() and (bhi <= hi + 1e-6).all()
            stack.append((c, blo, bhi))
    assert (seen == 1).all(), "every world prim is referenced by exactly one leaf"
    assert i["max_leaf"] <= 16
    return nodes, refs, bounds


@pytest.mark.parametrize("name", ["cornell", "book1", "book2", "quads", "model:96x24"])
def test_bvh_invariants(rt, name):
    t, cam, w, l = rt.demo_scene(name)
    with rt.Scene(t, w, l) as sc:
        bvh_invariants(sc)


def bvh8_invariants(sc):
    """host_bvh8.cpp: every world prim has exactly one BVH8 leaf record, every node is
    reached once through child_base + rank, and every child box dequantised with the
    device's fp32 arithmetic (origin + q * 2^(E-127)) contains what is below it."""
    nodes, refs8 = sc.export_bvh8()
    _, refs, _, bounds = sc.export_bvh()
    assert len(nodes) > 0
    assert sorted(refs8.tolist()) == sorted(refs.tolist())
    bound_of = {int(r): bounds[i] for i, r in enumerate(refs)}
    visits = np.zeros(len(nodes), np.int32)
    f32 = np.float32
    stack = [(0, np.full(3, -np.inf, f32), np.full(3, np.inf, f32))]
    while stack:
        ni, plo, phi = stack.pop()
        visits[ni] += 1
        w = nodes[ni]
        origin = w[0:3].view(np.float32)
        ex = [(int(w[3]) >> (8 * a)) & 0xFF for a in range(3)]
        scale = np.array([np.uint32(e << 23) for e in ex], np.uint32).view(np.float32)
        child_base, leaf_base = int(w[4]), int(w[5])
        meta = [(int(w[6 + k // 4]) >> (8 * (k % 4))) & 0xFF for k in range(8)]
        q = np.zeros((6, 8), np.uint32)
        for f in range(6):
            for k in range(8):
                word = int(w[8 + 4 * f + k // 2])
                q[f, k] = (word >> (16 * (k & 1))) & 0xFFFF
        for k, m in enumerate(meta):
            if m == 0xFF:
                continue
            lo = np.array([f32(origin[a]) + f32(q[2 * a, k]) * scale[a] for a in range(3)], f32)
            hi = np.array([f32(origin[a]) + f32(q[2 * a + 1, k]) * scale[a] for a in range(3)], f32)
            assert (lo <= hi).all()
            if m & 0x80:
                stack.append((child_base + (m & 7), np.maximum(lo, plo), np.minimum(hi, phi)))
            else:
                first, cnt = leaf_base + (m & 31), ((m >> 5) & 3) + 1
                for r in refs8[first:first + cnt]:
                    b = bound_of[int(r)]
                    assert (b[:3] >= lo).all() and (b[3:] <= hi).all()
                    assert (b[:3] >= plo).all() and (b[3:] <= phi).all()
    assert (visits == 1).all(), "every BVH8 node is reached exactly once"
    return nodes, refs8


@pytest.mark.parametrize("name", ["book2", "model:96x24"])
def test_bvh8_invariants(rt, name, tune):
    tune("RT_BVH8", "1")  # the wide tree is opt-in
    t, cam, w, l = rt.demo_scene(name)
    with rt.Scene(t, w, l) as sc:
        nodes, _ = bvh8_invariants(sc)
    assert len(nodes) >= 2


def test_bvh8_only_when_asked_and_large(rt, tune):
    t, cam, w, l = rt.demo_scene("book2")
    with rt.Scene(t, w, l) as sc:  # default: no BVH8
        assert len(sc.export_bvh8()[0]) == 0
    tune("RT_BVH8", "1")
    t, cam, w, l = rt.demo_scene("book1")  # 485 prims: the BVH4 (LDS-sized scenes)
    with rt.Scene(t, w, l) as sc:
        assert len(sc.export_bvh8()[0]) == 0


def test_light_table_matches_nested_picks(rt):
    """lights = list(list(a, b), c): the flattened pick intervals must select
    exactly what nested rand.Intn picks select (hittable.go:98-103)."""
    import ctypes as C
    t, cam, w, l = scenes.nested_lights(rt)
    with rt.Scene(t, w, l) as sc:
        assert sc.info()["n_lights"] == 3
    # reproduce the table from the interval rule and compare with nested picks
    for u24 in list(range(0, 1 << 24, 99991)) + [(1 << 24) - 1, (1 << 23), (1 << 24) // 3]:
        top = (u24 * 2) >> 24
        if top == 0:
            r = (u24 * 2) & 0xFFFFFF
            expect = (r * 2) >> 24  # a or b
        else:
            expect = 2  # c
        lo = [0, -(-(1 << 24) // 4), -(-(1 << 24) // 2)]  # ceil(i/4), ceil(2/4) boundaries
        got = max(i for i in range(3) if lo[i] <= u24)
        assert got == expect


def test_lights_must_have_pdf(rt):
    t = rt.Tree()
    m = t.lambertian((1, 1, 1))
    s = t.sphere((0, 0, 0), 1, m)
    world = t.list(s)
    for bad in (t.translate(s, (1, 0, 0)), t.bvh(t.list(s)), t.rotate_y(s, 10)):
        with pytest.raises(rt.RtError) as e:
            rt.Scene(t, world, bad)
        assert e.value.code == -2  # defaultPdfImpl log.Fatal in the reference


def test_rotated_transforms_baked(rt):
    """Translate(RotateY(box)) quads end up where rotateY/translate map them."""
    t = rt.Tree()
    m = t.lambertian((1, 1, 1))
    b = t.translate(t.rotate_y(t.box((0, 0, 0), (1, 2, 3), m), 90), (10, 0, 0))
    with rt.Scene(t, b, -1) as sc:
        nodes, refs, root, bounds = sc.export_bvh()
    lo, hi = bounds[:, :3].min(0), bounds[:, 3:].max(0)
    # Ry(90): x' = z, z' = -x  -> box spans x in [0,3]+10, z in [-1,0]
    assert np.allclose(lo, [10, 0, -1], atol=1e-4) and np.allclose(hi, [13, 2, 0], atol=1e-4)


def test_demo_scene_numbers(rt):
    import ctypes as C
    name = C.c_char_p()
    assert rt.lib().rt_demo_scene_name(6, C.byref(name)) == 0 and name.value == b"cornell"
    assert rt.lib().rt_demo_scene_name(8, C.byref(name)) == 0 and name.value == b"model"
    assert rt.lib().rt_demo_scene_name(9, C.byref(name)) < 0


def test_bvh_build_is_thread_count_invariant(rt, tune):
    """The SAH build runs its top levels with threaded loops and the subtrees in
    parallel (host_bvh.cpp); min/max box growth and integer bin counts make the
    tree bit-identical for any thread count."""
    out = {}
    for th in ("1", "3", "8"):
        tune("RT_THREADS", th)
        t, cam, w, l = rt.demo_scene("model:256x64")
        with rt.Scene(t, w, l) as sc:
            nodes, refs, root, bounds = sc.export_bvh()
        out[th] = (nodes.tobytes(), refs.tobytes(), int(root), bounds.tobytes())
    assert out["1"] == out["3"] == out["8"]


def test_box_leaves_kept_only_where_they_pay(rt, tune):
    """NewBox becomes one BVH leaf (rt_device.h "box leaf") in large scenes whose kernel
    set has FT_BOX; small scenes and lean sets keep the six quads, so their trees and
    images are exactly the per-quad ones."""
    import os
    from tests import scenes
    assets = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
    t, cam, w, l = scenes.box_leaves(rt, assets)
    with rt.Scene(t, w, l) as sc:
        i = sc.info()
        bvh_invariants(sc)
    assert i["features"] & rt.RT_FT_BOX and i["n_world_prims"] == 64 + 3 + 1 + 1
    tune("RT_BOX_LEAVES", "0")
    with rt.Scene(t, w, l) as sc:
        j = sc.info()
    assert not j["features"] & rt.RT_FT_BOX and j["n_world_prims"] == 6 * 64 + 3 + 1 + 1
    assert j["n_quads"] == i["n_quads"]  # the same quads either way
    tune("RT_BOX_LEAVES", None)
    for name in ("cornell", "quads"):  # small: no box leaves
        assert not info(rt, name)["features"] & rt.RT_FT_BOX
    t, cam, w, l = scenes.boxes(rt)  # 216 quads, lean set: expanded
    with rt.Scene(t, w, l) as sc:
        assert not sc.info()["features"] & rt.RT_FT_BOX


def qbvh_invariants(sc):
    """host_qbvh.cpp: the compressed BVH4 mirrors the BVH4 item by item -- every BVH4 node
    is one 64-B node item, every single-prim leaf one leaf record (its bit set in the node's
    leaf mask), every 2-4-prim leaf one node over its prims -- and every child box it encodes
    (fp32 corner + fp16 offsets, exact in float64) contains the fp32 box it replaces, so the
    traversal culls no more than the BVH4's (the images are bit-identical on the GPU,
    test_compressed_bvh_renders_like_bvh4).  Empty slots decode to inverted infinite boxes."""
    items, nodes4, root4 = sc.export_qbvh()
    _, refs, _, bounds = sc.export_bvh()
    assert len(items) > 0 and len(nodes4) > 0
    LEAF, EMPTY = 0x80000000, 0xFFFFFFFE

    def planes(item):
        w = items[item]
        corner = w[0:3].view(np.float32).astype(np.float64)
        half = w[4:16].view(np.float16).astype(np.float64).reshape(3, 4, 2)  # [axis][word][half]
        lo = np.stack([half[:, 0, 0], half[:, 0, 1], half[:, 1, 0], half[:, 1, 1]], 1)  # [axis][k]
        hi = np.stack([half[:, 2, 0], half[:, 2, 1], half[:, 3, 0], half[:, 3, 1]], 1)
        return corner, lo, hi, int(w[3]) & 0x0FFFFFFF, int(w[3]) >> 28

    seen_nodes = np.zeros(len(nodes4), np.int32)
    seen_refs = np.zeros(len(refs), np.int32)
    used = np.zeros(len(items), np.int32)
    used[0] = 1
    stack = [(0, ("node", root4))]
    while stack:
        item, (kind, what) = stack.pop()
        corner, lo, hi, base, lmask = planes(item)
        if kind == "node":
            seen_nodes[what] += 1
            nd = nodes4[what].view(np.float32).reshape(8, 4)  # [field][child]
            codes = nodes4[what][0:4]
            kids = []
            for k in range(4):
                c = int(codes[k])
                blo = np.array([nd[1 + 2 * a, k] for a in range(3)], np.float64)
                bhi = np.array([nd[2 + 2 * a, k] for a in range(3)], np.float64)
                if c == EMPTY or not (blo <= bhi).all():
                    kids.append(None)
                elif c & LEAF:
                    first, count = (c >> 4) & 0x7FFFFFF, (c & 15) + 1
                    kids.append((blo, bhi, ("leaf", first) if count == 1 else ("group", (first, count))))
                else:
                    kids.append((blo, bhi, ("node", c)))
        else:  # a node over the prims of one 2-4-prim BVH4 leaf
            first, count = what
            kids = [(bounds[first + k][:3].astype(np.float64), bounds[first + k][3:].astype(np.float64),
                     ("leaf", first + k)) if k < count else None for k in range(4)]
        for k, kid in enumerate(kids):
            if kid is None:
                assert (lo[:, k] == np.inf).all() and (hi[:, k] == -np.inf).all(), (item, k)
                used[base + k] += 1  # its (unused) slot of the node's four
                continue
            blo, bhi, nxt = kid
            assert (corner + lo[:, k] <= blo).all() and (corner + hi[:, k] >= bhi).all(), (item, k)
            child = base + k
            used[child] += 1
            if nxt[0] == "leaf":
                assert (lmask >> k) & 1, (item, k)
                seen_refs[nxt[1]] += 1
            else:
                assert not (lmask >> k) & 1, (item, k)
                stack.append((child, nxt))
    assert (seen_nodes == 1).all(), "every BVH4 node is encoded exactly once"
    assert (seen_refs == 1).all(), "every prim has exactly one leaf record"
    assert (used == 1).all(), "every item is one node's child slot, exactly once"


@pytest.mark.parametrize("name", ["book1", "book2", "model:96x24", "model:256x32"])
def test_qbvh_invariants(rt, name):
    t, cam, w, l = rt.demo_scene(name)
    with rt.Scene(t, w, l) as sc:
        qbvh_invariants(sc)
