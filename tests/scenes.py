"""Small hand-built scenes, each isolating one reference feature (tests only)."""
import numpy as np


def _cam(rt, look_from, look_at, vfov=40.0, width=32, spp=16, depth=20, bg=(0.0, 0.0, 0.0),
         aspect=1.0, defocus=0.0, focus=0.0, maxc=0.0):
    c = rt.Camera(AspectRatio=aspect, Width=width, SamplesPerPixel=spp, MaxDepth=depth,
                  VerticalFOV=vfov, Background=bg, DefocusAngle=defocus, FocusDistance=focus,
                  MaxContribution=maxc)
    c.PositionCamera(look_from, look_at, (0, 1, 0))
    return c


def _room(t):
    """floor + back wall + ceiling light (quads), returns (world list, lights list)."""
    white = t.lambertian((0.73, 0.73, 0.73))
    world = t.list()
    t.add(world, t.quad((-10, 0, -10), (20, 0, 0), (0, 0, 20), white))
    t.add(world, t.quad((-10, 0, 10), (20, 0, 0), (0, 10, 0), white))
    light = t.quad((-2, 9.9, -2), (4, 0, 0), (0, 0, 4), t.light((10, 10, 10)))
    t.add(world, light)
    lights = t.list(light)
    return world, lights


def fog(rt):
    """camera inside a huge constant medium (book2 fog, main.go:139-140)."""
    t = rt.Tree(1)
    world, lights = _room(t)
    b = t.sphere((0, 0, 0), 500, t.dielectric(1.5))
    t.add(world, t.medium(b, 0.05, (1, 1, 1)))
    return t, _cam(rt, (0, 3, -8), (0, 2, 0)), world, lights


def water(rt):
    """dielectric sphere holding a medium, both in the world (main.go:134-136)."""
    t = rt.Tree(1)
    world, lights = _room(t)
    b = t.sphere((0, 2, 0), 2, t.dielectric(1.5))
    t.add(world, b)
    t.add(world, t.medium(b, 0.4, (0.2, 0.4, 0.9)))
    return t, _cam(rt, (0, 3, -9), (0, 2, 0)), world, lights


def earth(rt, asset_dir):
    """image-textured sphere, rotated (UV in object space) and translated."""
    with open(f"{asset_dir}/earthmap.ppm", "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    w, h = map(int, parts[1].split())
    rgb = np.frombuffer(parts[3], np.uint8).reshape(h, w, 3)
    t = rt.Tree(1)
    world, lights = _room(t)
    em = t.lambertian(t.image(rgb))
    t.add(world, t.translate(t.rotate_y(t.sphere((0, 0, 0), 2, em), 70), (1, 2, 0)))
    return t, _cam(rt, (0, 3, -9), (0, 2, 0)), world, lights


def cluster(rt):
    """Translate(RotateY(BVH(spheres))) cluster (main.go:151-161)."""
    t = rt.Tree(3)
    world, lights = _room(t)
    white = t.lambertian((0.73, 0.73, 0.73))
    box = t.list()
    for _ in range(200):
        t.add(box, t.sphere((t.rand_range(0, 4), t.rand_range(0, 4), t.rand_range(0, 4)), 0.3, white))
    t.add(world, t.translate(t.rotate_y(t.bvh(box), 15), (-2, 0.5, -1)))
    # 64 x 64 at 32 spp (at 32 x 32 x 16 its 3,072 channels left the
    # named bar a 0.7-sigma margin)
    return t, _cam(rt, (0, 3, -9), (0, 2, 0), width=64, spp=32), world, lights


def metal_fuzz(rt):
    """metal spheres of fuzz 1.0 / 0.3 / 0 (main.go:131, :63-66)."""
    t = rt.Tree(1)
    world, lights = _room(t)
    for i, fz in enumerate((1.0, 0.3, 0.0)):
        t.add(world, t.sphere((-3 + 3 * i, 1, 0), 1, t.metal((0.8, 0.8, 0.9), fz)))
    return t, _cam(rt, (0, 3, -9), (0, 2, 0)), world, lights


def glass(rt):
    """dielectric spheres, including a hollow one (main.go:35,70,78,128)."""
    t = rt.Tree(1)
    world, lights = _room(t)
    g = t.dielectric(1.5)
    t.add(world, t.sphere((-2, 1.5, 0), 1.5, g))
    t.add(world, t.sphere((2, 1.5, 0), 1.5, g))
    t.add(world, t.sphere((2, 1.5, 0), 1.2, t.dielectric(1 / 1.5)))
    return t, _cam(rt, (0, 3, -9), (0, 2, 0)), world, lights


def boxes(rt):
    """book2 floor boxes: a BVH of NewBox (main.go:95-113)."""
    t = rt.Tree(5)
    world, lights = _room(t)
    ground = t.lambertian((0.48, 0.83, 0.53))
    bl = t.list()
    for i in range(6):
        for j in range(6):
            x0, z0 = -6 + 2 * i, -6 + 2 * j
            t.add(bl, t.box((x0, 0, z0), (x0 + 2, t.rand_range(0.2, 2), z0 + 2), ground))
    t.add(world, t.bvh(bl))
    return t, _cam(rt, (0, 6, -12), (0, 1, 0)), world, lights


def marble(rt):
    """marble / turbulent / perlin noise spheres (texture.go:112-125)."""
    t = rt.Tree(9)
    world, lights = _room(t)
    for i, (sc, var) in enumerate(((0.2, rt.RT_NOISE_MARBLE), (4, rt.RT_NOISE_TURBULENT),
                                   (4, rt.RT_NOISE_PERLIN))):
        t.add(world, t.sphere((-3 + 3 * i, 1, 0), 1, t.lambertian(t.noise(sc, var))))
    return t, _cam(rt, (0, 3, -9), (0, 2, 0)), world, lights


def motion(rt):
    """moving spheres (NewMotionSphere objects.go:30-37) + defocus blur."""
    t = rt.Tree(1)
    world, lights = _room(t)
    m = t.lambertian((0.7, 0.3, 0.1))
    t.add(world, t.motion_sphere((-1, 1, 0), (1, 1.5, 0), 1, m))
    return t, _cam(rt, (0, 3, -9), (0, 2, 0), defocus=2.0, focus=9.0), world, lights


def sphere_light(rt):
    """a spherical light (book1 sun / model sun, main.go:85-87, :387)."""
    t = rt.Tree(1)
    white = t.lambertian((0.73, 0.73, 0.73))
    world = t.list()
    t.add(world, t.sphere((0, -100, 0), 100, white))
    sun = t.sphere((3, 6, 2), 1.5, t.light((8, 8, 8)))
    t.add(world, sun)
    t.add(world, t.sphere((0, 1, 0), 1, white))
    return t, _cam(rt, (0, 2, -8), (0, 1, 0)), world, t.list(sun)


def tri_mesh(rt):
    """smooth-normal + textured triangles as lights and geometry (objects.go:242-465)."""
    t = rt.Tree(1)
    world, lights = _room(t)
    red = t.lambertian((0.65, 0.05, 0.05))
    v = [(-2, 0.5, 0), (2, 0.5, 0), (0, 3.5, 1)]
    n = [(0, 0, -1), (0.3, 0, -1), (0, 0.3, -1)]
    n = [np.array(x) / np.linalg.norm(x) for x in n]
    t.add(world, t.triangle(v, red, normals=n))
    lt = t.triangle([(-1, 6, -1), (1, 6, -1), (0, 6, 1)], t.light((6, 6, 6)), uv=[0, 0, 1, 0, 0, 1])
    t.add(world, lt)
    t.add(lights, lt)
    return t, _cam(rt, (0, 3, -9), (0, 2, 0)), world, lights


def nested_lights(rt):
    """lights = list(list(a, b), c): nested rand.Intn picks (hittable.go:98-103)."""
    t = rt.Tree(1)
    white = t.lambertian((0.73, 0.73, 0.73))
    world = t.list()
    t.add(world, t.quad((-10, 0, -10), (20, 0, 0), (0, 0, 20), white))
    lm = t.light((5, 5, 5))
    a = t.quad((-3, 5, -1), (2, 0, 0), (0, 0, 2), lm)
    b = t.quad((1, 5, -1), (2, 0, 0), (0, 0, 2), lm)
    c = t.sphere((0, 6, 3), 0.7, lm)
    for o in (a, b, c):
        t.add(world, o)
    lights = t.list(t.list(a, b), c)
    return t, _cam(rt, (0, 3, -9), (0, 1, 0)), world, lights


def smoke_box(rt):
    """constant media bounded by rotated boxes inside a BVH (main.go:323-367)."""
    t = rt.Tree(1)
    world, lights = _room(t)
    wl = t.list()
    b1 = t.translate(t.rotate_y(t.box((0, 0, 0), (2, 4, 2), t.lambertian((1, 1, 1))), 15), (-3, 0, 0))
    b2 = t.translate(t.rotate_y(t.box((0, 0, 0), (2, 2, 2), t.lambertian((1, 1, 1))), -18), (1, 0, -1))
    t.add(wl, t.medium(b1, 0.5, (0, 0, 0)))
    t.add(wl, t.medium(b2, 0.5, (1, 1, 1)))
    t.add(wl, world)
    return t, _cam(rt, (0, 3, -9), (0, 2, 0)), t.bvh(wl), lights


def dup_medium(rt):
    """a medium in a span-1 BVH leaf is tested twice (bvh.go:44-46, H2)."""
    t = rt.Tree(1)
    world, lights = _room(t)
    # the boundary has the smallest z-min, so the sort puts it in the span-1 leaf
    b = t.sphere((0, 2, 0), 11, t.dielectric(1.5))
    wl = t.list(world, t.medium(b, 0.03, (0.9, 0.9, 0.9)), t.quad((5, 0, 5), (1, 0, 0), (0, 1, 0),
                                                                   t.lambertian((1, 0, 0))))
    return t, _cam(rt, (0, 3, -9), (0, 2, 0)), t.bvh(wl), lights


def no_lights(rt):
    """an empty lights list: Random -> vec.Random(), PdfValue -> 0 (hittable.go:89-103)."""
    t = rt.Tree(1)
    world, _ = _room(t)
    return t, _cam(rt, (0, 3, -9), (0, 2, 0), bg=(0.5, 0.6, 0.9)), world, t.list()


def checker(rt):
    """checker of checkers on the book1 ground sphere (texture.go:50-60)."""
    t = rt.Tree(1)
    a = t.checker(0.5, t.solid(0.2, 0.3, 0.1), t.solid(0.9, 0.9, 0.9))
    b = t.checker(0.32, a, t.solid(0.8, 0.1, 0.1))
    world = t.list()
    t.add(world, t.sphere((0, -1000, 0), 1000, t.lambertian(b)))
    sun = t.sphere((0, 100, 0), 50, t.light((5, 5, 5)))
    t.add(world, sun)
    return t, _cam(rt, (13, 2, 3), (0, 0, 0), vfov=20, bg=(0.7, 0.8, 1.0)), world, t.list(sun)


def obj_mixed(rt, asset_dir):
    """tests/golden/obj/mixed.obj through the OBJ/MTL loader (objLoader.go:72-538):
    every ConvertToRaytracerMaterial branch, smooth normals, uvs, emissive and
    image-textured triangles, rotated like modelExample (main.go:384)."""
    import os
    fix = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "obj")
    obj = open(os.path.join(fix, "mixed.obj"), "rb").read()
    tex = os.path.join(asset_dir, "earthmap.ppm")
    mtl = open(os.path.join(fix, "mixed.mtl"), "rb").read().replace(b"@TEX@", tex.encode())
    t = rt.Tree(1)
    world, room_lights = _room(t)
    o = rt.LoadObjOptions(Debug=False, ScaleFactor=1.5, Position=(0.0, 2.5, 0.0))
    model, lights = t.LoadObjWithOptions(os.path.join(fix, "mixed.obj"), o, mtl_text=mtl,
                                         obj_text=obj)
    t.add(world, t.rotate_y(model, 150))
    light = t.quad((-2, 9.9, -2), (4, 0, 0), (0, 0, 4), t.light((10, 10, 10)))
    t.add(world, light)
    t.add(lights, light)  # as modelExample adds its sun to the loader's light list
    # spp 25, not 16: with 16 samples a pixel mean of exactly 1/16, 1/4 or 9/16 (one
    # clamped (1,1,1) sample, ...) sits on a PrintColor truncation boundary (sqrt*256
    # integral), where the last fp32 ulp of the sum flips the 8-bit output by one
    return t, _cam(rt, (0, 3, -9), (0, 2.5, 0), spp=25), world, lights


def box_leaves(rt, asset_dir):
    """64 NewBoxes (384 quads: above the box-leaf threshold) with RotateY/Translate and
    an image texture on some (alpha, beta of a box face), plus a metal sphere and a
    triangle (so the all-features kernel runs, the one with FT_BOX): the world BVH holds
    box leaves (host_flatten.cpp; rt_kernels.h hit_box_rec)."""
    with open(f"{asset_dir}/earthmap.ppm", "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    w, h = map(int, parts[1].split())
    rgb = np.frombuffer(parts[3], np.uint8).reshape(h, w, 3)
    t = rt.Tree(7)
    world, lights = _room(t)
    green = t.lambertian((0.48, 0.83, 0.53))
    em = t.lambertian(t.image(rgb))
    bl = t.list()
    for i in range(8):
        for j in range(8):
            x0, z0 = -8 + 2 * i, -8 + 2 * j
            b = t.box((0, 0, 0), (1.6, t.rand_range(0.3, 2.5), 1.2), em if (i + j) % 3 == 0 else green)
            t.add(bl, t.translate(t.rotate_y(b, 37 * i + 11 * j), (x0 + 0.5, 0, z0 + 0.5)))
    t.add(world, t.bvh(bl))
    t.add(world, t.sphere((0, 3.5, 0), 1, t.metal((0.8, 0.8, 0.9), 0.1)))
    t.add(world, t.triangle([(-6, 0.5, 8), (6, 0.5, 8), (0, 5, 8.5)], t.lambertian((0.65, 0.05, 0.05))))
    return t, _cam(rt, (0, 7, -13), (0, 1, 0)), world, lights


FEATURES = ["fog", "water", "earth", "cluster", "metal_fuzz", "glass", "boxes", "marble", "motion",
            "sphere_light", "tri_mesh", "nested_lights", "smoke_box", "dup_medium", "no_lights",
            "checker", "obj_mixed", "box_leaves"]


def build(rt, name, asset_dir):
    fn = globals()[name]
    if name in ("earth", "obj_mixed", "box_leaves"):
        return fn(rt, asset_dir)
    return fn(rt)


def book2_variant(rt, asset_dir, drop=()):
    """main.go:94-174 rebuilt through the Python API with components removable (bisection)."""
    t = rt.Tree(1)
    boxes1 = t.list()
    ground = t.lambertian((.48, .83, .53))
    for i in range(20):
        for j in range(20):
            w = 100.0
            x0, z0 = -1000.0 + i * w, -1000.0 + j * w
            y1 = t.rand_range(1, 101)
            if "boxes" not in drop:
                t.add(boxes1, t.box((x0, 0, z0), (x0 + w, y1, z0 + w), ground))
    world = t.list()
    if "boxes" not in drop:
        t.add(world, t.bvh(boxes1))
    light = t.quad((123, 554, 147), (300, 0, 0), (0, 0, 265), t.light((7, 7, 7)))
    t.add(world, light)
    lights = t.list(light)
    if "motion" not in drop:
        t.add(world, t.motion_sphere((400, 400, 200), (430, 400, 200), 50, t.lambertian((.7, .3, .1))))
    if "glass" not in drop:
        t.add(world, t.sphere((260, 150, 45), 50, t.dielectric(1.5)))
    if "metal" not in drop:
        t.add(world, t.sphere((0, 150, 145), 50, t.metal((0.8, 0.8, 0.9), 1.0)))
    if "water" not in drop:
        b = t.sphere((360, 150, 145), 70, t.dielectric(1.5))
        t.add(world, b)
        t.add(world, t.medium(b, .2, (0.2, 0.4, 0.9)))
    if "fog" not in drop:
        b2 = t.sphere((0, 0, 0), 5000, t.dielectric(1.5))
        t.add(world, t.medium(b2, .0001, (1, 1, 1)))
    if "earth" not in drop:
        with open(f"{asset_dir}/earthmap.ppm", "rb") as f:
            parts = f.read().split(b"\n", 3)
        wd, ht = map(int, parts[1].split())
        rgb = np.frombuffer(parts[3], np.uint8).reshape(ht, wd, 3)
        t.add(world, t.sphere((400, 200, 400), 100, t.lambertian(t.image(rgb))))
    p = t.noise(.2, rt.RT_NOISE_MARBLE)
    if "marble" not in drop:
        t.add(world, t.sphere((220, 280, 300), 80, t.lambertian(p)))
    boxes2 = t.list()
    white = t.lambertian((.73, .73, .73))
    for _ in range(1000):
        c = (t.rand_range(0, 165), t.rand_range(0, 165), t.rand_range(0, 165))
        if "cluster" not in drop:
            t.add(boxes2, t.sphere(c, 10, white))
    if "cluster" not in drop:
        t.add(world, t.translate(t.rotate_y(t.bvh(boxes2), 15), (-100, 270, 395)))
    cam = rt.Camera(AspectRatio=1.0, Width=48, SamplesPerPixel=9, MaxDepth=40, VerticalFOV=40)
    cam.PositionCamera((478, 278, -600), (278, 278, 0), (0, 1, 0))
    return t, cam, world, lights
