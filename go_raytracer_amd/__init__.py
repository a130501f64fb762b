"""go_raytracer_amd — MI355X-native drop-in for go_raytracer's render loop.

Python face of the C ABI (include/rt_abi.h).  The object model mirrors the
reference package API: ``Tree`` methods are the hittable constructors
(NewSphere, NewQuad, NewBox, RotateY, Translate, ConstantMedium, BuildBVH, ...),
``Camera`` mirrors camera.Camera's public fields (camera.go:26-36) with the
same zero-means-default rules, and ``Camera.Render(world, lights)`` renders
through the HIP path (camera.go:156).  There is no CPU render path here: the
HIP library must be built and a GPU present, otherwise calls raise.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import (RT_FT_ALL, RT_FT_BOX, RT_NOISE_MARBLE, RT_NOISE_PERLIN,  # noqa: F401
                   RT_NOISE_TURBULENT, RtCamera,
                   RtCameraDerived, RtError, RtRenderOpts, RtSceneInfo, RtStats, RtTreeView,
                   check, lib)

__all__ = ["Tree", "Camera", "Scene", "quantize", "format_ppm", "device_count", "RtError",
           "tune", "untune", "tuning", "tune_knobs", "tune_from_env",
           "demo_scene", "DEMO_SCENES", "LoadObjOptions", "DefaultLoadOptions", "quantize_device",
           "format_ppm_device"]

DEMO_SCENES = ("book1", "book2", "book3", "simple_light", "quads", "cornell", "cornell_smoke",
               "model")


def _d3(v):
    return _lib.D3(*[float(x) for x in v])


class Tree:
    """A scene under construction (rt_tree).  Handles are plain ints."""

    def __init__(self, seed=1):
        p = C.c_void_p()
        check(lib().rt_tree_create(C.byref(p)))
        self._p = p
        # bound now: at interpreter shutdown module globals (lib) may already be None
        self._destroy = lib().rt_tree_destroy
        check(lib().rt_tree_seed(self._p, seed))

    def __del__(self):
        if getattr(self, "_p", None):
            self._destroy(self._p)
            self._p = None

    @property
    def ptr(self):
        return self._p

    # scene RNG (replaces math/rand for scene content)
    def rand(self):
        return lib().rt_tree_rand(self._p)

    def rand_range(self, lo, hi):
        return lib().rt_tree_rand_range(self._p, lo, hi)

    def randn(self, n):
        return lib().rt_tree_randn(self._p, n)

    # textures
    def solid(self, r, g, b):
        return check(lib().rt_tex_solid(self._p, r, g, b))

    def checker(self, scale, even, odd):
        return check(lib().rt_tex_checker(self._p, scale, even, odd))

    def image(self, rgb):
        a = np.ascontiguousarray(rgb, dtype=np.uint8)
        h, w = a.shape[:2]
        return check(lib().rt_tex_image(self._p, a.ctypes.data, w, h))

    def noise(self, scale, variant=RT_NOISE_PERLIN):
        return check(lib().rt_tex_noise(self._p, scale, variant))

    def noise_tables(self, scale, variant, ranvec, perm):
        rv = np.ascontiguousarray(ranvec, dtype=np.float64).reshape(256, 3)
        pm = np.ascontiguousarray(perm, dtype=np.int32).reshape(3, 256)
        return check(lib().rt_tex_noise_tables(
            self._p, scale, variant, rv.ctypes.data_as(C.POINTER(C.c_double)),
            pm.ctypes.data_as(C.POINTER(C.c_int32))))

    # materials (a colour tuple means NewLambertian / NewDiffuseLight / NewIsotropic)
    def _tex(self, t):
        return t if isinstance(t, int) else self.solid(*t)

    def lambertian(self, tex):
        return check(lib().rt_mat_lambertian(self._p, self._tex(tex)))

    def metal(self, albedo, fuzz):
        return check(lib().rt_mat_metal(self._p, *[float(x) for x in albedo], fuzz))

    def dielectric(self, ior):
        return check(lib().rt_mat_dielectric(self._p, ior))

    def light(self, tex):
        return check(lib().rt_mat_diffuse_light(self._p, self._tex(tex)))

    def isotropic(self, tex):
        return check(lib().rt_mat_isotropic(self._p, self._tex(tex)))

    # hittables
    def list(self, *objs):
        h = check(lib().rt_new_list(self._p))
        for o in objs:
            self.add(h, o)
        return h

    def add(self, lst, obj):
        check(lib().rt_list_add(self._p, lst, obj))

    def bvh(self, lst):
        return check(lib().rt_build_bvh(self._p, lst))

    def sphere(self, center, radius, mat):
        return check(lib().rt_new_sphere(self._p, _d3(center), radius, mat))

    def motion_sphere(self, c1, c2, radius, mat):
        return check(lib().rt_new_motion_sphere(self._p, _d3(c1), _d3(c2), radius, mat))

    def quad(self, Q, u, v, mat):
        return check(lib().rt_new_quad(self._p, _d3(Q), _d3(u), _d3(v), mat))

    def box(self, a, b, mat):
        return check(lib().rt_new_box(self._p, _d3(a), _d3(b), mat))

    def triangle(self, verts, mat, normals=None, uv=None):
        v = np.ascontiguousarray(verts, dtype=np.float64).reshape(9)
        n = None if normals is None else np.ascontiguousarray(normals, dtype=np.float64).reshape(9)
        t = None if uv is None else np.ascontiguousarray(uv, dtype=np.float64).reshape(6)
        dp = C.POINTER(C.c_double)
        return check(lib().rt_new_triangle(
            self._p, v.ctypes.data_as(dp), None if n is None else n.ctypes.data_as(dp),
            None if t is None else t.ctypes.data_as(dp), mat))

    def triangles(self, verts, mats, normals=None, uv=None):
        v = np.ascontiguousarray(verts, dtype=np.float64).reshape(-1, 9)
        n_tri = v.shape[0]
        m = np.ascontiguousarray(np.broadcast_to(np.asarray(mats, dtype=np.int32), (n_tri,)))
        dp = C.POINTER(C.c_double)
        n = None if normals is None else np.ascontiguousarray(normals, dtype=np.float64).reshape(-1, 9)
        t = None if uv is None else np.ascontiguousarray(uv, dtype=np.float64).reshape(-1, 6)
        return check(lib().rt_new_triangles(
            self._p, n_tri, v.ctypes.data_as(dp), None if n is None else n.ctypes.data_as(dp),
            None if t is None else t.ctypes.data_as(dp), m.ctypes.data_as(C.POINTER(C.c_int32))))

    def translate(self, obj, offset):
        return check(lib().rt_translate(self._p, obj, _d3(offset)))

    def rotate_y(self, obj, degrees):
        return check(lib().rt_rotate_y(self._p, obj, degrees))

    def medium(self, boundary, density, tex):
        return check(lib().rt_constant_medium(self._p, boundary, density, self._tex(tex)))

    # OBJ/MTL loader (objLoader.go:63-538)
    def LoadObjWithOptions(self, filename, options=None, mtl_text=None, obj_text=None):
        """LoadObjWithOptions objLoader.go:72: returns (model, lights) node ids —
        BuildBVH over every triangle and the list of emissive (and, with
        FindWindows, dielectric) triangles.  ``obj_text``/``mtl_text`` load from
        memory instead of the files.  Image maps the C loader cannot decode
        (anything but binary PPM) are decoded here with PIL, when importable."""
        o = options if options is not None else DefaultLoadOptions()
        c, keep = o.to_c(self, filename, mtl_text)
        model, lights, info = C.c_int(-1), C.c_int(-1), _lib.RtObjInfo()
        if obj_text is None:
            check(lib().rt_load_obj(self._p, filename.encode(), C.byref(c), C.byref(model),
                                    C.byref(lights), C.byref(info)))
        else:
            ob = obj_text.encode() if isinstance(obj_text, str) else bytes(obj_text)
            mb = None if mtl_text is None else (
                mtl_text.encode() if isinstance(mtl_text, str) else bytes(mtl_text))
            check(lib().rt_load_obj_memory(
                self._p, ob, len(ob), mb, 0 if mb is None else len(mb),
                None if filename is None else filename.encode(), C.byref(c), C.byref(model),
                C.byref(lights), C.byref(info)))
        del keep
        self.last_obj_info = info
        return model.value, lights.value

    def LoadObj(self, filename, mat=-1):
        """LoadObj objLoader.go:64: default options with DefaultMaterial = mat."""
        o = DefaultLoadOptions()
        o.DefaultMaterial = mat
        return self.LoadObjWithOptions(filename, o)

    def view(self):
        v = RtTreeView()
        check(lib().rt_tree_get_view(self._p, C.byref(v)))
        return v


class LoadObjOptions:
    """LoadObjOptions objLoader.go:18-29 (DefaultMaterial: a material id, -1 = nil)."""

    def __init__(self, **kw):
        self.ScaleFactor = 1.0
        self.FlipYZ = False
        self.Debug = True
        self.IgnoreNormals = False
        self.Center = True
        self.FlipFaces = False
        self.Position = (0.0, 0.0, 0.0)
        self.DefaultMaterial = -1
        self.IgnoreMtl = False
        self.FindWindows = False
        for k, v in kw.items():
            if not hasattr(self, k):
                raise AttributeError(k)
            setattr(self, k, v)

    def to_c(self, tree, filename, mtl_text=None):
        c = _lib.RtObjOptions()
        check(lib().rt_obj_default_options(C.byref(c)))
        c.scale_factor = float(self.ScaleFactor)
        c.flip_yz, c.debug = int(bool(self.FlipYZ)), int(bool(self.Debug))
        c.ignore_normals, c.center = int(bool(self.IgnoreNormals)), int(bool(self.Center))
        c.flip_faces = int(bool(self.FlipFaces))
        c.default_material = int(self.DefaultMaterial)
        c.position = _d3(self.Position)
        c.ignore_mtl, c.find_windows = int(bool(self.IgnoreMtl)), int(bool(self.FindWindows))
        keep = []
        names = [] if self.IgnoreMtl else _mtl_image_names(filename, mtl_text)
        imgs = []
        for n in names:
            rgb = _decode_image(n)
            if rgb is None:
                continue
            keep.append(rgb)
            imgs.append(_lib.RtObjImage(n.encode(), rgb.ctypes.data, rgb.shape[1], rgb.shape[0]))
        if imgs:
            arr = (_lib.RtObjImage * len(imgs))(*imgs)
            keep.append(arr)
            c.n_images, c.images = len(imgs), C.cast(arr, C.POINTER(_lib.RtObjImage))
        return c, keep


def DefaultLoadOptions():
    """DefaultLoadOptions objLoader.go:32-45."""
    return LoadObjOptions()


def _mtl_image_names(filename, mtl_text):
    """map_Kd / map_Ka names of the MTL an OBJ references (mtlLoader.go:174-184)."""
    import os
    text = mtl_text
    if text is None:
        if filename is None or not os.path.exists(filename):
            return []
        import re
        with open(filename, "rb") as f:
            data = f.read()
        k = data.find(b"mtllib")  # C-speed scan first: most meshes have none
        m = None if k < 0 else re.search(rb"^[ \t]*mtllib[ \t]+([^\r\n]+)",
                                         data[max(0, data.rfind(b"\n", 0, k) + 1):], re.M)
        if m is None:
            return []
        lib_name = " ".join(m.group(1).decode("utf-8", "replace").split())
        path = os.path.join(os.path.dirname(filename), lib_name)
        if not os.path.exists(path):
            return []
        with open(path, "rb") as f:
            text = f.read()
    if isinstance(text, bytes):
        text = text.decode("utf-8", "replace")
    names = []
    for line in text.splitlines():
        p = line.split()
        if len(p) >= 2 and p[0] in ("map_Kd", "map_Ka"):
            names.append(" ".join(p[1:]))
    return names


def _decode_image(name):
    """image.Decode of a map file (imageLoader.go:29-46) for formats the C loader
    does not read; None leaves the file to the C loader (PPM, or its error)."""
    import os
    if not os.path.exists(name):
        return None
    with open(name, "rb") as f:
        if f.read(2) == b"P6":
            return None
    try:
        from PIL import Image
    except ImportError:
        return None
    return np.ascontiguousarray(np.asarray(Image.open(name).convert("RGB")), dtype=np.uint8)


class Camera:
    """camera.Camera (camera.go:24-62): public fields, 0 means default."""

    _FIELDS = ("AspectRatio", "Width", "SamplesPerPixel", "MaxDepth", "MaxThreads", "VerticalFOV",
               "DefocusAngle", "FocusDistance", "Background", "MaxContribution")

    def __init__(self, **kw):
        self.AspectRatio = 0.0
        self.Width = 0
        self.SamplesPerPixel = 0
        self.MaxDepth = 0
        self.MaxThreads = 0
        self.VerticalFOV = 0.0
        self.DefocusAngle = 0.0
        self.FocusDistance = 0.0
        self.Background = (0.0, 0.0, 0.0)
        self.MaxContribution = 0.0
        self._pos = None
        for k, v in kw.items():
            if k not in self._FIELDS:
                raise AttributeError(k)
            setattr(self, k, v)

    def PositionCamera(self, lookFrom=None, lookAt=None, vup=None):  # camera.go:65-81
        self._pos = (tuple(lookFrom) if lookFrom is not None else (0.0, 0.0, 0.0),
                     tuple(lookAt) if lookAt is not None else (0.0, 0.0, -1.0),
                     tuple(vup) if vup is not None else (0.0, 1.0, 0.0))

    def to_c(self):
        c = RtCamera()
        c.aspect_ratio = self.AspectRatio
        c.width = int(self.Width)
        c.samples_per_pixel = int(self.SamplesPerPixel)
        c.max_depth = int(self.MaxDepth)
        c.max_threads = int(self.MaxThreads)
        c.vertical_fov = self.VerticalFOV
        c.defocus_angle = self.DefocusAngle
        c.focus_distance = self.FocusDistance
        c.background = _d3(self.Background)
        c.max_contribution = self.MaxContribution
        if self._pos is not None:
            c.positioned = 1
            c.look_from, c.look_at, c.vup = (_d3(x) for x in self._pos)
        return c

    @classmethod
    def from_c(cls, c):
        cam = cls()
        cam.AspectRatio = c.aspect_ratio
        cam.Width = c.width
        cam.SamplesPerPixel = c.samples_per_pixel
        cam.MaxDepth = c.max_depth
        cam.MaxThreads = c.max_threads
        cam.VerticalFOV = c.vertical_fov
        cam.DefocusAngle = c.defocus_angle
        cam.FocusDistance = c.focus_distance
        cam.Background = tuple(c.background)
        cam.MaxContribution = c.max_contribution
        if c.positioned:
            cam._pos = (tuple(c.look_from), tuple(c.look_at), tuple(c.vup))
        return cam

    def derived(self):
        d = RtCameraDerived()
        c = self.to_c()
        check(lib().rt_camera_derive(C.byref(c), C.byref(d)))
        return d

    def image_size(self):
        d = self.derived()
        return d.width, d.height, d.spp_sqrt

    def Render(self, tree, world, lights, seed=1, device=0):
        """Render the full image on one GPU -> float32 [H, W, 3] linear mean RGB."""
        with Scene(tree, world, lights) as sc:
            img, _ = sc.render(self, seed=seed, device=device)
        return img


class Scene:
    """A flattened scene (rt_scene): BVH built on the host, uploaded on first render."""

    def __init__(self, tree, world, lights=-1):
        p = C.c_void_p()
        check(lib().rt_scene_create(tree.ptr, world, lights, C.byref(p)))
        self._p = p
        self._destroy = lib().rt_scene_destroy  # usable at interpreter shutdown
        self.tree = tree

    def close(self):
        if getattr(self, "_p", None):
            self._destroy(self._p)
            self._p = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def progress(self):
        """(samples done, samples total) of the render in flight (rt_progress);
        callable from another thread while render() blocks."""
        d, t = C.c_uint64(0), C.c_uint64(0)
        check(lib().rt_progress(self._p, C.byref(d), C.byref(t)))
        return d.value, t.value

    def info(self):
        i = RtSceneInfo()
        check(lib().rt_scene_info_get(self._p, C.byref(i)))
        return {f: getattr(i, f) for f, _ in RtSceneInfo._fields_}

    def export_bvh(self):
        nn, nr, root = C.c_int32(), C.c_int32(), C.c_uint32()
        check(lib().rt_scene_export_bvh(self._p, None, C.byref(nn), None, C.byref(nr), C.byref(root)))
        nodes = np.zeros((max(nn.value, 0), 16), np.float32)
        refs = np.zeros(max(nr.value, 0), np.uint32)
        check(lib().rt_scene_export_bvh(self._p, nodes.ctypes.data or None, C.byref(nn),
                                        refs.ctypes.data or None, C.byref(nr), C.byref(root)))
        n = C.c_int32()
        check(lib().rt_scene_export_prim_bounds(self._p, None, C.byref(n)))
        bounds = np.zeros((n.value, 6), np.float32)
        check(lib().rt_scene_export_prim_bounds(self._p, bounds.ctypes.data or None, C.byref(n)))
        return nodes, refs, int(root.value), bounds

    def export_bvh8(self):
        """(nodes uint32 [N, 32] in the rt_device.h BVH8 layout, refs8 uint32 [R])."""
        nn, nr = C.c_int32(), C.c_int32()
        check(lib().rt_scene_export_bvh8(self._p, None, C.byref(nn), None, C.byref(nr)))
        nodes = np.zeros((max(nn.value, 0), 32), np.uint32)
        refs = np.zeros(max(nr.value, 0), np.uint32)
        check(lib().rt_scene_export_bvh8(self._p, nodes.ctypes.data or None, C.byref(nn),
                                         refs.ctypes.data or None, C.byref(nr)))
        return nodes, refs

    def export_qbvh(self):
        """(items uint32 [N, 16]: the compressed BVH4's 64-B items, nodes4 uint32 [M, 32]:
        the BVH4 they encode, root4) -- rt_device.h layouts, for structural tests."""
        ni, nn, root = C.c_int32(), C.c_int32(), C.c_uint32()
        check(lib().rt_scene_export_qbvh(self._p, None, C.byref(ni), None, C.byref(nn), C.byref(root)))
        items = np.zeros((max(ni.value, 0), 16), np.uint32)
        nodes = np.zeros((max(nn.value, 0), 32), np.uint32)
        check(lib().rt_scene_export_qbvh(self._p, items.ctypes.data or None, C.byref(ni),
                                         nodes.ctypes.data or None, C.byref(nn), C.byref(root)))
        return items, nodes, int(root.value)

    MODES = {"auto": 0, "wavefront": 1, "fused": 2}

    @staticmethod
    def _opts(seed, device, rank, nranks, path_slots, chunk, profile, stream, mode="auto"):
        o = RtRenderOpts()
        o.mode = Scene.MODES[mode]
        o.seed = seed
        o.device = device
        o.rank = rank
        o.nranks = nranks
        o.path_slots = path_slots
        o.chunk = chunk
        o.flags = _lib.RT_FLAG_PROFILE if profile else 0
        o.stream = stream
        return o

    def render(self, camera, seed=1, device=0, rank=0, nranks=1, path_slots=0, chunk=0,
               profile=False, trace=None, mode="auto", progress_slices=0):
        """Render this rank's rows -> (float32 [rows, W, 3], stats dict).

        progress_slices=S runs the fused render as S launches so that progress()
        (from another thread) advances per slice; the image is the same.

        trace=(pixel, sample) additionally returns stats["trace"]: float32 [V, 12]
        {o.xyz, time, d.xyz, vertex, t, u, v, ref bits} per world.Hit of that sample.
        """
        d = camera.derived()
        rows = len(range(rank, d.height, nranks))
        out = np.zeros((rows, d.width, 3), np.float32)
        st = RtStats()
        c = camera.to_c()
        o = self._opts(seed, device, rank, nranks, path_slots, chunk, profile, None, mode)
        o.progress_slices = progress_slices
        tbuf = None
        if trace is not None:
            tbuf = np.zeros((d.max_depth + 1, 12), np.float32)
            o.trace_pixel, o.trace_sample = int(trace[0]), int(trace[1])
            o.trace_cap = tbuf.shape[0]
            o.trace_out = tbuf.ctypes.data
        check(lib().rt_render(self._p, C.byref(c), C.byref(o), out.ctypes.data, C.byref(st)))
        res = {f: getattr(st, f) for f, _ in RtStats._fields_}
        if tbuf is not None:
            res["trace"] = tbuf[tbuf[:, 7] >= 0]
        return out, res

    def render_multi(self, camera, devices, seed=1, path_slots=0, chunk=0, profile=False,
                     mode="auto", rccl=False):
        """The whole image over several devices (rt_render_multi: row r on
        devices[r % n], gathered to devices[0] by peer copies, or by one RCCL
        ncclGather with rccl=True) -> (float32 [H, W, 3], stats)."""
        d = camera.derived()
        out = np.zeros((d.height, d.width, 3), np.float32)
        st = _multi(self, camera, devices, (out.ctypes.data, False), seed, path_slots, chunk,
                    profile, mode, rccl)
        return out, st

    def render_multi_device(self, camera, devices, out_ptr, seed=1, path_slots=0, chunk=0,
                            profile=False, mode="auto", rccl=False):
        """rt_render_multi_device: the whole image into a device buffer on devices[0]."""
        return _multi(self, camera, devices, (out_ptr, True), seed, path_slots, chunk, profile,
                      mode, rccl)

    def render_device(self, camera, out_ptr, seed=1, device=0, rank=0, nranks=1, path_slots=0,
                      chunk=0, profile=False, stream=None, mode="auto"):
        """Render into a device buffer (e.g. torch tensor .data_ptr()) on `stream`."""
        st = RtStats()
        c = camera.to_c()
        o = self._opts(seed, device, rank, nranks, path_slots, chunk, profile, stream, mode)
        check(lib().rt_render_device(self._p, C.byref(c), C.byref(o), C.c_void_p(out_ptr),
                                     C.byref(st)))
        return {f: getattr(st, f) for f, _ in RtStats._fields_}


def _multi(scene, camera, devices, out_ptr, seed, path_slots, chunk, profile, mode, rccl=False):
    devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
    st = RtStats()
    c = camera.to_c()
    o = scene._opts(seed, int(devices[0]) if len(devices) else 0, 0, 1, path_slots, chunk,
                    profile, None, mode)
    if rccl:
        o.flags |= _lib.RT_FLAG_GATHER_RCCL
    fn = lib().rt_render_multi_device if out_ptr[1] else lib().rt_render_multi
    check(fn(scene._p, C.byref(c), C.byref(o), devs, len(devices), C.c_void_p(out_ptr[0]),
             C.byref(st)))
    return {f: getattr(st, f) for f, _ in RtStats._fields_}


def demo_scene(name, seed=1, asset_dir=None):
    """Build a main.go scene -> (tree, camera, world, lights)."""
    import os
    if asset_dir is None:
        asset_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                 "assets")
    t = Tree(seed)
    cam = RtCamera()
    w, l = C.c_int(), C.c_int()
    check(lib().rt_demo_scene(t.ptr, name.encode(), asset_dir.encode(), C.byref(cam), C.byref(w),
                              C.byref(l)))
    return t, Camera.from_c(cam), w.value, l.value


def substitute_mesh_obj(nu=0, nv=0):
    """The "model" scene's dragon.obj substitute as OBJ bytes (rt_substitute_mesh_obj)."""
    n = check(int(lib().rt_substitute_mesh_obj(nu, nv, None, 0)))
    buf = C.create_string_buffer(n)
    check(int(lib().rt_substitute_mesh_obj(nu, nv, buf, n)))
    return buf.raw[:n]


def quantize(rgb):
    """PrintColor (vec/color.go:23-46) on a float32 [..., 3] image -> uint8."""
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    out = np.zeros(a.shape, np.uint8)
    check(lib().rt_quantize(a.ctypes.data, a.size // 3, out.ctypes.data))
    return out


def format_ppm(rgb):
    """PPM P3 text exactly as the reference writes it (camera.go:160 + PrintColor)."""
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = a.shape[:2]
    n = lib().rt_format_ppm(a.ctypes.data, w, h, None, 0)
    check(int(n))
    buf = C.create_string_buffer(int(n))
    check(int(lib().rt_format_ppm(a.ctypes.data, w, h, buf, n)))
    return buf.raw[:n]


def _stream_of(t):
    import torch
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def quantize_device(rgb):
    """PrintColor on a device float32 [..., 3] torch tensor -> device uint8 tensor
    (HIP kernel, rt_quantize_device)."""
    import torch
    a = rgb.contiguous().to(torch.float32)
    out = torch.empty(a.shape, dtype=torch.uint8, device=a.device)
    check(lib().rt_quantize_device(a.data_ptr(), a.numel() // 3, out.data_ptr(),
                                   a.device.index or 0, _stream_of(a)))
    return out


def format_ppm_device(rgb, to_host=True):
    """The P3 text of camera.go:160 built on the GPU from a device float32
    [H, W, 3] tensor (rt_format_ppm_device).  Returns bytes, or the device
    uint8 tensor when to_host is False."""
    import torch
    a = rgb.contiguous().to(torch.float32)
    h, w = a.shape[:2]
    dev, st = a.device.index or 0, _stream_of(a)
    n = int(lib().rt_format_ppm_device(a.data_ptr(), w, h, None, 0, dev, st))
    check(n)
    out = torch.empty(n, dtype=torch.uint8, device=a.device)
    check(int(lib().rt_format_ppm_device(a.data_ptr(), w, h, out.data_ptr(), n, dev, st)))
    return out.cpu().numpy().tobytes() if to_host else out


def device_count():
    return lib().rt_device_count()


# ---- tuning knobs (rt_tune_set): the library never reads the process environment ----
def tune_knobs():
    """{knob name: changes_image_bits} for every knob the library consults."""
    n = lib().rt_tune_list(-1, None, None)
    out = {}
    for i in range(n):
        name, bits = C.c_char_p(), C.c_int32()
        check(lib().rt_tune_list(i, C.byref(name), C.byref(bits)))
        out[name.value.decode()] = bool(bits.value)
    return out


def tune(name, value):
    """Set knob `name` (e.g. "RT_TAIL_FRAC") to `value`; None clears it."""
    v = None if value is None else str(value).encode()
    check(lib().rt_tune_set(name.encode(), v))


def tune_get(name):
    """The text knob `name` is set to, or None when it is at its default."""
    n = int(lib().rt_tune_get(name.encode(), None, 0))
    check(n)
    if n == 0:
        return None
    buf = C.create_string_buffer(n)
    check(int(lib().rt_tune_get(name.encode(), buf, n)))
    return buf.value.decode()


def untune(name=None):
    """Clear one knob, or every knob (name None)."""
    check(lib().rt_tune_set(None if name is None else name.encode(), None))


class tuning:
    """Context manager: ``with rt.tuning(RT_SPLIT_MIN=0): ...`` sets knobs, then puts back the
    values they had on entry (cleared if they were unset)."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.saved = {}

    def __enter__(self):
        self.saved = {k: tune_get(k) for k in self.knobs}
        try:
            for k, v in self.knobs.items():
                tune(k, v)
        except BaseException:
            self.__exit__()
            raise
        return self

    def __exit__(self, *a):
        for k, v in self.saved.items():
            tune(k, v)


def tune_from_env(environ=None):
    """Dev tools only (tools/*): copy RT_* knobs from the environment into the library, an
    explicit opt-in of the calling process.  Returns the knobs set."""
    import os
    env = os.environ if environ is None else environ
    got = {k: env[k] for k in tune_knobs() if env.get(k)}
    for k, v in got.items():
        tune(k, v)
    return got
