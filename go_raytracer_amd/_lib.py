"""ctypes binding of the C ABI in include/rt_abi.h (librt_amd.so).

The library is built in-tree (go_raytracer_amd/csrc/Makefile, or
``__graft_entry__.build()``).  There is no fallback: if the shared object is
missing, importing the binding raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT_AMD_LIB") or os.path.join(_HERE, "librt_amd.so")  # env: dev A/B

RT_OK = 0
RT_ERR_INVALID = -1
RT_ERR_UNSUPPORTED = -2
RT_ERR_DEVICE = -3
RT_ERR_OOM = -4
RT_ERR_IO = -5

RT_TEX_SOLID, RT_TEX_CHECKER, RT_TEX_IMAGE, RT_TEX_NOISE = range(4)
RT_NOISE_PERLIN, RT_NOISE_MARBLE, RT_NOISE_TURBULENT = 1, 2, 3
(RT_MAT_LAMBERTIAN, RT_MAT_METAL, RT_MAT_DIELECTRIC, RT_MAT_DIFFUSE_LIGHT,
 RT_MAT_ISOTROPIC) = range(5)
(RT_NODE_LIST, RT_NODE_BVH, RT_NODE_SPHERE, RT_NODE_QUAD, RT_NODE_TRIANGLE,
 RT_NODE_TRANSLATE, RT_NODE_ROTATE_Y, RT_NODE_MEDIUM) = range(8)
RT_FLAG_PROFILE = 1
RT_FLAG_GATHER_RCCL = 2  # rt_render_multi: one RCCL ncclGather instead of peer copies
RT_FT_SPHERE, RT_FT_TRI, RT_FT_METAL, RT_FT_DIEL = 1, 2, 4, 8
RT_FT_MEDIA, RT_FT_CHECKER, RT_FT_IMAGE, RT_FT_NOISE = 16, 32, 64, 128
RT_FT_BOX = 256
RT_FT_ALL = 511
RT_MODE_AUTO, RT_MODE_WAVEFRONT, RT_MODE_FUSED = 0, 1, 2

D3 = C.c_double * 3


class RtCamera(C.Structure):
    _fields_ = [
        ("aspect_ratio", C.c_double), ("width", C.c_int32),
        ("samples_per_pixel", C.c_int32), ("max_depth", C.c_int32),
        ("max_threads", C.c_int32), ("vertical_fov", C.c_double),
        ("defocus_angle", C.c_double), ("focus_distance", C.c_double),
        ("background", D3), ("max_contribution", C.c_double),
        ("look_from", D3), ("look_at", D3), ("vup", D3),
        ("positioned", C.c_int32), ("_pad", C.c_int32),
    ]


class RtCameraDerived(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("spp_sqrt", C.c_int32),
        ("max_depth", C.c_int32), ("pixel_samples_scale", C.c_double),
        ("recip_spp_sqrt", C.c_double), ("center", D3), ("pixel00", D3),
        ("delta_u", D3), ("delta_v", D3), ("defocus_u", D3), ("defocus_v", D3),
        ("defocus_angle", C.c_double), ("max_contribution", C.c_double),
        ("background", D3),
    ]


class RtSceneInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "n_spheres", "n_quads", "n_triangles", "n_world_prims", "n_media",
        "n_lights", "n_bvh_nodes", "bvh_depth", "max_leaf", "n_materials",
        "n_textures", "n_images", "n_perlins", "medium_draws")] + [
        ("device_bytes", C.c_int64), ("features", C.c_int32), ("bvh_builder", C.c_int32),
        ("tuned", C.c_int32), ("_pad", C.c_int32)]


class RtRenderOpts(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64), ("device", C.c_int32), ("rank", C.c_int32),
        ("nranks", C.c_int32), ("path_slots", C.c_int32), ("chunk", C.c_int32),
        ("flags", C.c_int32), ("mode", C.c_int32), ("stream", C.c_void_p),
        ("trace_pixel", C.c_int64), ("trace_sample", C.c_int32), ("trace_cap", C.c_int32),
        ("trace_out", C.c_void_p), ("progress_slices", C.c_int32), ("_pad3", C.c_int32),
    ]


class RtStats(C.Structure):
    _fields_ = [
        ("samples", C.c_uint64), ("segments", C.c_uint64),
        ("stack_pushes", C.c_uint64), ("extend_rays", C.c_uint64),
        ("shade_rays", C.c_uint64), ("ms_total", C.c_double),
        ("ms_extend", C.c_double), ("ms_shade", C.c_double),
        ("ms_other", C.c_double), ("n_extend_launches", C.c_int32),
        ("n_shade_launches", C.c_int32), ("iterations", C.c_int32),
        ("rows", C.c_int32), ("mode", C.c_int32), ("path_slots", C.c_int32),
        ("ms_fused", C.c_double),
        ("kernel_features", C.c_int32), ("scene_features", C.c_int32),
        ("tree_width", C.c_int32), ("lds_scene", C.c_int32),
        ("chunk_samples", C.c_int32), ("record_boxes", C.c_int32),
        ("overflow_samples", C.c_uint64),
        ("tuned", C.c_int32), ("chunk_records", C.c_int32),
    ]


class RtTreeView(C.Structure):
    _fields_ = [
        ("nodes", C.c_void_p), ("n_nodes", C.c_int32),
        ("children", C.c_void_p), ("n_children", C.c_int32),
        ("tris", C.c_void_p), ("n_tris", C.c_int32),
        ("materials", C.c_void_p), ("n_materials", C.c_int32),
        ("textures", C.c_void_p), ("n_textures", C.c_int32),
        ("images", C.c_void_p), ("n_images", C.c_int32),
        ("perlins", C.c_void_p), ("n_perlins", C.c_int32),
    ]


class RtObjImage(C.Structure):
    _fields_ = [("name", C.c_char_p), ("rgb", C.c_void_p), ("w", C.c_int32), ("h", C.c_int32)]


class RtObjOptions(C.Structure):  # LoadObjOptions objLoader.go:18-29
    _fields_ = [
        ("scale_factor", C.c_double), ("flip_yz", C.c_int32), ("debug", C.c_int32),
        ("ignore_normals", C.c_int32), ("center", C.c_int32), ("flip_faces", C.c_int32),
        ("default_material", C.c_int32), ("position", D3), ("ignore_mtl", C.c_int32),
        ("find_windows", C.c_int32), ("n_images", C.c_int32), ("_pad", C.c_int32),
        ("images", C.POINTER(RtObjImage)),
    ]


class RtObjInfo(C.Structure):
    _fields_ = [
        ("n_vertices", C.c_int64), ("n_normals", C.c_int64), ("n_texcoords", C.c_int64),
        ("n_triangles", C.c_int64), ("n_lights", C.c_int64), ("n_materials", C.c_int32),
        ("default_material", C.c_int32), ("bounds_min", D3), ("bounds_max", D3), ("center", D3),
    ]


_P = C.c_void_p
_I = C.c_int
_DP = C.POINTER(C.c_double)

# name -> (restype, argtypes); every symbol declared in include/rt_abi.h
SIGNATURES = {
    "rt_last_error": (C.c_char_p, []),
    "rt_abi_version": (_I, []),
    "rt_tune_set": (_I, [C.c_char_p, C.c_char_p]),
    "rt_tune_get": (_I, [C.c_char_p, C.c_char_p, C.c_int32]),
    "rt_tune_list": (_I, [C.c_int32, C.POINTER(C.c_char_p), C.POINTER(C.c_int32)]),
    "rt_tree_create": (_I, [C.POINTER(_P)]),
    "rt_tree_destroy": (_I, [_P]),
    "rt_tree_seed": (_I, [_P, C.c_uint64]),
    "rt_tree_rand": (C.c_double, [_P]),
    "rt_tree_rand_range": (C.c_double, [_P, C.c_double, C.c_double]),
    "rt_tree_randn": (_I, [_P, _I]),
    "rt_tex_solid": (_I, [_P, C.c_double, C.c_double, C.c_double]),
    "rt_tex_checker": (_I, [_P, C.c_double, _I, _I]),
    "rt_tex_image": (_I, [_P, C.c_void_p, _I, _I]),
    "rt_tex_noise": (_I, [_P, C.c_double, _I]),
    "rt_tex_noise_tables": (_I, [_P, C.c_double, _I, _DP, C.POINTER(C.c_int32)]),
    "rt_mat_lambertian": (_I, [_P, _I]),
    "rt_mat_metal": (_I, [_P, C.c_double, C.c_double, C.c_double, C.c_double]),
    "rt_mat_dielectric": (_I, [_P, C.c_double]),
    "rt_mat_diffuse_light": (_I, [_P, _I]),
    "rt_mat_isotropic": (_I, [_P, _I]),
    "rt_new_list": (_I, [_P]),
    "rt_list_add": (_I, [_P, _I, _I]),
    "rt_build_bvh": (_I, [_P, _I]),
    "rt_new_sphere": (_I, [_P, D3, C.c_double, _I]),
    "rt_new_motion_sphere": (_I, [_P, D3, D3, C.c_double, _I]),
    "rt_new_quad": (_I, [_P, D3, D3, D3, _I]),
    "rt_new_box": (_I, [_P, D3, D3, _I]),
    "rt_new_triangle": (_I, [_P, _DP, _DP, _DP, _I]),
    "rt_new_triangles": (_I, [_P, _I, _DP, _DP, _DP, C.POINTER(C.c_int32)]),
    "rt_translate": (_I, [_P, _I, D3]),
    "rt_rotate_y": (_I, [_P, _I, C.c_double]),
    "rt_constant_medium": (_I, [_P, _I, C.c_double, _I]),
    "rt_obj_default_options": (_I, [C.POINTER(RtObjOptions)]),
    "rt_load_obj": (_I, [_P, C.c_char_p, C.POINTER(RtObjOptions), C.POINTER(_I), C.POINTER(_I),
                         C.POINTER(RtObjInfo)]),
    "rt_load_obj_memory": (_I, [_P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p,
                                C.POINTER(RtObjOptions), C.POINTER(_I), C.POINTER(_I),
                                C.POINTER(RtObjInfo)]),
    "rt_tree_get_view": (_I, [_P, C.POINTER(RtTreeView)]),
    "rt_camera_derive": (_I, [C.POINTER(RtCamera), C.POINTER(RtCameraDerived)]),
    "rt_scene_create": (_I, [_P, _I, _I, C.POINTER(_P)]),
    "rt_scene_destroy": (_I, [_P]),
    "rt_scene_info_get": (_I, [_P, C.POINTER(RtSceneInfo)]),
    "rt_scene_export_bvh": (_I, [_P, C.c_void_p, C.POINTER(C.c_int32), C.c_void_p,
                                 C.POINTER(C.c_int32), C.POINTER(C.c_uint32)]),
    "rt_scene_export_bvh8": (_I, [_P, C.c_void_p, C.POINTER(C.c_int32), C.c_void_p,
                                  C.POINTER(C.c_int32)]),
    "rt_scene_export_qbvh": (_I, [_P, C.c_void_p, C.POINTER(C.c_int32), C.c_void_p,
                                  C.POINTER(C.c_int32), C.POINTER(C.c_uint32)]),
    "rt_scene_export_prim_bounds": (_I, [_P, C.c_void_p, C.POINTER(C.c_int32)]),
    "rt_render": (_I, [_P, C.POINTER(RtCamera), C.POINTER(RtRenderOpts), C.c_void_p,
                       C.POINTER(RtStats)]),
    "rt_render_device": (_I, [_P, C.POINTER(RtCamera), C.POINTER(RtRenderOpts), C.c_void_p,
                              C.POINTER(RtStats)]),
    "rt_render_multi": (_I, [_P, C.POINTER(RtCamera), C.POINTER(RtRenderOpts),
                             C.POINTER(C.c_int32), C.c_int32, C.c_void_p, C.POINTER(RtStats)]),
    "rt_render_multi_device": (_I, [_P, C.POINTER(RtCamera), C.POINTER(RtRenderOpts),
                                    C.POINTER(C.c_int32), C.c_int32, C.c_void_p,
                                    C.POINTER(RtStats)]),
    "rt_quantize": (_I, [C.c_void_p, C.c_int64, C.c_void_p]),
    "rt_format_ppm": (C.c_int64, [C.c_void_p, _I, _I, C.c_void_p, C.c_int64]),
    "rt_progress": (_I, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "rt_quantize_device": (_I, [C.c_void_p, C.c_int64, C.c_void_p, _I, C.c_void_p]),
    "rt_format_ppm_device": (C.c_int64, [C.c_void_p, _I, _I, C.c_void_p, C.c_int64, _I,
                                         C.c_void_p]),
    "rt_demo_scene": (_I, [_P, C.c_char_p, C.c_char_p, C.POINTER(RtCamera), C.POINTER(_I),
                           C.POINTER(_I)]),
    "rt_demo_scene_name": (_I, [_I, C.POINTER(C.c_char_p)]),
    "rt_substitute_mesh_obj": (C.c_int64, [_I, _I, C.c_void_p, C.c_int64]),
    "rt_device_count": (_I, []),
}

_lib = None


def lib():
    """Load librt_amd.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built: run `make -C go_raytracer_amd/csrc` "
                          "or __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("RT_AMD_LIB") and not hasattr(L, name):
                continue  # dev A/B against an older build that predates the symbol
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class RtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rt error {code}: {msg}")
        self.code = code


def check(rc):
    """Raise RtError for a negative status, else return rc (a handle or RT_OK)."""
    if rc < 0:
        raise RtError(rc, lib().rt_last_error().decode(errors="replace"))
    return rc
