/*
 * rt_abi.h — C ABI of the MI355X path-tracing hot path (go_raytracer_amd).
 *
 * Drop-in boundary for the reference's per-pixel render loop
 *     (*Camera).Render(world, lights hittable.Hittable)   internal/camera/camera.go:156
 * The reference has no FFI; the seam is its Go interfaces (Hittable
 * hittable.go:60-65, Material materials.go:19-27, Texture texture.go:10-12).
 * A cgo shim walks the Go object tree with the rt_new_* /
 * rt_mat_* / rt_tex_* constructors below — one call per Go constructor — and
 * then calls rt_scene_create + rt_render instead of Camera.Render.
 *
 * Conventions: every function returns RT_OK (0) or a negative RT_ERR_* code,
 * or a non-negative handle.  Nothing aborts the process (the reference calls
 * log.Fatal, camera.go:188, hittable.go:70, imageLoader.go:32-36); the message
 * of the last failure on the calling thread is in rt_last_error().
 * All inputs are copied; callers may free them after the call returns.
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 4

enum {
  RT_OK = 0,
  RT_ERR_INVALID = -1,     /* bad argument / handle */
  RT_ERR_UNSUPPORTED = -2, /* e.g. a BVH or transform used as a light (hittable.go:69-72) */
  RT_ERR_DEVICE = -3,      /* HIP runtime failure or no GPU */
  RT_ERR_OOM = -4,
  RT_ERR_IO = -5
};

const char* rt_last_error(void);
int rt_abi_version(void);

/* Tuning overrides (A/B experiments and tests; the knobs and their measured defaults are
 * listed in DESIGN.md §6).  The library never reads the process environment: a knob
 * differs from its default only after the caller sets it here, and rt_scene_info.tuned /
 * rt_stats.tuned report how many knobs were set when the scene was created / the render
 * ran (the reference is configured through Camera fields only, camera.go:181-207).
 * value: a number as text (or a file path for RT_WAVE_TIMES, host|device|auto for
 * RT_BVH_BUILDER); NULL clears the knob; name NULL clears every knob.  Unknown names, text
 * that is not one whole number, and numbers outside the knob's range (e.g. RT_STEP_BUDGET
 * below 1) return RT_ERR_INVALID and leave the knob as it was.  Process-wide. */
int rt_tune_set(const char* name, const char* value);
/* The value knob `name` is set to: returns 0 when it is not set, else the value's length + 1
 * (the buffer size it needs), copying at most cap - 1 bytes and a NUL into buf when buf is not
 * NULL and cap > 0.  Unknown names return RT_ERR_INVALID. */
int rt_tune_get(const char* name, char* buf, int32_t cap);
/* Knob i's name and whether it may change image bits (the others move work only); returns
 * the number of knobs (i < 0: just the count). */
int rt_tune_list(int32_t i, const char** name, int32_t* changes_bits);

/* ------------------------------------------------------------------------ */
/* Scene tree: one constructor per reference constructor.                    */
/* ------------------------------------------------------------------------ */
typedef struct rt_tree rt_tree;

int rt_tree_create(rt_tree** out);
int rt_tree_destroy(rt_tree* t);

/* Scene-construction randomness (the reference uses the global math/rand for
 * random scene content, main.go:38-75,107,155, and perlin tables,
 * perlin.go:20-31).  A per-tree splitmix64 stream replaces it. */
int rt_tree_seed(rt_tree* t, uint64_t seed);
double rt_tree_rand(rt_tree* t);             /* rand.Float64()        */
double rt_tree_rand_range(rt_tree* t, double lo, double hi); /* util.RangeRange utilities.go:12 */
int rt_tree_randn(rt_tree* t, int n);        /* rand.Intn(n)          */

/* textures — texture.go */
enum { RT_TEX_SOLID = 0, RT_TEX_CHECKER = 1, RT_TEX_IMAGE = 2, RT_TEX_NOISE = 3 };
enum { RT_NOISE_PERLIN = 1, RT_NOISE_MARBLE = 2, RT_NOISE_TURBULENT = 3 }; /* texture.go:88-95 */
int rt_tex_solid(rt_tree* t, double r, double g, double b);                 /* NewSolidColor texture.go:18 */
int rt_tex_checker(rt_tree* t, double scale, int even_tex, int odd_tex);    /* NewCheckerboard texture.go:37 */
/* NewImageTexture texture.go:66 with the image already decoded to RGB8
 * rows (RTImage.bdata layout imageLoader.go:52-62); w*h*3 bytes copied. */
int rt_tex_image(rt_tree* t, const uint8_t* rgb, int w, int h);
/* NewNoiseTextureWithType texture.go:108: perlin tables drawn from the tree RNG
 * in NewPerlin's order (perlin.go:20-31, 81-90). */
int rt_tex_noise(rt_tree* t, double scale, int variant);
/* same, with explicit tables (ranvec[256][3] doubles, perm[3][256]) */
int rt_tex_noise_tables(rt_tree* t, double scale, int variant, const double* ranvec,
                        const int32_t* perm);

/* materials — materials.go */
enum {
  RT_MAT_LAMBERTIAN = 0,
  RT_MAT_METAL = 1,
  RT_MAT_DIELECTRIC = 2,
  RT_MAT_DIFFUSE_LIGHT = 3,
  RT_MAT_ISOTROPIC = 4
};
int rt_mat_lambertian(rt_tree* t, int tex);                               /* NewTexturedLambertian :40 */
int rt_mat_metal(rt_tree* t, double r, double g, double b, double fuzz); /* NewMetal :65 */
int rt_mat_dielectric(rt_tree* t, double ior);                            /* NewDielectric :89 */
int rt_mat_diffuse_light(rt_tree* t, int tex);                            /* NewDiffuseLightTextured :139 */
int rt_mat_isotropic(rt_tree* t, int tex);                                /* NewIsotropicTexture :165 */

/* hittables — hittable.go, bvh.go, objects.go, transformation.go, medium.go */
enum {
  RT_NODE_LIST = 0,
  RT_NODE_BVH = 1,
  RT_NODE_SPHERE = 2,
  RT_NODE_QUAD = 3,
  RT_NODE_TRIANGLE = 4,
  RT_NODE_TRANSLATE = 5,
  RT_NODE_ROTATE_Y = 6,
  RT_NODE_MEDIUM = 7
};
int rt_new_list(rt_tree* t);                        /* NewHittableList hittable.go:84 */
int rt_list_add(rt_tree* t, int list, int obj);     /* HittableList.Add hittable.go:113 */
int rt_build_bvh(rt_tree* t, int list);             /* BuildBVH bvh.go:21 */
int rt_new_sphere(rt_tree* t, const double center[3], double radius, int mat); /* objects.go:23 */
int rt_new_motion_sphere(rt_tree* t, const double c1[3], const double c2[3], double radius,
                         int mat);                  /* NewMotionSphere objects.go:30 */
int rt_new_quad(rt_tree* t, const double Q[3], const double u[3], const double v[3],
                int mat);                           /* NewQuad objects.go:129 */
int rt_new_box(rt_tree* t, const double a[3], const double b[3], int mat); /* NewBox objects.go:208 */
/* NewTriangle / NewTriangleWithNormals / NewTexturedTriangle[WithNormals]
 * objects.go:257-316.  normals (9) and uv (6) may be NULL. */
int rt_new_triangle(rt_tree* t, const double v[9], const double* normals, const double* uv,
                    int mat);
/* bulk form for meshes: n triangles, returns a LIST node holding them */
int rt_new_triangles(rt_tree* t, int n, const double* v, const double* normals,
                     const double* uv, const int32_t* mats);
int rt_translate(rt_tree* t, int obj, const double offset[3]);  /* Translate transformation.go:20 */
int rt_rotate_y(rt_tree* t, int obj, double degrees);           /* RotateY transformation.go:48 */
int rt_constant_medium(rt_tree* t, int boundary, double density, int tex); /* medium.go:20 */

/* ------------------------------------------------------------------------ */
/* OBJ/MTL loader — LoadObjWithOptions internal/objLoader/objLoader.go:72-538, */
/* LoadMTL + ConvertToRaytracerMaterial mtlLoader.go:53-326.  Builds the same  */
/* triangles (bit-identical fp64 vertices/normals/uvs), the same materials and */
/* the same two Hittables as the Go loader: *model = BuildBVH(all triangles),  */
/* *lights = list of the emissive (and, with find_windows, dielectric) ones.   */
/* ------------------------------------------------------------------------ */
typedef struct {
  const char* name;   /* map_Kd / map_Ka string exactly as written in the MTL */
  const uint8_t* rgb; /* w*h*3, decoded by the caller (image.Decode imageLoader.go:34) */
  int32_t w, h;
} rt_obj_image;

typedef struct {                /* LoadObjOptions objLoader.go:18-29 */
  double scale_factor;          /* ScaleFactor */
  int32_t flip_yz;              /* FlipYZ */
  int32_t debug;                /* Debug: print the loader's diagnostics to stdout */
  int32_t ignore_normals;       /* IgnoreNormals */
  int32_t center;               /* Center (Position is applied only when set, :243-248) */
  int32_t flip_faces;           /* FlipFaces */
  int32_t default_material;     /* DefaultMaterial; -1 = nil -> Lambertian(.8,.8,.8) :88-90 */
  double position[3];           /* Position */
  int32_t ignore_mtl;           /* IgnoreMtl */
  int32_t find_windows;         /* FindWindows */
  /* image textures named by map_Kd / map_Ka: looked up here by exact name
   * first; otherwise the file is opened as written (binary PPM only). */
  int32_t n_images;
  int32_t _pad;
  const rt_obj_image* images;
} rt_obj_options;

typedef struct {
  int64_t n_vertices, n_normals, n_texcoords, n_triangles, n_lights;
  int32_t n_materials;      /* materials in the MTL library */
  int32_t default_material; /* material id used for faces without a known usemtl */
  double bounds_min[3], bounds_max[3], center[3]; /* after scale/flip, before centring */
} rt_obj_info;

int rt_obj_default_options(rt_obj_options* o); /* DefaultLoadOptions objLoader.go:32-45 */
int rt_load_obj(rt_tree* t, const char* filename, const rt_obj_options* opts, int* model,
                int* lights, rt_obj_info* info);
/* Same from memory (e.g. a Go embed.FS); mtl_text, when non-NULL, replaces the file
 * named by mtllib; filename (may be NULL) only resolves the mtllib directory. */
int rt_load_obj_memory(rt_tree* t, const char* obj_text, size_t obj_len, const char* mtl_text,
                       size_t mtl_len, const char* filename, const rt_obj_options* opts,
                       int* model, int* lights, rt_obj_info* info);

/* ------------------------------------------------------------------------ */
/* Read-only view of a tree (consumed by the CPU oracle and the cgo shim).  */
/* ------------------------------------------------------------------------ */
typedef struct {
  int32_t kind;  /* RT_NODE_* */
  int32_t mat;   /* material id (prims), phase material (medium) */
  int32_t a, b;  /* LIST/BVH: children[a .. a+b); TRANSLATE/ROTATE_Y: a = child;
                    MEDIUM: a = boundary; TRIANGLE: a = index into tris */
  double p[10];  /* SPHERE: c1[3] c2[3] r moving; QUAD: Q u v; TRANSLATE: off;
                    ROTATE_Y: degrees; MEDIUM: density */
} rt_node;

typedef struct {
  double v[9];   /* 3 vertices */
  double n[9];   /* vertex normals (if flags & 1) */
  double uv[6];  /* texture coords (if flags & 2) */
  int32_t flags; /* 1 = has vertex normals, 2 = has uv */
  int32_t mat;
} rt_tri;

typedef struct {
  int32_t kind;   /* RT_MAT_* */
  int32_t tex;    /* lambertian / light / isotropic */
  double albedo[3];
  double fuzz;
  double ior;
} rt_material;

typedef struct {
  int32_t kind;    /* RT_TEX_* */
  int32_t a, b;    /* CHECKER: even, odd; IMAGE: image id; NOISE: perlin id */
  int32_t variant; /* NOISE */
  double color[3]; /* SOLID */
  double scale;    /* CHECKER: inv_scale (= 1/scale as texture.go:39); NOISE: scale */
} rt_texture;

typedef struct {
  int32_t w, h;
  const uint8_t* rgb; /* w*h*3 */
} rt_image;

typedef struct {
  double ranvec[256][3];
  int32_t perm[3][256];
} rt_perlin;

typedef struct {
  const rt_node* nodes;
  int32_t n_nodes;
  const int32_t* children;
  int32_t n_children;
  const rt_tri* tris;
  int32_t n_tris;
  const rt_material* materials;
  int32_t n_materials;
  const rt_texture* textures;
  int32_t n_textures;
  const rt_image* images;
  int32_t n_images;
  const rt_perlin* perlins;
  int32_t n_perlins;
} rt_tree_view;

int rt_tree_get_view(const rt_tree* t, rt_tree_view* out);

/* ------------------------------------------------------------------------ */
/* Camera — public fields of Camera camera.go:26-36 + PositionCamera :65.    */
/* Zero means "use the reference default" exactly as initialize() :181-207. */
/* ------------------------------------------------------------------------ */
typedef struct {
  double aspect_ratio;        /* 0 -> 1.0 */
  int32_t width;              /* 0 -> 100 */
  int32_t samples_per_pixel;  /* 0 -> 100 (truncated to floor(sqrt)^2, camera.go:211) */
  int32_t max_depth;          /* 0 -> 10 */
  int32_t max_threads;        /* -N; unused by the GPU path (kept for API parity) */
  double vertical_fov;        /* 0 -> 90 */
  double defocus_angle;       /* 0 -> 0 */
  double focus_distance;      /* 0 -> 10 */
  double background[3];       /* Background (nil in Go == black here) */
  double max_contribution;    /* 0 -> 1.5 */
  double look_from[3];        /* PositionCamera; a never-positioned camera uses */
  double look_at[3];          /*   lookFrom (0,0,0), lookAt (0,0,-1), vup (0,1,0) */
  double vup[3];
  int32_t positioned;         /* 0 -> the defaults above */
  int32_t _pad;
} rt_camera;

/* Derived geometry, initialize() camera.go:179-253 (fp64). */
typedef struct {
  int32_t width, height, spp_sqrt, max_depth;
  double pixel_samples_scale, recip_spp_sqrt;
  double center[3], pixel00[3], delta_u[3], delta_v[3], defocus_u[3], defocus_v[3];
  double defocus_angle, max_contribution;
  double background[3];
} rt_camera_derived;

int rt_camera_derive(const rt_camera* cam, rt_camera_derived* out);

/* ------------------------------------------------------------------------ */
/* Flattened scene + render.                                                 */
/* ------------------------------------------------------------------------ */
typedef struct rt_scene rt_scene;

/* Flatten world/lights (transforms baked, media separated, light table built)
 * and build the device BVH (BuildBVH bvh.go:21-61 + the world list).  Scenes of
 * >= 65536 world prims build it on the calling thread's current HIP device (PLOC,
 * DESIGN.md "BVH"; the current device is left unchanged) when one is
 * present, otherwise with the host binned-SAH builder; the knobs RT_BVH_BUILDER
 * (host|device) and RT_BVH_DEVICE_MIN (rt_tune_set) override.  lights may be -1. */
int rt_scene_create(const rt_tree* t, int world, int lights, rt_scene** out);
int rt_scene_destroy(rt_scene* s);

typedef struct {
  int32_t n_spheres, n_quads, n_triangles;
  int32_t n_world_prims, n_media, n_lights;
  int32_t n_bvh_nodes, bvh_depth, max_leaf;
  int32_t n_materials, n_textures, n_images, n_perlins;
  int32_t medium_draws; /* total free-flight draws per vertex */
  int64_t device_bytes; /* scene bytes uploaded to HBM */
  int32_t features;     /* RT_FT_* bits the scene needs (selects the fused kernel) */
  int32_t bvh_builder;  /* 0: host binned SAH, 1: device PLOC (rt_scene_create) */
  int32_t tuned;        /* rt_tune_set knobs set when the scene was created (0: defaults) */
  int32_t _pad;
} rt_scene_info;

/* scene features (rt_scene_info.features, rt_stats.kernel_features) */
enum {
  RT_FT_SPHERE = 1, RT_FT_TRI = 2, RT_FT_METAL = 4, RT_FT_DIEL = 8, RT_FT_MEDIA = 16,
  RT_FT_CHECKER = 32, RT_FT_IMAGE = 64, RT_FT_NOISE = 128,
  RT_FT_BOX = 256 /* box leaves (NewBox as one BVH leaf; scenes above 256 world prims) */
};
int rt_scene_info_get(const rt_scene* s, rt_scene_info* out);

/* BVH export for structural tests: nodes as 16 floats
 * {b0min[3], b0max[3], b1min[3], b1max[3], child0 bits, child1 bits, 0, 0},
 * leaf child encoding documented in DESIGN.md.  Pass NULL to query counts. */
int rt_scene_export_bvh(const rt_scene* s, float* nodes, int32_t* n_nodes, uint32_t* prim_refs,
                        int32_t* n_refs, uint32_t* root);
/* the wide tree large scenes render with: BVH8 nodes as 32 floats
 * (rt_device.h "BVH8 node", 16-bit planes) and the prim ref of each of its leaf
 * records; 0 nodes when the scene has none.  Pass NULL to query counts. */
int rt_scene_export_bvh8(const rt_scene* s, float* nodes, int32_t* n_nodes, uint32_t* refs8,
                         int32_t* n_refs8);
/* world-prim float AABBs in prim-ref order (6 floats each) */
int rt_scene_export_prim_bounds(const rt_scene* s, float* bounds, int32_t* n);
/* the compressed BVH4 the fused kernels read through L1/L2 (rt_device.h "compressed BVH4
 * node", 64-B items: nodes with fp16 child planes and single-prim leaf records; 0 items when
 * the scene's tree is not encodable) and the BVH4 it encodes (8 float4 per node), for
 * structural tests.  NULL pointers query the counts. */
int rt_scene_export_qbvh(const rt_scene* s, float* items, int32_t* n_items, float* nodes4,
                         int32_t* n_nodes4, uint32_t* root4);

enum {
  RT_FLAG_PROFILE = 1,     /* time every kernel with HIP events */
  RT_FLAG_GATHER_RCCL = 2  /* rt_render_multi: gather the shares with one RCCL ncclGather
                              (communicators over the device list, cached per scene;
                              the devices must be distinct) instead of peer copies */
};

/* execution strategy of the same per-vertex code (DESIGN.md "Kernels"):
 *   WAVEFRONT: queue-driven extend / shade kernels, path state in HBM (SoA)
 *   FUSED:     one persistent kernel, path state in registers
 *   AUTO:      the faster one for the scene */
enum { RT_MODE_AUTO = 0, RT_MODE_WAVEFRONT = 1, RT_MODE_FUSED = 2 };

typedef struct {
  uint64_t seed;       /* render_seed */
  int32_t device;      /* HIP device ordinal */
  int32_t rank;        /* row-interleaved shard: rows r with r % nranks == rank */
  int32_t nranks;
  int32_t path_slots;  /* wavefront capacity; 0 = auto */
  int32_t chunk;       /* samples per work chunk; 0 = auto */
  int32_t flags;       /* RT_FLAG_* */
  int32_t mode;        /* RT_MODE_* */
  void* stream;        /* hipStream_t to enqueue on; NULL = library stream */
  /* path trace of one sample (debugging): when trace_out != NULL the vertices
   * of sample trace_sample of global pixel trace_pixel are written as 12 floats
   * {o.xyz, time, d.xyz, vertex, t, u, v, prim-ref bits} per world.Hit call,
   * up to trace_cap vertices; unused entries have vertex = -1. */
  int64_t trace_pixel;
  int32_t trace_sample;
  int32_t trace_cap;
  float* trace_out;
  /* rt_progress granularity: the fused render runs as this many launches over
   * consecutive chunk ranges (same image, bit for bit) and rt_progress advances
   * as each completes.  0/1 = one launch, progress only reports start and end. */
  int32_t progress_slices;
  int32_t _pad3;
} rt_render_opts;

typedef struct {
  uint64_t samples;      /* W*rows*spp_sqrt^2 rendered by this call */
  uint64_t segments;     /* closest-hit queries (world.Hit calls, camera.go:300) */
  uint64_t stack_pushes; /* clamp-vertex weights stored (0 unless built with RT_COUNT_PUSHES) */
  uint64_t extend_rays;  /* total rays processed by extend launches */
  uint64_t shade_rays;
  double ms_total;       /* render wall time (host, incl. sync) */
  double ms_extend;      /* summed extend-kernel time (RT_FLAG_PROFILE) */
  double ms_shade;
  double ms_other;
  int32_t n_extend_launches;
  int32_t n_shade_launches;
  int32_t iterations;
  int32_t rows;          /* rows rendered by this rank */
  int32_t mode;          /* RT_MODE_* actually used */
  int32_t path_slots;    /* concurrent paths (wavefront slots / fused lanes) */
  double ms_fused;       /* fused-kernel time (RT_FLAG_PROFILE) */
  int32_t kernel_features; /* RT_FT_* set compiled into the fused kernel that ran */
  int32_t scene_features;  /* RT_FT_* set the scene needs */
  int32_t tree_width;      /* tree the kernels traversed: 0 none (record loop), 2 BVH2, 4 BVH4,
                              5 BVH4 with 64-B compressed nodes (large trees) */
  int32_t lds_scene;       /* 1: nodes (and leaf records) ran from the LDS cache */
  int32_t chunk_samples;   /* samples per work chunk (opts.chunk or the adaptive choice) */
  int32_t record_boxes;    /* boxes the record loop tested as one slab test each (0: none) */
  /* sample channels with |v| >= 2^31 / spp_sqrt^2 (outside the exact fixed-point pixel
   * sum; added in fp64 instead — the image is then order-dependent in those pixels) */
  uint64_t overflow_samples;
  int32_t tuned;           /* rt_tune_set knobs set when the render ran (0: defaults) */
  int32_t chunk_records;   /* 1: per-chunk sum records, 0: pixel atomics (record buffer
                              over its cap or not allocatable: same image) */
} rt_stats;

/* Render this rank's rows; out_rgb (host) receives linear mean RGB
 * [rows][W][3] fp32, rows = rows r with r % nranks == rank in increasing order.
 * Replaces (*Camera).Render's pixel loop, camera.go:156 -> :90-153 (one process,
 * one device; rank/nranks = the row partition of camera.go:119-122 across processes).
 * Threading: an rt_scene keeps one device copy per device ordinal and one set of
 * render buffers per device; rt_render / rt_render_device may run concurrently from
 * different threads for DIFFERENT devices of one scene; calls for the same device
 * serialise (the second waits for the first). */
int rt_render(rt_scene* s, const rt_camera* cam, const rt_render_opts* opts, float* out_rgb,
              rt_stats* stats);
/* Same, but out_rgb is a device pointer on opts->device (e.g. a torch tensor);
 * work is enqueued on opts->stream and the call returns after it completes. */
int rt_render_device(rt_scene* s, const rt_camera* cam, const rt_render_opts* opts,
                     float* out_rgb_device, rt_stats* stats);

/* Render the WHOLE image on n devices from one process (the north_star's 8-GPU tile
 * split, camera.go:119-122 row partition): device devices[i] renders rows
 * r % n == i, each share on its own host thread, stream and render buffers (a
 * device may repeat: {0, 0, 0} renders three shares on device 0); the shares are
 * copied to devices[0] (peer copies over xGMI) and de-interleaved there by a kernel.
 * out_rgb (host) receives [H][W][3]; the _device form writes a device pointer on
 * devices[0].  The image is bit-identical to rt_render's for any n (per-sample
 * fixed-point pixel sums).  opts->rank/nranks must be 0/1 and opts->stream NULL;
 * stats sum samples/segments over shares, ms_fused is the slowest share's.
 * opts->flags & RT_FLAG_GATHER_RCCL: each share renders into a padded send buffer on
 * its device and ONE ncclGather (RCCL over xGMI, root devices[0]) collects them, the
 * survey's collective for this step; same image bits.
 * One rt_render_multi per scene at a time (a second call waits). */
int rt_render_multi(rt_scene* s, const rt_camera* cam, const rt_render_opts* opts,
                    const int32_t* devices, int32_t n, float* out_rgb, rt_stats* stats);
int rt_render_multi_device(rt_scene* s, const rt_camera* cam, const rt_render_opts* opts,
                           const int32_t* devices, int32_t n, float* out_rgb_device,
                           rt_stats* stats);

/* Progress of the render in flight on scene s (the reference's progress bar,
 * camera.go:106-108 + internal/progress): may be polled from any thread while
 * rt_render blocks in another.  *total = samples of the current (or last)
 * render; *done = samples of the completed slices (opts.progress_slices), or
 * for rt_render_multi the samples of the completed shares, and *total once the
 * render returned.  A render refused before it starts leaves no render in
 * flight. */
int rt_progress(const rt_scene* s, uint64_t* done, uint64_t* total);

/* Output: PrintColor vec/color.go:23-46 (NaN->0, sqrt gamma, clamp .99999, x256). */
int rt_quantize(const float* rgb, int64_t n_pixels, uint8_t* out);
/* PPM P3 text exactly as camera.go:160 + PrintColor; returns bytes written
 * (call with out = NULL to size). */
int64_t rt_format_ppm(const float* rgb, int w, int h, char* out, int64_t cap);

/* On-device output (HIP): the same PrintColor bytes / P3 text, produced by kernels
 * from an image already in HBM (rgb_dev: device fp32 [n][3] on `device`; out_dev:
 * device memory; stream: hipStream_t or NULL).  The calls return after the work
 * completes.  rt_format_ppm_device returns the byte count (out_dev = NULL to size). */
int rt_quantize_device(const float* rgb_dev, int64_t n_pixels, uint8_t* out_dev, int device,
                       void* stream);
int64_t rt_format_ppm_device(const float* rgb_dev, int w, int h, char* out_dev, int64_t cap,
                             int device, void* stream);

/* Demo scenes mirroring main.go (by name or the main.go -S number).
 * names: book1, book2, book3, simple_light, quads, cornell, cornell_smoke, model
 * The camera receives the scene's settings; override fields afterwards. */
int rt_demo_scene(rt_tree* t, const char* name, const char* asset_dir, rt_camera* cam,
                  int* world, int* lights);
int rt_demo_scene_name(int s_number, const char** name_out);
/* The "model" scene's substitute for dragon.obj (absent from the reference) as OBJ
 * text: nu x nv grid of a torus-knot tube (nu, nv <= 0: 2048 x 256 = 1M triangles).
 * Returns the byte count; call with out = NULL to size.  Writing it to
 * <asset_dir>/dragon.obj lets "model" load it from disk like the real mesh. */
int64_t rt_substitute_mesh_obj(int nu, int nv, char* out, int64_t cap);

/* Number of HIP devices visible (0 on a CPU-only host; never aborts). */
int rt_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* RT_ABI_H */
