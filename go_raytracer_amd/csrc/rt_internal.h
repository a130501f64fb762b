// rt_internal.h — host-side structures behind the opaque rt_tree / rt_scene handles.
#pragma once
#include <stdint.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "rt_device.h"

namespace rt {

// thread-local error slot (rt_last_error)
int set_error(int code, const char* fmt, ...);

// host_tune.cpp: tuning overrides set by the caller through rt_tune_set (the library never
// reads the process environment).  The value of knob `name`, or `dflt` when it is not set.
bool tune_str(const char* name, std::string* out);
double tune_num(const char* name, double dflt);
int tune_int(const char* name, int dflt);
int32_t tune_count();  // knobs currently set (rt_scene_info.tuned, rt_stats.tuned)

struct Tree {
  // nodes as created; LIST/BVH children live in lists[node.a]
  std::vector<rt_node> nodes;
  std::vector<std::vector<int32_t>> lists;
  std::vector<rt_tri> tris;
  std::vector<rt_material> materials;
  std::vector<rt_texture> textures;
  std::vector<std::vector<uint8_t>> image_data;
  std::vector<rt_image> images;
  std::vector<rt_perlin> perlins;
  uint64_t rng = 0x853c49e6748fea9bull;

  // packed view (rebuilt lazily when dirty)
  bool dirty = true;
  std::vector<rt_node> v_nodes;
  std::vector<int32_t> v_children;

  double rand01();
  int randn(int n);
  void pack();
};

// Host copy of the flattened scene plus its device mirror.
// World spheres this large stay out of the BVH and are tested in fp64 at the start of every
// ray (trav_init): the BVH's sphere leaves are then all small and tested in fp32
constexpr double kBigSphereR = 256.0;
struct HostScene {
  std::vector<F4> sph_cr, sph_mv;
  std::vector<F2> sph_uv;
  std::vector<F4> quad;      // 5 per quad
  std::vector<F4> tri;       // 3 per tri
  std::vector<F4> tri_attr;  // 6 per tri
  std::vector<F4> box_recs;  // 4 per box leaf: the leaf record (rt_device.h), ref in [0].w
  std::vector<F4> nodes;     // BVH2, 4 per node (export / structural tests)
  std::vector<F4> nodes4;    // BVH4 the kernels traverse, 8 per node (rt_device.h)
  uint32_t root4 = PRIM_NONE;
  std::vector<F4> nodes8;    // BVH8, 8 F4 per node, root = node 0 (large scenes, host_bvh8.cpp)
  std::vector<uint32_t> refs8;  // the BVH8's leaf records in node order (prim refs)
  std::vector<uint32_t> refs;
  uint32_t root = PRIM_NONE;
  std::vector<float> prim_bounds;  // 6 per world ref (export/tests)
  std::vector<DevMedium> media;
  std::vector<uint32_t> medium_refs;
  std::vector<uint32_t> big_refs;  // world spheres of radius >= kBigSphereR: tested in fp64
                                   // by every ray before the BVH (not BVH prims)
  int32_t medium_draws = 0;
  std::vector<DevLight> lights;
  std::vector<DevMaterial> mats;
  std::vector<DevTexture> texs;
  std::vector<uint8_t> texels;
  std::vector<DevImage> images;
  std::vector<DevPerlin> perlins;
  int32_t n_world_prims = 0;
  int32_t bvh_depth = 0;
  int32_t max_leaf = 0;
  int32_t bvh_builder = 0;  // 0 host binned SAH, 1 device PLOC
  uint32_t features = 0;    // scene_features(), computed once by rt_scene_create
  bool noise_table0 = true; // every reachable noise texture uses perlin table 0 (scene_features)
  int32_t tuned = 0;        // tuning knobs set when the scene was created (rt_scene_info.tuned)
};

struct DeviceScene;  // defined in the HIP translation unit
struct RenderState;

// Progress of the tracked render (rt_progress): written by the rendering thread,
// read by any polling thread under `mu`.  One render is tracked at a time: the
// rt_render / rt_render_multi call that finds `busy` clear claims it, and
// only that render updates and clears it, so concurrent renders of one scene on
// other devices neither reset nor finish another render's record.
struct Progress {
  std::mutex mu;
  int busy = 0;                 // 1 while the tracked render is in flight
  int device = -1;
  uint64_t total = 0;           // samples of the current / last render
  uint64_t done = 0;            // samples of the last render once it returned
  std::vector<void*> events;    // hipEvent_t recorded after each slice
  std::vector<uint64_t> cum;    // samples complete when event i has fired
};

// Render buffers of one (device, slot): slot 0 serves rt_render / rt_render_device,
// slots 1..n the shares of rt_render_multi (so {0, 0, 0} gets three of them).  The
// mutex is held for the whole render: one render in flight per (scene, device, slot).
struct SlotState {
  std::mutex mu;
  RenderState* st = nullptr;
};

// A device's copy of the scene.  `mu` is held while it is uploaded, so uploads to
// different devices run concurrently (rt_render_multi's share threads), and a
// render on a device whose copy is being uploaded waits for that copy only.
struct DeviceSlot {
  std::mutex mu;
  DeviceScene* ds = nullptr;  // null until the upload succeeded
};

struct Scene {
  HostScene h;
  std::mutex mu;                                    // guards the maps (not the renders)
  std::map<int, DeviceSlot*> devs;                  // per device ordinal, uploaded lazily
  std::map<std::pair<int, int>, SlotState*> slots;  // per (device, slot)
  std::mutex multi_mu;                              // one rt_render_multi at a time
  void* multi_buf = nullptr;                        // gather + image buffer on the first device
  size_t multi_bytes = 0;
  int multi_dev = -1;
  void* rccl = nullptr;                             // RCCL gather state (rt_render.hip RcclGather)
  Progress prog;
  // the compressed BVH4 (host_qbvh.cpp), built on the host once, at the first render that
  // can traverse it (rt_render.hip ensure_qbvh), then uploaded per device
  std::mutex qb_mu;
  bool qb_built = false;
  std::vector<F4> qb;
  size_t qb_items = 0;
};

// host_flatten.cpp
int flatten_scene(const Tree& t, int world, int lights, HostScene& out);
// host_bvh.cpp
int build_bvh(HostScene& s, const std::vector<F4>& lo, const std::vector<F4>& hi,
              const std::vector<uint32_t>& prims);
// host_bvh8.cpp: the BVH8 of s.nodes (the binary tree) -> s.nodes8 / s.refs8
constexpr size_t kBvh8MinRefs = 1024;
int build_bvh8(HostScene& s);
// host_qbvh.cpp: s's BVH4 as 64-B compressed nodes with the single-prim leaf records inline
// (rt_device.h "compressed BVH4 node"); *n_items = 0 when the tree is not encodable
int build_qbvh(const HostScene& s, const std::vector<F4>& recs, std::vector<F4>* out,
               size_t* n_items);
// rt_build.hip: the same outputs as build_bvh, built by PLOC on `device` (-1: the calling
// thread's current device; the current device is restored on return)
int build_bvh_device(HostScene& s, const std::vector<F4>& lo, const std::vector<F4>& hi,
                     const std::vector<uint32_t>& prims, int device);
bool bvh_device_available();
// box leaves only in scenes of more world prims than this (counting faces; host_flatten.cpp)
constexpr size_t kBoxLeafMinPrims = 256;
// host_scene.cpp: RT_FT_* features a flattened scene needs
uint32_t scene_features(const HostScene& h, bool* noise_table0 = nullptr);
// rt_render.hip
void release_device(Scene* s);

}  // namespace rt

struct rt_tree {
  rt::Tree t;
};
struct rt_scene {
  rt::Scene s;
};
