// host_tune.cpp — tuning overrides (rt_tune_set): the A/B and test switches of the library.
//
// The library never reads the process environment.  Every knob below has a measured default
// (DESIGN.md §6 "Tuning knobs"); a knob differs from it only after the caller sets it through
// rt_tune_set, and rt_scene_info.tuned / rt_stats.tuned report how many knobs were set when
// the scene was built / the render ran.  A Go host that inherits an environment therefore
// gets the default kernels, trees and schedules whatever RT_* variables it carries.
#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>

#include "rt_internal.h"

namespace rt {
namespace {

// every knob the library consults; `bits` = it may change image bits (the others only move
// work: exact fixed-point pixel sums make the image independent of them)
struct Knob {
  const char* name;
  bool bits;
};
constexpr Knob kKnobs[] = {
    // scene creation (host_flatten.cpp, host_bvh.cpp, host_scene.cpp, rt_build.hip)
    {"RT_BOX_LEAVES", true},       // 0: expand box leaves into six quad leaves
    {"RT_BIG_SPHERE_R", true},     // spheres of at least this radius are tested before the BVH
    {"RT_BVH_BUILDER", false},     // host | device | auto (closest hits do not depend on the tree)
    {"RT_BVH_DEVICE_MIN", false},  // world prims from which "auto" builds on the device
    {"RT_BVH8", false},            // 1: also build the BVH8 (kernels only with -DRT_BVH8_KERNELS)
    {"RT_BVH_LEAF", false},        // host SAH: leaf target
    {"RT_BVH_CT", false},          // host SAH: traversal cost
    {"RT_BVH_CI", false},          // host SAH: intersection cost
    {"RT_BVH_TOP", false},         // PLOC: clusters left to the host SAH top
    {"RT_THREADS", false},         // host BVH build threads (bit-identical for any count)
    {"RT_FEATURES_ALL", true},     // 1: count every material/texture (bigger kernel)
    // first upload of a scene to a device (rt_render.hip upload_scene)
    {"RT_BRUTE_MAX", true},        // record-loop scenes: up to this many leaf entries
    {"RT_BRUTE_AXIS", false},      // 0: no axis-aligned record groups
    {"RT_BRUTE_VERT", false},      // 0: no y-parallel record group
    {"RT_BRUTE_BOX", true},        // 0: boxes as six records instead of one slab test
    {"RT_BRUTE_MIXED", false},     // 0: two odd axis-aligned records join the general pairs
    {"RT_SHADE_LDS", false},       // 0: no LDS shade table for the lean record loop
    // every render (rt_render.hip render_impl)
    {"RT_TREE", true},             // 2 / 4: force the BVH2 / BVH4 over the record loop
    {"RT_BRUTE_SMEM", false},      // 1: record loop through the scalar cache
    {"RT_QBVH", false},            // 0: 128-B BVH4 nodes instead of the compressed 64-B ones
    {"RT_CHUNK_NEED", false},      // chunks per lane that pick the chunk size
    {"RT_TAIL_FRAC", false},       // tail phase: 1 / fraction of the samples
    {"RT_TAIL_K", false},          // tail phase chunk size
    {"RT_CSUM", false},            // 0: pixel atomics instead of per-chunk records
    {"RT_CSUM_MAX_MB", false},     // per-chunk record buffer cap (MiB)
    {"RT_CHUNK_ROWS", false},      // rows per chunk-order group
    {"RT_STEP_BUDGET", false},     // traversal steps per scheduling round
    {"RT_SHADE_MIN", false},       // ready lanes before a wave shades
    {"RT_GRAB_MIN", false},        // chunks per refill of a wave's batch
    {"RT_SPLIT_MIN", false},       // drain: samples a lane must have left to share (0: off)
    {"RT_PARTS_LOG2", false},      // chunk-counter partitions (log2)
    {"RT_GRAN_LOG2", false},       // partition granule (log2 chunks)
    {"RT_WAVE_TIMES", false},      // debug: write per-wave records to this file
    {"RT_TIMING", false},          // debug: host phase timings on stderr
};

std::mutex g_mu;
std::map<std::string, std::string> g_set;

const Knob* find_knob(const char* name) {
  for (const Knob& k : kKnobs)
    if (strcmp(k.name, name) == 0) return &k;
  return nullptr;
}

}  // namespace

bool tune_str(const char* name, std::string* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_set.find(name);
  if (it == g_set.end()) return false;
  if (out) *out = it->second;
  return true;
}

double tune_num(const char* name, double dflt) {
  std::string v;
  if (!tune_str(name, &v) || v.empty()) return dflt;
  return atof(v.c_str());
}

int tune_int(const char* name, int dflt) {
  std::string v;
  if (!tune_str(name, &v) || v.empty()) return dflt;
  return atoi(v.c_str());
}

int32_t tune_count() {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int32_t)g_set.size();
}

}  // namespace rt

extern "C" {

int rt_tune_set(const char* name, const char* value) {
  if (!name) {
    std::lock_guard<std::mutex> lk(rt::g_mu);
    rt::g_set.clear();
    return RT_OK;
  }
  if (!rt::find_knob(name)) return rt::set_error(RT_ERR_INVALID, "rt_tune_set: unknown knob %s", name);
  std::lock_guard<std::mutex> lk(rt::g_mu);
  if (value) rt::g_set[name] = value;
  else rt::g_set.erase(name);
  return RT_OK;
}

int rt_tune_list(int32_t i, const char** name, int32_t* changes_bits) {
  const int32_t n = (int32_t)(sizeof(rt::kKnobs) / sizeof(rt::kKnobs[0]));
  if (i < 0) return n;
  if (i >= n) return rt::set_error(RT_ERR_INVALID, "rt_tune_list: index %d of %d", i, n);
  if (name) *name = rt::kKnobs[i].name;
  if (changes_bits) *changes_bits = rt::kKnobs[i].bits ? 1 : 0;
  return n;
}

}  // extern "C"
