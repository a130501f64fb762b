// host_tune.cpp — tuning overrides (rt_tune_set): the A/B and test switches of the library.
//
// The library never reads the process environment.  Every knob below has a measured default
// (DESIGN.md §6 "Tuning knobs"); a knob differs from it only after the caller sets it through
// rt_tune_set, and rt_scene_info.tuned / rt_stats.tuned report how many knobs were set when
// the scene was built / the render ran.  A Go host that inherits an environment therefore
// gets the default kernels, trees and schedules whatever RT_* variables it carries.
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>

#include "rt_internal.h"

namespace rt {
namespace {

// every knob the library consults; `bits` = it may change image bits (the others only move
// work: exact fixed-point pixel sums make the image independent of them)
// kind: 'i' integer, 'f' number, 's' string; numeric values outside [lo, hi] are refused by
// rt_tune_set (RT_ERR_INVALID), so every knob a render reads is in range
struct Knob {
  const char* name;
  bool bits;
  char kind;
  double lo, hi;
};
constexpr double kBig = 1e30;
constexpr Knob kKnobs[] = {
    // scene creation (host_flatten.cpp, host_bvh.cpp, host_scene.cpp, rt_build.hip)
    {"RT_BOX_LEAVES", true, 'i', 0, 1},       // 0: expand box leaves into six quad leaves
    {"RT_BIG_SPHERE_R", true, 'f', 0, kBig},     // spheres of at least this radius are tested before the BVH
    {"RT_BVH_BUILDER", false, 's', 0, 0},     // host | device | auto (closest hits do not depend on the tree)
    {"RT_BVH_DEVICE_MIN", false, 'f', 0, kBig},  // world prims from which "auto" builds on the device
    {"RT_BVH8", false, 'i', 0, 1},            // 1: also build the BVH8 (kernels only with -DRT_BVH8_KERNELS)
    {"RT_BVH_LEAF", false, 'i', 1, 64},        // host SAH: leaf target
    {"RT_BVH_CT", false, 'f', 1e-06, 1000000.0},          // host SAH: traversal cost
    {"RT_BVH_CI", false, 'f', 1e-06, 1000000.0},          // host SAH: intersection cost
    {"RT_BVH_TOP", false, 'i', 1, 1073741824},         // PLOC: clusters left to the host SAH top
    {"RT_THREADS", false, 'i', 1, 1024},         // host BVH build threads (bit-identical for any count)
    {"RT_FEATURES_ALL", true, 'i', 0, 1},     // 1: count every material/texture (bigger kernel)
    // first upload of a scene to a device (rt_render.hip upload_scene)
    {"RT_BRUTE_MAX", true, 'i', 0, 1048576},        // record-loop scenes: up to this many leaf entries
    {"RT_BRUTE_AXIS", false, 'i', 0, 1},      // 0: no axis-aligned record groups
    {"RT_BRUTE_VERT", false, 'i', 0, 1},      // 0: no y-parallel record group
    {"RT_BRUTE_BOX", true, 'i', 0, 1},        // 0: boxes as six records instead of one slab test
    {"RT_BRUTE_MIXED", false, 'i', 0, 1},     // 0: two odd axis-aligned records join the general pairs
    {"RT_SHADE_LDS", false, 'i', 0, 1},       // 0: no LDS shade table for the lean record loop
    // every render (rt_render.hip render_impl)
    {"RT_TREE", true, 'i', -1, 4},             // 2 / 4: force the BVH2 / BVH4 over the record loop
    {"RT_BRUTE_SMEM", false, 'i', -1, 1},      // 1: record loop through the scalar cache
    {"RT_QBVH", false, 'i', 0, 1},            // 0: 128-B BVH4 nodes instead of the compressed 64-B ones
    {"RT_CHUNK_NEED", false, 'i', 1, 1048576},      // chunks per lane that pick the chunk size
    {"RT_TAIL_FRAC", false, 'i', -1, 1024},       // tail phase: 1 / fraction of the samples
    {"RT_TAIL_K", false, 'i', 1, 4096},          // tail phase chunk size
    {"RT_CSUM", false, 'i', 0, 1},            // 0: pixel atomics instead of per-chunk records
    {"RT_CSUM_MAX_MB", false, 'i', 0, 16777216},     // per-chunk record buffer cap (MiB)
    {"RT_CHUNK_ROWS", false, 'i', -1, 1073741824},      // rows per chunk-order group
    {"RT_SWEEP", false, 's', 0, 0},           // chunk-group sweep order: forward | reverse
    {"RT_STEP_BUDGET", false, 'i', 1, 1073741824},     // traversal steps per scheduling round
    {"RT_SHADE_MIN", false, 'i', 1, 64},       // ready lanes before a wave shades
    {"RT_GRAB_MIN", false, 'i', 1, 1048576},        // chunks per refill of a wave's batch
    {"RT_SPLIT_MIN", false, 'i', 0, 1048576},       // drain: samples a lane must have left to share (0: off)
    {"RT_PARTS_LOG2", false, 'i', 0, 6},      // chunk-counter partitions (log2)
    {"RT_GRAN_LOG2", false, 'i', 0, 20},       // partition granule (log2 chunks)
    {"RT_WAVE_TIMES", false, 's', 0, 0},      // debug: write per-wave records to this file
    {"RT_TIMING", false, 'i', 0, 1},          // debug: host phase timings on stderr
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
  const rt::Knob* k = rt::find_knob(name);
  if (!k) return rt::set_error(RT_ERR_INVALID, "rt_tune_set: unknown knob %s", name);
  if (value && k->kind != 's') {
    // the whole string must be one number (strtol / strtod with an end-pointer check) inside
    // the knob's range: a step budget of 0, say, would leave traversal without steps
    char* end = nullptr;
    errno = 0;
    const double v = k->kind == 'i' ? (double)strtoll(value, &end, 10) : strtod(value, &end);
    if (end == value || *end != '\0' || errno == ERANGE || !(v >= k->lo && v <= k->hi))
      return rt::set_error(RT_ERR_INVALID, "rt_tune_set: %s=\"%s\" is not a number in [%g, %g]",
                           name, value, k->lo, k->hi);
  }
  if (value && strcmp(name, "RT_BVH_BUILDER") == 0 && strcmp(value, "host") != 0 &&
      strcmp(value, "device") != 0 && strcmp(value, "auto") != 0 && value[0] != '\0')
    return rt::set_error(RT_ERR_INVALID, "rt_tune_set: RT_BVH_BUILDER=\"%s\" (host | device | auto)",
                         value);
  if (value && strcmp(name, "RT_SWEEP") == 0 && strcmp(value, "forward") != 0 &&
      strcmp(value, "reverse") != 0 && value[0] != '\0')
    return rt::set_error(RT_ERR_INVALID, "rt_tune_set: RT_SWEEP=\"%s\" (forward | reverse)", value);
  std::lock_guard<std::mutex> lk(rt::g_mu);
  if (value) rt::g_set[name] = value;
  else rt::g_set.erase(name);
  return RT_OK;
}

int rt_tune_get(const char* name, char* buf, int32_t cap) {
  if (!name || !rt::find_knob(name)) return rt::set_error(RT_ERR_INVALID, "rt_tune_get: unknown knob %s", name ? name : "(null)");
  std::string v;
  if (!rt::tune_str(name, &v)) return 0;
  if (buf && cap > 0) {
    const size_t n = std::min<size_t>(v.size(), (size_t)cap - 1);
    memcpy(buf, v.data(), n);
    buf[n] = '\0';
  }
  return (int)v.size() + 1;
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
