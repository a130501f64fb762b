// host_scene.cpp — rt_scene_create / info / export (host side, no GPU needed).
#include <string.h>

#include "rt_internal.h"

using rt::set_error;

namespace rt {

static uint32_t fbits_host(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
// Prim types reachable by traversal, shading or light sampling, material kinds
// and texture kinds present: selects the fused-kernel instantiation.
// Features of what a render can reach: the world's and lights' prims, the media,
// the materials of those prims and media, and the textures of those materials
// (through checker children).  Materials and textures that are built but never
// placed (book1's perlin orbs, main.go:52-60) do not count, so such a scene runs a
// leaner kernel.  The knob RT_FEATURES_ALL=1 counts every table entry (A/B).
// *noise_table0: every reachable noise texture uses perlin table 0, the one the
// feature-set kernels stage in LDS (others need the all-features kernel).
uint32_t scene_features(const HostScene& h, bool* noise_table0) {
  uint32_t f = 0;
  if (noise_table0) *noise_table0 = true;
  std::vector<char> mat_used(h.mats.size(), 0);
  auto use_mat = [&](int m) {
    if (m >= 0 && (size_t)m < mat_used.size()) mat_used[m] = 1;
  };
  auto prim = [&](uint32_t ref) {
    if (ref == PRIM_NONE) return;
    const uint32_t type = ref >> 30, idx = ref & 0x3FFFFFFFu;
    if (type == PRIM_SPHERE) {
      f |= FT_SPHERE;
      if (idx < h.sph_mv.size()) use_mat((int)fbits_host(h.sph_mv[idx].w));
    } else if (type == PRIM_QUAD) {
      if (5 * (size_t)idx + 2 < h.quad.size()) use_mat((int)fbits_host(h.quad[5 * (size_t)idx + 2].w));
    } else if (type == PRIM_TRI) {
      f |= FT_TRI;
      if (3 * (size_t)idx < h.tri.size()) use_mat((int)fbits_host(h.tri[3 * (size_t)idx].w));
    } else {
      f |= FT_MEDIA;
    }
  };
  for (uint32_t r : h.refs) {
    if (r != PRIM_NONE && (r >> 30) == PRIM_BOX) {  // a box leaf: its six face quads
      f |= FT_BOX;
      const F4* b = &h.box_recs[4 * (size_t)(r & 0x3FFFFFFFu)];
      const float fr[6] = {b[2].y, b[2].z, b[2].w, b[3].x, b[3].y, b[3].z};
      for (float x : fr) {
        uint32_t q;
        memcpy(&q, &x, 4);
        prim(q);
      }
      continue;
    }
    prim(r);
  }
  for (uint32_t r : h.medium_refs) prim(r);
  for (uint32_t r : h.big_refs) prim(r);
  for (const DevLight& l : h.lights) prim(l.ref);
  if (!h.media.empty()) f |= FT_MEDIA;
  for (const DevMedium& m : h.media) use_mat(m.phase_mat);
  const bool every = tune_int("RT_FEATURES_ALL", 0) != 0;
  std::vector<char> tex_used(h.texs.size(), 0);
  std::vector<int> st;
  for (size_t i = 0; i < h.mats.size(); ++i) {
    if (!mat_used[i] && !every) continue;
    const DevMaterial& m = h.mats[i];
    if (m.kind == RT_MAT_METAL) f |= FT_METAL;
    if (m.kind == RT_MAT_DIELECTRIC) f |= FT_DIEL;
    if (m.kind == RT_MAT_ISOTROPIC) f |= FT_MEDIA;
    if (m.kind != RT_MAT_METAL && m.kind != RT_MAT_DIELECTRIC && m.tex >= 0) st.push_back(m.tex);
  }
  if (every)
    for (size_t i = 0; i < h.texs.size(); ++i) st.push_back((int)i);
  while (!st.empty()) {
    const int t = st.back();
    st.pop_back();
    if (t < 0 || (size_t)t >= h.texs.size() || tex_used[t]) continue;
    tex_used[t] = 1;
    const DevTexture& T = h.texs[t];
    if (T.kind == RT_TEX_CHECKER) {
      f |= FT_CHECKER;
      st.push_back(T.a);
      st.push_back(T.b);
    }
    if (T.kind == RT_TEX_IMAGE) f |= FT_IMAGE;
    if (T.kind == RT_TEX_NOISE) {
      f |= FT_NOISE;
      if (T.a != 0 && noise_table0) *noise_table0 = false;
    }
  }
  return f;
}
}  // namespace rt

extern "C" {

int rt_scene_create(const rt_tree* t, int world, int lights, rt_scene** out) {
  if (!t || !out) return set_error(RT_ERR_INVALID, "rt_scene_create: null");
  *out = nullptr;
  rt_scene* s = new (std::nothrow) rt_scene();
  if (!s) return set_error(RT_ERR_OOM, "rt_scene_create: out of memory");
  int rc = rt::flatten_scene(t->t, world, lights, s->s.h);
  if (rc) {
    delete s;
    return rc;
  }
  s->s.h.features = rt::scene_features(s->s.h, &s->s.h.noise_table0);  // walks every prim: once, not per render
  s->s.h.tuned = rt::tune_count();
  *out = s;
  return RT_OK;
}

int rt_scene_destroy(rt_scene* s) {
  if (!s) return RT_OK;
  rt::release_device(&s->s);
  delete s;
  return RT_OK;
}

int rt_scene_info_get(const rt_scene* sc, rt_scene_info* o) {
  if (!sc || !o) return set_error(RT_ERR_INVALID, "rt_scene_info_get: null");
  const rt::HostScene& h = sc->s.h;
  memset(o, 0, sizeof *o);
  o->n_spheres = (int32_t)h.sph_cr.size();
  o->n_quads = (int32_t)(h.quad.size() / 5);
  o->n_triangles = (int32_t)(h.tri.size() / 3);
  o->n_world_prims = h.n_world_prims;
  o->n_media = (int32_t)h.media.size();
  o->n_lights = (int32_t)h.lights.size();
  o->n_bvh_nodes = (int32_t)(h.nodes.size() / 4);
  o->bvh_depth = h.bvh_depth;
  o->max_leaf = h.max_leaf;
  o->n_materials = (int32_t)h.mats.size();
  o->n_textures = (int32_t)h.texs.size();
  o->n_images = (int32_t)h.images.size();
  o->n_perlins = (int32_t)h.perlins.size();
  o->medium_draws = h.medium_draws;
  int64_t b = 0;
  b += h.sph_cr.size() * 16 + h.sph_mv.size() * 16 + h.sph_uv.size() * 8;
  b += h.quad.size() * 16 + h.tri.size() * 16 + h.tri_attr.size() * 16;
  b += h.nodes.size() * 16 + h.refs.size() * 4;
  b += h.media.size() * sizeof(rt::DevMedium) + h.medium_refs.size() * 4;
  b += h.lights.size() * sizeof(rt::DevLight) + h.mats.size() * sizeof(rt::DevMaterial);
  b += h.texs.size() * sizeof(rt::DevTexture) + h.texels.size();
  b += h.images.size() * sizeof(rt::DevImage) + h.perlins.size() * sizeof(rt::DevPerlin);
  o->device_bytes = b;
  o->features = (int32_t)h.features;
  o->bvh_builder = h.bvh_builder;
  o->tuned = h.tuned;
  return RT_OK;
}

int rt_scene_export_bvh(const rt_scene* sc, float* nodes, int32_t* n_nodes, uint32_t* prim_refs,
                        int32_t* n_refs, uint32_t* root) {
  if (!sc) return set_error(RT_ERR_INVALID, "rt_scene_export_bvh: null");
  const rt::HostScene& h = sc->s.h;
  if (n_nodes) *n_nodes = (int32_t)(h.nodes.size() / 4);
  if (n_refs) *n_refs = (int32_t)h.refs.size();
  if (root) *root = h.root;
  if (nodes && !h.nodes.empty()) memcpy(nodes, h.nodes.data(), h.nodes.size() * 16);
  if (prim_refs && !h.refs.empty()) memcpy(prim_refs, h.refs.data(), h.refs.size() * 4);
  return RT_OK;
}

int rt_scene_export_bvh8(const rt_scene* sc, float* nodes, int32_t* n_nodes, uint32_t* refs8,
                         int32_t* n_refs8) {
  if (!sc) return set_error(RT_ERR_INVALID, "rt_scene_export_bvh8: null");
  const rt::HostScene& h = sc->s.h;
  if (n_nodes) *n_nodes = (int32_t)(h.nodes8.size() / 8);
  if (n_refs8) *n_refs8 = (int32_t)h.refs8.size();
  if (nodes && !h.nodes8.empty()) memcpy(nodes, h.nodes8.data(), h.nodes8.size() * 16);
  if (refs8 && !h.refs8.empty()) memcpy(refs8, h.refs8.data(), h.refs8.size() * 4);
  return RT_OK;
}

int rt_scene_export_prim_bounds(const rt_scene* sc, float* bounds, int32_t* n) {
  if (!sc) return set_error(RT_ERR_INVALID, "rt_scene_export_prim_bounds: null");
  const rt::HostScene& h = sc->s.h;
  if (n) *n = (int32_t)(h.prim_bounds.size() / 6);
  if (bounds && !h.prim_bounds.empty())
    memcpy(bounds, h.prim_bounds.data(), h.prim_bounds.size() * 4);
  return RT_OK;
}

}  // extern "C"
