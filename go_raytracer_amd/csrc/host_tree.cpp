// host_tree.cpp — the scene tree: one C-ABI constructor per reference constructor.
//
// Mirrors internal/hittable's constructors (objects.go, materials.go,
// texture.go, transformation.go, medium.go, bvh.go, hittable.go).  Nothing here
// renders: the tree is the input consumed by the flattener (product) and by the
// CPU oracle (tests).
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "rt_internal.h"

namespace rt {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

// splitmix64: the scene-content stream replacing Go's global math/rand
static inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

double Tree::rand01() { return (double)(splitmix64(rng) >> 11) * 0x1.0p-53; }

int Tree::randn(int n) {
  if (n <= 0) return 0;
  int r = (int)(rand01() * (double)n);
  return r >= n ? n - 1 : r;
}

void Tree::pack() {
  if (!dirty) return;
  v_nodes = nodes;
  v_children.clear();
  for (auto& nd : v_nodes) {
    if (nd.kind == RT_NODE_LIST || nd.kind == RT_NODE_BVH) {
      const auto& ch = lists[nd.a];
      nd.a = (int32_t)v_children.size();
      nd.b = (int32_t)ch.size();
      v_children.insert(v_children.end(), ch.begin(), ch.end());
    }
  }
  dirty = false;
}

}  // namespace rt

using rt::set_error;

#define TREE_OR_FAIL(t) \
  if (!(t)) return set_error(RT_ERR_INVALID, "%s: null tree", __func__)

static bool valid_node(const rt_tree* t, int id) { return id >= 0 && id < (int)t->t.nodes.size(); }
static bool valid_mat(const rt_tree* t, int id) {
  return id >= 0 && id < (int)t->t.materials.size();
}
static bool valid_tex(const rt_tree* t, int id) {
  return id >= 0 && id < (int)t->t.textures.size();
}

static int add_node(rt_tree* t, const rt_node& n) {
  t->t.nodes.push_back(n);
  t->t.dirty = true;
  return (int)t->t.nodes.size() - 1;
}

extern "C" {

const char* rt_last_error(void) { return rt::g_err; }
int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_tree_create(rt_tree** out) {
  if (!out) return set_error(RT_ERR_INVALID, "rt_tree_create: null out");
  *out = new (std::nothrow) rt_tree();
  if (!*out) return set_error(RT_ERR_OOM, "rt_tree_create: out of memory");
  return RT_OK;
}

int rt_tree_destroy(rt_tree* t) {
  delete t;
  return RT_OK;
}

int rt_tree_seed(rt_tree* t, uint64_t seed) {
  TREE_OR_FAIL(t);
  t->t.rng = seed;
  return RT_OK;
}

double rt_tree_rand(rt_tree* t) { return t ? t->t.rand01() : 0.0; }

double rt_tree_rand_range(rt_tree* t, double lo, double hi) {
  // util.RangeRange utilities.go:12-14
  return lo + (hi - lo) * rt_tree_rand(t);
}

int rt_tree_randn(rt_tree* t, int n) { return t ? t->t.randn(n) : 0; }

// ---------------------------------------------------------------- textures
int rt_tex_solid(rt_tree* t, double r, double g, double b) {
  TREE_OR_FAIL(t);
  rt_texture x{};
  x.kind = RT_TEX_SOLID;
  x.color[0] = r;
  x.color[1] = g;
  x.color[2] = b;
  t->t.textures.push_back(x);
  return (int)t->t.textures.size() - 1;
}

int rt_tex_checker(rt_tree* t, double scale, int even_tex, int odd_tex) {
  TREE_OR_FAIL(t);
  if (!valid_tex(t, even_tex) || !valid_tex(t, odd_tex))
    return set_error(RT_ERR_INVALID, "rt_tex_checker: bad child texture");
  rt_texture x{};
  x.kind = RT_TEX_CHECKER;
  x.a = even_tex;
  x.b = odd_tex;
  x.scale = 1.0 / scale;  // inv_scale, texture.go:39
  t->t.textures.push_back(x);
  return (int)t->t.textures.size() - 1;
}

int rt_tex_image(rt_tree* t, const uint8_t* rgb, int w, int h) {
  TREE_OR_FAIL(t);
  if (w < 0 || h < 0 || (w * (int64_t)h > 0 && !rgb))
    return set_error(RT_ERR_INVALID, "rt_tex_image: bad image");
  t->t.image_data.emplace_back(rgb ? std::vector<uint8_t>(rgb, rgb + (size_t)w * h * 3)
                                   : std::vector<uint8_t>());
  rt_image im{};
  im.w = w;
  im.h = h;
  t->t.images.push_back(im);
  rt_texture x{};
  x.kind = RT_TEX_IMAGE;
  x.a = (int)t->t.images.size() - 1;
  t->t.textures.push_back(x);
  t->t.dirty = true;
  return (int)t->t.textures.size() - 1;
}

int rt_tex_noise_tables(rt_tree* t, double scale, int variant, const double* ranvec,
                        const int32_t* perm) {
  TREE_OR_FAIL(t);
  if (!ranvec || !perm) return set_error(RT_ERR_INVALID, "rt_tex_noise_tables: null tables");
  rt_perlin p;
  memcpy(p.ranvec, ranvec, sizeof p.ranvec);
  memcpy(p.perm, perm, sizeof p.perm);
  for (int a = 0; a < 3; ++a)
    for (int i = 0; i < 256; ++i)
      if (p.perm[a][i] < 0 || p.perm[a][i] > 255)
        return set_error(RT_ERR_INVALID, "rt_tex_noise_tables: perm out of range");
  t->t.perlins.push_back(p);
  rt_texture x{};
  x.kind = RT_TEX_NOISE;
  x.a = (int)t->t.perlins.size() - 1;
  x.variant = (variant >= 1 && variant <= 3) ? variant : RT_NOISE_PERLIN;  // texture.go:121
  x.scale = scale;
  t->t.textures.push_back(x);
  return (int)t->t.textures.size() - 1;
}

int rt_tex_noise(rt_tree* t, double scale, int variant) {
  TREE_OR_FAIL(t);
  // NewPerlin perlin.go:20-31: 256 x RangeRandom(-1,1).UnitVector(), then the
  // three permutations, each a Sattolo shuffle with rand.Intn(i) (perlin.go:85-90)
  double ranvec[256][3];
  int32_t perm[3][256];
  for (int i = 0; i < 256; ++i) {
    double x = rt_tree_rand_range(t, -1, 1), y = rt_tree_rand_range(t, -1, 1),
           z = rt_tree_rand_range(t, -1, 1);
    double inv = 1.0 / sqrt(x * x + y * y + z * z);
    ranvec[i][0] = x * inv;
    ranvec[i][1] = y * inv;
    ranvec[i][2] = z * inv;
  }
  for (int a = 0; a < 3; ++a) {
    for (int i = 0; i < 256; ++i) perm[a][i] = i;
    for (int i = 255; i > 0; --i) {
      int target = t->t.randn(i);
      std::swap(perm[a][i], perm[a][target]);
    }
  }
  return rt_tex_noise_tables(t, scale, variant, &ranvec[0][0], &perm[0][0]);
}

// --------------------------------------------------------------- materials
static int add_mat(rt_tree* t, const rt_material& m) {
  t->t.materials.push_back(m);
  return (int)t->t.materials.size() - 1;
}

int rt_mat_lambertian(rt_tree* t, int tex) {
  TREE_OR_FAIL(t);
  if (!valid_tex(t, tex)) return set_error(RT_ERR_INVALID, "rt_mat_lambertian: bad texture");
  rt_material m{};
  m.kind = RT_MAT_LAMBERTIAN;
  m.tex = tex;
  return add_mat(t, m);
}

int rt_mat_metal(rt_tree* t, double r, double g, double b, double fuzz) {
  TREE_OR_FAIL(t);
  rt_material m{};
  m.kind = RT_MAT_METAL;
  m.tex = -1;
  m.albedo[0] = r;
  m.albedo[1] = g;
  m.albedo[2] = b;
  m.fuzz = fuzz;  // NewMetal stores fuzz as given (materials.go:65-67)
  return add_mat(t, m);
}

int rt_mat_dielectric(rt_tree* t, double ior) {
  TREE_OR_FAIL(t);
  rt_material m{};
  m.kind = RT_MAT_DIELECTRIC;
  m.tex = -1;
  m.ior = ior;
  return add_mat(t, m);
}

int rt_mat_diffuse_light(rt_tree* t, int tex) {
  TREE_OR_FAIL(t);
  if (!valid_tex(t, tex)) return set_error(RT_ERR_INVALID, "rt_mat_diffuse_light: bad texture");
  rt_material m{};
  m.kind = RT_MAT_DIFFUSE_LIGHT;
  m.tex = tex;
  return add_mat(t, m);
}

int rt_mat_isotropic(rt_tree* t, int tex) {
  TREE_OR_FAIL(t);
  if (!valid_tex(t, tex)) return set_error(RT_ERR_INVALID, "rt_mat_isotropic: bad texture");
  rt_material m{};
  m.kind = RT_MAT_ISOTROPIC;
  m.tex = tex;
  return add_mat(t, m);
}

// -------------------------------------------------------------- hittables
int rt_new_list(rt_tree* t) {
  TREE_OR_FAIL(t);
  rt_node n{};
  n.kind = RT_NODE_LIST;
  n.mat = -1;
  t->t.lists.emplace_back();
  n.a = (int)t->t.lists.size() - 1;
  return add_node(t, n);
}

int rt_list_add(rt_tree* t, int list, int obj) {
  TREE_OR_FAIL(t);
  if (!valid_node(t, list) || t->t.nodes[list].kind != RT_NODE_LIST)
    return set_error(RT_ERR_INVALID, "rt_list_add: %d is not a list", list);
  if (!valid_node(t, obj)) return set_error(RT_ERR_INVALID, "rt_list_add: bad object %d", obj);
  t->t.lists[t->t.nodes[list].a].push_back(obj);
  t->t.dirty = true;
  return RT_OK;
}

int rt_build_bvh(rt_tree* t, int list) {
  TREE_OR_FAIL(t);
  if (!valid_node(t, list) || t->t.nodes[list].kind != RT_NODE_LIST)
    return set_error(RT_ERR_INVALID, "rt_build_bvh: %d is not a list", list);
  const auto& ch = t->t.lists[t->t.nodes[list].a];
  if (ch.empty())  // bvhHelper on an empty span dereferences objects[start] (bvh.go:44)
    return set_error(RT_ERR_INVALID, "rt_build_bvh: empty list");
  rt_node n{};
  n.kind = RT_NODE_BVH;
  n.mat = -1;
  t->t.lists.push_back(ch);  // BuildBVH snapshots the list (sorting is topology only)
  n.a = (int)t->t.lists.size() - 1;
  return add_node(t, n);
}

int rt_new_sphere(rt_tree* t, const double c[3], double r, int mat) {
  TREE_OR_FAIL(t);
  if (!c || !valid_mat(t, mat)) return set_error(RT_ERR_INVALID, "rt_new_sphere: bad args");
  rt_node n{};
  n.kind = RT_NODE_SPHERE;
  n.mat = mat;
  for (int i = 0; i < 3; ++i) n.p[i] = n.p[3 + i] = c[i];
  n.p[6] = r;
  n.p[7] = 0;  // not moving
  return add_node(t, n);
}

int rt_new_motion_sphere(rt_tree* t, const double c1[3], const double c2[3], double r, int mat) {
  TREE_OR_FAIL(t);
  if (!c1 || !c2 || !valid_mat(t, mat))
    return set_error(RT_ERR_INVALID, "rt_new_motion_sphere: bad args");
  rt_node n{};
  n.kind = RT_NODE_SPHERE;
  n.mat = mat;
  for (int i = 0; i < 3; ++i) {
    n.p[i] = c1[i];
    n.p[3 + i] = c2[i];
  }
  n.p[6] = r;
  n.p[7] = 1;
  return add_node(t, n);
}

int rt_new_quad(rt_tree* t, const double Q[3], const double u[3], const double v[3], int mat) {
  TREE_OR_FAIL(t);
  if (!Q || !u || !v || !valid_mat(t, mat))
    return set_error(RT_ERR_INVALID, "rt_new_quad: bad args");
  rt_node n{};
  n.kind = RT_NODE_QUAD;
  n.mat = mat;
  for (int i = 0; i < 3; ++i) {
    n.p[i] = Q[i];
    n.p[3 + i] = u[i];
    n.p[6 + i] = v[i];
  }
  return add_node(t, n);
}

int rt_new_box(rt_tree* t, const double a[3], const double b[3], int mat) {
  TREE_OR_FAIL(t);
  if (!a || !b || !valid_mat(t, mat)) return set_error(RT_ERR_INVALID, "rt_new_box: bad args");
  // NewBox objects.go:208-240: six quads in this order, then BuildBVH
  double mn[3], mx[3];
  for (int i = 0; i < 3; ++i) {
    mn[i] = std::min(a[i], b[i]);
    mx[i] = std::max(a[i], b[i]);
  }
  const double dx[3] = {mx[0] - mn[0], 0, 0}, dy[3] = {0, mx[1] - mn[1], 0},
               dz[3] = {0, 0, mx[2] - mn[2]};
  const double ndx[3] = {-dx[0], -dx[1], -dx[2]}, ndz[3] = {-dz[0], -dz[1], -dz[2]};
  int sides = rt_new_list(t);
  const double q0[3] = {mn[0], mn[1], mx[2]}, q1[3] = {mx[0], mn[1], mx[2]},
               q2[3] = {mx[0], mn[1], mn[2]}, q3[3] = {mn[0], mn[1], mn[2]},
               q4[3] = {mn[0], mx[1], mx[2]}, q5[3] = {mn[0], mn[1], mn[2]};
  rt_list_add(t, sides, rt_new_quad(t, q0, dx, dy, mat));   // front
  rt_list_add(t, sides, rt_new_quad(t, q1, ndz, dy, mat));  // right
  rt_list_add(t, sides, rt_new_quad(t, q2, ndx, dy, mat));  // back
  rt_list_add(t, sides, rt_new_quad(t, q3, dz, dy, mat));   // left
  rt_list_add(t, sides, rt_new_quad(t, q4, dx, ndz, mat));  // top
  rt_list_add(t, sides, rt_new_quad(t, q5, dx, dz, mat));   // bottom
  return rt_build_bvh(t, sides);
}

int rt_new_triangle(rt_tree* t, const double v[9], const double* normals, const double* uv,
                    int mat) {
  TREE_OR_FAIL(t);
  if (!v || !valid_mat(t, mat)) return set_error(RT_ERR_INVALID, "rt_new_triangle: bad args");
  rt_tri tr{};
  memcpy(tr.v, v, sizeof tr.v);
  if (normals) {
    memcpy(tr.n, normals, sizeof tr.n);
    tr.flags |= 1;
  }
  if (uv) {
    memcpy(tr.uv, uv, sizeof tr.uv);
    tr.flags |= 2;
  }
  tr.mat = mat;
  t->t.tris.push_back(tr);
  rt_node n{};
  n.kind = RT_NODE_TRIANGLE;
  n.mat = mat;
  n.a = (int)t->t.tris.size() - 1;
  return add_node(t, n);
}

int rt_new_triangles(rt_tree* t, int n, const double* v, const double* normals,
                     const double* uv, const int32_t* mats) {
  TREE_OR_FAIL(t);
  if (n < 0 || (n > 0 && (!v || !mats)))
    return set_error(RT_ERR_INVALID, "rt_new_triangles: bad args");
  int list = rt_new_list(t);
  auto& ch = t->t.lists[t->t.nodes[list].a];
  ch.reserve(n);
  t->t.tris.reserve(t->t.tris.size() + n);
  t->t.nodes.reserve(t->t.nodes.size() + n);
  for (int i = 0; i < n; ++i) {
    int id = rt_new_triangle(t, v + 9 * (size_t)i, normals ? normals + 9 * (size_t)i : nullptr,
                             uv ? uv + 6 * (size_t)i : nullptr, mats[i]);
    if (id < 0) return id;
    t->t.lists[t->t.nodes[list].a].push_back(id);
  }
  return list;
}

int rt_translate(rt_tree* t, int obj, const double off[3]) {
  TREE_OR_FAIL(t);
  if (!valid_node(t, obj) || !off) return set_error(RT_ERR_INVALID, "rt_translate: bad args");
  rt_node n{};
  n.kind = RT_NODE_TRANSLATE;
  n.mat = -1;
  n.a = obj;
  for (int i = 0; i < 3; ++i) n.p[i] = off[i];
  return add_node(t, n);
}

int rt_rotate_y(rt_tree* t, int obj, double degrees) {
  TREE_OR_FAIL(t);
  if (!valid_node(t, obj)) return set_error(RT_ERR_INVALID, "rt_rotate_y: bad object");
  rt_node n{};
  n.kind = RT_NODE_ROTATE_Y;
  n.mat = -1;
  n.a = obj;
  n.p[0] = degrees;
  return add_node(t, n);
}

int rt_constant_medium(rt_tree* t, int boundary, double density, int tex) {
  TREE_OR_FAIL(t);
  if (!valid_node(t, boundary)) return set_error(RT_ERR_INVALID, "rt_constant_medium: bad boundary");
  int mat = rt_mat_isotropic(t, tex);  // phaseFunction = NewIsotropicTexture (medium.go:20-25)
  if (mat < 0) return mat;
  rt_node n{};
  n.kind = RT_NODE_MEDIUM;
  n.mat = mat;
  n.a = boundary;
  n.p[0] = density;
  return add_node(t, n);
}

int rt_tree_get_view(const rt_tree* tc, rt_tree_view* out) {
  if (!tc || !out) return set_error(RT_ERR_INVALID, "rt_tree_get_view: null");
  rt_tree* t = const_cast<rt_tree*>(tc);
  t->t.pack();
  for (size_t i = 0; i < t->t.images.size(); ++i)
    t->t.images[i].rgb = t->t.image_data[i].empty() ? nullptr : t->t.image_data[i].data();
  out->nodes = t->t.v_nodes.data();
  out->n_nodes = (int32_t)t->t.v_nodes.size();
  out->children = t->t.v_children.data();
  out->n_children = (int32_t)t->t.v_children.size();
  out->tris = t->t.tris.data();
  out->n_tris = (int32_t)t->t.tris.size();
  out->materials = t->t.materials.data();
  out->n_materials = (int32_t)t->t.materials.size();
  out->textures = t->t.textures.data();
  out->n_textures = (int32_t)t->t.textures.size();
  out->images = t->t.images.data();
  out->n_images = (int32_t)t->t.images.size();
  out->perlins = t->t.perlins.data();
  out->n_perlins = (int32_t)t->t.perlins.size();
  return RT_OK;
}

}  // extern "C"
