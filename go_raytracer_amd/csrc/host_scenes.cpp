// host_scenes.cpp — the demo scenes of main.go, built through the C ABI exactly
// as a Go caller would (one rt_* call per reference constructor).
//
// Scene content that the reference draws from math/rand (main.go:38-75, 107,
// 155; perlin tables perlin.go:20-31) is drawn from the tree's seeded stream
// (rt_tree_seed) in the same order, so a scene is a pure function of its seed.
//
// main.go:371-409 (modelExample) needs dragon.obj, which the reference does not
// ship (.gitignore:5).  "model" loads <asset_dir>/dragon.obj through the OBJ
// loader (host_obj.cpp) when it is there; otherwise it substitutes a
// procedurally generated (2,3) torus-knot tube with smooth vertex normals
// (~1.05 M triangles), written as OBJ text and passed through the same
// LoadObjWithOptions (scale, centre, position, objLoader.go:146-265) and the same
// scene wrapper.  It is labelled as a substitute everywhere it is reported.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "rt_internal.h"

using rt::set_error;

namespace {

struct V {
  double x, y, z;
};

#define CHECK(expr)            \
  do {                         \
    int _rc = (expr);          \
    if (_rc < 0) return _rc;   \
  } while (0)

int solid_lambert(rt_tree* t, double r, double g, double b) {  // NewLambertian :35
  int tex = rt_tex_solid(t, r, g, b);
  if (tex < 0) return tex;
  return rt_mat_lambertian(t, tex);
}
int solid_light(rt_tree* t, double r, double g, double b) {  // NewDiffuseLight :136
  int tex = rt_tex_solid(t, r, g, b);
  if (tex < 0) return tex;
  return rt_mat_diffuse_light(t, tex);
}
int sphere(rt_tree* t, V c, double r, int mat) {
  double cc[3] = {c.x, c.y, c.z};
  return rt_new_sphere(t, cc, r, mat);
}
int quad(rt_tree* t, V Q, V u, V v, int mat) {
  double q[3] = {Q.x, Q.y, Q.z}, a[3] = {u.x, u.y, u.z}, b[3] = {v.x, v.y, v.z};
  return rt_new_quad(t, q, a, b, mat);
}
int box(rt_tree* t, V a, V b, int mat) {
  double p[3] = {a.x, a.y, a.z}, q[3] = {b.x, b.y, b.z};
  return rt_new_box(t, p, q, mat);
}
int translate(rt_tree* t, int obj, V off) {
  double o[3] = {off.x, off.y, off.z};
  return rt_translate(t, obj, o);
}
void position(rt_camera* c, V from, V at, V up) {
  c->positioned = 1;
  c->look_from[0] = from.x, c->look_from[1] = from.y, c->look_from[2] = from.z;
  c->look_at[0] = at.x, c->look_at[1] = at.y, c->look_at[2] = at.z;
  c->vup[0] = up.x, c->vup[1] = up.y, c->vup[2] = up.z;
}
void background(rt_camera* c, V b) {
  c->background[0] = b.x, c->background[1] = b.y, c->background[2] = b.z;
}

// binary PPM (P6) decoded from the reference's JPEG by tools/make_assets.py
int load_image_texture(rt_tree* t, const char* asset_dir, const char* name) {
  std::string path = std::string(asset_dir ? asset_dir : "assets") + "/" + name;
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return set_error(RT_ERR_IO, "Could not open %s", path.c_str());  // imageLoader.go:31-33
  char magic[3] = {0};
  int w = 0, h = 0, mx = 0;
  if (fscanf(f, "%2s %d %d %d", magic, &w, &h, &mx) != 4 || strcmp(magic, "P6") || mx != 255 ||
      w <= 0 || h <= 0) {
    fclose(f);
    return set_error(RT_ERR_IO, "Error while decoding %s", path.c_str());
  }
  fgetc(f);
  std::vector<uint8_t> px((size_t)w * h * 3);
  size_t got = fread(px.data(), 1, px.size(), f);
  fclose(f);
  if (got != px.size()) return set_error(RT_ERR_IO, "Error while decoding %s: short read", path.c_str());
  return rt_tex_image(t, px.data(), w, h);
}

// ------------------------------------------------------------- main.go:19-91
int book1(rt_tree* t, const char*, rt_camera* c, int* world_out, int* lights_out) {
  c->aspect_ratio = 16.0 / 9.0;
  c->width = 400;
  c->samples_per_pixel = 100;
  c->max_depth = 50;
  c->vertical_fov = 20;
  position(c, {13, 2, 3}, {0, 0, 0}, {0, 1, 0});
  c->defocus_angle = 0.6;
  c->focus_distance = 10.0;
  background(c, {0.70, 0.80, 1.00});

  int world = rt_new_list(t);
  int lights = rt_new_list(t);
  int glass = rt_mat_dielectric(t, 1.5);
  int even = rt_tex_solid(t, .2, .3, .1), odd = rt_tex_solid(t, .9, .9, .9);
  int checker = rt_tex_checker(t, 0.32, even, odd);
  CHECK(rt_list_add(t, world, sphere(t, {0, -1000, 0}, 1000, rt_mat_lambertian(t, checker))));
  for (int a = -11; a < 11; ++a) {
    for (int b = -11; b < 11; ++b) {
      double mat = rt_tree_rand(t);
      double cx = a + 0.9 * rt_tree_rand(t);
      double cz = b + 0.9 * rt_tree_rand(t);
      V center = {cx, 0.2, cz};
      double dx = center.x - 4, dy = center.y - 0.2, dz = center.z - 0;
      if (sqrt(dx * dx + dy * dy + dz * dz) > 0.9) {
        if (mat < 0.6) {
          // albedo := vec.Random().Multiply(vec.Random())
          double r1 = rt_tree_rand(t), g1 = rt_tree_rand(t), b1 = rt_tree_rand(t);
          double r2 = rt_tree_rand(t), g2 = rt_tree_rand(t), b2 = rt_tree_rand(t);
          int m = solid_lambert(t, r1 * r2, g1 * g2, b1 * b2);
          double up = rt_tree_rand_range(t, 0, 0.5);
          double c1[3] = {center.x, center.y, center.z};
          double c2[3] = {center.x + 0, center.y + up, center.z + 0};
          CHECK(rt_list_add(t, world, rt_new_motion_sphere(t, c1, c2, 0.2, m)));
        } else if (mat < 0.8) {
          // perlin orbs: the material is built but never added (main.go:52-60)
          int variant = mat < .65 ? RT_NOISE_MARBLE : (mat < .7 ? RT_NOISE_TURBULENT : RT_NOISE_PERLIN);
          double scale = (double)rt_tree_randn(t, 10);
          CHECK(rt_mat_lambertian(t, rt_tex_noise(t, scale, variant)));
        } else if (mat < 0.95) {
          double ar = rt_tree_rand_range(t, 0.5, 1.0), ag = rt_tree_rand_range(t, 0.5, 1.0),
                 ab = rt_tree_rand_range(t, 0.5, 1.0);
          double fuzz = rt_tree_rand(t);
          CHECK(rt_list_add(t, world, sphere(t, center, 0.2, rt_mat_metal(t, ar, ag, ab, fuzz))));
        } else {
          CHECK(rt_list_add(t, world, sphere(t, center, 0.2, glass)));
        }
      }
    }
  }
  CHECK(rt_list_add(t, world, sphere(t, {0, 1, 0}, 1.0, glass)));
  CHECK(rt_list_add(t, world, sphere(t, {-4, 1, 0}, 1.0, solid_lambert(t, 0.4, 0.2, 0.1))));
  CHECK(rt_list_add(t, world, sphere(t, {4, 1, 0}, 1.0, rt_mat_metal(t, .7, .6, .5, 0))));
  int sun = sphere(t, {0, 100, 0}, 50, solid_light(t, 5, 5, 5));
  CHECK(rt_list_add(t, world, sun));
  CHECK(rt_list_add(t, lights, sun));
  *world_out = rt_build_bvh(t, world);
  *lights_out = lights;
  return *world_out < 0 ? *world_out : RT_OK;
}

// ------------------------------------------------------------ main.go:94-174
int book2(rt_tree* t, const char* assets, rt_camera* c, int* world_out, int* lights_out) {
  int boxes1 = rt_new_list(t);
  int ground = solid_lambert(t, .48, .83, .53);
  for (int i = 0; i < 20; ++i) {
    for (int j = 0; j < 20; ++j) {
      double w = 100.0;
      double x0 = -1000.0 + i * w, z0 = -1000.0 + j * w, y0 = 0.0;
      double x1 = x0 + w, y1 = rt_tree_rand_range(t, 1, 101), z1 = z0 + w;
      CHECK(rt_list_add(t, boxes1, box(t, {x0, y0, z0}, {x1, y1, z1}, ground)));
    }
  }
  int world = rt_new_list(t);
  CHECK(rt_list_add(t, world, rt_build_bvh(t, boxes1)));
  int lights = rt_new_list(t);
  int light = quad(t, {123, 554, 147}, {300, 0, 0}, {0, 0, 265}, solid_light(t, 7, 7, 7));
  CHECK(rt_list_add(t, world, light));
  CHECK(rt_list_add(t, lights, light));
  double c1[3] = {400, 400, 200}, c2[3] = {430, 400, 200};
  CHECK(rt_list_add(t, world, rt_new_motion_sphere(t, c1, c2, 50, solid_lambert(t, .7, .3, .1))));
  CHECK(rt_list_add(t, world, sphere(t, {260, 150, 45}, 50, rt_mat_dielectric(t, 1.5))));
  CHECK(rt_list_add(t, world, sphere(t, {0, 150, 145}, 50, rt_mat_metal(t, 0.8, 0.8, 0.9, 1.0))));
  int boundary = sphere(t, {360, 150, 145}, 70, rt_mat_dielectric(t, 1.5));
  CHECK(rt_list_add(t, world, boundary));
  CHECK(rt_list_add(t, world, rt_constant_medium(t, boundary, .2, rt_tex_solid(t, 0.2, 0.4, 0.9))));
  int b2 = sphere(t, {0, 0, 0}, 5000, rt_mat_dielectric(t, 1.5));
  CHECK(rt_list_add(t, world, rt_constant_medium(t, b2, .0001, rt_tex_solid(t, 1, 1, 1))));
  int earth = load_image_texture(t, assets, "earthmap.ppm");
  CHECK(earth);
  CHECK(rt_list_add(t, world, sphere(t, {400, 200, 400}, 100, rt_mat_lambertian(t, earth))));
  int marble = rt_tex_noise(t, .2, RT_NOISE_MARBLE);
  CHECK(rt_list_add(t, world, sphere(t, {220, 280, 300}, 80, rt_mat_lambertian(t, marble))));
  int boxes2 = rt_new_list(t);
  int white = solid_lambert(t, .73, .73, .73);
  for (int k = 0; k < 1000; ++k) {
    double x = rt_tree_rand_range(t, 0, 165), y = rt_tree_rand_range(t, 0, 165),
           z = rt_tree_rand_range(t, 0, 165);
    CHECK(rt_list_add(t, boxes2, sphere(t, {x, y, z}, 10, white)));
  }
  CHECK(rt_list_add(t, world, translate(t, rt_rotate_y(t, rt_build_bvh(t, boxes2), 15), {-100, 270, 395})));
  c->aspect_ratio = 1.0;
  c->width = 800;
  c->samples_per_pixel = 100;
  c->max_depth = 40;
  background(c, {0, 0, 0});
  c->vertical_fov = 40;
  position(c, {478, 278, -600}, {278, 278, 0}, {0, 1, 0});
  c->defocus_angle = 0;
  *world_out = world;
  *lights_out = lights;
  return RT_OK;
}

int cornell_walls(rt_tree* t, int world, int* white_out, int* light_mat) {
  int red = solid_lambert(t, .65, .05, .05);
  int white = solid_lambert(t, .73, .73, .73);
  int green = solid_lambert(t, .12, .45, .15);
  *light_mat = solid_light(t, 15, 15, 15);
  CHECK(rt_list_add(t, world, quad(t, {555, 0, 0}, {0, 555, 0}, {0, 0, 555}, green)));
  CHECK(rt_list_add(t, world, quad(t, {0, 0, 0}, {0, 555, 0}, {0, 0, 555}, red)));
  CHECK(rt_list_add(t, world, quad(t, {0, 0, 0}, {555, 0, 0}, {0, 0, 555}, white)));
  CHECK(rt_list_add(t, world, quad(t, {555, 555, 555}, {-555, 0, 0}, {0, 0, -555}, white)));
  CHECK(rt_list_add(t, world, quad(t, {0, 0, 555}, {555, 0, 0}, {0, 555, 0}, white)));
  *white_out = white;
  return RT_OK;
}

void cornell_camera(rt_camera* c, int width, int spp) {
  c->aspect_ratio = 1.0;
  c->width = width;
  c->samples_per_pixel = spp;
  c->max_depth = 50;
  background(c, {0, 0, 0});
  c->vertical_fov = 40;
  position(c, {278, 278, -800}, {278, 278, 0}, {0, 1, 0});
  c->defocus_angle = 0;
}

// ------------------------------------------------------------ main.go:177-218
int book3(rt_tree* t, const char*, rt_camera* c, int* world_out, int* lights_out) {
  int world = rt_new_list(t), white, lm;
  CHECK(cornell_walls(t, world, &white, &lm));
  int lights = rt_new_list(t);
  CHECK(rt_list_add(t, lights, quad(t, {343, 550, 332}, {-130, 0, 0}, {0, 0, -105}, lm)));
  CHECK(rt_list_add(t, world, lights));
  int b1 = box(t, {0, 0, 0}, {165, 330, 165}, white);
  b1 = translate(t, rt_rotate_y(t, b1, 15), {265, 0, 295});
  CHECK(rt_list_add(t, world, b1));
  int s = sphere(t, {190, 90, 190}, 90, rt_mat_dielectric(t, 1.5));
  CHECK(rt_list_add(t, lights, s));
  CHECK(rt_list_add(t, world, s));
  cornell_camera(c, 600, 10);
  *world_out = rt_build_bvh(t, world);
  *lights_out = lights;
  return *world_out < 0 ? *world_out : RT_OK;
}

// ------------------------------------------------------------ main.go:220-247
int quads(rt_tree* t, const char* assets, rt_camera* c, int* world_out, int* lights_out) {
  int world = rt_new_list(t);
  int lights = rt_new_list(t);
  int earth = load_image_texture(t, assets, "earthmap.ppm");
  CHECK(earth);
  int left_earth = rt_mat_lambertian(t, earth);
  int back_light = solid_light(t, 3, 3, 3);
  int right_perlin = rt_mat_lambertian(t, rt_tex_noise(t, 5, RT_NOISE_MARBLE));
  int upper_metal = rt_mat_metal(t, 0.8, 0.6, 0.2, 0);
  int lower_teal = solid_lambert(t, 0.2, 0.8, 0.8);
  CHECK(rt_list_add(t, world, quad(t, {-3, -2, 5}, {0, 0, -4}, {0, 4, 0}, left_earth)));
  int light = quad(t, {-2, -2, 0}, {4, 0, 0}, {0, 4, 0}, back_light);
  CHECK(rt_list_add(t, world, light));
  CHECK(rt_list_add(t, world, quad(t, {3, -2, 1}, {0, 0, 4}, {0, 4, 0}, right_perlin)));
  CHECK(rt_list_add(t, world, quad(t, {-2, 3, 1}, {4, 0, 0}, {0, 0, 4}, upper_metal)));
  CHECK(rt_list_add(t, world, quad(t, {-2, -3, 5}, {4, 0, 0}, {0, 0, -4}, lower_teal)));
  int bvh = rt_build_bvh(t, world);
  CHECK(rt_list_add(t, lights, light));
  c->aspect_ratio = 1.0;
  c->width = 400;
  c->samples_per_pixel = 100;
  c->max_depth = 50;
  background(c, {0.70, 0.80, 1.00});
  c->vertical_fov = 80;
  position(c, {0, 0, 9}, {0, 0, 0}, {0, 1, 0});
  c->defocus_angle = 0;
  *world_out = bvh;
  *lights_out = lights;
  return bvh < 0 ? bvh : RT_OK;
}

// ------------------------------------------------------------ main.go:249-275
int simple_light(rt_tree* t, const char*, rt_camera* c, int* world_out, int* lights_out) {
  int world = rt_new_list(t);
  int p = rt_tex_noise(t, 4, RT_NOISE_MARBLE);
  int l = solid_light(t, 4, 4, 4);
  int s1 = sphere(t, {0, -1000, 0}, 1000, rt_mat_lambertian(t, p));
  int s2 = sphere(t, {0, 2, 0}, 2, rt_mat_lambertian(t, p));
  int q = quad(t, {3, 1, -2}, {2, 0, 0}, {0, 2, 0}, l);
  int s = sphere(t, {0, 7, 0}, 2, l);
  CHECK(rt_list_add(t, world, s1));
  CHECK(rt_list_add(t, world, s));
  CHECK(rt_list_add(t, world, q));
  CHECK(rt_list_add(t, world, s2));
  c->aspect_ratio = 16.0 / 9.0;
  c->width = 400;
  c->samples_per_pixel = 100;
  c->max_depth = 50;
  background(c, {0, 0, 0});
  c->vertical_fov = 20;
  position(c, {26, 3, 6}, {0, 2, 0}, {0, 1, 0});
  c->defocus_angle = 0;
  *world_out = world;
  *lights_out = q;  // Render(world, q): a bare quad as the lights Hittable
  return RT_OK;
}

// ------------------------------------------------------------ main.go:278-320
int cornell(rt_tree* t, const char*, rt_camera* c, int* world_out, int* lights_out) {
  int world = rt_new_list(t), white, lm;
  CHECK(cornell_walls(t, world, &white, &lm));
  int lights = rt_new_list(t);
  CHECK(rt_list_add(t, lights, quad(t, {343, 550, 332}, {-130, 0, 0}, {0, 0, -105}, lm)));
  CHECK(rt_list_add(t, world, lights));
  int b1 = box(t, {0, 0, 0}, {165, 330, 165}, white);
  b1 = translate(t, rt_rotate_y(t, b1, 15), {265, 0, 295});
  int b2 = box(t, {0, 0, 0}, {165, 165, 165}, white);
  b2 = translate(t, rt_rotate_y(t, b2, -18), {130, 0, 65});
  CHECK(rt_list_add(t, world, b1));
  CHECK(rt_list_add(t, world, b2));
  cornell_camera(c, 600, 100);
  *world_out = rt_build_bvh(t, world);
  *lights_out = lights;
  return *world_out < 0 ? *world_out : RT_OK;
}

// ------------------------------------------------------------ main.go:323-367
int cornell_smoke(rt_tree* t, const char*, rt_camera* c, int* world_out, int* lights_out) {
  int world = rt_new_list(t);
  int lights = rt_new_list(t);
  int red = solid_lambert(t, .65, .05, .05);
  int white = solid_lambert(t, .73, .73, .73);
  int green = solid_lambert(t, .12, .45, .15);
  int lm = solid_light(t, 15, 15, 15);
  CHECK(rt_list_add(t, world, quad(t, {555, 0, 0}, {0, 555, 0}, {0, 0, 555}, green)));
  CHECK(rt_list_add(t, world, quad(t, {0, 0, 0}, {0, 555, 0}, {0, 0, 555}, red)));
  int lq = quad(t, {343, 550, 332}, {-130, 0, 0}, {0, 0, -105}, lm);
  CHECK(rt_list_add(t, world, lq));
  CHECK(rt_list_add(t, lights, lq));
  CHECK(rt_list_add(t, world, quad(t, {0, 0, 0}, {555, 0, 0}, {0, 0, 555}, white)));
  CHECK(rt_list_add(t, world, quad(t, {555, 555, 555}, {-555, 0, 0}, {0, 0, -555}, white)));
  CHECK(rt_list_add(t, world, quad(t, {0, 0, 555}, {555, 0, 0}, {0, 555, 0}, white)));
  int b1 = box(t, {0, 0, 0}, {165, 330, 165}, white);
  b1 = translate(t, rt_rotate_y(t, b1, 15), {265, 0, 295});
  int b2 = box(t, {0, 0, 0}, {165, 165, 165}, white);
  b2 = translate(t, rt_rotate_y(t, b2, -18), {130, 0, 65});
  CHECK(rt_list_add(t, world, rt_constant_medium(t, b1, .01, rt_tex_solid(t, 0, 0, 0))));
  CHECK(rt_list_add(t, world, rt_constant_medium(t, b2, .01, rt_tex_solid(t, 1, 1, 1))));
  cornell_camera(c, 600, 10);
  *world_out = rt_build_bvh(t, world);
  *lights_out = lights;
  return *world_out < 0 ? *world_out : RT_OK;
}

// ------------------------------------------------------------ main.go:371-409
// Substitute mesh: (2,3) torus-knot tube in "OBJ units", nu x nv quads -> 2 tris.
void knot_point(double s, double* p) {
  const double P = 2, Q = 3;
  double r = 2.0 + cos(Q * s);
  p[0] = r * cos(P * s) * 0.18;
  p[1] = -sin(Q * s) * 0.31;
  p[2] = r * sin(P * s) * 0.18;
}

// The substitute as OBJ text ("OBJ units", before LoadObjWithOptions' scale),
// 9 significant digits like a typical exported mesh:
// nu*nv vertices with vertex normals and one quad face per grid cell, which the
// loader fans into the triangles (a,b,c), (a,c,d) (objLoader.go:396-397).
std::string substitute_dragon_obj(int nu, int nv) {
  // tube radius / frame by finite differences + parallel transport
  const double a = 0.055;
  std::string out;
  out.reserve((size_t)nu * nv * 190);
  out += "# go_raytracer_amd substitute for dragon.obj: (2,3) torus-knot tube\n";
  std::vector<double> norms((size_t)nu * nv * 3);
  char line[256];
  double prev_n[3] = {0, 1, 0};
  for (int i = 0; i < nu; ++i) {
    double s = 2 * M_PI * i / nu, ds = 1e-4;
    double c0[3], c1[3];
    knot_point(s, c0);
    knot_point(s + ds, c1);
    double T[3] = {c1[0] - c0[0], c1[1] - c0[1], c1[2] - c0[2]};
    double tl = sqrt(T[0] * T[0] + T[1] * T[1] + T[2] * T[2]);
    for (double& x : T) x /= tl;
    // N = normalize(prev_n - (prev_n.T) T), B = T x N
    double d = prev_n[0] * T[0] + prev_n[1] * T[1] + prev_n[2] * T[2];
    double N[3] = {prev_n[0] - d * T[0], prev_n[1] - d * T[1], prev_n[2] - d * T[2]};
    double nl = sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
    for (double& x : N) x /= nl;
    double B[3] = {T[1] * N[2] - T[2] * N[1], T[2] * N[0] - T[0] * N[2], T[0] * N[1] - T[1] * N[0]};
    memcpy(prev_n, N, sizeof N);
    // a "scaly" radius modulation gives the surface dragon-like detail
    for (int j = 0; j < nv; ++j) {
      double phi = 2 * M_PI * j / nv;
      double rr = a * (1.0 + 0.18 * sin(7 * phi) * sin(23 * s));
      double dir[3];
      for (int k = 0; k < 3; ++k) dir[k] = cos(phi) * N[k] + sin(phi) * B[k];
      snprintf(line, sizeof line, "v %.9g %.9g %.9g\n", c0[0] + rr * dir[0],
               c0[1] + rr * dir[1], c0[2] + rr * dir[2]);
      out += line;
      memcpy(&norms[3 * ((size_t)i * nv + j)], dir, sizeof dir);
    }
  }
  for (size_t v = 0; v < norms.size(); v += 3) {
    snprintf(line, sizeof line, "vn %.9g %.9g %.9g\n", norms[v], norms[v + 1], norms[v + 2]);
    out += line;
  }
  auto id = [&](int i, int j) { return (long)(i % nu) * nv + (j % nv) + 1; };
  for (int i = 0; i < nu; ++i)
    for (int j = 0; j < nv; ++j) {
      long q[4] = {id(i, j), id(i + 1, j), id(i + 1, j + 1), id(i, j + 1)};
      snprintf(line, sizeof line, "f %ld//%ld %ld//%ld %ld//%ld %ld//%ld\n", q[0], q[0], q[1], q[1],
               q[2], q[2], q[3], q[3]);
      out += line;
    }
  return out;
}

// modelExample main.go:371-409: LoadObjWithOptions("dragon.obj") with ScaleFactor 5,
// Center, Position (0, 1.8, 0), a gold Metal default material; the real file is
// used when asset_dir holds dragon.obj, otherwise the substitute mesh goes
// through the same loader from memory.
int model(rt_tree* t, const char* asset_dir, rt_camera* c, int* world_out, int* lights_out,
          int nu, int nv) {
  int world = rt_new_list(t);
  int ground = sphere(t, {0, -1000, 0}, 1000, solid_lambert(t, .4, .4, .4));
  CHECK(rt_list_add(t, world, ground));
  rt_obj_options opt;
  rt_obj_default_options(&opt);
  opt.scale_factor = 5;
  opt.center = 1;
  opt.position[0] = 0, opt.position[1] = 1.8, opt.position[2] = 0;
  opt.debug = 0;  // the reference prints its loader diagnostics (Debug = true); silent here
  opt.default_material = rt_mat_metal(t, 255.0 / 255.0, 215.0 / 255.0, 0, 0.5);
  CHECK(opt.default_material);
  int mdl = -1, lights = -1;
  std::string path = std::string(asset_dir ? asset_dir : "assets") + "/dragon.obj";
  FILE* f = nu < 0 ? fopen(path.c_str(), "rb") : nullptr;
  if (f) {
    fclose(f);
    CHECK(rt_load_obj(t, path.c_str(), &opt, &mdl, &lights, nullptr));
  } else {
    const bool timing = rt::tune_int("RT_TIMING", 0) != 0;
    auto t0 = std::chrono::steady_clock::now();
    std::string obj = substitute_dragon_obj(nu < 0 ? 2048 : nu, nv < 0 ? 256 : nv);
    auto t1 = std::chrono::steady_clock::now();
    CHECK(rt_load_obj_memory(t, obj.data(), obj.size(), nullptr, 0, "dragon.obj", &opt, &mdl,
                             &lights, nullptr));
    if (timing)
      fprintf(stderr, "[rt] substitute OBJ text %.3f s (%zu bytes), LoadObj %.3f s\n",
              std::chrono::duration<double>(t1 - t0).count(), obj.size(),
              std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
  }
  CHECK(rt_list_add(t, world, rt_rotate_y(t, mdl, 180)));
  // the sun joins the model's light list (main.go:385-391)
  int light = sphere(t, {7, 13, 7}, 5, solid_light(t, 4, 4, 4));
  CHECK(rt_list_add(t, world, light));
  CHECK(rt_list_add(t, lights, light));
  c->aspect_ratio = 16.0 / 9.0;
  c->width = 600;
  c->samples_per_pixel = 250;
  c->max_depth = 50;
  background(c, {0, 0, 0});
  c->vertical_fov = 40;
  c->max_contribution = 2.0;
  position(c, {10, 5, 10}, {0, 0, 0}, {0, 1, 0});
  c->defocus_angle = .1;
  *world_out = world;
  *lights_out = lights;
  return RT_OK;
}

const char* kNames[] = {nullptr, "book1", "book2", "book3", "simple_light",
                        "quads", "cornell", "cornell_smoke", "model"};

}  // namespace

extern "C" {

int64_t rt_substitute_mesh_obj(int nu, int nv, char* out, int64_t cap) {
  const std::string obj = substitute_dragon_obj(nu > 0 ? nu : 2048, nv > 0 ? nv : 256);
  if (out) {
    if (cap < (int64_t)obj.size())
      return set_error(RT_ERR_INVALID, "rt_substitute_mesh_obj: buffer of %lld < %zu bytes",
                       (long long)cap, obj.size());
    memcpy(out, obj.data(), obj.size());
  }
  return (int64_t)obj.size();
}

int rt_demo_scene_name(int s, const char** name_out) {
  if (!name_out) return set_error(RT_ERR_INVALID, "rt_demo_scene_name: null");
  if (s < 1 || s > 8) return set_error(RT_ERR_INVALID, "no scene %d (main.go:449-476)", s);
  *name_out = kNames[s];
  return RT_OK;
}

int rt_demo_scene(rt_tree* t, const char* name, const char* asset_dir, rt_camera* cam, int* world,
                  int* lights) {
  if (!t || !name || !cam || !world || !lights)
    return set_error(RT_ERR_INVALID, "rt_demo_scene: null argument");
  memset(cam, 0, sizeof *cam);
  std::string n(name);
  if (n == "book1") return book1(t, asset_dir, cam, world, lights);
  if (n == "book2") return book2(t, asset_dir, cam, world, lights);
  if (n == "book3") return book3(t, asset_dir, cam, world, lights);
  if (n == "simple_light") return simple_light(t, asset_dir, cam, world, lights);
  if (n == "quads") return quads(t, asset_dir, cam, world, lights);
  if (n == "cornell") return cornell(t, asset_dir, cam, world, lights);
  if (n == "cornell_smoke") return cornell_smoke(t, asset_dir, cam, world, lights);
  if (n == "model") return model(t, asset_dir, cam, world, lights, -1, -1);
  int nu = 0, nv = 0;
  if (sscanf(name, "model:%dx%d", &nu, &nv) == 2 && nu >= 3 && nv >= 3)
    return model(t, asset_dir, cam, world, lights, nu, nv);
  return set_error(RT_ERR_INVALID, "unknown scene '%s'", name);
}

}  // extern "C"
