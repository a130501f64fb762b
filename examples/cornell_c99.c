/* cornell_c99.c — the C side of the cgo shim, as plain C99.
 *
 * cgo compiles its preamble and every call through it as C, not C++, so this is the
 * call sequence a Go caller's shim makes, compiled the same way: the Go scene
 * cornellBox (main.go:278-320) lowered one constructor call per Go constructor
 * (NewLambertian, NewDiffuseLight, NewQuad, NewBox, RotateY, Translate, the lights
 * HittableList, BuildBVH), then (*Camera).Render (camera.go:156) as rt_scene_create +
 * rt_render + rt_format_ppm.
 *
 *   cornell_c99 info                      flatten + BVH only (no GPU): prints scene counts
 *   cornell_c99 render W SPP SEED OUT.f32 render on device 0: linear RGB [H][W][3] fp32
 *   cornell_c99 ppm W SPP SEED OUT.ppm    render and write the P3 stream (camera.go:160)
 *
 * Build: gcc -std=c99 -pedantic -Wall -Wextra -Werror -I include examples/cornell_c99.c \
 *          -L go_raytracer_amd -lrt_amd -Wl,-rpath,<dir of librt_amd.so>   (tests/test_c_client.py)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_abi.h"

/* every rt_* call returns a handle >= 0 or a negative RT_ERR_* code (the Go shim's
 * errors.New(C.GoString(C.rt_last_error()))) */
static int must(int rc, const char* what) {
  if (rc < 0) {
    fprintf(stderr, "%s: %d (%s)\n", what, rc, rt_last_error());
    exit(2);
  }
  return rc;
}

static int lambertian(rt_tree* t, double r, double g, double b) { /* NewLambertian materials.go:35 */
  return must(rt_mat_lambertian(t, must(rt_tex_solid(t, r, g, b), "tex")), "lambertian");
}
static int light(rt_tree* t, double r, double g, double b) { /* NewDiffuseLight materials.go:136 */
  return must(rt_mat_diffuse_light(t, must(rt_tex_solid(t, r, g, b), "tex")), "light");
}
static int quad(rt_tree* t, double qx, double qy, double qz, double ux, double uy, double uz,
                double vx, double vy, double vz, int mat) { /* NewQuad objects.go:129 */
  const double Q[3] = {qx, qy, qz}, u[3] = {ux, uy, uz}, v[3] = {vx, vy, vz};
  return must(rt_new_quad(t, Q, u, v, mat), "quad");
}
static int box(rt_tree* t, double x, double y, double z, int mat) { /* NewBox objects.go:208 */
  const double a[3] = {0, 0, 0}, b[3] = {x, y, z};
  return must(rt_new_box(t, a, b, mat), "box");
}
static int placed(rt_tree* t, int obj, double deg, double x, double y, double z) {
  const double off[3] = {x, y, z}; /* Translate(RotateY(obj, deg), off) transformation.go:20,48 */
  return must(rt_translate(t, must(rt_rotate_y(t, obj, deg), "rotate_y"), off), "translate");
}

/* cornellBox, main.go:278-320 */
static void cornell(rt_tree* t, int* world_out, int* lights_out, rt_camera* c) {
  int world = must(rt_new_list(t), "list");
  int red = lambertian(t, .65, .05, .05), white = lambertian(t, .73, .73, .73);
  int green = lambertian(t, .12, .45, .15), lm = light(t, 15, 15, 15);
  int lights, b1, b2;
  must(rt_list_add(t, world, quad(t, 555, 0, 0, 0, 555, 0, 0, 0, 555, green)), "add");
  must(rt_list_add(t, world, quad(t, 0, 0, 0, 0, 555, 0, 0, 0, 555, red)), "add");
  must(rt_list_add(t, world, quad(t, 0, 0, 0, 555, 0, 0, 0, 0, 555, white)), "add");
  must(rt_list_add(t, world, quad(t, 555, 555, 555, -555, 0, 0, 0, 0, -555, white)), "add");
  must(rt_list_add(t, world, quad(t, 0, 0, 555, 555, 0, 0, 0, 555, 0, white)), "add");
  lights = must(rt_new_list(t), "list");
  must(rt_list_add(t, lights, quad(t, 343, 550, 332, -130, 0, 0, 0, 0, -105, lm)), "add");
  must(rt_list_add(t, world, lights), "add");
  b1 = placed(t, box(t, 165, 330, 165, white), 15, 265, 0, 295);
  b2 = placed(t, box(t, 165, 165, 165, white), -18, 130, 0, 65);
  must(rt_list_add(t, world, b1), "add");
  must(rt_list_add(t, world, b2), "add");
  memset(c, 0, sizeof *c);
  c->aspect_ratio = 1.0;
  c->width = 600;
  c->samples_per_pixel = 100;
  c->max_depth = 50;
  c->vertical_fov = 40;
  c->positioned = 1; /* PositionCamera(lookFrom, lookAt, vup) camera.go:65-81 */
  c->look_from[0] = 278, c->look_from[1] = 278, c->look_from[2] = -800;
  c->look_at[0] = 278, c->look_at[1] = 278, c->look_at[2] = 0;
  c->vup[1] = 1;
  *world_out = must(rt_build_bvh(t, world), "bvh"); /* BuildBVH bvh.go:21 */
  *lights_out = lights;
}

int main(int argc, char** argv) {
  rt_tree* tree = NULL;
  rt_scene* scene = NULL;
  rt_camera cam;
  rt_camera_derived d;
  int world, lights;
  if (argc < 2) {
    fprintf(stderr, "usage: %s info | render W SPP SEED OUT | ppm W SPP SEED OUT\n", argv[0]);
    return 2;
  }
  must(rt_tree_create(&tree), "tree");
  cornell(tree, &world, &lights, &cam);
  must(rt_scene_create(tree, world, lights, &scene), "scene");
  if (strcmp(argv[1], "info") == 0) {
    rt_scene_info in;
    must(rt_scene_info_get(scene, &in), "info");
    printf("{\"abi\": %d, \"n_quads\": %d, \"n_world_prims\": %d, \"n_lights\": %d, "
           "\"n_materials\": %d, \"n_textures\": %d, \"n_bvh_nodes\": %d, \"features\": %d}\n",
           rt_abi_version(), (int)in.n_quads, (int)in.n_world_prims, (int)in.n_lights,
           (int)in.n_materials, (int)in.n_textures, (int)in.n_bvh_nodes, (int)in.features);
  } else if (argc == 6 && (strcmp(argv[1], "render") == 0 || strcmp(argv[1], "ppm") == 0)) {
    rt_render_opts opts;
    rt_stats st;
    float* rgb;
    size_t n;
    FILE* f;
    cam.width = atoi(argv[2]);
    cam.samples_per_pixel = atoi(argv[3]);
    must(rt_camera_derive(&cam, &d), "derive");
    n = (size_t)d.width * (size_t)d.height * 3u;
    rgb = (float*)malloc(n * sizeof(float));
    if (!rgb) return 2;
    memset(&opts, 0, sizeof opts);
    opts.seed = strtoull(argv[4], NULL, 10);
    opts.nranks = 1;
    must(rt_render(scene, &cam, &opts, rgb, &st), "render");
    f = fopen(argv[5], "wb");
    if (!f) return 2;
    if (argv[1][0] == 'r') {
      fwrite(rgb, sizeof(float), n, f);
    } else {
      const int64_t len = rt_format_ppm(rgb, d.width, d.height, NULL, 0);
      char* text = (char*)malloc((size_t)len);
      if (!text || rt_format_ppm(rgb, d.width, d.height, text, len) != len) return 2;
      fwrite(text, 1, (size_t)len, f);
      free(text);
    }
    fclose(f);
    printf("{\"width\": %d, \"height\": %d, \"samples\": %llu, \"segments\": %llu}\n", (int)d.width,
           (int)d.height, (unsigned long long)st.samples, (unsigned long long)st.segments);
    free(rgb);
  } else {
    fprintf(stderr, "bad arguments\n");
    return 2;
  }
  must(rt_scene_destroy(scene), "destroy");
  must(rt_tree_destroy(tree), "destroy");
  return 0;
}
