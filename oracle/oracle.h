/*
 * oracle.h — CPU restatement of the reference path tracer.  TEST INFRASTRUCTURE
 * ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * as the checker; never linked into or called by the product library.
 *
 * It restates, function by function, the Go code of nsp5488/go_raytracer
 * (internal/camera/camera.go, internal/hittable/ *.go, internal/vec, aabb,
 * interval, ray, util) in C++ with the same object structure: a recursive
 * rayColor, virtual Hit/PdfValue/Random, the reference's own median-split BVH
 * with duplicated span-1 leaves, Translate/RotateY wrappers applied at hit time.
 *
 * Pinning: the Go toolchain is absent, so the reference cannot
 * be compiled or run here.  The oracle's leaf functions are pinned by the
 * reference's own unit-test vectors (vec_test.go, interval_test.go,
 * ray_test.go, imageLoader_test.go) — see tests/test_oracle_golden.py.  Render
 * outputs have no reference fixture ("render parity unpinned at the reference
 * level"); the random stream is the shared counter RNG of include/rt_rng.h.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#include "rt_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint64_t samples;
  uint64_t segments; /* world.Hit calls that were made (camera.go:300) */
  double seconds;
  int32_t threads;
} oracle_stats;

/* precision: 64 = faithful fp64 restatement, 32 = fp32 twin.
 * out: [rows of rank][W][3] linear mean RGB (pixelColor.Scale, camera.go:103).
 * max_rows > 0 renders only the first max_rows rows of the rank (CPU-baseline
 * sampling). */
int oracle_render(const rt_tree_view* tree, int world, int lights, const rt_camera* cam,
                  uint64_t seed, int precision, int threads, int rank, int nranks, int max_rows,
                  float* out, oracle_stats* stats);

/* One sample of one global pixel, recording every world.Hit call as 12 floats
 * {o.xyz, time, d.xyz, vertex, t, u, v, material kind (-1 = miss)}; returns the
 * number of records (<= cap) or a negative error. */
int oracle_trace(const rt_tree_view* tree, int world, int lights, const rt_camera* cam,
                 uint64_t seed, int precision, int64_t pixel, int sample, float* out, int cap);

/* the reference's unit-level functions, for the golden-vector tests */
enum {
  ORACLE_VEC_ADD = 0, ORACLE_VEC_SUB, ORACLE_VEC_MUL, ORACLE_VEC_DIV, ORACLE_VEC_NEG,
  ORACLE_VEC_DOT, ORACLE_VEC_CROSS, ORACLE_VEC_SCALE, ORACLE_VEC_LEN, ORACLE_VEC_LENSQ,
  ORACLE_VEC_UNIT, ORACLE_VEC_NEARZERO, ORACLE_VEC_REFLECT, ORACLE_VEC_REFRACT
};
int oracle_vec_op(int op, const double* a, const double* b, double s, double* out);
int oracle_print_color(double r, double g, double b, char* out, int cap); /* PrintColor */
int oracle_interval(int op, double mn, double mx, double x, double* out);  /* 0 contains 1 surrounds 2 clamp */
int oracle_ray_at(const double* o, const double* d, double t, double* out);
int oracle_camera(const rt_camera* cam, rt_camera_derived* out); /* initialize() */

#ifdef __cplusplus
}
#endif
#endif
