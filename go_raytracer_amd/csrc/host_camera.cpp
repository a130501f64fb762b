// host_camera.cpp — Camera.initialize (camera.go:179-253) and the output
// quantizer PrintColor (vec/color.go:11-46).
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "rt_internal.h"

using rt::set_error;

namespace {

struct D3 {
  double x, y, z;
};
inline D3 d3(const double* p) { return {p[0], p[1], p[2]}; }
inline D3 sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline D3 add(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline D3 scale(D3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline D3 cross(D3 a, D3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline D3 unit(D3 a) { return scale(a, 1.0 / sqrt(a.x * a.x + a.y * a.y + a.z * a.z)); }
inline void put(double* o, D3 a) {
  o[0] = a.x;
  o[1] = a.y;
  o[2] = a.z;
}

// linearToGamma + Interval{0,.99999}.Clamp + int(x*256), color.go:11-43
inline uint8_t quant(float v) {
  double x = (double)v;
  if (isnan(x)) x = 0.0;
  x = x <= 0 ? 0.0 : sqrt(x);
  if (x < 0) x = 0;
  if (x > 0.99999) x = 0.99999;
  return (uint8_t)(int)(x * 256);
}

}  // namespace

extern "C" {

int rt_camera_derive(const rt_camera* c, rt_camera_derived* o) {
  if (!c || !o) return set_error(RT_ERR_INVALID, "rt_camera_derive: null");
  memset(o, 0, sizeof *o);
  // defaults, camera.go:181-207
  double aspect = c->aspect_ratio == 0 ? 1.0 : c->aspect_ratio;
  int width = c->width == 0 ? 100 : c->width;
  int spp = c->samples_per_pixel == 0 ? 100 : c->samples_per_pixel;
  int max_depth = c->max_depth == 0 ? 10 : c->max_depth;
  double vfov = c->vertical_fov == 0 ? 90 : c->vertical_fov;
  double focus = c->focus_distance == 0 ? 10 : c->focus_distance;
  double maxc = c->max_contribution == 0 ? 1.5 : c->max_contribution;
  if (width < 0 || spp < 0 || aspect < 0)
    return set_error(RT_ERR_INVALID, "rt_camera_derive: negative size");
  if (max_depth < 0 || max_depth > 254)
    return set_error(RT_ERR_UNSUPPORTED, "rt_camera_derive: max_depth %d outside [1,254]",
                     max_depth);
  int height = std::max(1, (int)((double)width / aspect));  // camera.go:209
  int s = (int)sqrt((double)spp);                              // camera.go:211
  if (s < 1) return set_error(RT_ERR_INVALID, "rt_camera_derive: spp_sqrt < 1");
  if (s > 4095) return set_error(RT_ERR_UNSUPPORTED, "rt_camera_derive: spp too large");
  o->width = width;
  o->height = height;
  o->spp_sqrt = s;
  o->max_depth = max_depth;
  o->pixel_samples_scale = 1.0 / (double)(s * s);
  o->recip_spp_sqrt = 1.0 / (double)s;

  // PositionCamera(nil, nil, nil) defaults, camera.go:65-81
  D3 from = {0, 0, 0}, at = {0, 0, -1}, vup = {0, 1, 0};
  if (c->positioned) {
    from = d3(c->look_from);
    at = d3(c->look_at);
    vup = d3(c->vup);
  }
  D3 center = from;
  double theta = vfov * M_PI / 180.0;  // util.DegressToRadians
  double h = tan(theta / 2);
  double vh = 2.0 * h * focus;
  double vw = vh * ((double)width / (double)height);
  D3 w = unit(sub(from, at));
  D3 u = unit(cross(vup, w));
  D3 v = cross(w, u);
  D3 vpU = scale(u, vw);
  D3 vpV = scale(scale(v, -1.0), vh);
  D3 du = scale(vpU, 1.0 / (double)width);
  D3 dv = scale(vpV, 1.0 / (double)height);
  D3 top_left = sub(sub(sub(center, scale(w, focus)), scale(vpU, 0.5)), scale(vpV, 0.5));
  D3 p00 = add(top_left, scale(add(du, dv), 0.5));
  double dr = focus * tan((c->defocus_angle / 2.0) * M_PI / 180.0);
  put(o->center, center);
  put(o->pixel00, p00);
  put(o->delta_u, du);
  put(o->delta_v, dv);
  put(o->defocus_u, scale(u, dr));
  put(o->defocus_v, scale(v, dr));
  o->defocus_angle = c->defocus_angle;
  o->max_contribution = maxc;
  for (int i = 0; i < 3; ++i) o->background[i] = c->background[i];
  return RT_OK;
}

int rt_quantize(const float* rgb, int64_t n, uint8_t* out) {
  if (n < 0 || (n > 0 && (!rgb || !out))) return set_error(RT_ERR_INVALID, "rt_quantize: null");
  for (int64_t i = 0; i < 3 * n; ++i) out[i] = quant(rgb[i]);
  return RT_OK;
}

int64_t rt_format_ppm(const float* rgb, int w, int h, char* out, int64_t cap) {
  if (w < 0 || h < 0 || (w * (int64_t)h > 0 && !rgb))
    return set_error(RT_ERR_INVALID, "rt_format_ppm: bad args");
  char line[64];
  int64_t pos = 0;
  auto emit = [&](const char* s, int len) {
    if (out && pos + len <= cap) memcpy(out + pos, s, len);
    pos += len;
  };
  int len = snprintf(line, sizeof line, "P3\n%d %d\n255\n", w, h);  // camera.go:160
  emit(line, len);
  for (int64_t i = 0; i < (int64_t)w * h; ++i) {
    len = snprintf(line, sizeof line, "%d %d %d\n", quant(rgb[3 * i]), quant(rgb[3 * i + 1]),
                   quant(rgb[3 * i + 2]));
    emit(line, len);
  }
  if (out && pos > cap) return set_error(RT_ERR_INVALID, "rt_format_ppm: buffer too small");
  return pos;
}

}  // extern "C"
