// host_obj.cpp — Wavefront OBJ/MTL loader.
//
// Builds, through the rt_* tree constructors, exactly the objects the reference's
// loader builds:
//   LoadObjWithOptions   internal/objLoader/objLoader.go:72-538
//   LoadMTL              internal/objLoader/mtlLoader.go:53-230
//   ConvertToRaytracerMaterial                          mtlLoader.go:233-326
// i.e. one triangle per fan triangle of every face (objLoader.go:393-468), all of
// them in a list handed to BuildBVH (:489-512), and a second list holding the
// emissive (and, with FindWindows, dielectric) triangles for light sampling
// (:491-510).  Numbers are parsed with Go's strconv grammar (ParseFloat / Atoi),
// lines split like bufio.Scanner + strings.TrimSpace/Fields, and vertex
// arithmetic (scale, flip, centre, position, normal normalisation) is done in
// fp64 in the reference's operation order, so the triangles are bit-identical
// to the Go loader's.  Non-fatal problems print the reference's warnings only
// when options.debug is set; fatal ones (log.Fatalf in Go) return an error code.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "rt_internal.h"

using rt::set_error;

namespace {

using sv = std::string_view;

// ----------------------------------------------------------------- strings
// unicode.IsSpace over UTF-8 (strings.TrimSpace / strings.Fields): returns the
// byte length of the space rune at p, 0 if p does not start one.
inline int space_len(const char* p, const char* e) {
  unsigned char c = (unsigned char)*p;
  if (c < 0x80) return (c == ' ' || (c >= '\t' && c <= '\r')) ? 1 : 0;
  if (c == 0xC2 && p + 1 < e) {
    unsigned char d = (unsigned char)p[1];
    return (d == 0x85 || d == 0xA0) ? 2 : 0;  // U+0085 NEL, U+00A0 NBSP
  }
  if ((c == 0xE1 || c == 0xE2 || c == 0xE3) && p + 2 < e) {
    unsigned char d = (unsigned char)p[1], f = (unsigned char)p[2];
    if (c == 0xE1 && d == 0x9A && f == 0x80) return 3;                     // U+1680
    if (c == 0xE2 && d == 0x80 && (f <= 0x8A || f == 0xA8 || f == 0xA9 || f == 0xAF))
      return 3;                                                            // U+2000-200A, 2028/9, 202F
    if (c == 0xE2 && d == 0x81 && f == 0x9F) return 3;                     // U+205F
    if (c == 0xE3 && d == 0x80 && f == 0x80) return 3;                     // U+3000
  }
  return 0;
}

sv trim_space(sv s) {
  const char* b = s.data();
  const char* e = b + s.size();
  for (int n; b < e && (n = space_len(b, e)) > 0;) b += n;
  // ASCII tail (the common case): strip backwards
  const char* t = e;
  while (t > b && (unsigned char)t[-1] < 0x80 && space_len(t - 1, e)) --t;
  if (t == b || (unsigned char)t[-1] < 0x80) return sv(b, t - b);
  // trailing: scan forward remembering the end of the last non-space rune
  const char* last = b;
  for (const char* p = b; p < e;) {
    int n = space_len(p, e);
    if (n) {
      p += n;
    } else {
      ++p;
      last = p;
    }
  }
  return sv(b, last - b);
}

void fields(sv s, std::vector<sv>& out) {
  out.clear();
  const char* p = s.data();
  const char* e = p + s.size();
  while (p < e) {
    int n;
    while (p < e && (n = space_len(p, e)) > 0) p += n;
    if (p >= e) break;
    const char* b = p;
    while (p < e && space_len(p, e) == 0) ++p;
    out.emplace_back(b, p - b);
  }
}

// the first field of a trimmed, non-empty line (strings.Fields(line)[0])
inline sv first_field(sv s) {
  const char* b = s.data();
  const char* e = b + s.size();
  const char* p = b;
  while (p < e && space_len(p, e) == 0) ++p;
  return sv(b, p - b);
}

void split_slash(sv s, std::vector<sv>& out) {  // strings.Split(s, "/")
  out.clear();
  size_t b = 0;
  for (size_t i = 0; i <= s.size(); ++i)
    if (i == s.size() || s[i] == '/') {
      out.push_back(s.substr(b, i - b));
      b = i + 1;
    }
}

// bufio.Scanner with ScanLines: '\n'-separated, one trailing '\r' dropped; a line
// that does not fit the scanner's 64 KiB buffer stops the scan with ErrTooLong.
struct Lines {
  sv buf;
  size_t pos = 0;
  bool too_long = false;
  explicit Lines(sv b) : buf(b) {}
  bool next(sv& line) {
    if (pos >= buf.size() || too_long) return false;
    size_t nl = buf.find('\n', pos);
    size_t end = nl == sv::npos ? buf.size() : nl;
    if (end - pos >= 65536) {
      too_long = true;
      return false;
    }
    line = buf.substr(pos, end - pos);
    if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
    pos = nl == sv::npos ? buf.size() : nl + 1;
    return true;
  }
};

// ------------------------------------------------------------ Go strconv
char lower(char c) { return (char)(c | 0x20); }

bool ieq_prefix_len(sv s, const char* word, size_t* n) {
  size_t i = 0;
  while (i < s.size() && word[i] && lower(s[i]) == word[i]) ++i;
  *n = i;
  return true;
}

// underscoreOK (strconv/atoi.go)
bool underscore_ok(sv s) {
  char saw = '^';
  size_t i = 0;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) s.remove_prefix(1);
  bool hex = false;
  if (s.size() >= 2 && s[0] == '0' &&
      (lower(s[1]) == 'b' || lower(s[1]) == 'o' || lower(s[1]) == 'x')) {
    i = 2;
    saw = '0';
    hex = lower(s[1]) == 'x';
  }
  for (; i < s.size(); ++i) {
    char c = s[i];
    if ((c >= '0' && c <= '9') || (hex && lower(c) >= 'a' && lower(c) <= 'f')) {
      saw = '0';
      continue;
    }
    if (c == '_') {
      if (saw != '0') return false;
      saw = '_';
      continue;
    }
    if (saw == '_') return false;
    saw = '!';
  }
  return saw != '_';
}

// strconv.ParseFloat(s, 64).  Returns false on error; *out is then what Go
// returns alongside the error (0 for a syntax error, ±Inf for ErrRange).
bool go_parse_float(sv s, double* out) {
  *out = 0;
  if (s.empty()) return false;
  {  // special(): [+-]inf / infinity, or nan (no sign)
    size_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') {
      neg = s[0] == '-';
      i = 1;
    }
    sv r = s.substr(i);
    if (!r.empty() && lower(r[0]) == 'i') {
      size_t n;
      ieq_prefix_len(r, "infinity", &n);
      if (n > 3 && n < 8) n = 3;
      if (n == 3 || n == 8) {
        if (n != r.size()) return false;  // trailing bytes: syntax error
        *out = neg ? -INFINITY : INFINITY;
        return true;
      }
    } else if (i == 0 && !r.empty() && lower(r[0]) == 'n') {
      size_t n;
      ieq_prefix_len(r, "nan", &n);
      if (n == 3) {
        if (s.size() != 3) return false;
        *out = NAN;
        return true;
      }
    }
  }
  // readFloat()
  size_t i = 0;
  if (s[0] == '+' || s[0] == '-') ++i;
  bool hex = false;
  if (i + 2 < s.size() && s[i] == '0' && lower(s[i + 1]) == 'x') {
    hex = true;
    i += 2;
  }
  bool underscores = false, sawdot = false, sawdigits = false;
  for (; i < s.size(); ++i) {
    char c = s[i];
    if (c == '_') {
      underscores = true;
      continue;
    }
    if (c == '.') {
      if (sawdot) break;
      sawdot = true;
      continue;
    }
    if ((c >= '0' && c <= '9') || (hex && lower(c) >= 'a' && lower(c) <= 'f')) {
      sawdigits = true;
      continue;
    }
    break;
  }
  if (!sawdigits) return false;
  const char exp_char = hex ? 'p' : 'e';
  if (i < s.size() && lower(s[i]) == exp_char) {
    ++i;
    if (i >= s.size()) return false;
    if (s[i] == '+' || s[i] == '-') ++i;
    if (i >= s.size() || s[i] < '0' || s[i] > '9') return false;
    for (; i < s.size() && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_'); ++i)
      if (s[i] == '_') underscores = true;
  } else if (hex) {
    return false;  // a hexadecimal mantissa requires a 'p' exponent
  }
  if (underscores && !underscore_ok(s.substr(0, i))) return false;
  if (i != s.size()) return false;
  // the grammar matched.  Clinger's fast path when it is exact: a decimal
  // mantissa M <= 2^53 and |exp10| <= 22 give M * 10^e (or M / 10^-e) with ONE
  // rounding, i.e. the correctly rounded value Go returns; else strtod (also
  // correctly rounded).  Typical OBJ coordinates (<= 15 digits) take the fast path.
  if (!hex && !underscores) {
    static const double kP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                    1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                    1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    size_t k = 0;
    const bool neg = s[0] == '-';
    if (s[0] == '+' || s[0] == '-') ++k;
    uint64_t m = 0;
    int nd = 0, e10 = 0;
    bool ok = true, dot = false;
    for (; k < s.size(); ++k) {
      const char c = s[k];
      if (c == '.') {
        dot = true;
        continue;
      }
      if (c < '0' || c > '9') break;
      if (m == 0 && c == '0') {  // leading zeros carry no digits
        if (dot) --e10;
        continue;
      }
      if (++nd > 16) {
        ok = false;
        break;
      }
      m = m * 10 + (uint64_t)(c - '0');
      if (dot) --e10;
    }
    if (ok && k < s.size()) {  // exponent
      ++k;
      bool eneg = false;
      if (s[k] == '+' || s[k] == '-') eneg = s[k++] == '-';
      int ev = 0;
      for (; k < s.size() && ev < 10000; ++k) ev = ev * 10 + (s[k] - '0');
      if (k < s.size()) ok = false;
      e10 += eneg ? -ev : ev;
    }
    if (ok && m <= (1ull << 53) && e10 >= -22 && e10 <= 22) {
      double v = (double)m;
      v = e10 >= 0 ? v * kP10[e10] : v / kP10[-e10];
      *out = neg ? -v : v;
      return true;
    }
  }
  // strtod needs a NUL-terminated copy without underscores; tokens are short
  char buf[128];
  std::string big;
  char* q = buf;
  if (s.size() >= sizeof buf) {
    big.resize(s.size() + 1);
    q = &big[0];
  }
  size_t nq = 0;
  for (char c : s)
    if (c != '_') q[nq++] = c;
  q[nq] = 0;
  double v = strtod(q, nullptr);
  *out = v;
  return !isinf(v);  // overflow: ErrRange with ±Inf (underflow is not an error)
}

// strconv.Atoi: [+-]digits (base 10, no underscores).  *out is what Go returns:
// 0 on a syntax error, the clamped value on ErrRange.
bool go_atoi(sv s, int64_t* out) {
  *out = 0;
  size_t i = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '+' || s[0] == '-')) {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  unsigned __int128 v = 0;
  bool range = false;
  for (; i < s.size(); ++i) {
    char c = s[i];
    if (c < '0' || c > '9') return false;
    if (!range) {
      v = v * 10 + (unsigned)(c - '0');
      if (v > ((unsigned __int128)1 << 63)) range = true;
    }
  }
  if (range || (!neg && v == ((unsigned __int128)1 << 63))) {
    *out = neg ? INT64_MIN : INT64_MAX;
    return false;
  }
  *out = neg ? -(int64_t)(uint64_t)v : (int64_t)(uint64_t)v;
  return true;
}

// math.Min / math.Max (NaN-propagating, -0 < +0)
double go_min(double x, double y) {
  if (isinf(x) && x < 0) return x;
  if (isinf(y) && y < 0) return y;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0 && x == y) return signbit(x) ? x : y;
  return x < y ? x : y;
}
double go_max(double x, double y) {
  if (isinf(x) && x > 0) return x;
  if (isinf(y) && y > 0) return y;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0 && x == y) return signbit(x) ? y : x;
  return x > y ? x : y;
}

// fixIndex objLoader.go:47-61 (Go int is 64-bit)
int64_t fix_index(int64_t i, int64_t length, bool debug) {
  if (i < 0)
    i = length + i;
  else
    i = i - 1;
  if (i < 0 || i >= length) {
    if (debug)
      printf("Warning: Index %lld out of bounds (0-%lld), clamping\n", (long long)i,
             (long long)(length - 1));
    i = (int64_t)go_max(0, go_min((double)i, (double)(length - 1)));
  }
  return i;
}

bool read_file(const std::string& path, std::string& out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  out.clear();
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
  fclose(f);
  return true;
}

std::string dir_of(const std::string& p) {  // filepath.Dir (enough for Join below)
  size_t s = p.find_last_of('/');
  if (s == std::string::npos) return ".";
  if (s == 0) return "/";
  return p.substr(0, s);
}

std::string join_path(const std::string& dir, const std::string& name) {  // filepath.Join
  if (name.empty()) return dir;
  if (!name.empty() && name[0] == '/') return dir == "/" ? name : dir + name;
  if (dir == ".") return name;
  return dir + "/" + name;
}

// ----------------------------------------------------------------- MTL
struct MtlMaterial {  // mtlLoader.go:18-35
  std::string name;
  double Ka[3] = {0.2, 0.2, 0.2}, Kd[3] = {0.8, 0.8, 0.8}, Ks[3] = {0, 0, 0}, Ke[3] = {0, 0, 0},
         Tf[3] = {0, 0, 0};
  double Ns = 0.0, d = 1.0, Ni = 1.0;
  int64_t illum = 2;
  std::string map_Kd, map_Ka, map_Ks, map_Ns, map_bump;
  int material = -1;
};

struct Loader {
  rt_tree* t;
  rt_obj_options o;
  std::unordered_map<std::string, int> image_tex;  // decoded image textures by map name

  double pf(sv s) {  // `v, _ := strconv.ParseFloat(s, 64)`
    double v;
    go_parse_float(s, &v);
    return v;
  }

  // NewImageTexture(filename) texture.go:66 -> ImageLoader.LoadImage imageLoader.go:29-46
  // (the path is opened as written, relative to the working directory).  Images
  // the caller decoded are looked up by the exact map string first; binary PPM
  // (P6) files are decoded here; anything else is the fatal decode error.
  int image_texture(const std::string& name) {
    auto it = image_tex.find(name);
    if (it != image_tex.end()) return it->second;
    for (int k = 0; k < o.n_images; ++k)
      if (o.images[k].name && name == o.images[k].name) {
        int id = rt_tex_image(t, o.images[k].rgb, o.images[k].w, o.images[k].h);
        if (id >= 0) image_tex[name] = id;
        return id;
      }
    std::string data;
    if (!read_file(name, data)) return set_error(RT_ERR_IO, "Could not open %s", name.c_str());
    int w = 0, h = 0, mx = 0, off = 0;
    if (sscanf(data.c_str(), "P6 %d %d %d%n", &w, &h, &mx, &off) != 3 || mx != 255 || w <= 0 ||
        h <= 0 || (size_t)off + 1 + (size_t)w * h * 3 > data.size())
      return set_error(RT_ERR_IO,
                       "Error while decoding %s: not a binary PPM (pass other formats decoded "
                       "in rt_obj_options.images)",
                       name.c_str());
    int id = rt_tex_image(t, (const uint8_t*)data.data() + off + 1, w, h);
    if (id >= 0) image_tex[name] = id;
    return id;
  }

  int solid(const double c[3]) { return rt_tex_solid(t, c[0], c[1], c[2]); }

  // ConvertToRaytracerMaterial mtlLoader.go:233-326
  int convert(const MtlMaterial& m) {
    if ((m.d < 0.95 && m.Ni > 1.0) || m.illum == 4 || m.illum == 6 || m.illum == 7) {
      double ri = m.Ni;
      if (ri <= 1.01) ri = 1.5;
      return rt_mat_dielectric(t, ri);
    }
    if (m.d < 0.95) {
      int tex = solid(m.Kd);
      return tex < 0 ? tex : rt_mat_isotropic(t, tex);
    }
    double emissive = m.Ke[0] + m.Ke[1] + m.Ke[2];
    if (emissive > 0.1) {
      int tex;
      if (!m.map_Kd.empty())
        tex = image_texture(m.map_Kd);
      else if (!m.map_Ka.empty())
        tex = image_texture(m.map_Ka);
      else
        tex = solid(m.Ke);
      return tex < 0 ? tex : rt_mat_diffuse_light(t, tex);
    }
    double spec = m.Ks[0] + m.Ks[1] + m.Ks[2];
    double diff = m.Kd[0] + m.Kd[1] + m.Kd[2];
    if (spec > 0.1 && spec > diff * 0.5) {
      double rough;
      if (m.Ns <= 0.0) {
        rough = 1.0;
      } else if (m.Ns >= 1000.0) {
        rough = 0.0;
      } else {
        double b = 1.0 - m.Ns / 1000.0;
        rough = b * b;  // math.Pow(b, 2.0): Go's Pow squares the mantissa exactly like b*b
        rough = go_max(0.0, go_min(1.0, rough));
      }
      double c[3] = {m.Ks[0], m.Ks[1], m.Ks[2]};
      if (spec < 0.2) {
        double blend = 1.0 - (spec / 0.2);
        for (int k = 0; k < 3; ++k) c[k] = (1.0 - blend) * m.Ks[k] + blend * m.Kd[k];
      }
      return rt_mat_metal(t, c[0], c[1], c[2], rough);
    }
    int tex;
    switch (m.illum) {
      case 3: case 4: case 5:
        return rt_mat_metal(t, m.Ks[0], m.Ks[1], m.Ks[2], 0.3);
      default:  // 0, 1, 2 and anything else: diffuse
        if (!m.map_Kd.empty())
          tex = image_texture(m.map_Kd);
        else if (!m.map_Ka.empty())
          tex = image_texture(m.map_Ka);
        else
          tex = solid(m.Kd);
        return tex < 0 ? tex : rt_mat_lambertian(t, tex);
    }
  }

  // LoadMTL mtlLoader.go:53-230.  The scanner's error is not checked there, so a
  // too-long line silently ends the material list.
  int load_mtl(sv text, std::unordered_map<std::string, MtlMaterial>& lib) {
    Lines lines(text);
    sv line;
    std::vector<sv> p;
    MtlMaterial* cur = nullptr;
    auto rgb = [&](double (MtlMaterial::*dst)[3]) {  // `r, _ := strconv.ParseFloat(...)` x3
      if (!cur || p.size() < 4) return;
      for (int k = 0; k < 3; ++k) (cur->*dst)[k] = pf(p[1 + k]);
    };
    auto rest = [&](std::string MtlMaterial::*dst) {  // strings.Join(parts[1:], " ")
      if (!cur || p.size() < 2) return;
      std::string& d = cur->*dst;
      d.clear();
      for (size_t k = 1; k < p.size(); ++k) {
        if (k > 1) d.push_back(' ');
        d.append(p[k]);
      }
    };
    while (lines.next(line)) {
      sv s = trim_space(line);
      if (s.empty() || s[0] == '#') continue;
      fields(s, p);
      if (p.empty()) continue;
      sv k = p[0];
      if (k == "newmtl") {
        if (p.size() < 2) continue;
        std::string name(p[1]);
        MtlMaterial m;
        m.name = name;
        lib[name] = m;  // a redefinition replaces the map entry (mtlLoader.go:99)
        cur = &lib[name];
      } else if (k == "Ka") {
        rgb(&MtlMaterial::Ka);
      } else if (k == "Kd") {
        rgb(&MtlMaterial::Kd);
      } else if (k == "Ks") {
        rgb(&MtlMaterial::Ks);
      } else if (k == "Ke") {
        rgb(&MtlMaterial::Ke);
      } else if (k == "Ns") {
        if (cur && p.size() >= 2) cur->Ns = pf(p[1]);
      } else if (k == "d") {
        if (cur && p.size() >= 2) cur->d = pf(p[1]);
      } else if (k == "Ni") {
        if (cur && p.size() >= 2) cur->Ni = pf(p[1]);
      } else if (k == "Tf") {
        if (!cur || p.size() < 4) continue;
        double r = pf(p[1]), g = pf(p[2]), b = pf(p[3]);
        cur->Tf[0] = r, cur->Tf[1] = g, cur->Tf[2] = b;
        cur->d = (r + g + b) / 3.0;
      } else if (k == "illum") {
        if (!cur || p.size() < 2) continue;
        int64_t v;
        go_atoi(p[1], &v);
        cur->illum = v;
      } else if (k == "map_Kd") {
        rest(&MtlMaterial::map_Kd);
      } else if (k == "map_Ka") {
        rest(&MtlMaterial::map_Ka);
      } else if (k == "map_Ks") {
        rest(&MtlMaterial::map_Ks);
      } else if (k == "map_Ns") {
        rest(&MtlMaterial::map_Ns);
      } else if (k == "map_bump" || k == "bump") {
        rest(&MtlMaterial::map_bump);
      }
    }
    // every material of the library is converted (mtlLoader.go:207-209), used or not
    for (auto& kv : lib) {
      int m = convert(kv.second);
      if (m < 0) return m;
      kv.second.material = m;
    }
    if (o.debug) printf("=== MTL SUMMARY ===\nLoaded %zu materials\n", lib.size());
    return RT_OK;
  }
};

struct Face {
  std::vector<const double*> v, n;
  std::vector<const double*> tc;
};

}  // namespace

extern "C" {

int rt_obj_default_options(rt_obj_options* o) {  // DefaultLoadOptions objLoader.go:32-45
  if (!o) return set_error(RT_ERR_INVALID, "rt_obj_default_options: null");
  memset(o, 0, sizeof *o);
  o->scale_factor = 1.0;
  o->flip_yz = 0;
  o->debug = 1;
  o->ignore_normals = 0;
  o->center = 1;
  o->flip_faces = 0;
  o->default_material = -1;
  o->ignore_mtl = 0;
  o->find_windows = 0;
  return RT_OK;
}

int rt_load_obj_memory(rt_tree* t, const char* obj_text, size_t obj_len, const char* mtl_text,
                       size_t mtl_len, const char* filename, const rt_obj_options* opts,
                       int* model_out, int* lights_out, rt_obj_info* info) {
  if (!t || (!obj_text && obj_len) || !model_out || !lights_out)
    return set_error(RT_ERR_INVALID, "rt_load_obj: null argument");
  Loader L{t, {}, {}};
  if (opts)
    L.o = *opts;
  else
    rt_obj_default_options(&L.o);
  const rt_obj_options& o = L.o;
  const bool debug = o.debug != 0;
  std::string fname = filename ? filename : "";
  sv text(obj_text ? obj_text : "", obj_len);

  int default_mat = o.default_material;
  if (default_mat < 0) {  // objLoader.go:88-90
    int tex = rt_tex_solid(t, 0.8, 0.8, 0.8);
    if (tex < 0) return tex;
    default_mat = rt_mat_lambertian(t, tex);
    if (default_mat < 0) return default_mat;
  }

  // mtllib scan + LoadMTL (objLoader.go:104-142)
  std::unordered_map<std::string, MtlMaterial> lib;
  bool have_lib = false;
  std::vector<sv> p;
  sv line;
  if (!o.ignore_mtl) {
    std::string mtl_name;
    Lines lines(text);
    while (lines.next(line)) {
      sv s = trim_space(line);
      if (s.empty() || s[0] == '#') continue;
      if (first_field(s) != "mtllib") continue;
      fields(s, p);
      if (p.empty()) continue;
      if (p[0] == "mtllib" && p.size() >= 2) {
        for (size_t k = 1; k < p.size(); ++k) {
          if (k > 1) mtl_name.push_back(' ');
          mtl_name.append(p[k]);
        }
        break;
      }
    }
    if (!mtl_name.empty()) {
      std::string mtl_path = join_path(dir_of(fname.empty() ? "." : fname), mtl_name);
      std::string data;
      bool ok = true;
      if (mtl_text) {
        data.assign(mtl_text, mtl_len);
      } else if (!read_file(mtl_path, data)) {
        ok = false;
        if (debug)
          printf("Warning: Could not load MTL file: could not open MTL file %s\n",
                 mtl_path.c_str());
      }
      if (ok) {
        if (debug) printf("Loading MTL file: %s\n", mtl_path.c_str());
        int rc = L.load_mtl(data, lib);
        if (rc < 0) return rc;
        have_lib = true;
      }
    }
  }

  // pass 1: texture coordinates and vertices, bounds (objLoader.go:144-208)
  std::vector<double> raw;  // 3 per vertex
  std::vector<double> tcs;  // 2 per texcoord
  const double kMax = 1.7976931348623157e308;  // math.MaxFloat64 (objLoader.go:98-99)
  double mn[3] = {kMax, kMax, kMax}, mx[3] = {-kMax, -kMax, -kMax};
  {
    Lines lines(text);
    while (lines.next(line)) {
      sv s = trim_space(line);
      if (s.empty() || s[0] == '#') continue;
      const sv head = first_field(s);
      if (head != "v" && head != "vt") continue;  // the only keys this pass reads
      fields(s, p);
      if (p.empty()) continue;
      if (p[0] == "vt") {
        if (p.size() < 3) continue;
        double u, v;
        bool okU = go_parse_float(p[1], &u), okV = go_parse_float(p[2], &v);
        if (!okU || !okV) continue;
        tcs.push_back(u);
        tcs.push_back(v);
      }
      if (p[0] == "v") {
        if (p.size() < 4) continue;
        double x, y, z;
        bool okX = go_parse_float(p[1], &x), okY = go_parse_float(p[2], &y),
             okZ = go_parse_float(p[3], &z);
        if (!okX || !okY || !okZ) continue;
        x *= o.scale_factor;
        y *= o.scale_factor;
        z *= o.scale_factor;
        if (o.flip_yz) std::swap(y, z);
        raw.push_back(x), raw.push_back(y), raw.push_back(z);
        mn[0] = go_min(mn[0], x), mn[1] = go_min(mn[1], y), mn[2] = go_min(mn[2], z);
        mx[0] = go_max(mx[0], x), mx[1] = go_max(mx[1], y), mx[2] = go_max(mx[2], z);
      }
    }
  }
  const double center[3] = {(mn[0] + mx[0]) / 2, (mn[1] + mx[1]) / 2, (mn[2] + mx[2]) / 2};
  if (debug) {
    printf("=== OBJ MODEL DIMENSIONS ===\n");
    printf("Min bounds: [%f, %f, %f]\n", mn[0], mn[1], mn[2]);
    printf("Max bounds: [%f, %f, %f]\n", mx[0], mx[1], mx[2]);
    printf("Center: [%f, %f, %f]\n", center[0], center[1], center[2]);
  }
  // centring + position (objLoader.go:238-251): v + (-center), then + Position
  std::vector<double> verts(raw);
  if (o.center)
    for (size_t i = 0; i < verts.size(); i += 3)
      for (int k = 0; k < 3; ++k) {
        verts[i + k] += -center[k];
        verts[i + k] += o.position[k];
      }
  const int64_t nverts = (int64_t)(verts.size() / 3), ntcs = (int64_t)(tcs.size() / 2);

  // pass 2: normals, materials, faces (objLoader.go:285-470)
  std::vector<double> normals;  // 3 per normal, grows while faces are read
  normals.reserve(verts.size());
  std::vector<int32_t> tri_nodes;
  std::vector<int32_t> light_nodes;
  int cur_mat = default_mat;
  int cur_kind = -1;  // material kind of cur_mat, for the light list
  auto mat_kind = [&](int m) { return t->t.materials[m].kind; };
  cur_kind = mat_kind(cur_mat);
  std::vector<sv> idx;
  // face corners as indices (the normals vector may reallocate while reading)
  std::vector<int64_t> fv, ft, fn;
  {
    Lines lines(text);
    while (lines.next(line)) {
      sv s = trim_space(line);
      if (s.empty() || s[0] == '#') continue;
      const sv head = first_field(s);
      if (head != "vn" && head != "f" && head != "usemtl") continue;
      fields(s, p);
      if (p.empty()) continue;
      sv k = p[0];
      if (k == "vn") {
        if (p.size() < 4) continue;
        double nx, ny, nz;
        bool okX = go_parse_float(p[1], &nx), okY = go_parse_float(p[2], &ny),
             okZ = go_parse_float(p[3], &nz);
        if (!okX || !okY || !okZ) continue;
        if (o.flip_yz) std::swap(ny, nz);
        double len = sqrt(nx * nx + ny * ny + nz * nz);
        double n[3] = {nx, ny, nz};
        if (len > 0) {
          double inv = 1.0 / len;  // normal.ScaleInplace(1.0 / length)
          for (double& c : n) c *= inv;
        }
        normals.insert(normals.end(), n, n + 3);
      } else if (k == "usemtl") {
        if (o.ignore_mtl || !have_lib || p.size() < 2) continue;
        auto it = lib.find(std::string(p[1]));
        if (it != lib.end()) {
          cur_mat = it->second.material;
          if (debug) printf("Switched to material: %s\n", it->first.c_str());
        } else {
          if (debug) printf("Material not found: %.*s, using default\n", (int)p[1].size(), p[1].data());
          cur_mat = default_mat;
        }
        cur_kind = mat_kind(cur_mat);
      } else if (k == "f") {
        if (p.size() < 4) continue;
        fv.clear(), ft.clear(), fn.clear();
        const int64_t nnorm = (int64_t)(normals.size() / 3);
        for (size_t i = 1; i < p.size(); ++i) {
          split_slash(p[i], idx);
          if (!idx.empty() && !idx[0].empty()) {
            int64_t id;
            if (!go_atoi(idx[0], &id)) continue;
            int64_t vi = fix_index(id, nverts, debug);
            if (vi >= 0 && vi < nverts)
              fv.push_back(vi);
            else
              continue;
          }
          if (idx.size() > 1 && !idx[1].empty() && ntcs > 0) {
            int64_t id;
            if (go_atoi(idx[1], &id)) {
              int64_t ti = fix_index(id, ntcs, debug);
              if (ti >= 0 && ti < ntcs) ft.push_back(ti);
            }
          }
          if (idx.size() > 2 && !idx[2].empty() && nnorm > 0 && !o.ignore_normals) {
            int64_t id;
            if (go_atoi(idx[2], &id)) {
              int64_t ni = fix_index(id, nnorm, debug);
              if (ni >= 0 && ni < nnorm) fn.push_back(ni);
            }
          }
        }
        const size_t nf = fv.size();
        for (size_t i = 2; i < nf; ++i) {  // fan triangulation
          int64_t a = fv[0], b = fv[i - 1], c = fv[i];
          bool has_tc = ft.size() >= nf && ft.size() > i;
          bool has_n = fn.size() >= nf && fn.size() > i && !o.ignore_normals;
          int64_t ta = 0, tb = 0, tc = 0, na = 0, nb = 0, nc = 0;
          if (has_tc) ta = ft[0], tb = ft[i - 1], tc = ft[i];
          if (has_n) na = fn[0], nb = fn[i - 1], nc = fn[i];
          if (o.flip_faces) {
            std::swap(b, c);
            std::swap(tb, tc);
            std::swap(nb, nc);
          }
          double v9[9], n9[9], uv6[6];
          const int64_t vs[3] = {a, b, c}, ns[3] = {na, nb, nc}, ts[3] = {ta, tb, tc};
          for (int q = 0; q < 3; ++q)
            for (int r = 0; r < 3; ++r) {
              v9[3 * q + r] = verts[3 * vs[q] + r];
              n9[3 * q + r] = has_n ? normals[3 * ns[q] + r] : 0.0;
            }
          for (int q = 0; q < 3; ++q)
            for (int r = 0; r < 2; ++r) uv6[2 * q + r] = has_tc ? tcs[2 * ts[q] + r] : 0.0;
          int id = rt_new_triangle(t, v9, has_n ? n9 : nullptr, has_tc ? uv6 : nullptr, cur_mat);
          if (id < 0) return id;
          tri_nodes.push_back(id);
          // light list (objLoader.go:496-509): emissive, or dielectric with FindWindows
          if (cur_kind == RT_MAT_DIFFUSE_LIGHT || (cur_kind == RT_MAT_DIELECTRIC && o.find_windows))
            light_nodes.push_back(id);
        }
      }
    }
    if (lines.too_long)
      return set_error(RT_ERR_IO, "Error reading file %s: bufio.Scanner: token too long",
                       fname.c_str());
  }
  if (debug)
    printf("=== MODEL SUMMARY ===\nLoaded %lld vertices, %zu normals, %zu triangles\n",
           (long long)nverts, normals.size() / 3, tri_nodes.size());
  if (tri_nodes.empty()) return set_error(RT_ERR_INVALID, "No triangles found in OBJ file");

  int model = rt_new_list(t);
  if (model < 0) return model;
  for (int id : tri_nodes) {
    int rc = rt_list_add(t, model, id);
    if (rc < 0) return rc;
  }
  int lights = rt_new_list(t);
  if (lights < 0) return lights;
  for (int id : light_nodes) {
    int rc = rt_list_add(t, lights, id);
    if (rc < 0) return rc;
  }
  int bvh = rt_build_bvh(t, model);  // objLoader.go:512
  if (bvh < 0) return bvh;
  if (debug) printf("%zu Light sources found\n", light_nodes.size());
  *model_out = bvh;
  *lights_out = lights;
  if (info) {
    memset(info, 0, sizeof *info);
    info->n_vertices = nverts;
    info->n_normals = (int64_t)(normals.size() / 3);
    info->n_texcoords = ntcs;
    info->n_triangles = (int64_t)tri_nodes.size();
    info->n_lights = (int64_t)light_nodes.size();
    info->n_materials = (int32_t)lib.size();
    info->default_material = default_mat;
    for (int k = 0; k < 3; ++k) {
      info->bounds_min[k] = mn[k];
      info->bounds_max[k] = mx[k];
      info->center[k] = center[k];
    }
  }
  return RT_OK;
}

int rt_load_obj(rt_tree* t, const char* filename, const rt_obj_options* opts, int* model_out,
                int* lights_out, rt_obj_info* info) {
  if (!t || !filename) return set_error(RT_ERR_INVALID, "rt_load_obj: null argument");
  if (!opts || opts->debug) printf("Attempting to load %s . . .\n", filename);
  std::string data;
  if (!read_file(filename, data))  // objLoader.go:74-77
    return set_error(RT_ERR_IO, "Could not open file %s", filename);
  return rt_load_obj_memory(t, data.data(), data.size(), nullptr, 0, filename, opts, model_out,
                            lights_out, info);
}

}  // extern "C"
