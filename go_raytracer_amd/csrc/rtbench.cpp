// rtbench: the reference's command line (main.go:414-478) over the C ABI.
//
//   rtbench [-o image.ppm] [-N cores] [-S scene] [-cpuprofile file] [extensions]
//
// Same flags, defaults and effects as main.go: -S picks the scene function
// (1 book1 .. 8 model, main.go:447-472; anything else is defaultScene, which
// renders nothing, so the output file is created and left empty), -o names the
// output file (created before the render, main.go:434-439), -N is
// Camera.MaxThreads (the GPU path ignores it; kept in rt_camera.max_threads).
// Flag syntax follows Go's flag package: -name value, -name=value, --name;
// bool flags take no value; parsing stops at "--" or the first non-flag;
// an unknown flag or a bad value prints the usage and exits 2, -h exits 0.
//
// Extensions beyond main.go (defaults leave the reference scene unchanged):
// -device, -width, -spp, -depth (camera overrides), -seed (render seed),
// -tree-seed (the scene's rand seed), -mode auto|fused|wavefront, -assets DIR,
// -progress (a progress line on stderr, the reference's bubbletea bar,
// camera.go:106-108), -slices N (rt_progress granularity), -stats (one JSON
// line of rt_stats on stderr).  -cpuprofile has no pprof to drive on the GPU
// path: the file receives the same JSON statistics instead.
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rt_abi.h"

namespace {

struct Flag {
  const char* name;
  const char* usage;
  enum Kind { STR, INT, U64, BOOL } kind;
  void* dst;
  const char* def;  // shown in the usage, Go style
};

struct Args {
  std::string cpuprofile, out = "image.ppm", mode = "auto", assets;
  long long N = 1, S = -1, device = 0, width = 0, spp = 0, depth = 0, slices = 0;
  unsigned long long seed = 1, tree_seed = 1;
  bool progress = false, stats = false;
};

std::vector<Flag> flags(Args& a) {
  return {
      {"N", "Set the number of cores to allocate to rendering", Flag::INT, &a.N, "1"},
      {"S", "Set the scene to render, default will render a custom scene function", Flag::INT,
       &a.S, "-1"},
      {"assets", "directory holding earthmap.jpg / dragon.obj (default: <exe dir>/../assets)",
       Flag::STR, &a.assets, ""},
      {"cpuprofile", "Write cpu profile to file (here: render statistics as JSON)", Flag::STR,
       &a.cpuprofile, ""},
      {"depth", "override Camera.MaxDepth (0 = the scene's)", Flag::INT, &a.depth, "0"},
      {"device", "HIP device ordinal", Flag::INT, &a.device, "0"},
      {"mode", "kernel strategy: auto, fused or wavefront", Flag::STR, &a.mode, "auto"},
      {"o", "Specify a custom output file", Flag::STR, &a.out, "image.ppm"},
      {"progress", "print render progress on stderr", Flag::BOOL, &a.progress, ""},
      {"seed", "render seed (Philox key)", Flag::U64, &a.seed, "1"},
      {"slices", "progress granularity: launches per render (0 = 20 with -progress)", Flag::INT,
       &a.slices, "0"},
      {"spp", "override Camera.SamplesPerPixel (0 = the scene's)", Flag::INT, &a.spp, "0"},
      {"stats", "print render statistics (JSON) on stderr", Flag::BOOL, &a.stats, ""},
      {"tree-seed", "seed of the scene builder's rand (main.go's math/rand)", Flag::U64,
       &a.tree_seed, "1"},
      {"width", "override Camera.Width (0 = the scene's)", Flag::INT, &a.width, "0"},
  };
}

void usage(const char* prog, const std::vector<Flag>& fl) {
  fprintf(stderr, "Usage of %s:\n", prog);
  for (const Flag& f : fl) {
    const char* ty = f.kind == Flag::STR ? " string" : f.kind == Flag::INT ? " int"
                     : f.kind == Flag::U64 ? " uint" : "";
    fprintf(stderr, "  -%s%s\n    \t%s", f.name, ty, f.usage);
    if (f.def && *f.def && !(f.kind == Flag::INT && !strcmp(f.def, "0")))
      fprintf(stderr, f.kind == Flag::STR ? " (default \"%s\")" : " (default %s)", f.def);
    fprintf(stderr, "\n");
  }
}

// strconv.ParseInt(s, 0, 64) / ParseUint / ParseBool as flag.Value.Set uses them
bool set_value(const Flag& f, const std::string& v) {
  errno = 0;
  char* end = nullptr;
  switch (f.kind) {
    case Flag::STR: *(std::string*)f.dst = v; return true;
    case Flag::INT: {
      long long x = strtoll(v.c_str(), &end, 0);
      if (v.empty() || *end || errno) return false;
      *(long long*)f.dst = x;
      return true;
    }
    case Flag::U64: {
      if (v.empty() || v[0] == '-') return false;
      unsigned long long x = strtoull(v.c_str(), &end, 0);
      if (*end || errno) return false;
      *(unsigned long long*)f.dst = x;
      return true;
    }
    case Flag::BOOL: {
      static const char* t[] = {"1", "t", "T", "true", "TRUE", "True"};
      static const char* n[] = {"0", "f", "F", "false", "FALSE", "False"};
      for (const char* s : t) if (v == s) return *(bool*)f.dst = true, true;
      for (const char* s : n) if (v == s) return *(bool*)f.dst = false, true;
      return false;
    }
  }
  return false;
}

// flag.FlagSet.Parse with ExitOnError: returns the exit code, or -1 to go on
int parse(int argc, char** argv, Args& a) {
  std::vector<Flag> fl = flags(a);
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    if (s.size() < 2 || s[0] != '-') break;  // first non-flag argument
    size_t dashes = s[1] == '-' ? 2 : 1;
    if (dashes == 2 && s.size() == 2) break;  // "--" terminates
    std::string name = s.substr(dashes), val;
    bool has_val = false;
    if (name.empty() || name[0] == '-' || name[0] == '=') {
      fprintf(stderr, "bad flag syntax: %s\n", s.c_str());
      usage(argv[0], fl);
      return 2;
    }
    size_t eq = name.find('=');
    if (eq != std::string::npos) val = name.substr(eq + 1), name = name.substr(0, eq), has_val = true;
    if (name == "h" || name == "help") {
      usage(argv[0], fl);
      return 0;
    }
    const Flag* f = nullptr;
    for (const Flag& c : fl)
      if (name == c.name) f = &c;
    if (!f) {
      fprintf(stderr, "flag provided but not defined: -%s\n", name.c_str());
      usage(argv[0], fl);
      return 2;
    }
    if (f->kind == Flag::BOOL && !has_val) {
      val = "true";
    } else if (!has_val) {
      if (i + 1 >= argc) {
        fprintf(stderr, "flag needs an argument: -%s\n", name.c_str());
        usage(argv[0], fl);
        return 2;
      }
      val = argv[++i];
    }
    if (!set_value(*f, val)) {
      fprintf(stderr, "invalid value \"%s\" for flag -%s: parse error\n", val.c_str(),
              name.c_str());
      usage(argv[0], fl);
      return 2;
    }
  }
  return -1;
}

std::string exe_dir() {
  char buf[4096];
  ssize_t n = readlink("/proc/self/exe", buf, sizeof buf - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p = buf;
  size_t k = p.rfind('/');
  return k == std::string::npos ? "." : p.substr(0, k);
}

int fail(const char* what, int rc) {
  fprintf(stderr, "rtbench: %s failed (%d): %s\n", what, rc, rt_last_error());
  return 1;
}

std::string stats_json(const rt_stats& st, const rt_camera_derived& d, const char* scene,
                       double wall_s) {
  char b[1024];
  snprintf(b, sizeof b,
           "{\"scene\": \"%s\", \"width\": %d, \"height\": %d, \"spp\": %d, \"max_depth\": %d, "
           "\"samples\": %" PRIu64 ", \"segments\": %" PRIu64 ", \"ms_render\": %.3f, "
           "\"samples_per_s\": %.6g, \"mode\": %d, \"tree_width\": %d, \"chunk_samples\": %d, "
           "\"wall_s\": %.3f}",
           scene, d.width, d.height, d.spp_sqrt * d.spp_sqrt, d.max_depth, st.samples,
           st.segments, st.ms_total, st.ms_total > 0 ? st.samples / (st.ms_total * 1e-3) : 0.0,
           st.mode, st.tree_width, st.chunk_samples, wall_s);
  return b;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  int rc = parse(argc, argv, a);
  if (rc >= 0) return rc;
  auto t0 = std::chrono::steady_clock::now();

  // main.go:434-439: the output file exists before anything renders
  FILE* out = fopen(a.out.c_str(), "wb");
  if (!out) {
    fprintf(stderr, "Error creating output file\n");
    return 1;
  }
  const char* scene = nullptr;
  if (a.S < 1 || a.S > 8 || rt_demo_scene_name((int)a.S, &scene) != RT_OK || !scene) {
    fclose(out);  // defaultScene (main.go:412-414): nothing rendered, empty file
    return 0;
  }
  int mode = a.mode == "auto" ? RT_MODE_AUTO : a.mode == "fused" ? RT_MODE_FUSED
             : a.mode == "wavefront" ? RT_MODE_WAVEFRONT : -1;
  if (mode < 0) {
    fprintf(stderr, "invalid value \"%s\" for flag -mode\n", a.mode.c_str());
    fclose(out);
    return 2;
  }
  std::string assets = a.assets.empty() ? exe_dir() + "/../assets" : a.assets;
  if (a.assets.empty() && getenv("RT_ASSET_DIR")) assets = getenv("RT_ASSET_DIR");

  rt_tree* tree = nullptr;
  rt_scene* sc = nullptr;
  if ((rc = rt_tree_create(&tree)) != RT_OK) return fail("rt_tree_create", rc);
  rt_tree_seed(tree, a.tree_seed);
  rt_camera cam;
  memset(&cam, 0, sizeof cam);
  int world = -1, lights = -1;
  if ((rc = rt_demo_scene(tree, scene, assets.c_str(), &cam, &world, &lights)) != RT_OK)
    return fail("rt_demo_scene", rc);
  cam.max_threads = (int32_t)a.N;
  if (a.width > 0) cam.width = (int32_t)a.width;
  if (a.spp > 0) cam.samples_per_pixel = (int32_t)a.spp;
  if (a.depth > 0) cam.max_depth = (int32_t)a.depth;
  rt_camera_derived d;
  if ((rc = rt_camera_derive(&cam, &d)) != RT_OK) return fail("rt_camera_derive", rc);
  if ((rc = rt_scene_create(tree, world, lights, &sc)) != RT_OK)
    return fail("rt_scene_create", rc);

  rt_render_opts o;
  memset(&o, 0, sizeof o);
  o.seed = a.seed;
  o.device = (int32_t)a.device;
  o.nranks = 1;
  o.mode = mode;
  o.trace_pixel = -1;
  o.progress_slices = (int32_t)(a.slices > 0 ? a.slices : a.progress ? 20 : 0);
  std::vector<float> rgb((size_t)d.width * d.height * 3);
  rt_stats st;
  memset(&st, 0, sizeof st);

  std::atomic<bool> rendering{true};
  std::thread bar;
  if (a.progress) {
    bar = std::thread([&] {
      uint64_t done = 0, total = 0;
      while (rendering.load()) {
        if (rt_progress(sc, &done, &total) == RT_OK && total)
          fprintf(stderr, "\rrendering %s: %5.1f%%", scene, 100.0 * done / total);
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
      }
    });
  }
  rc = rt_render(sc, &cam, &o, rgb.data(), &st);
  rendering = false;
  if (bar.joinable()) bar.join();
  if (a.progress) fprintf(stderr, "\rrendering %s: 100.0%%\n", scene);
  if (rc != RT_OK) return fail("rt_render", rc);

  // camera.go:160 header + PrintColor per pixel, then main.go:477's single write
  int64_t n = rt_format_ppm(rgb.data(), d.width, d.height, nullptr, 0);
  std::vector<char> text((size_t)(n > 0 ? n : 0));
  if (n < 0 || rt_format_ppm(rgb.data(), d.width, d.height, text.data(), n) != n)
    return fail("rt_format_ppm", (int)n);
  if (fwrite(text.data(), 1, text.size(), out) != text.size() || fclose(out) != 0) {
    fprintf(stderr, "rtbench: writing %s failed\n", a.out.c_str());
    return 1;
  }
  double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::string js = stats_json(st, d, scene, wall);
  if (a.stats) fprintf(stderr, "%s\n", js.c_str());
  if (!a.cpuprofile.empty()) {
    FILE* p = fopen(a.cpuprofile.c_str(), "w");
    if (!p) {
      fprintf(stderr, "rtbench: cannot create %s\n", a.cpuprofile.c_str());
      return 1;
    }
    fprintf(p, "%s\n", js.c_str());
    fclose(p);
  }
  rt_scene_destroy(sc);
  rt_tree_destroy(tree);
  return 0;
}
