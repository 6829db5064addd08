// h2s_cube.cpp — the BT.2020->BT.709 lattice and .cube text (host C++).
//
// Replaces the reference's offline generator tools/generate_lut.py:28-119
// (whose output src/luts/rec2020_to_rec709.cube is missing from the mount,
// .MISSING_LARGE_BLOBS:1) and the .cube reader of ffmpeg's lut3d filter that
// lut3d=file=... (src/utils.py:40) invokes.  The generator is restated
// operation for operation in double precision so the text is byte-identical
// (pinned by sha256 in tests/golden/lut_hashes.json).
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "../../include/h2s.h"

namespace {

// tools/generate_lut.py:36-40
const double kM[3][3] = {
    {1.6604910021, -0.5876411388, -0.0728498633},
    {-0.1245504745, 1.1328998971, -0.0083494226},
    {-0.0181507634, -0.1005788980, 1.1187296614},
};

// Python's max(0.0, min(1.0, v)) (tools/generate_lut.py:71-72), including
// which operand wins a tie (-0.0 -> 0.0).
double clamp01_py(double v) {
  double t = v < 1.0 ? v : 1.0;
  return t > 0.0 ? t : 0.0;
}

// tools/generate_lut.py:75-90 _convert
void convert(double r, double g, double b, double out[3]) {
  const double lr = pow(r, 2.4), lg = pow(g, 2.4), lb = pow(b, 2.4);
  double o[3];
  for (int i = 0; i < 3; i++) o[i] = kM[i][0] * lr + kM[i][1] * lg + kM[i][2] * lb;
  const double inv = 1 / 2.4;
  for (int i = 0; i < 3; i++) out[i] = pow(clamp01_py(o[i]), inv);
}

template <class Fn>
void for_each_point(int n, Fn fn) {
  // tools/generate_lut.py:97-109: blue slowest, red fastest
  for (int bi = 0; bi < n; bi++) {
    const double b = bi / (double)(n - 1);
    for (int gi = 0; gi < n; gi++) {
      const double g = gi / (double)(n - 1);
      for (int ri = 0; ri < n; ri++) {
        const double r = ri / (double)(n - 1);
        double o[3];
        convert(r, g, b, o);
        fn(o);
      }
    }
  }
}

}  // namespace

extern "C" {

int64_t h2s_cube_format(int n, char* buf, int64_t cap) {
  if (n < 2 || n > 256) return H2S_E_INVALID_ARG;
  std::string s;
  s.reserve((size_t)n * n * n * 27 + 32);
  char line[96];
  snprintf(line, sizeof line, "LUT_3D_SIZE %d\n", n);
  s += line;
  for_each_point(n, [&](const double* o) {
    snprintf(line, sizeof line, "%.6f %.6f %.6f\n", o[0], o[1], o[2]);
    s += line;
  });
  if (buf && cap > 0) memcpy(buf, s.data(), (size_t)((int64_t)s.size() < cap ? (int64_t)s.size() : cap));
  return (int64_t)s.size();
}

int h2s_cube_generate(int n, float* rgb) {
  if (n < 2 || n > 256 || !rgb) return H2S_E_INVALID_ARG;
  size_t i = 0;
  char txt[32];
  for_each_point(n, [&](const double* o) {
    // round through the "%.6f" text the reference writes, then parse the way
    // lut3d does (decimal -> double -> float)
    for (int c = 0; c < 3; c++) {
      snprintf(txt, sizeof txt, "%.6f", o[c]);
      rgb[i++] = (float)strtod(txt, nullptr);
    }
  });
  return 0;
}

int h2s_cube_parse(const char* text, int64_t len, float* rgb, int64_t cap_floats, int* n_out) {
  if (!text || len < 0 || !n_out) return H2S_E_INVALID_ARG;
  *n_out = 0;
  int n = 0;
  int64_t want = 0, got = 0;
  const char* p = text;
  const char* end = text + len;
  std::string line;
  while (p < end) {
    const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
    const char* le = nl ? nl : end;
    line.assign(p, (size_t)(le - p));
    p = nl ? nl + 1 : end;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    size_t s = line.find_first_not_of(" \t");
    if (s == std::string::npos || line[s] == '#') continue;
    const char* l = line.c_str() + s;
    if (!strncmp(l, "TITLE", 5)) continue;
    if (!strncmp(l, "LUT_3D_SIZE", 11)) {
      n = atoi(l + 11);
      if (n < 2 || n > 256) return H2S_E_PARSE;
      want = (int64_t)n * n * n * 3;
      *n_out = n;
      if (!rgb) return 0;
      if (cap_floats < want) return H2S_E_INVALID_ARG;
      continue;
    }
    if (!strncmp(l, "LUT_1D_SIZE", 11)) return H2S_E_UNSUPPORTED;
    if (!strncmp(l, "DOMAIN_MIN", 10) || !strncmp(l, "DOMAIN_MAX", 10)) {
      const bool mx = l[8] == 'A';
      double v[3];
      if (sscanf(l + 10, "%lf %lf %lf", &v[0], &v[1], &v[2]) != 3) return H2S_E_PARSE;
      for (int c = 0; c < 3; c++)
        if (v[c] != (mx ? 1.0 : 0.0)) return H2S_E_UNSUPPORTED;
      continue;
    }
    if (!n) return H2S_E_PARSE;  // data before the size header
    if (got >= want) return H2S_E_PARSE;
    char* e = nullptr;
    const char* q = l;
    for (int c = 0; c < 3; c++) {
      errno = 0;
      const double v = strtod(q, &e);
      if (e == q) return H2S_E_PARSE;
      rgb[got++] = (float)v;
      q = e;
    }
  }
  if (!n || got != want) return H2S_E_PARSE;
  return 0;
}

}  // extern "C"
