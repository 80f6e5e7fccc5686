// Host build of the device pupil math (ort_pupil.h) for tests/test_pupil_host.py.
//   pupil_main sincos < doubles            -> (sin, cos) pairs
//   pupil_main pupil  < spec + tables      -> (px, py) pairs
// spec: int64 kind, positive_only, n, n_points, n_rows, n_chunks, then row_start[n_rows],
// row_col[2 n_rows], rng_chunk[4 n_chunks], rng_lane[4 * 256] (uint64 as int64).
#define ORT_HD
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../optiland_pr_amd/csrc/ort_pupil.h"

static std::vector<int64_t> read_i64(size_t n) {
  std::vector<int64_t> v(n);
  if (n && fread(v.data(), sizeof(int64_t), n, stdin) != n) v.clear();
  return v;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "sincos")) {
    double v;
    while (fread(&v, sizeof v, 1, stdin) == 1) {
      double s, c;
      ort::cr_sincos(v, s, c);
      fwrite(&s, sizeof s, 1, stdout);
      fwrite(&c, sizeof c, 1, stdout);
    }
    return 0;
  }
  std::vector<int64_t> h = read_i64(6);
  if (h.size() != 6) return 2;
  std::vector<int64_t> rs = read_i64(h[4]), rc = read_i64(2 * h[4]);
  std::vector<int64_t> ch = read_i64(4 * h[5]), ln = read_i64(h[5] ? 4 * 256 : 0);
  ort_pupil d{};
  d.kind = (int32_t)h[0];
  d.positive_only = (int32_t)h[1];
  d.n = h[2];
  d.n_points = h[3];
  d.n_rows = (int32_t)h[4];
  d.row_start = rs.data();
  d.row_col = rc.data();
  d.rng_chunk = (const uint64_t*)ch.data();
  d.rng_lane = (const uint64_t*)ln.data();
  for (int64_t k = 0; k < d.n_points; ++k) {
    double x, y;
    ort::pupil_point(d, k, x, y);
    fwrite(&x, sizeof x, 1, stdout);
    fwrite(&y, sizeof y, 1, stdout);
  }
  return 0;
}
