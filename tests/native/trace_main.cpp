// Host build of the trace core's per-ray arithmetic (csrc/ort_core.h: the same functions
// the HIP kernels call) behind a small driver, for tests/test_host_core.py: the golden
// lens cases traced on the CPU with g++ (-ffp-contract=off) and compared with the
// reference's outputs and the oracle, plus an AddressSanitizer / UBSan build of the same
// driver. The surface loop restates trace_kernel (csrc/ort_kernels.h) for one ray at a
// time; the Newton surfaces follow the reference's global stop rule
// (newton_raphson.py:137-166) directly, lockstep over the rays of a (field, lambda)
// segment, the way the reference evaluates it. Closed-form surfaces use the exact path
// (ort_core.h); the device-only fast sequences (ort_fastpath.h) are not host code.
//
// stdin (little-endian):
//   int64 head[16] = n_surf, n_cs, n_coef, n_zern, n_lambda, n_mat, final_mat, n_seg,
//                    n_pupil, mode (0: generated from the shared pupil, 1: resident rays),
//                    start_surface, record, has_apod, 0, 0, 0
//   double final_thickness
//   ort_surface[n_surf], ort_cs_op[n_cs], double coef[n_coef], ort_zernike_term[n_zern],
//   double n_tab[n_lambda][n_mat], double alpha_tab[n_lambda][n_mat],
//   ort_surface_optics[n_lambda][n_surf], ort_segment[n_seg], ort_apodization (has_apod),
//   mode 0: double px[n_pupil], py[n_pupil]; mode 1: double rays[8][n_seg * n_pupil]
// stdout: double rays[8][n] (x y z L M N i opd), int32 updates[n_seg][n_surf] (-1: not a
//   Newton surface), int32 status, record: double rec[n_surf][8][n]
#define ORT_HD
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../optiland_pr_amd/csrc/ort_core.h"

using ort::Ray;

template <class T>
static bool read_vec(std::vector<T>& v, size_t n) {
  v.resize(n);
  return n == 0 || fread(v.data(), sizeof(T), n, stdin) == n;
}

struct Lens {
  std::vector<ort_surface> surf;
  std::vector<ort_cs_op> cs;
  std::vector<double> coef;
  std::vector<ort_zernike_term> zern;
  std::vector<double> n_tab, alpha_tab;
  std::vector<ort_surface_optics> optics;
  int n_surf, n_mat, final_mat;
  double final_thickness;
};

static void localize(const Lens& L, const ort_surface& s, Ray& r) {
  r.x = r.x + -s.cs_t[0];
  r.y = r.y + -s.cs_t[1];
  r.z = r.z + -s.cs_t[2];
  for (int c = 0; c < s.n_cs_loc; ++c) ort::apply_cs_op(r, L.cs[s.cs_loc_off + c]);
}

static void globalize(const Lens& L, const ort_surface& s, Ray& r) {
  for (int c = 0; c < s.n_cs_glob; ++c) ort::apply_cs_op(r, L.cs[s.cs_glob_off + c]);
  r.x = r.x + s.cs_t[0];
  r.y = r.y + s.cs_t[1];
  r.z = r.z + s.cs_t[2];
}

static bool is_newton(int g) {
  return g != ORT_GEOM_PLANE && g != ORT_GEOM_STANDARD && g != ORT_GEOM_NURBS;
}

// one reference trace call over rays [0, n) of a segment at wavelength row lam
static int trace_segment(const Lens& L, std::vector<Ray>& rays, int lam, int start,
                         int32_t* updates, double* rec, int64_t rec_stride, int64_t rec_off,
                         int& status) {
  constexpr unsigned KM =
      ort::KM_EVEN | ort::KM_ODD | ort::KM_ZERN | ort::KM_FREE | ort::KM_NURBS;
  const double* coef = L.coef.data();
  const ort_zernike_term* zern = L.zern.data();
  const size_t n = rays.size();
  std::vector<double> t(n);
  for (int si = start; si < L.n_surf; ++si) {
    const ort_surface& s = L.surf[si];
    const ort_surface_optics& o = L.optics[(size_t)lam * L.n_surf + si];
    updates[si] = -1;
    for (auto& r : rays) localize(L, s, r);
    if (s.geometry == ORT_GEOM_PLANE) {
      for (size_t k = 0; k < n; ++k) t[k] = ort::distance_plane(rays[k]);
    } else if (s.geometry == ORT_GEOM_GRID_SAG) {
      return 3;  // the grid sag's own Newton is not restated here
    } else if (s.geometry == ORT_GEOM_NURBS) {  // its per-ray (u, v) solve (ort_nurbs.h)
      for (size_t k = 0; k < n; ++k)
        t[k] = ort::nurbs_distance(ort::nurbs_view(coef + s.coef_off), s.tol, s.max_iter,
                                   rays[k]);
    } else {
      const bool rinf = (s.flags & ORT_SURF_RADIUS_INF) != 0;
      for (size_t k = 0; k < n; ++k) t[k] = ort::distance_conic(rays[k], s.radius, s.conic, rinf);
      if (is_newton(s.geometry)) {
        // newton_raphson.py:137-166: stop when max |f| < tol over the whole call
        int j = 0;
        std::vector<double> f(n), nx(n), ny(n), nz(n);
        for (;; ++j) {
          double fmax = 0.0;
          bool nan = false;
          for (size_t k = 0; k < n; ++k) {
            bool rerr = false;
            f[k] = ort::newton_eval<KM>(s, s.radius, s.conic, coef, zern, ort::ZSeed{nullptr, 0},
                                        rays[k], t[k], true, rerr, nx[k], ny[k], nz[k]);
            if (rerr && (j < s.max_iter)) status |= ORT_STATUS_ZERNIKE_RANGE;
            const double a = fabs(f[k]);
            if (a != a) nan = true;
            else if (a > fmax) fmax = a;
          }
          if (j >= s.max_iter || (!nan && fmax < s.tol)) break;
          for (size_t k = 0; k < n; ++k)
            t[k] = ort::newton_step(rays[k], t[k], f[k], nx[k], ny[k], nz[k]);
        }
        updates[si] = j;
      }
    }
    for (size_t k = 0; k < n; ++k) {
      ort::finish_surface<KM>(rays[k], s, s.radius, s.conic, coef, zern, ort::ZSeed{nullptr, 0},
                              t[k], o.n_pre, o.u, o.alpha_pre);
      globalize(L, s, rays[k]);
    }
    if (rec) {
      for (size_t k = 0; k < n; ++k) {
        double* b = rec + (int64_t)si * 8 * rec_stride + rec_off + (int64_t)k;
        const Ray& r = rays[k];
        b[0] = r.x;
        b[rec_stride] = r.y;
        b[2 * rec_stride] = r.z;
        b[3 * rec_stride] = r.L;
        b[4 * rec_stride] = r.M;
        b[5 * rec_stride] = r.N;
        b[6 * rec_stride] = ort::intensity(r);
        b[7 * rec_stride] = r.opd;
      }
    }
  }
  if (L.final_mat >= 0) {
    const double alpha = L.alpha_tab[(size_t)lam * L.n_mat + L.final_mat];
    for (auto& r : rays) ort::propagate(r, L.final_thickness, alpha);
  }
  return 0;
}

int main() {
  int64_t head[16];
  if (fread(head, sizeof head, 1, stdin) != 1) return 2;
  Lens L;
  L.n_surf = (int)head[0];
  const int64_t n_cs = head[1], n_coef = head[2], n_zern = head[3], n_lambda = head[4];
  L.n_mat = (int)head[5];
  L.final_mat = (int)head[6];
  const int64_t n_seg = head[7], n_pupil = head[8], mode = head[9];
  const int start = (int)head[10];
  const bool record = head[11] != 0, has_apod = head[12] != 0;
  if (L.n_surf < 0 || L.n_surf > ORT_MAX_SURFACES || n_seg < 1 || n_pupil < 0) return 2;
  if (fread(&L.final_thickness, sizeof(double), 1, stdin) != 1) return 2;
  std::vector<ort_segment> seg;
  ort_apodization apod{};
  if (!read_vec(L.surf, L.n_surf) || !read_vec(L.cs, n_cs) || !read_vec(L.coef, n_coef) ||
      !read_vec(L.zern, n_zern) || !read_vec(L.n_tab, n_lambda * L.n_mat) ||
      !read_vec(L.alpha_tab, n_lambda * L.n_mat) || !read_vec(L.optics, n_lambda * L.n_surf) ||
      !read_vec(seg, n_seg))
    return 2;
  if (has_apod && fread(&apod, sizeof apod, 1, stdin) != 1) return 2;
  const int64_t n = n_seg * n_pupil;
  std::vector<double> px, py, in;
  if (mode == 0) {
    if (!read_vec(px, n_pupil) || !read_vec(py, n_pupil)) return 2;
  } else if (!read_vec(in, 8 * n)) {
    return 2;
  }
  std::vector<double> out(8 * n);
  std::vector<int32_t> updates(n_seg * L.n_surf, -1);
  std::vector<double> rec(record ? (size_t)L.n_surf * 8 * n : 0);
  int status = 0;
  for (int64_t g = 0; g < n_seg; ++g) {
    std::vector<Ray> rays(n_pupil);
    for (int64_t p = 0; p < n_pupil; ++p) {
      const int64_t r = g * n_pupil + p;
      if (mode == 0) {
        rays[p] = ort::generate_ray(seg[g], px[p], py[p], has_apod ? &apod : nullptr);
      } else {
        Ray& q = rays[p];
        q.x = in[r];
        q.y = in[n + r];
        q.z = in[2 * n + r];
        q.L = in[3 * n + r];
        q.M = in[4 * n + r];
        q.N = in[5 * n + r];
        q.i = in[6 * n + r];
        q.opd = in[7 * n + r];
        q.att = 0.0;
      }
    }
    const int rc = trace_segment(L, rays, seg[g].lambda_idx, start, &updates[g * L.n_surf],
                                 record ? rec.data() : nullptr, n, g * n_pupil, status);
    if (rc) return rc;
    for (int64_t p = 0; p < n_pupil; ++p) {
      const int64_t r = g * n_pupil + p;
      const Ray& q = rays[p];
      out[r] = q.x;
      out[n + r] = q.y;
      out[2 * n + r] = q.z;
      out[3 * n + r] = q.L;
      out[4 * n + r] = q.M;
      out[5 * n + r] = q.N;
      out[6 * n + r] = ort::intensity(q);
      out[7 * n + r] = q.opd;
    }
  }
  fwrite(out.data(), sizeof(double), out.size(), stdout);
  fwrite(updates.data(), sizeof(int32_t), updates.size(), stdout);
  fwrite(&status, sizeof status, 1, stdout);
  if (record) fwrite(rec.data(), sizeof(double), rec.size(), stdout);
  return 0;
}
