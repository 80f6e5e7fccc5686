// ort_adjoint.h -- reverse-mode (adjoint) VJP of the fused pupil trace.
//
// The forward-mode VJP (vjp_kernel, ort_kernels.h) re-traces the lens once per chunk of
// P parameter tangents, so its cost grows with the number of parameters. This kernel
// computes the same vector-Jacobian product in one launch whatever the parameter count:
//
//   forward   the primal trace in double (same code, same values as ort_trace_pupil),
//             taping each traced surface's incoming global ray (x, y, z, L, M, N), its
//             intersection distance t and (Newton surfaces) the iterates before the
//             last kHist updates to a workspace in HBM ([S][11][n_rays], coalesced);
//   reverse   from the image back to the first surface, the adjoint of every step of
//             Surface.trace (standard_surface.py:186-233): globalize, refract / reflect
//             with the aligned normal, the normal at the hit point, OPD and absorption,
//             propagation, the intersection distance, localize.
//
// Closed-form intersections (plane, conic) are differentiated through their implicit
// equations (the derivative of the closed form, up to rounding). Newton intersections
// are differentiated like torch autograd does it, through the unrolled updates
// t' = t - f(t) / f'(t) (newton_raphson.py:137-166) -- not through the converged root:
// the last update starts ~sqrt(tol) from the root, so the two differ at the 1e-5 level.
// The reverse sweep replays the last kHist updates from taped iterates and then the
// conic initial guess; with more updates the earliest are dropped (their share is
// scaled by products of converged residuals). The standard / noll Zernike normal omits
// the normalisation constant, so its Newton slope is not the sag's derivative and the
// iteration converges linearly: the host keeps the forward-mode VJP for those lenses.
//
// Local derivatives of the surface at the hit point (normal and sag w.r.t. x, y and,
// with P = 4, the radius and conic) come from one forward-mode evaluation with dual
// numbers seeded on those inputs; the Zernike coefficients from one transposed pass
// over the terms (ort::zernike_coef_adjoint). Each per-ray contribution to a parameter
// "slot" (radius / conic / vertex z of each surface, each Zernike term, the image-space
// propagation distance) is summed over the wave and written to partial[slot][wave] (every
// needed (slot, wave) entry by this launch: no memset); adj_param_reduce_kernel sums, per
// parameter, the waves of its slots in a fixed order (deterministic) weighted by the
// tangent tables.
#pragma once

#include "ort_kernels.h"

namespace ortk {

struct AArgs {
  const int32_t* zparam;    // [n_zern] parameter per Zernike term (< 0: constant)
  const double* tan_surf;   // [n_param][n_surf][3]: d radius, d conic, d vertex z
  const double* tan_final;  // [n_param]: d final_thickness
  int32_t n_param;
  int32_t n_zern;
  int32_t n_slot;           // 3 n_surf + n_zern + 1
  int32_t n_surf;
  int64_t n_wave;           // waves of the main launch
  ort_rays cot;             // cotangents of the outputs (NULL field: zero)
  // cotangents of the per-surface record buffer [n_rec][8][n_rays] (NULL: zero) and the
  // primal's record buffer (its intensity rows weight the absorption adjoint)
  const double* rec_cot;
  const double* rec;
  ort_rays gin;             // RES: d / d rays_in (NULL field: not wanted)
  double* tape;             // [n_surf][kTapeRows][n_rays]
  double* partial;          // [n_slot][n_wave]
  double* slot_sum;         // [n_slot]
  const int32_t* need;      // [n_slot]: some parameter depends on this slot
  int32_t zero_partials;    // adj_run: memset the partials first (start_surface > 0: the
                            // earlier surfaces' slots are never written)
  int32_t tape_ready;       // the primal trace wrote the tape (F_TAPE): reverse sweep only,
  ort_rays primal;          // the final ray state read from its outputs (L, M, N, i)
  double* grad;             // [n_param], accumulated (grad_store: overwritten)
  int32_t grad_store;
};

// d(slot) / d(parameter p)
__device__ inline double slot_weight(const AArgs& j, int slot, int p) {
  const int ns = 3 * j.n_surf;
  if (slot < ns) return j.tan_surf ? j.tan_surf[(int64_t)p * ns + slot] : 0.0;
  if (slot < ns + j.n_zern) return (j.zparam && j.zparam[slot - ns] == p) ? 1.0 : 0.0;
  return j.tan_final ? j.tan_final[p] : 0.0;
}

// adjoint of a coordinate-system op: rotations transpose (sin -> -sin), translations
// are constant offsets (identity on the adjoint)
__device__ inline void adj_cs_op(ort::Ray& b, const ort_cs_op& op) {
  if (op.kind == ORT_CS_TRANSLATE) return;
  ort_cs_op t = op;
  t.p[1] = -op.p[1];
  ort::apply_cs_op(b, t);
}


// Distance along the ray to surface s in its local frame, as the primal computes it
// (ort_trace_pupil with ORT_NEWTON_SCHEDULE: exactly sched[group][si] Newton updates),
// keeping the iterates before the last kHist updates: hist[m] = t_{U-1-m}.
template <uint32_t KM>
__device__ inline double replay_distance(const KArgs& a, const ort_surface& s, int si,
                                         const ort::Ray& r, int64_t group,
                                         double (&hist)[kHist]) {
#pragma unroll
  for (int h = 0; h < kHist; ++h) hist[h] = 0.0;
  if (s.geometry == ORT_GEOM_PLANE) return ort::distance_plane(r);
  double t = ort::distance_conic(r, s.radius, s.conic, (s.flags & ORT_SURF_RADIUS_INF) != 0);
  if (s.geometry == ORT_GEOM_STANDARD) return t;
  if constexpr (KM != 0) {
    const int U = a.sched ? a.sched[group * a.n_surf + si] : s.max_iter;
    bool rerr = false;
    for (int it = 0; it < U; ++it) {
#pragma unroll
      for (int h = kHist - 1; h > 0; --h) hist[h] = hist[h - 1];
      hist[0] = t;
      double nx, ny, nz;
      const double f = ort::newton_eval<KM>(s, s.radius, s.conic, cst(a.coef), cst(a.zern),
                                            kNoSeed, r, t, true, rerr, nx, ny, nz);
      t = ort::newton_step(r, t, f, nx, ny, nz);
    }
  }
  return t;
}

// P = 2: duals seeded on the point (x, y); P = 4: also on the radius and conic.
//
// Occupancy: the Zernike kernels without freeform kinds (KM 4-7, P = 2) need ~230 VGPRs,
// i.e. 2 waves per SIMD; capped at 128 VGPRs (4 waves, ~400 B of scratch per lane) they
// run 11% faster on the MI355X (TMA 1M rays: 1283 -> 1135 us per adjoint launch,
// rocprofv3); 3 waves: 1177 us, 5 waves: 1719 us. Other kernels keep the compiler's
// choice. ORT_ADJ_WAVES overrides the target for A/B builds.
template <uint32_t KM, int P>
struct AdjWaves {
  static constexpr int value = (P == 2 && (KM & ort::KM_ZERN) != 0 && KM < ort::KM_FREE) ? 4 : 1;
};
#ifdef ORT_ADJ_WAVES
#define ORT_ADJ_OCC __attribute__((amdgpu_waves_per_eu(ORT_ADJ_WAVES)))
#else
#define ORT_ADJ_OCC __attribute__((amdgpu_waves_per_eu(AdjWaves<KM, P>::value)))
#endif
// RES = false: rays generated from pupil samples (ort_trace_pupil_vjp);
// RES = true: resident input rays a.in (ort_trace_sequential_vjp, SurfaceGroup.trace under
// autograd), optionally with per-ray wavelengths (a.w), and the cotangents of the input
// rays written to j.gin. The forward then runs with i = 1, so intensity(r) is the factor
// d i_out / d i_in (0 when clipped, exp(att) otherwise; i_in times it is the primal's
// intensity, operation for operation).
template <uint32_t KM, int P, bool RES>
__global__ __launch_bounds__(kBlock) ORT_ADJ_OCC void adj_kernel(const KArgs a, const AArgs j) {
  using D = ort::Dual<P>;
  const int64_t rid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool active = rid < a.n_rays;
  const int64_t r_ld = active ? rid : 0;
  const int64_t wave = rid >> 6;
  const int64_t NR = a.n_rays;
  const int64_t sidx = (RES && !a.seg) ? 0 : r_ld / a.seg_len;
  int lam = 0;
  double wl = 0.0, i_in = 1.0;
  ort::Ray r;
  if constexpr (RES) {
    if (a.seg) lam = a.seg[sidx].lambda_idx;
    if (a.w) wl = a.w[r_ld];
    r.x = a.in.x[r_ld];
    r.y = a.in.y[r_ld];
    r.z = a.in.z[r_ld];
    r.L = a.in.L[r_ld];
    r.M = a.in.M[r_ld];
    r.N = a.in.N[r_ld];
    i_in = a.in.i[r_ld];
    r.i = 1.0;
    r.opd = a.in.opd[r_ld];
    r.att = 0.0;
  } else {
    const ort_segment sg = a.seg[sidx];
    lam = sg.lambda_idx;
    const int64_t p = a.pupil_per_ray ? r_ld : (r_ld - sidx * a.seg_len);
    r = ort::generate_ray(sg, a.px[p], a.py[p], a.apod);
  }
  const int64_t group = r_ld / a.group_len;
  // optical constants of surface si at this ray's wavelength (table row, or per ray)
  auto optics_of = [&](const ort_surface& s, int si) -> ort_surface_optics {
    if constexpr (RES) {
      if (a.w) return optics_ray(a, s, wl);
    }
    return optics_at(a, lam, si);
  };

  // wave sum of a per-ray contribution into its slot (one writer per slot and wave).
  // first: the slot's first contribution from this wave -- a plain store instead of a
  // read-modify-write whose load the wave would wait for (the same value: 0 + w == w)
  auto emit = [&](int slot, double v, bool first) {
    if (!cst(j.need)[slot]) return;  // uniform
    const double w = wave_sum(active ? v : 0.0);
    if ((threadIdx.x & 63) == 0) {
      double* dst = j.partial + (int64_t)slot * j.n_wave + wave;
      if (first)
        *dst = w;
      else
        *dst += w;
    }
  };

  // sag and normal of surface s at local (x, y) as duals (sag only for Newton kinds)
  auto sagnorm = [&](const ort_surface& s, double x, double y, D& nx, D& ny, D& nz) -> D {
    D X(x), Y(y);
    X.d[0] = 1.0;
    Y.d[1] = 1.0;
    if (s.geometry == ORT_GEOM_PLANE) {
      nx = D(0.0);
      ny = D(0.0);
      nz = D(1.0);
      return D(0.0);
    }
    if (s.geometry == ORT_GEOM_STANDARD) {
      if (s.flags & ORT_SURF_RADIUS_INF) {  // standard.py with R = inf: (0, 0, -1)
        nx = D(0.0);
        ny = D(0.0);
        nz = D(-1.0);
      } else if constexpr (P == 4) {
        D Rd(s.radius), Kd(s.conic);
        Rd.d[2] = 1.0;
        Kd.d[3] = 1.0;
        ort::normal_conic(X, Y, Rd, Kd, nx, ny, nz);
      } else {
        ort::normal_conic(X, Y, s.radius, s.conic, nx, ny, nz);
      }
      return D(0.0);
    }
    bool rerr = false;
    if constexpr (KM == 0) {
      nx = ny = nz = D(__builtin_nan(""));
      return D(__builtin_nan(""));
    } else if constexpr (P == 4) {
      D Rd(s.radius), Kd(s.conic);
      Rd.d[2] = 1.0;
      Kd.d[3] = 1.0;
      return ort::newton_sagnorm<KM>(s, Rd, Kd, cst(a.coef), cst(a.zern), kNoSeed, X, Y, true,
                                     rerr, nx, ny, nz);
    } else {
      return ort::newton_sagnorm<KM>(s, s.radius, s.conic, cst(a.coef), cst(a.zern), kNoSeed,
                                     X, Y, true, rerr, nx, ny, nz);
    }
  };

  // Zernike coefficients at local (x, y): w_sag * d sag / d c plus the slopes' share of
  // the normal's adjoint bn (n = (dzdx, dzdy, -1) / q, q = -1 / nz)
  auto zern_adj = [&](const ort_surface& s, bool on, bool first, double x, double y,
                      double w_sag, double bnx, double bny, double bnz, double nxv,
                      double nyv, double nzv) {
    if constexpr ((KM & ort::KM_ZERN) != 0) {
      if (s.geometry == ORT_GEOM_ZERNIKE && j.zparam) {
        const double bn = bnx * nxv + bny * nyv + bnz * nzv;
        const double bdx = -nzv * (bnx - nxv * bn);
        const double bdy = -nzv * (bny - nyv * bn);
        const int base = 3 * a.n_surf;
        ort::zernike_coef_adjoint(x, y, s.norm_radius, cst(a.zern), s.coef_off, s.n_coef,
                                  cst(a.coef), w_sag, bdx, bdy,
                                  [&](int term, double g) {
                                    emit(base + term, on ? g : 0.0, first);
                                  });
      }
    }
  };

  // distance of the closed forms through their implicit equations: plane / flat conic
  // F = -z (plane.py:61-77), conic x^2 + y^2 + (1 + k) z^2 - 2 R z = 0
  // (standard.py:89-140); tb = adjoint of t, at the point q + t D
  auto closed_adj = [&](const ort_surface& s, const ort::Ray& q, double t, double tb,
                        ort::Ray& b, double& bR, double& bk) {
    const double x = q.x + t * q.L, y = q.y + t * q.M, z = q.z + t * q.N;
    double Gx = 0.0, Gy = 0.0, Gz = -1.0, GR = 0.0, Gk = 0.0;
    if (s.geometry != ORT_GEOM_PLANE && !(s.flags & ORT_SURF_RADIUS_INF)) {
      Gx = 2.0 * x;
      Gy = 2.0 * y;
      Gz = 2.0 * (1.0 + s.conic) * z - 2.0 * s.radius;
      GR = -2.0 * z;
      Gk = z * z;
    }
    const double lm = -tb / (Gx * q.L + Gy * q.M + Gz * q.N);
    b.x += lm * Gx;
    b.y += lm * Gy;
    b.z += lm * Gz;
    b.L += lm * t * Gx;
    b.M += lm * t * Gy;
    b.N += lm * t * Gz;
    bR += lm * GR;
    bk += lm * Gk;
  };

  // ---- forward: the primal trace, taping (incoming ray, t, Newton iterates) per surface;
  // skipped when the primal launch wrote the tape itself (F_TAPE, tape_ready): the final
  // state is then that launch's output (the same values, operation for operation)
  double gi = 0.0;  // RES: d (recorded intensities) / d i_in, contracted with rec_cot
  bool replay = true;
  if constexpr (!RES) replay = !j.tape_ready;
  if (replay) {
    for (int si = a.start_surface; si < a.n_surf; ++si) {
      const ort_surface s = cst(a.surf)[si];
      const ort_surface_optics o = optics_of(s, si);
      double* tp = j.tape + (int64_t)si * kTapeRows * NR + rid;
      if (active) {
        tp[0] = r.x;
        tp[NR] = r.y;
        tp[2 * NR] = r.z;
        tp[3 * NR] = r.L;
        tp[4 * NR] = r.M;
        tp[5 * NR] = r.N;
      }
      localize(a, s, r);
      double hist[kHist];
      const double t = replay_distance<KM>(a, s, si, r, group, hist);
      if (active) {
        tp[6 * NR] = t;
        if (s.geometry != ORT_GEOM_PLANE && s.geometry != ORT_GEOM_STANDARD) {
#pragma unroll
          for (int h = 0; h < kHist; ++h) tp[(7 + h) * NR] = hist[h];
        }
      }
      ort::finish_surface<KM>(r, s, s.radius, s.conic, cst(a.coef), cst(a.zern), kNoSeed, t,
                              o.n_pre, o.u, o.alpha_pre);
      globalize(a, s, r);
      if constexpr (RES) {
        if (j.rec_cot && (s.flags & ORT_SURF_RECORD) && active)
          gi += j.rec_cot[((int64_t)s.rec_slot * 8 + 6) * NR + rid] * ort::intensity(r);
      }
    }
  } else {
    r.L = j.primal.L[r_ld];
    r.M = j.primal.M[r_ld];
    r.N = j.primal.N[r_ld];
    r.i = j.primal.i[r_ld];  // the stored intensity: i exp(att), apodization included
    r.att = 0.0;
  }
  double alpha_f = 0.0;
  if (a.final_mat >= 0) {
    if (RES && a.w)
      alpha_f = ort::absorption_alpha(ort::material_k(cst(a.mats)[a.final_mat], a.coef, wl), wl);
    else
      alpha_f = tab(a.alpha_tab, a.n_lambda, a.n_mat, lam, a.final_mat);
    if (replay) ort::propagate(r, a.final_thickness, alpha_f);
  }

  // ---- output cotangents (intensity = i exp(att): d/d att = intensity)
  ort::Ray b;
  b.x = b.y = b.z = b.L = b.M = b.N = 0.0;
  b.i = b.opd = b.att = 0.0;
  double bopd = 0.0, batt = 0.0;
  if (active) {
    if (j.cot.x) b.x = j.cot.x[rid];
    if (j.cot.y) b.y = j.cot.y[rid];
    if (j.cot.z) b.z = j.cot.z[rid];
    if (j.cot.L) b.L = j.cot.L[rid];
    if (j.cot.M) b.M = j.cot.M[rid];
    if (j.cot.N) b.N = j.cot.N[rid];
    if (j.cot.opd) bopd = j.cot.opd[rid];
    if (j.cot.i) batt = j.cot.i[rid] * (RES ? i_in * ort::intensity(r) : ort::intensity(r));
  }
  const double factor_f = ort::intensity(r);  // RES: d i_out / d i_in
  // image-space propagate (real_ray_tracer.py:84-89): x = x' + d L, ...
  if (a.final_mat >= 0) {
    double bd = b.x * r.L + b.y * r.M + b.z * r.N;
    if (alpha_f > 0.0) bd += batt * (-alpha_f * 1e3);
    emit(3 * a.n_surf + j.n_zern, bd, true);
    const double d = a.final_thickness;
    b.L += d * b.x;
    b.M += d * b.y;
    b.N += d * b.z;
  }

  // ---- reverse over the surfaces
  // LDS slots of this lane's adjoint state, parked across the Newton replay's dual-number
  // evaluation (see there): 10 x 256 doubles = 20 KB per block
  __shared__ double park[10][kBlock];
  for (int si = a.n_surf - 1; si >= a.start_surface; --si) {
    const ort_surface s = cst(a.surf)[si];
    const ort_surface_optics o = optics_of(s, si);
    // cotangent of this surface's record (the state after its globalize): the adjoint of
    // the state there gains it; its intensity row through att (d I / d att = I, the
    // primal's recorded value)
    if (j.rec_cot && (s.flags & ORT_SURF_RECORD) && active) {
      const double* rc = j.rec_cot + (int64_t)s.rec_slot * 8 * NR + rid;
      b.x += rc[0];
      b.y += rc[NR];
      b.z += rc[2 * NR];
      b.L += rc[3 * NR];
      b.M += rc[4 * NR];
      b.N += rc[5 * NR];
      bopd += rc[7 * NR];
      const double ci = rc[6 * NR];
      if (ci != 0.0) batt += ci * j.rec[((int64_t)s.rec_slot * 8 + 6) * NR + rid];
    }
    const double* tp = j.tape + (int64_t)si * kTapeRows * NR + r_ld;
    ort::Ray q;
    q.x = tp[0];
    q.y = tp[NR];
    q.z = tp[2 * NR];
    q.L = tp[3 * NR];
    q.M = tp[4 * NR];
    q.N = tp[5 * NR];
    q.i = 1.0;
    q.opd = 0.0;
    q.att = 0.0;
    const double t = tp[6 * NR];
    localize(a, s, q);
    const double x1 = q.x + t * q.L;
    const double y1 = q.y + t * q.M;
    D nx, ny, nz;
    (void)sagnorm(s, x1, y1, nx, ny, nz);

    // globalize adjoint: + cs_t, then the op list transposed in reverse
    double bCZ = b.z;
    for (int c = s.n_cs_glob - 1; c >= 0; --c) {
      const ort_cs_op op = cst(a.cs)[s.cs_glob_off + c];
      adj_cs_op(b, op);
    }

    // interaction adjoint with the aligned normal m = sign(D.n) n, dot = D.m
    // (real_rays.py:141-181, :511-547)
    const double dr = q.L * nx.v + q.M * ny.v + q.N * nz.v;
    const double sgn = dr > 0.0 ? 1.0 : (dr < 0.0 ? -1.0 : (dr == dr ? 0.0 : dr));
    const double mx = nx.v * sgn, my = ny.v * sgn, mz = nz.v * sgn;
    const double dot = fabs(dr);
    double bmx, bmy, bmz, bdot;
    if (s.flags & ORT_SURF_REFLECTIVE) {  // D' = D - 2 dot m
      bdot = -2.0 * (b.L * mx + b.M * my + b.N * mz);
      bmx = -2.0 * dot * b.L;
      bmy = -2.0 * dot * b.M;
      bmz = -2.0 * dot * b.N;
    } else {  // D' = u D + m (root - u dot), root = sqrt(1 - u^2 (1 - dot^2))
      const double u = o.u;
      const double root = sqrt(1.0 - u * u * (1.0 - dot * dot));
      const double fac = root - u * dot;
      const double bs = b.L * mx + b.M * my + b.N * mz;
      bmx = b.L * fac;
      bmy = b.M * fac;
      bmz = b.N * fac;
      bdot = bs * (u * u * dot / root - u);
      b.L *= u;
      b.M *= u;
      b.N *= u;
    }
    b.L += bdot * mx;
    b.M += bdot * my;
    b.N += bdot * mz;
    bmx += bdot * q.L;
    bmy += bdot * q.M;
    bmz += bdot * q.N;
    const double bnx = sgn * bmx, bny = sgn * bmy, bnz = sgn * bmz;

    // normal adjoint -> hit point, radius, conic, Zernike coefficients
    const double bx1 = b.x + bnx * nx.d[0] + bny * ny.d[0] + bnz * nz.d[0];
    const double by1 = b.y + bnx * nx.d[1] + bny * ny.d[1] + bnz * nz.d[1];
    const double bz1 = b.z;
    double bR = 0.0, bk = 0.0;
    if constexpr (P == 4) {
      bR = bnx * nx.d[2] + bny * ny.d[2] + bnz * nz.d[2];
      bk = bnx * nx.d[3] + bny * ny.d[3] + bnz * nz.d[3];
    }
    zern_adj(s, true, true, x1, y1, 0.0, bnx, bny, bnz, nx.v, ny.v, nz.v);

    // propagation, OPD (|t n|) and absorption adjoint -> t
    double bt = bx1 * q.L + by1 * q.M + bz1 * q.N;
    const double tn = t * o.n_pre;
    bt += bopd * (tn > 0.0 ? o.n_pre : (tn < 0.0 ? -o.n_pre : 0.0));
    if (o.alpha_pre > 0.0) bt += batt * (-o.alpha_pre * 1e3);
    b.x = bx1;
    b.y = by1;
    b.z = bz1;
    b.L += t * bx1;
    b.M += t * by1;
    b.N += t * bz1;

    // intersection distance adjoint
    if (s.geometry == ORT_GEOM_PLANE || s.geometry == ORT_GEOM_STANDARD) {
      closed_adj(s, q, t, bt, b, bR, bk);
    } else if constexpr (KM != 0) {
      // the unrolled Newton updates t' = t - f / f' (newton_raphson.py:140-166) in
      // reverse, newest first, from the taped iterates; then the conic initial guess
      const int U = a.sched ? a.sched[group * a.n_surf + si] : s.max_iter;
      const int Uk = U < kHist ? U : kHist;
      const int m_end = wave_max_i32(active ? Uk : 0);
      double tb = bt;
      for (int m = 0; m < m_end; ++m) {
        const bool on = m < Uk;
        const double tk = tp[(7 + m) * NR];
        const double xk = q.x + tk * q.L, yk = q.y + tk * q.M, zk = q.z + tk * q.N;
        D kx, ky, kz;
        // The dual-number sag / normal alone needs ~124 VGPRs (the plain one 42), so with the
        // adjoint state live across it the kernel spills at its 128-VGPR cap. The state is
        // parked in LDS instead (the empty asm is a compiler memory barrier: the values are
        // reloaded, their registers are free during the evaluation): TMA adjoint 909 ->
        // 851 us per 1M-ray launch (rocprofv3 A/B); parking more values, or at the hit-point
        // and coefficient evaluations too, measured no better.
        park[0][threadIdx.x] = b.x;
        park[1][threadIdx.x] = b.y;
        park[2][threadIdx.x] = b.z;
        park[3][threadIdx.x] = b.L;
        park[4][threadIdx.x] = b.M;
        park[5][threadIdx.x] = b.N;
        park[6][threadIdx.x] = bopd;
        park[7][threadIdx.x] = batt;
        park[8][threadIdx.x] = tb;
        park[9][threadIdx.x] = bCZ;
        asm volatile("" ::: "memory");
        const D sk = sagnorm(s, xk, yk, kx, ky, kz);
        asm volatile("" ::: "memory");
        b.x = park[0][threadIdx.x];
        b.y = park[1][threadIdx.x];
        b.z = park[2][threadIdx.x];
        b.L = park[3][threadIdx.x];
        b.M = park[4][threadIdx.x];
        b.N = park[5][threadIdx.x];
        bopd = park[6][threadIdx.x];
        batt = park[7][threadIdx.x];
        tb = park[8][threadIdx.x];
        bCZ = park[9][threadIdx.x];
        const double f = sk.v - zk;
        const bool zg = fabs(kz.v) > 1e-14;
        const double nzs = zg ? kz.v : 1e-14;
        const double fx = -kx.v / nzs, fy = -ky.v / nzs;
        const double df = fx * q.L + fy * q.M - q.N;
        const bool dg = fabs(df) > 1e-14;
        const double dfs = dg ? df : 1e-14;
        const double tbo = on ? tb : 0.0;
        const double bf = -tbo / dfs;
        const double bdfs = dg ? tbo * f / (dfs * dfs) : 0.0;
        const double bfx = bdfs * q.L, bfy = bdfs * q.M;
        const double knx = -bfx / nzs, kny = -bfy / nzs;
        const double knz = zg ? (bfx * kx.v + bfy * ky.v) / (nzs * nzs) : 0.0;
        if (on) {
          b.L += bdfs * fx;
          b.M += bdfs * fy;
          b.N -= bdfs;
          const double bxk = bf * sk.d[0] + knx * kx.d[0] + kny * ky.d[0] + knz * kz.d[0];
          const double byk = bf * sk.d[1] + knx * kx.d[1] + kny * ky.d[1] + knz * kz.d[1];
          const double bzk = -bf;
          if constexpr (P == 4) {
            bR += bf * sk.d[2] + knx * kx.d[2] + kny * ky.d[2] + knz * kz.d[2];
            bk += bf * sk.d[3] + knx * kx.d[3] + kny * ky.d[3] + knz * kz.d[3];
          }
          b.x += bxk;
          b.y += byk;
          b.z += bzk;
          b.L += tk * bxk;
          b.M += tk * byk;
          b.N += tk * bzk;
          tb = tbo + bxk * q.L + byk * q.M + bzk * q.N;
        }
        zern_adj(s, on, false, xk, yk, bf, knx, kny, knz, kx.v, ky.v, kz.v);
      }
      // initial guess: the base conic's closed form (newton_raphson.py:131-135). More than
      // kHist updates: the earlier ones are dropped -- their share is scaled by the
      // products of f f'' / f'^2 over the kept updates, i.e. by converged residuals
      const double t0 = U == 0 ? t : tp[(int64_t)(7 + (U <= kHist ? U - 1 : 0)) * NR];
      closed_adj(s, q, t0, U <= kHist ? tb : 0.0, b, bR, bk);
    }

    // localize adjoint: the op list transposed in reverse, then - cs_t
    for (int c = s.n_cs_loc - 1; c >= 0; --c) {
      const ort_cs_op op = cst(a.cs)[s.cs_loc_off + c];
      adj_cs_op(b, op);
    }
    bCZ -= b.z;
    emit(3 * si + 0, bR, true);
    emit(3 * si + 1, bk, true);
    emit(3 * si + 2, bCZ, true);
  }
  // no image-space propagate: the final-thickness slot still gets its (zero) partial,
  // so every needed (slot, wave) partial is written by this launch (no memset)
  if (a.final_mat < 0) emit(3 * a.n_surf + j.n_zern, 0.0, true);
  if constexpr (RES) {
    // cotangents of the input rays: the adjoint state at the first traced surface; opd
    // passes straight through, i through the clip / absorption factors
    if (active) {
      if (j.gin.x) j.gin.x[rid] = b.x;
      if (j.gin.y) j.gin.y[rid] = b.y;
      if (j.gin.z) j.gin.z[rid] = b.z;
      if (j.gin.L) j.gin.L[rid] = b.L;
      if (j.gin.M) j.gin.M[rid] = b.M;
      if (j.gin.N) j.gin.N[rid] = b.N;
      if (j.gin.opd) j.gin.opd[rid] = bopd;
      if (j.gin.i) j.gin.i[rid] = (j.cot.i ? j.cot.i[rid] * factor_f : 0.0) + gi;
    }
  }
}

typedef void (*AdjFn)(const KArgs, const AArgs);
AdjFn select_adj2(uint32_t km);   // ort_k_adj2.hip   (generated rays)
AdjFn select_adj4(uint32_t km);   // ort_k_adj4.hip
AdjFn select_adj2r(uint32_t km);  // ort_k_adj2r.hip  (resident rays)
AdjFn select_adj4r(uint32_t km);  // ort_k_adj4r.hip
// zero the partials, flag the needed slots, run the adjoint kernel, reduce, contract
// (ort_k_adj.hip)
int adj_run(const KArgs& a, AArgs j, int32_t* need_ws, int tangents, uint32_t km,
            bool resident, int64_t blocks, hipStream_t stream);

}  // namespace ortk
