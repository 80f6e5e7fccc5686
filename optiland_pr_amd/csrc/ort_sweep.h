// ort_sweep.h -- the per-ray sweeps shared by the HIP kernels and the host build.
//
// Everything here is plain per-ray C++ (ORT_HD: __host__ __device__ under hipcc, plain
// functions under g++): the kernel argument block KArgs and its unpacking from the C ABI
// structs (fill_args), frame changes, the optical constants of a surface at a ray's
// wavelength, and the two derivative sweeps of the trace --
//
//   adj_ray  the reverse-mode (adjoint) VJP of one ray (ort_trace_*_vjp, ORT_VJP_ADJOINT);
//   vjp_ray  the forward-mode (dual number) VJP of one ray (ORT_VJP_UNROLLED).
//
// The GPU kernels (ort_adjoint.h adj_kernel, ort_kernels.h vjp_kernel) run them one ray
// per lane; the host library (ort_host.cpp: the CPU dispatch key of the torch custom ops)
// runs them one ray per loop iteration. What differs between the two is behind a small
// "lane" policy object: where a per-ray contribution to a parameter slot goes (a wave sum
// into partial[slot][wave] on the device, a per-chunk accumulator on the host), where the
// adjoint tape lives (HBM rows [S][11][n_rays] on the device, a per-ray scratch array on
// the host) and how a wave-uniform loop bound is formed. The arithmetic is the same source, so the host gradients follow the GPU's operation for
// operation (the reductions over rays run in a different fixed order).
//
// Reference files are cited as path:line under optiland/.
#pragma once

#include "ort_core.h"
#include "ort_interact.h"
#include "ort_material.h"

namespace ortk {

// Lens tables are read-only for the whole launch and indexed by wave-uniform values, so
// the kernels read them through the constant address space: the compiler then emits
// scalar loads (s_load -> SGPRs) instead of per-lane vector loads. Identity on the host.
#if defined(__HIP_DEVICE_COMPILE__)
#define ORT_CONST_AS __attribute__((address_space(4)))
#else
#define ORT_CONST_AS
#endif
template <class T>
using cptr = const ORT_CONST_AS T*;
template <class T>
ORT_INLINE cptr<T> cst(const T* p) {
  return (cptr<T>)(p);
}
using PD = cptr<double>;
using PZ = cptr<ort_zernike_term>;
constexpr ort::ZSeed kNoSeed{nullptr, 0};

// Kernel specialisation bits: bits 0-3 = Newton kinds present (ort::KM_*), bit 4 = rays
// generated in-kernel from pupil coordinates.
enum : uint32_t {
  F_KM = 15u | ort::KM_NURBS,  // the kinds (bits 0-3 and KM_NURBS = bit 16)
  F_GEN = 1u << 4,
  F_REC = 1u << 5,   // some surfaces are recorded (standard_surface.py:266-286)
  F_MONO = 1u << 6,  // the wavelength row is wave-uniform (one wavelength in the lens
                     // tables, or segments aligned to 64 rays): scalar table loads
  F_WRAY = 1u << 7,  // per-ray wavelengths: n, k from lens.materials (ort_batch.w)
  F_IA = 1u << 8,    // thin-lens / phase / grating interactions (ort_interaction)
  F_AXIAL = 1u << 9, // ORT_LENS_AXIAL: every frame a +z translation (closed-form kernels)
  F_TAPE = 1u << 10, // write the adjoint tape as the trace runs (ort_options.tape)
  F_SPOT = 1u << 11, // closed-form kernel: spot pass 1 in the epilogue (ort_trace_spot)
  F_RMS = 1u << 12,  // taped Newton kernel: the rms spot size's workgroup rows in the
                     // epilogue (ort_options.rms_part)
  F_STRIDE = 1u << 13,  // Newton kernel of a verify-and-re-trace round: a grid of at most
                        // kVerifyGrid workgroups strides over the blocks of rays
};

// Adjoint tape (adj_ray): per surface, rows of n_rays doubles -- the incoming global
// x y z L M N, the distance t (7 rows), and for a Newton surface kHist more: the iterates
// before the last kHist updates, row 7 + m = t_{U-1-m} for m < min(U, kHist), the initial
// guess t_0 in the rows m >= U (ABI v19: closed-form surfaces take no iterate rows, and
// every row of the tape is written -- it is the trace op's output, ops.py)
constexpr int kTapeRows = 11;  // the most rows of one surface
constexpr int kHist = 4;

// tape rows of surface s, and the first row of surface si (the surfaces before it)
ORT_INLINE int tape_rows(const ort_surface& s) {
  return (s.geometry == ORT_GEOM_PLANE || s.geometry == ORT_GEOM_STANDARD) ? 7 : kTapeRows;
}
ORT_INLINE int64_t tape_row0(const ort_surface* surf, int si) {
  int64_t r = 0;
  for (int k = 0; k < si; ++k) r += tape_rows(cst(surf)[k]);
  return r;
}

struct KArgs {
  // lens
  const ort_surface* surf;
  const ort_cs_op* cs;
  const double* coef;
  const ort_zernike_term* zern;
  const double* n_tab;
  const double* alpha_tab;
  const ort_surface_optics* optics;
  int32_t n_surf;
  int32_t n_lambda;
  int32_t n_mat;
  int32_t final_mat;
  double final_thickness;
  // rays
  ort_rays in;
  ort_rays out;
  const double* px;
  const double* py;
  // batch
  int64_t n_rays;
  int64_t seg_len;
  int64_t group_len;
  const ort_segment* seg;
  int32_t n_seg;
  int32_t pupil_per_ray;
  // options
  int32_t newton_mode;
  int32_t start_surface;
  const int32_t* sched;
  int32_t conv_base;  // first stop index of the ort_newton_stat.conv_mask window
  // outputs
  double* rec;
  ort_newton_stat* stats;
  int32_t* status;
  // per-ray wavelengths (F_WRAY)
  const double* w;
  const ort_material* mats;
  // wavelength of each table row (F_IA: phase / grating interactions)
  const double* lambdas;
  // pupil apodization of generated rays (NULL: intensity 1)
  const ort_apodization* apod;
  // trace_kernel: blocks walk the pupil chunk by chunk over all (field, lambda) segments
  // (pair_major_ray); set by the host only when it is a bijection (see launch)
  int32_t block_remap;
  // nullable: the launch is a no-op unless *run_if == 1 (ort_options.run_if)
  const int32_t* run_if;
  int32_t no_init;  // host side only: ORT_OPT_NO_INIT (skip init_outputs)
  int32_t exact_only;  // ORT_OPT_EXACT: no deferred-check pass (trace_kernel)
  // verify-and-re-trace (ort_options.verify_*): the launch decides from vstats first
  const ort_newton_stat* vstats;
  const int32_t* vprev;
  int32_t* vflag;
  int32_t* sched_out;
  double* tape;     // F_TAPE: [sum of tape_rows][n_rays] (ort_options.tape)
  // F_SPOT (ort_trace_spot): block b traces chunk b % spot_chunks of pair b / spot_chunks
  // (kClosedBlock rays of seg_len, the tail lanes idle) and writes the chunk's count, sum x,
  // sum y of its i > 0 image points, in the image frame, to spot_part1[b][3] -- the rows
  // spot_sum_kernel would write (ort_k_spot.hip), by the same block reduction
  double* spot_part1;
  const ort_cs_op* spot_ops;
  int32_t spot_n_ops;
  int32_t spot_chunks;
  double* rms_part;  // F_RMS: [workgroup][4] (ort_options.rms_part)
};

// KArgs from the C ABI structs (argument checks included) and the kernel feature bits the
// lens and batch call for (F_KM kinds, F_REC, F_WRAY / F_MONO, F_IA, F_AXIAL).
inline int fill_args(KArgs& a, const ort_lens* lens, const ort_batch* batch,
                     const ort_options* opt, double* rec, ort_newton_stat* stats,
                     int32_t* status, uint32_t& feat) {
  if (!lens || !batch || !opt) return ORT_ERR_ARG;
  if (lens->n_surfaces < 0 || lens->n_surfaces > ORT_MAX_SURFACES) return ORT_ERR_SURFACES;
  if (lens->n_surfaces > 0 &&
      (!lens->surfaces || !lens->n_tab || !lens->alpha_tab || !lens->optics))
    return ORT_ERR_ARG;
  if (batch->n_rays < 0 || batch->seg_len < 1 || batch->group_len < 1) return ORT_ERR_ARG;
  if (lens->n_lambda < 1 || lens->n_mat < 1) return ORT_ERR_ARG;
  if (opt->start_surface < 0) return ORT_ERR_ARG;
  a.surf = lens->surfaces;
  a.cs = lens->cs_ops;
  a.coef = lens->coef;
  a.zern = lens->zern;
  a.n_tab = lens->n_tab;
  a.alpha_tab = lens->alpha_tab;
  a.optics = lens->optics;
  a.n_surf = lens->n_surfaces;
  a.n_lambda = lens->n_lambda;
  a.n_mat = lens->n_mat;
  a.final_mat = lens->final_mat;
  a.final_thickness = lens->final_thickness;
  a.n_rays = batch->n_rays;
  a.seg_len = batch->seg_len;
  a.group_len = batch->group_len;
  a.seg = batch->seg;
  a.n_seg = batch->n_seg;
  a.pupil_per_ray = batch->pupil_per_ray;
  a.apod = batch->apod;
  a.newton_mode = opt->newton_mode;
  a.start_surface = opt->start_surface;
  a.sched = opt->sched;
  a.conv_base = opt->conv_base;
  a.run_if = opt->run_if;
  a.no_init = (opt->flags & ORT_OPT_NO_INIT) != 0;
  a.exact_only = (opt->flags & ORT_OPT_EXACT) != 0;
  a.tape = opt->tape;
  a.rms_part = opt->rms_part;
  if (opt->conv_base < 0) return ORT_ERR_ARG;
  // geometry ids this library knows (enum ort_geometry): anything else is refused here
  // rather than traced as some other kind
  if (lens->geometry_mask & ~((2u << ORT_GEOM_NURBS) - 1u)) return ORT_ERR_ARG;
  a.rec = rec;
  a.stats = stats;
  a.status = status;
  feat = 0;
  if (lens->geometry_mask & (1u << ORT_GEOM_EVEN_ASPHERE)) feat |= ort::KM_EVEN;
  if (lens->geometry_mask & (1u << ORT_GEOM_ODD_ASPHERE)) feat |= ort::KM_ODD;
  if (lens->geometry_mask & (1u << ORT_GEOM_ZERNIKE)) feat |= ort::KM_ZERN;
  if (lens->geometry_mask & ((1u << ORT_GEOM_POLYNOMIAL) | (1u << ORT_GEOM_CHEBYSHEV) |
                             (1u << ORT_GEOM_BICONIC) | (1u << ORT_GEOM_TOROIDAL) |
                             (1u << ORT_GEOM_FORBES_QBFS) | (1u << ORT_GEOM_FORBES_Q2D) |
                             (1u << ORT_GEOM_GRID_SAG)))
    feat |= ort::KM_FREE;
  // NURBS lenses take the all-kinds kernels of ort_k_trace_ia.hip (the only trace kernels
  // with the NURBS solves compiled in)
  if (lens->geometry_mask & (1u << ORT_GEOM_NURBS))
    feat |= ort::KM_NURBS | F_IA | ort::KM_EVEN | ort::KM_ODD | ort::KM_ZERN | ort::KM_FREE;
  if (rec) feat |= F_REC;
  if (batch->w) {  // per-ray wavelengths: n, k from the material tables
    if (!lens->materials) return ORT_ERR_ARG;
    a.w = batch->w;
    a.mats = lens->materials;
    feat |= F_WRAY;
  } else if (lens->n_lambda == 1 || batch->n_seg <= 1 || batch->seg_len % 64 == 0) {
    // every wave reads one wavelength row: one row, one segment, or segment boundaries
    // on the 64-ray wave boundaries (ray r is in segment r / seg_len)
    feat |= F_MONO;
  }
  if (lens->interaction_mask & ~(1u << ORT_IA_REFRACT_REFLECT)) {
    feat |= F_IA;
    a.lambdas = lens->wavelengths;
    const uint32_t need_w = (1u << ORT_IA_PHASE) | (1u << ORT_IA_DIFFRACTIVE);
    if ((lens->interaction_mask & need_w) && !batch->w && !lens->wavelengths) return ORT_ERR_ARG;
  }
  if (lens->frame_flags & ORT_LENS_AXIAL) feat |= F_AXIAL;
  if (opt->newton_mode != ORT_NEWTON_SCHEDULE && opt->newton_mode != ORT_NEWTON_WAVE)
    return ORT_ERR_ARG;
  a.vstats = opt->verify_stats;
  a.vprev = opt->verify_prev_flag;
  a.vflag = opt->verify_flag;
  a.sched_out = opt->sched_out;
  if (opt->verify_stats) {  // verify-and-re-trace (see ort_options)
    const int64_t ng = (batch->n_rays + batch->group_len - 1) / batch->group_len;
    if ((feat & F_KM) == 0 || opt->newton_mode != ORT_NEWTON_SCHEDULE || !opt->sched ||
        !opt->verify_flag || !opt->sched_out || opt->sched_out == opt->sched ||
        !(opt->flags & ORT_OPT_NO_INIT) ||
        opt->run_if || ng * (int64_t)lens->n_surfaces > ORT_VERIFY_MAX_SCHED)
      return ORT_ERR_ARG;
  }
  return ORT_OK;
}

// Table lookup n_tab[lam][mat]: a uniform scalar load when the lens is traced at one
// wavelength (the common case), else a per-lane load of the small L1-resident table.
ORT_INLINE double tab(const double* t, int n_lambda, int n_mat, int lam, int mat) {
  if (n_lambda == 1) return cst(t)[mat];
  return t[lam * n_mat + mat];
}

// optical constants of surface si at wavelength row lam
ORT_INLINE ort_surface_optics optics_row(const KArgs& a, int lam, int si) {
  if (a.n_lambda == 1) return cst(a.optics)[si];
  return a.optics[lam * a.n_surf + si];
}

// F_WRAY: the surface's optical constants at this ray's own wavelength w, evaluated from
// the material tables as the reference evaluates material.n(rays.w) / .k(rays.w)
// (standard_surface.py:218, refractive_reflective_model.py:32-55, homogeneous.py:45-54)
ORT_INLINE ort_surface_optics optics_ray(const KArgs& a, const ort_surface& s, double w) {
  const ort_material mp = cst(a.mats)[s.mat_pre];
  const ort_material mq = cst(a.mats)[s.mat_post];
  ort_surface_optics o;
  o.n_pre = ort::material_n(mp, a.coef, w);
  o.n_post = ort::material_n(mq, a.coef, w);
  o.u = o.n_pre / o.n_post;
  o.u_sq = o.u * o.u;
  o.alpha_pre = ort::absorption_alpha(ort::material_k(mp, a.coef, w), w);
  return o;
}

// localize / globalize (coordinate_system.py:73-107): the root frame's translation
// (cs_t) inline and unconditional, the rest (rotations, reference_cs chains) through the
// op lists, which are empty for plain decentred surfaces (no branch, no register
// shuffling around one)
template <class T>
ORT_INLINE void localize(const KArgs& a, const ort_surface& s, ort::RayT<T>& r) {
  {
    r.x = r.x + -s.cs_t[0];
    r.y = r.y + -s.cs_t[1];
  }
  r.z = r.z + -s.cs_t[2];
  for (int c = 0; c < s.n_cs_loc; ++c) ort::apply_cs_op(r, cst(a.cs)[s.cs_loc_off + c]);
}

template <class T>
ORT_INLINE void globalize(const KArgs& a, const ort_surface& s, ort::RayT<T>& r) {
  for (int c = 0; c < s.n_cs_glob; ++c) ort::apply_cs_op(r, cst(a.cs)[s.cs_glob_off + c]);
  r.x = r.x + s.cs_t[0];
  r.y = r.y + s.cs_t[1];
  r.z = r.z + s.cs_t[2];
}

// =====================================================================================
// Reverse-mode (adjoint) VJP of one ray.
//
// The forward-mode VJP (vjp_ray) re-traces the lens once per chunk of P parameter
// tangents, so its cost grows with the number of parameters. The adjoint computes the
// same vector-Jacobian product in one sweep whatever the parameter count:
//
//   forward   the primal trace in double (same code, same values as ort_trace_pupil),
//             taping each traced surface's incoming global ray (x, y, z, L, M, N), its
//             intersection distance t and (Newton surfaces) the iterates before the
//             last kHist updates;
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
// iteration converges linearly: on those surfaces (ORT_SURF_SLOPE_INEXACT) the sweep is
// exact while U <= kHist (every iterate taped), and the host takes the forward-mode VJP
// for a longer schedule (autodiff.vjp_mode).
//
// Local derivatives of the surface at the hit point (normal and sag w.r.t. x, y and,
// with P = 4, the radius and conic) come from one forward-mode evaluation with dual
// numbers seeded on those inputs; the Zernike coefficients from one transposed pass
// over the terms (ort::zernike_coef_adjoint). Each per-ray contribution to a parameter
// "slot" (radius / conic / vertex z of each surface, each Zernike term, the image-space
// propagation distance) goes to lane.emit(slot, v, first); the per-parameter gradient is
// the sum over rays of its slots weighted by the tangent tables (slot_weight).
// =====================================================================================
// The adjoint's tape rows are read once: ORT_NT_LOAD (A/B builds) reads them non-temporal
// on the device -- measured no gain (config 5 adjoint 428 / 428 vs 436 / 430 us, A/B on the
// MI355X), so plain loads are the default.
#if defined(__HIP_DEVICE_COMPILE__) && defined(ORT_NT_LOAD)
#define ORT_TAPE_LD(x) __builtin_nontemporal_load(&(x))
#else
#define ORT_TAPE_LD(x) (x)
#endif

struct AArgs {
  const int32_t* zparam;    // [n_zern] parameter per Zernike term (< 0: constant)
  const double* tan_surf;   // [n_param][n_surf][3]: d radius, d conic, d vertex z
  const double* tan_final;  // [n_param]: d final_thickness
  int32_t n_param;
  int32_t n_zern;
  int32_t n_slot;           // 3 n_surf + n_zern + 1
  int32_t n_surf;
  int64_t n_wave;           // partial columns (GPU: one per block of the main launch)
  ort_rays cot;             // cotangents of the outputs (NULL field: zero)
  // cotangents of the per-surface record buffer [n_rec][8][n_rays] (NULL: zero) and the
  // primal's record buffer (its intensity rows weight the absorption adjoint)
  const double* rec_cot;
  const double* rec;
  ort_rays gin;             // RES: d / d rays_in (NULL field: not wanted)
  double* tape;             // [sum of tape_rows][n_rays]
  double* partial;          // [n_slot][n_wave]
  double* slot_sum;         // [n_slot]
  const int32_t* need;      // [n_slot]: some parameter depends on this slot
  int32_t zero_partials;    // adj_run: memset the partials first (start_surface > 0: the
                            // earlier surfaces' slots are never written)
  int32_t tape_ready;       // the primal trace wrote the tape (F_TAPE): reverse sweep only,
  ort_rays primal;          // the final ray state read from its outputs (L, M, N, i)
  double* grad;             // [n_param], accumulated (grad_store: overwritten)
  int32_t grad_store;
  // Zernike coefficient adjoints in the Cartesian monomial basis (ort_vjp_params.n_mono,
  // ABI v18): every Zernike surface with a Cartesian block (zm_deg >= 0) owns 2 K slots
  // after the final-thickness slot -- S_k = sum w_sag m_k and D_k = sum (a_x dm_k/dxn +
  // a_y dm_k/dyn) over its evaluations, m_k = xn^p yn^q in the block's order -- and the
  // parameter reduce applies the term matrices Ms / Mn once per launch (mono_weight).
  // mono_on: n_mono equals that count (mono_slots); otherwise the per-term slots serve.
  int32_t n_mono;
  int32_t mono_on;
  const ort_surface* surf;  // the lens tables the reduce reads the term matrices from
  const ort_zernike_term* zern;
  const double* coef;
  // an rms spot size's cotangent folded into the x, y cotangents (ort_vjp_params.rms_*)
  const double* rms_stats;
  const double* rms_grad;
};

// monomials of a Cartesian block of degree N
ORT_INLINE int mono_count(int N) { return (N + 1) * (N + 2) / 2; }
// the highest Cartesian-block degree with a specialised monomial adjoint (zmono_adjoint_deg;
// the host lowers blocks up to geometries.ZM_MAX_DEG = 6). A block of a higher degree --
// only through a hand-made ort_lens: the forward kernels evaluate any degree -- takes the
// per-term slots, so its coefficient adjoint stays exact.
constexpr int kMonoMaxDeg = 6;
// slots of a surface in the monomial basis (0: none)
ORT_INLINE int mono_slots(const ort_surface& s) {
  return (s.geometry == ORT_GEOM_ZERNIKE && s.zm_deg >= 0 && s.zm_deg <= kMonoMaxDeg)
             ? 2 * mono_count(s.zm_deg)
             : 0;
}
// the lens's monomial slot count (every surface, in order)
ORT_INLINE int mono_total(const ort_surface* surf, int n_surf) {
  int t = 0;
  for (int si = 0; si < n_surf; ++si) t += mono_slots(cst(surf)[si]);
  return t;
}

// the monomial slots serve (AArgs.mono_on): the caller's n_mono is the lens's count
ORT_INLINE bool mono_enabled(const AArgs& j) {
  return j.n_mono > 0 && j.zparam && j.surf && j.coef && j.zern &&
         mono_total(j.surf, j.n_surf) == j.n_mono;
}

// the traced surface whose Zernike terms include row `row` of lens.zern (-1: none)
ORT_INLINE int term_surface(const AArgs& j, int row) {
  for (int si = 0; si < j.n_surf; ++si) {
    const ort_surface s = cst(j.surf)[si];
    if (s.geometry == ORT_GEOM_ZERNIKE && row >= s.coef_off && row < s.coef_off + s.n_coef)
      return si;
  }
  return -1;
}

// d(monomial slot m) / d(parameter p): slot m (0-based after the final-thickness slot) is
// S_k or D_k of some surface; its weight is the sum over the surface's terms j that are
// parameter p of Ms[j][k] (the sag: d sag / d c_j = sum_k Ms[j][k] m_k) resp. Mn[j][k] (the
// normal's slopes; zero for c_j == 0, whose term the reference's normal skips,
// zernike.py:213-214)
ORT_INLINE double mono_weight(const AArgs& j, int m, int p) {
  int base = 0;
  for (int si = 0; si < j.n_surf; ++si) {
    const ort_surface s = cst(j.surf)[si];
    const int ms = mono_slots(s);
    if (m < base + ms) {
      const int K = mono_count(s.zm_deg), r = m - base;
      const bool sag = r < K;
      const int k = sag ? r : r - K;
      const int nt = s.n_coef;
      const double* Ms = j.coef + s.zm_off + 2 * K;
      const double* Mn = Ms + (int64_t)nt * K;
      double w = 0.0;
      for (int jt = 0; jt < nt; ++jt) {
        if (!j.zparam || j.zparam[s.coef_off + jt] != p) continue;
        if (sag)
          w = w + Ms[(int64_t)jt * K + k];
        else if (j.zern[s.coef_off + jt].c != 0.0)
          w = w + Mn[(int64_t)jt * K + k];
      }
      return w;
    }
    base += ms;
  }
  return 0.0;
}

// d(slot) / d(parameter p)
ORT_INLINE double slot_weight(const AArgs& j, int slot, int p) {
  const int ns = 3 * j.n_surf;
  if (slot < ns) return j.tan_surf ? j.tan_surf[(int64_t)p * ns + slot] : 0.0;
  if (slot < ns + j.n_zern) {
    if (!j.zparam || j.zparam[slot - ns] != p) return 0.0;
    // a term of a surface served by the monomial slots has no per-term slot of its own
    if (j.mono_on) {
      const int si = term_surface(j, slot - ns);
      if (si >= 0 && mono_slots(cst(j.surf)[si]) > 0) return 0.0;
    }
    return 1.0;
  }
  if (slot == ns + j.n_zern) return j.tan_final ? j.tan_final[p] : 0.0;
  return j.mono_on ? mono_weight(j, slot - ns - j.n_zern - 1, p) : 0.0;
}

// adjoint of a coordinate-system op: rotations transpose (sin -> -sin), translations
// are constant offsets (identity on the adjoint)
ORT_INLINE void adj_cs_op(ort::Ray& b, const ort_cs_op& op) {
  if (op.kind == ORT_CS_TRANSLATE) return;
  ort_cs_op t = op;
  t.p[1] = -op.p[1];
  ort::apply_cs_op(b, t);
}

// Distance along the ray to surface s in its local frame, as the primal computes it
// (ort_trace_pupil with ORT_NEWTON_SCHEDULE: exactly sched[group][si] Newton updates),
// keeping the iterates before the last kHist updates: hist[m] = t_{U-1-m}.
template <uint32_t KM>
ORT_INLINE double replay_distance(const KArgs& a, const ort_surface& s, int si,
                                  const ort::Ray& r, int64_t group, double (&hist)[kHist]) {
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
                                            kNoSeed, r, t, ort::kSlope, rerr, nx, ny, nz);
      t = ort::newton_step_any(r, t, f, nx, ny, nz);
    }
  }
  return t;
}

// One evaluation's Zernike coefficient adjoint in the monomial basis of a degree-N block
// (see AArgs.n_mono): at the normalised point (xn, yn) the sag's weight ws adds ws m_k to
// S_k (SAG; without it -- the hit point, where the sag has no adjoint -- the S slots are
// left alone) and the slopes' weights (ax, ay) -- the adjoint of the block gradient
// (Gx, Gy) the Cartesian normal is formed from -- add ax dm_k/dxn + ay dm_k/dyn to D_k;
// handed to the lane value by value (mono_put(base, i, v): slot base + i, i counting from
// 0), then mono_flush(base, n)
template <int N, bool SAG, class Lane>
ORT_INLINE void zmono_adjoint(Lane& ln, int slot0, double xn, double yn, double ws, double ax,
                              double ay) {
  constexpr int K = (N + 1) * (N + 2) / 2;
  double xp[N + 1], yp[N + 1];
  xp[0] = yp[0] = 1.0;
#pragma unroll
  for (int p = 1; p <= N; ++p) {
    xp[p] = xp[p - 1] * xn;
    yp[p] = yp[p - 1] * yn;
  }
  const int base = SAG ? slot0 : slot0 + K;
  int i = 0;
  if constexpr (SAG) {
#pragma unroll
    for (int p = 0; p <= N; ++p) {
#pragma unroll
      for (int q = 0; q <= N - p; ++q) ln.mono_put(base, i++, ws * (xp[p] * yp[q]));
    }
  }
#pragma unroll
  for (int p = 0; p <= N; ++p) {
#pragma unroll
    for (int q = 0; q <= N - p; ++q) {
      double d = 0.0;
      if (p > 0) d = ax * ((double)p * (xp[p - 1] * yp[q]));
      if (q > 0) d = d + ay * ((double)q * (xp[p] * yp[q - 1]));
      ln.mono_put(base, i++, d);
    }
  }
  ln.mono_flush(base, i);
}

template <bool SAG, class Lane>
ORT_INLINE void zmono_adjoint_deg(Lane& ln, int deg, int slot0, double xn, double yn, double ws,
                                  double ax, double ay) {
  switch (deg) {
    case 0: zmono_adjoint<0, SAG>(ln, slot0, xn, yn, ws, ax, ay); break;
    case 1: zmono_adjoint<1, SAG>(ln, slot0, xn, yn, ws, ax, ay); break;
    case 2: zmono_adjoint<2, SAG>(ln, slot0, xn, yn, ws, ax, ay); break;
    case 3: zmono_adjoint<3, SAG>(ln, slot0, xn, yn, ws, ax, ay); break;
    case 4: zmono_adjoint<4, SAG>(ln, slot0, xn, yn, ws, ax, ay); break;
    case 5: zmono_adjoint<5, SAG>(ln, slot0, xn, yn, ws, ax, ay); break;
    case 6: zmono_adjoint<6, SAG>(ln, slot0, xn, yn, ws, ax, ay); break;
    default:  // unreachable (mono_slots gives such a surface no monomial slots): never
              // another degree's layout -- a NaN in the surface's first slot instead
      ln.mono_put(slot0, 0, __builtin_nan(""));
      ln.mono_flush(slot0, 1);
      break;
  }
}

// The lane policy (Lane) adj_ray is written against:
//   void   emit(int slot, double v, bool first)  add the ray's v to parameter slot `slot`
//                                                 (first: the slot's first contribution
//                                                 from this ray / wave)
//   double* tape_at(int64_t row)                  this ray's entry of tape row `row`
//   int64_t tape_stride()                         distance between two tape rows
//   int    uniform_max(int v)                     max over the rays sharing control flow
//   void   zemit(int slot, int j, double v, bool first), zflush(int slot0, int nt)
//                                                 a Zernike term's contribution (term j of
//                                                 the surface; first: the surface's first);
//                                                 zflush after the surface's last one
//   void   mono_put(int slot0, int i, double v), mono_flush(int slot0, int n)
//                                                 one evaluation's monomial-basis values,
//                                                 v to slot slot0 + i (zmono_adjoint)
// RES = false: rays generated from pupil samples (ort_trace_pupil_vjp);
// RES = true: resident input rays a.in (ort_trace_sequential_vjp, SurfaceGroup.trace under
// autograd), optionally with per-ray wavelengths (a.w), and the cotangents of the input
// rays written to j.gin. The forward then runs with i = 1, so intensity(r) is the factor
// d i_out / d i_in (0 when clipped, exp(att) otherwise; i_in times it is the primal's
// intensity, operation for operation).
template <uint32_t KM, int P, bool RES, class Lane>
ORT_INLINE void adj_ray(const KArgs& a, const AArgs& j, Lane& ln, int64_t rid, bool active) {
  using D = ort::Dual<P>;
  const int64_t r_ld = active ? rid : 0;
  const int64_t NR = a.n_rays;
  const int64_t TS = ln.tape_stride();
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
    return optics_row(a, lam, si);
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
    if constexpr (P == 2 && (KM & ort::KM_ZERN) != 0) {
      // Zernike: the plain-double second-order model (ort::zernike_jet) instead of the
      // dual-number evaluation -- the same derivatives, a fraction of the registers
      if (KM == ort::KM_ZERN || s.geometry == ORT_GEOM_ZERNIKE) {
        ort::SurfJet J;
        ort::zernike_jet(x, y, s.radius, s.conic, s.norm_radius, cst(a.zern), s.coef_off,
                         s.n_coef, cst(a.coef), J, s.zm_off, s.zm_deg);
        ort::jet_normal(J, nx, ny, nz);
        D z(J.z);
        z.d[0] = J.zx;
        z.d[1] = J.zy;
        return z;
      }
    }
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

  // monomial-basis coefficient slots (AArgs.n_mono): the current surface's first slot
  // (mono_base, -1: per-term slots), walking back from the end of the slot table
  int mono_base = -1;
  int mono_end = 3 * a.n_surf + j.n_zern + 1 + (j.mono_on ? j.n_mono : 0);

  // Zernike coefficients at local (x, y): w_sag * d sag / d c plus the slopes' share of
  // the normal's adjoint bn (n = (dzdx, dzdy, -1) / q, q = -1 / nz)
  auto zern_adj = [&](const ort_surface& s, bool on, bool first, double x, double y,
                      double w_sag, double bnx, double bny, double bnz, double nxv,
                      double nyv, double nzv) {
    if constexpr ((KM & ort::KM_ZERN) != 0) {
#ifdef ORT_ADJ_NO_COEF  // timing builds only (A/B of the coefficient adjoint's cost): one
      // contribution per call instead of the term pass, so the sweep's data flow stays live
      if (s.geometry == ORT_GEOM_ZERNIKE && j.zparam)
        ln.zemit(3 * a.n_surf + s.coef_off, 0, on ? x * w_sag + y * bnx + bny + bnz : 0.0, first);
      return;
#endif
      if (s.geometry == ORT_GEOM_ZERNIKE && j.zparam) {
        const double bn = bnx * nxv + bny * nyv + bnz * nzv;
        const double bdx = -nzv * (bnx - nxv * bn);
        const double bdy = -nzv * (bny - nyv * bn);
        if (mono_base >= 0) {
          // the Cartesian normal's slopes (sagnorm_zernike): their adjoints (bdx, bdy)
          // pulled back to the block gradient (Gx, Gy) (derivative-only quotients: rdiv)
          const double inv_rn = ort::rrcp(s.norm_radius);
          const double xn = x * inv_rn, yn = y * inv_rn;
          // sagnorm_zernike's slopes: Gx / Rn, Gy / Rn off the disc rho^2 < kZernChainRho2
          // (their adjoint: (bdx, bdy) / Rn), the reference's chain on it
          const double rho2n = xn * xn + yn * yn;
          double ax, ay;
#ifndef ORT_ZERN_POLAR_CHAIN
          if (rho2n >= ort::kZernChainRho2) {
            ax = bdx * inv_rn;
            ay = bdy * inv_rn;
          } else
#endif
          {
            const double eps = 1e-14;
            const double rho = sqrt(rho2n);
            const double ire = ort::rrcp(rho + eps), iq = ort::rrcp(rho * rho + eps);
            const double drx = xn * inv_rn * ire, dry = yn * inv_rn * ire;
            const double qy = -(yn)*iq, qx = xn * iq;
            double cx = 0.0, cy = 0.0;  // xn / rho, yn / rho (Fr's factors)
            if (rho > 0.0) {
              const double ir = ort::rrcp(rho);
              cx = xn * ir;
              cy = yn * ir;
            }
            const double fr = bdx * drx + bdy * dry;        // adjoint of Fr
            const double g2 = (bdx * qy + bdy * qx) * inv_rn;  // adjoint of G2
            ax = fr * cx - g2 * yn;
            ay = fr * cy + g2 * xn;
          }
          const double wx = on ? ax : 0.0, wy = on ? ay : 0.0;
          if (first)  // the hit point: the normal only (w_sag == 0)
            zmono_adjoint_deg<false>(ln, s.zm_deg, mono_base, xn, yn, 0.0, wx, wy);
          else
            zmono_adjoint_deg<true>(ln, s.zm_deg, mono_base, xn, yn, on ? w_sag : 0.0, wx, wy);
          return;
        }
        const int base = 3 * a.n_surf;
        ort::zernike_coef_adjoint(x, y, s.norm_radius, cst(a.zern), s.coef_off, s.n_coef,
                                  cst(a.coef), w_sag, bdx, bdy,
                                  [&](int term, double g) {
                                    ln.zemit(base + term, term - s.coef_off, on ? g : 0.0,
                                             first);
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
    const double lm = ort::rdiv(-tb, Gx * q.L + Gy * q.M + Gz * q.N);
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
    int64_t trow = tape_row0(a.surf, a.start_surface);
    for (int si = a.start_surface; si < a.n_surf; ++si) {
      const ort_surface s = cst(a.surf)[si];
      const ort_surface_optics o = optics_of(s, si);
      double* tp = ln.tape_at(trow);
      trow += tape_rows(s);
      if (active) {
        tp[0] = r.x;
        tp[TS] = r.y;
        tp[2 * TS] = r.z;
        tp[3 * TS] = r.L;
        tp[4 * TS] = r.M;
        tp[5 * TS] = r.N;
      }
      localize(a, s, r);
      double hist[kHist];
      const double t = replay_distance<KM>(a, s, si, r, group, hist);
      if (active) {
        tp[6 * TS] = t;
        if (s.geometry != ORT_GEOM_PLANE && s.geometry != ORT_GEOM_STANDARD) {
#pragma unroll
          for (int h = 0; h < kHist; ++h) tp[(7 + h) * TS] = hist[h];
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
    if (j.rms_stats) {
      // d rms / d (x, y) = (x - mx, y - my) / (n rms) times the upstream gradient: the
      // ort_rms_spot_vjp kernel's operations, on the final point (the primal's outputs, or
      // the replayed state after the image-space propagate: the same values)
      const double px = replay ? r.x : j.primal.x[r_ld];
      const double py = replay ? r.y : j.primal.y[r_ld];
      const double w = cst(j.rms_grad)[0] / (cst(j.rms_stats)[0] * cst(j.rms_stats)[3]);
      b.x = b.x + (px - cst(j.rms_stats)[1]) * w;
      b.y = b.y + (py - cst(j.rms_stats)[2]) * w;
    }
  }
  const double factor_f = ort::intensity(r);  // RES: d i_out / d i_in
  // image-space propagate (real_ray_tracer.py:84-89): x = x' + d L, ...
  if (a.final_mat >= 0) {
    double bd = b.x * r.L + b.y * r.M + b.z * r.N;
    if (alpha_f > 0.0) bd += batt * (-alpha_f * 1e3);
    ln.emit(3 * a.n_surf + j.n_zern, bd, true);
    const double d = a.final_thickness;
    b.L += d * b.x;
    b.M += d * b.y;
    b.N += d * b.z;
  }

  // ---- reverse over the surfaces
  int64_t trow_end = tape_row0(a.surf, a.n_surf);  // (this surface's rows end here)
  for (int si = a.n_surf - 1; si >= a.start_surface; --si) {
    const ort_surface s = cst(a.surf)[si];
    const ort_surface_optics o = optics_of(s, si);
    trow_end -= tape_rows(s);
    const int64_t trow = trow_end;
    if constexpr ((KM & ort::KM_ZERN) != 0) {
      mono_base = -1;  // this surface's monomial slots (uniform), walking back from the end
      if (j.mono_on) {
        const int ms = mono_slots(s);
        if (ms > 0) {
          mono_end -= ms;
          mono_base = mono_end;
        }
      }
    }
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
    const double* tp = ln.tape_at(trow);
    ort::Ray q;
    q.x = ORT_TAPE_LD(tp[0]);
    q.y = ORT_TAPE_LD(tp[TS]);
    q.z = ORT_TAPE_LD(tp[2 * TS]);
    q.L = ORT_TAPE_LD(tp[3 * TS]);
    q.M = ORT_TAPE_LD(tp[4 * TS]);
    q.N = ORT_TAPE_LD(tp[5 * TS]);
    q.i = 1.0;
    q.opd = 0.0;
    q.att = 0.0;
    const double t = ORT_TAPE_LD(tp[6 * TS]);
    localize(a, s, q);
    const double x1 = q.x + t * q.L;
    const double y1 = q.y + t * q.M;
    D nx, ny, nz;
    (void)sagnorm(s, x1, y1, nx, ny, nz);

    // globalize adjoint: + cs_t, then the op list transposed in reverse
    // surface slots (radius, conic, vertex z) have tangents only with P = 4: the launch
    // takes P = 2 exactly when no surface tangent table is given (ort_api.hip vjp_run), so
    // then their adjoints are not carried at all
    constexpr bool kSurf = P == 4;
    double bCZ = kSurf ? b.z : 0.0;
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
      bdot = bs * (ort::rdiv(u * u * dot, root) - u);
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
      const int m_end = ln.uniform_max(active ? Uk : 0);
      // (a linearly converging surface past the tape: NaN, see the initial guess below)
      double tb = U > kHist && (s.flags & ORT_SURF_SLOPE_INEXACT) ? __builtin_nan("") : bt;
      for (int m = 0; m < m_end; ++m) {
        const bool on = m < Uk;
        // (loaded here, a second round trip per surface; loading the newest iterate with
        // the surface's rows measured the same: config 5 step 0.4917 / 0.4953 vs 0.4925 /
        // 0.4929 ms, tools/gpu_r05u.sh)
        const double tk = ORT_TAPE_LD(tp[(7 + m) * TS]);
        const double xk = q.x + tk * q.L, yk = q.y + tk * q.M, zk = q.z + tk * q.N;
        D kx, ky, kz;
        const D sk = sagnorm(s, xk, yk, kx, ky, kz);
        const double f = sk.v - zk;
        const bool zg = fabs(kz.v) > 1e-14;
        const double nzs = zg ? kz.v : 1e-14;
        const double inzs = ort::rrcp(nzs);  // (derivative-only quotients: rdiv)
        const double fx = -kx.v * inzs, fy = -ky.v * inzs;
        const double df = fx * q.L + fy * q.M - q.N;
        const bool dg = fabs(df) > 1e-14;
        const double dfs = dg ? df : 1e-14;
        const double tbo = on ? tb : 0.0;
        const double idfs = ort::rrcp(dfs);
        const double bf = -tbo * idfs;
        const double bdfs = dg ? tbo * f * (idfs * idfs) : 0.0;
        const double bfx = bdfs * q.L, bfy = bdfs * q.M;
        const double knx = -bfx * inzs, kny = -bfy * inzs;
        const double knz = zg ? (bfx * kx.v + bfy * ky.v) * (inzs * inzs) : 0.0;
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
      // products of f f'' / f'^2 over the kept updates, i.e. by converged residuals. Not so
      // where the Newton slope is not the sag's derivative (ORT_SURF_SLOPE_INEXACT: standard
      // / noll Zernike, linear convergence): the host takes the forward-mode VJP when it
      // knows of such a schedule (autodiff.vjp_mode), and a schedule only the device saw
      // (a device-verified round raised it) poisons the gradient with NaN instead of
      // truncating it silently
      const double t0 = U == 0 ? t : ORT_TAPE_LD(tp[(int64_t)(7 + (U <= kHist ? U - 1 : 0)) * TS]);
      closed_adj(s, q, t0, U <= kHist || (s.flags & ORT_SURF_SLOPE_INEXACT) ? tb : 0.0, b, bR,
                 bk);
    }

    if constexpr ((KM & ort::KM_ZERN) != 0) {
      if (s.geometry == ORT_GEOM_ZERNIKE && j.zparam && mono_base < 0)
        ln.zflush(3 * a.n_surf + s.coef_off, s.n_coef);
    }

    // localize adjoint: the op list transposed in reverse, then - cs_t
    for (int c = s.n_cs_loc - 1; c >= 0; --c) {
      const ort_cs_op op = cst(a.cs)[s.cs_loc_off + c];
      adj_cs_op(b, op);
    }
    if constexpr (kSurf) {
      bCZ -= b.z;
      ln.emit(3 * si + 0, bR, true);
      ln.emit(3 * si + 1, bk, true);
      ln.emit(3 * si + 2, bCZ, true);
    }
  }
  // no image-space propagate: the final-thickness slot still gets its (zero) partial,
  // so every needed (slot, wave) partial is written by this launch (no memset)
  if (a.final_mat < 0) ln.emit(3 * a.n_surf + j.n_zern, 0.0, true);
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

// =====================================================================================
// Forward-mode VJP of one ray w.r.t. lens parameters (the autograd backward; reference:
// torch autograd through the unrolled trace, backend/torch_backend.py +
// optimization/optimizer/torch/base.py:95-154): Zernike coefficients, surface radius and
// conic, surface vertex z (thickness variables) and the image-space propagation distance.
//
// The ray state carries P tangents (ort::Dual<P>), one per parameter of this chunk,
// through exactly the Newton update counts of the primal trace (opt.sched), so the
// derivative is that of the unrolled iteration the reference differentiates. The ray's
// contraction of its tangents with the ray cotangents is added to acc[0 .. P).
// =====================================================================================
struct JArgs {
  const int32_t* zparam;   // [n_zern_terms] parameter index per term, < 0: constant
  const double* tan_surf;  // [n_param][n_surf][3]: d radius, d conic, d vertex z
  const double* tan_final; // [n_param]: d final_thickness
  int32_t n_param;
  int32_t p0;              // first parameter of this launch
  ort_rays cot;            // cotangents of the outputs (NULL field: zero)
  const double* rec_cot;   // cotangents of the record buffer [n_rec][8][n_rays] (or NULL)
  double* grad;            // [n_param]
  double* partial;         // device: [n_block][P] block sums of this chunk (fixed-order
                           // reduction by vjp_reduce_kernel; no atomics)
};

template <int P>
ORT_INLINE void cot_acc(double (&acc)[P], const double* g, int64_t rid,
                        const ort::Dual<P>& v) {
  if (!g) return;
  const double c = g[rid];
#pragma unroll
  for (int k = 0; k < P; ++k) acc[k] += c * v.d[k];
}

// v with the tangents of this chunk's parameters: tan[p * stride + off] (uniform loads)
template <int P>
ORT_INLINE ort::Dual<P> seeded(double v, const double* tan, int64_t stride, int off,
                               const JArgs& j) {
  ort::Dual<P> r(v);
  if (tan) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int p = j.p0 + k;
      r.d[k] = p < j.n_param ? cst(tan)[(int64_t)p * stride + off] : 0.0;
    }
  }
  return r;
}

// a.px set: rays generated from pupil samples (ort_trace_pupil_vjp); NULL: resident input
// rays a.in (ort_trace_sequential_vjp), per-ray wavelengths when a.w is set
template <int P, uint32_t KM>
ORT_INLINE void vjp_ray(const KArgs& a, const JArgs& j, int64_t rid, bool active,
                        double (&acc)[P]) {
  using D = ort::Dual<P>;
  const int64_t r_ld = active ? rid : 0;
  const int64_t sidx = a.seg ? r_ld / a.seg_len : 0;
  int lam = 0;
  double wl = 0.0;
  ort::RayT<D> r;
  if (a.px) {
    const ort_segment sg = a.seg[sidx];
    lam = sg.lambda_idx;
    const int64_t p = a.pupil_per_ray ? r_ld : (r_ld - sidx * a.seg_len);
    r = ort::promote<D>(ort::generate_ray(sg, a.px[p], a.py[p], a.apod));
  } else {
    if (a.seg) lam = a.seg[sidx].lambda_idx;
    if (a.w) wl = a.w[r_ld];
    ort::Ray q;
    q.x = a.in.x[r_ld];
    q.y = a.in.y[r_ld];
    q.z = a.in.z[r_ld];
    q.L = a.in.L[r_ld];
    q.M = a.in.M[r_ld];
    q.N = a.in.N[r_ld];
    q.i = a.in.i[r_ld];
    q.opd = a.in.opd[r_ld];
    q.att = 0.0;
    r = ort::promote<D>(q);
  }
  const int64_t group = r_ld / a.group_len;
  const ort::ZSeed zs{j.zparam, j.p0};
  const int64_t ts = (int64_t)a.n_surf * 3;
  bool unnorm = false;  // a thin lens left the direction unnormalised (F_IA lenses)
#pragma unroll
  for (int k = 0; k < P; ++k) acc[k] = 0.0;

  for (int si = a.start_surface; si < a.n_surf; ++si) {
    const ort_surface s = cst(a.surf)[si];
    const ort_surface_optics o = a.w ? optics_ray(a, s, wl) : optics_row(a, lam, si);
    const D R = seeded<P>(s.radius, j.tan_surf, ts, si * 3 + 0, j);
    const D K = seeded<P>(s.conic, j.tan_surf, ts, si * 3 + 1, j);
    const D CZ = seeded<P>(s.cs_t[2], j.tan_surf, ts, si * 3 + 2, j);
    // localize (coordinate_system.py:73-107) with the vertex z as a parameter
    r.x = r.x + -s.cs_t[0];
    r.y = r.y + -s.cs_t[1];
    r.z = r.z + -CZ;
    for (int c = 0; c < s.n_cs_loc; ++c) ort::apply_cs_op(r, cst(a.cs)[s.cs_loc_off + c]);
    D t;
    if (s.geometry == ORT_GEOM_PLANE) {
      t = ort::distance_plane(r);
    } else {
      t = ort::distance_conic(r, R, K, (s.flags & ORT_SURF_RADIUS_INF) != 0);
      if (s.geometry != ORT_GEOM_STANDARD) {
        if constexpr (KM != 0) {
          // replay the primal's update count (newton_raphson.py:137-166)
          const int U = a.sched ? a.sched[group * a.n_surf + si] : s.max_iter;
          bool rerr = false;
          for (int it = 0; it < U; ++it) {
            D nx, ny, nz;
            const D f = ort::newton_eval<KM>(s, R, K, cst(a.coef), cst(a.zern), zs, r, t,
                                             ort::kSlope, rerr, nx, ny, nz);
            t = ort::newton_step_any(r, t, f, nx, ny, nz);
          }
        }
      }
    }
    bool done = false;
    if constexpr ((KM & 15u) == 15u) {
      // thin-lens / phase / grating surfaces (F_IA lenses take the all-kinds kernels):
      // trace_kernel<F_IA>'s surface step in duals -- propagate, the normalisation a thin
      // lens left pending (homogeneous.py:55-57), OPD, clipping, the interaction model
      if (s.interaction != ORT_IA_REFRACT_REFLECT || unnorm) {
        ort::propagate(r, t, o.alpha_pre);
        if (unnorm) {
          ort::normalize_dir(r);
          unnorm = false;
        }
        ort::add_opd(r, t, o.n_pre);
        if (s.flags & ORT_SURF_APERTURE) ort::clip_radial(r, s.ap_rmax2, s.ap_rmin2);
        if (s.flags & ORT_SURF_APERTURE_PROG) ort::clip_program(r, cst(a.coef) + s.ap_off, s.ap_len);
        const bool refl = (s.flags & ORT_SURF_REFLECTIVE) != 0;
        const PD ip = cst(a.coef) + s.ia_off;
        if (s.interaction == ORT_IA_THIN_LENS) {
          ort::thin_lens(r, ip[0], o.n_pre, refl ? -o.n_pre : o.n_post);
          unnorm = true;
        } else {
          D nx, ny, nz;
          ort::surface_normal<KM>(s, R, K, cst(a.coef), cst(a.zern), zs, r, nx, ny, nz);
          if (s.interaction == ORT_IA_REFRACT_REFLECT) {
            if (refl)
              ort::reflect(r, nx, ny, nz);
            else
              ort::refract(r, nx, ny, nz, o.u);
          } else {
            const double w = a.w ? wl : (a.n_lambda == 1 ? cst(a.lambdas)[0] : a.lambdas[lam]);
            if (s.interaction == ORT_IA_PHASE)
              ort::phase_interact(r, ip, nx, ny, nz, o.n_pre, refl ? o.n_pre : o.n_post, refl, w);
            else
              ort::diffract(r, ip, nx, ny, nz, o.n_pre, o.n_post, refl, w);
          }
        }
        done = true;
      }
    }
    if (!done)
      ort::finish_surface<KM>(r, s, R, K, cst(a.coef), cst(a.zern), zs, t, o.n_pre, o.u,
                              o.alpha_pre);
    for (int c = 0; c < s.n_cs_glob; ++c) ort::apply_cs_op(r, cst(a.cs)[s.cs_glob_off + c]);
    r.x = r.x + s.cs_t[0];
    r.y = r.y + s.cs_t[1];
    r.z = r.z + CZ;
    if (j.rec_cot && (s.flags & ORT_SURF_RECORD) && active) {  // this surface's record
      const double* rc = j.rec_cot + (int64_t)s.rec_slot * 8 * a.n_rays;
      cot_acc(acc, rc, rid, r.x);
      cot_acc(acc, rc + a.n_rays, rid, r.y);
      cot_acc(acc, rc + 2 * a.n_rays, rid, r.z);
      cot_acc(acc, rc + 3 * a.n_rays, rid, r.L);
      cot_acc(acc, rc + 4 * a.n_rays, rid, r.M);
      cot_acc(acc, rc + 5 * a.n_rays, rid, r.N);
      cot_acc(acc, rc + 6 * a.n_rays, rid, ort::intensity(r));
      cot_acc(acc, rc + 7 * a.n_rays, rid, r.opd);
    }
  }
  if (a.final_mat >= 0) {
    ort::propagate(r, seeded<P>(a.final_thickness, j.tan_final, 1, 0, j),
                   a.w ? ort::absorption_alpha(ort::material_k(cst(a.mats)[a.final_mat], a.coef, wl), wl)
                       : tab(a.alpha_tab, a.n_lambda, a.n_mat, lam, a.final_mat));
    if constexpr ((KM & 15u) == 15u) {
      if (unnorm) ort::normalize_dir(r);
    }
  }

  if (active) {
    cot_acc(acc, j.cot.x, rid, r.x);
    cot_acc(acc, j.cot.y, rid, r.y);
    cot_acc(acc, j.cot.z, rid, r.z);
    cot_acc(acc, j.cot.L, rid, r.L);
    cot_acc(acc, j.cot.M, rid, r.M);
    cot_acc(acc, j.cot.N, rid, r.N);
    if (j.cot.i) cot_acc(acc, j.cot.i, rid, ort::intensity(r));
    cot_acc(acc, j.cot.opd, rid, r.opd);
  }
}

}  // namespace ortk
