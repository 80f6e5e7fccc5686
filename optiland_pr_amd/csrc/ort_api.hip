// ort_api.hip -- the C ABI (include/optiland_rt.h): argument checks, lens / batch
// unpacking and kernel launches. Kernels are reached through the select_* functions of
// ort_kernels.h (their templates are instantiated in the ort_k_*.hip units).

#include "ort_adjoint.h"

namespace ortk {

int init_outputs(const KArgs& a, hipStream_t stream);

int launch_geom(const ort_lens* lens, int32_t surface, int64_t n, const ort_rays* rays,
                GArgs g, const ort_options* opt, ort_newton_stat* stats, int32_t* status,
                hipStream_t stream) {
  if (!lens || n < 0) return ORT_ERR_ARG;
  if (n == 0) return ORT_OK;
  if (surface < 0 || surface >= lens->n_surfaces) return ORT_ERR_ARG;
  const ort_options dflt{ORT_NEWTON_SCHEDULE, 0, nullptr, 0, 0};
  ort_batch b{};
  b.n_rays = n;
  b.seg_len = n;
  b.group_len = n;  // one reference call: the Newton stop rule spans all n rays
  KArgs a{};
  uint32_t feat = 0;
  if (opt && opt->verify_stats) return ORT_ERR_ARG;  // trace launches only
  int rc = fill_args(a, lens, &b, opt ? opt : &dflt, nullptr, stats, status, feat);
  if (rc) return rc;
  if (rays) a.in = *rays;
  if ((rc = init_outputs(a, stream))) return rc;
  const int64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 0x7fffffff) return ORT_ERR_ARG;
  g.surface = surface;
  hipLaunchKernelGGL(select_geom(feat & F_KM), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                     a, g);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

int launch(const KArgs& a_in, uint32_t feat, hipStream_t stream) {
  if (a_in.n_rays == 0) return ORT_OK;
  const bool closed = (feat & F_IA) == 0 && (feat & F_KM) == 0;
  KernelFn fn = (feat & F_IA) != 0 ? select_trace_ia(feat & ~F_AXIAL)
                : closed           ? select_closed(feat)
                                   : select_trace(feat & ~F_AXIAL);
  if (!fn) return ORT_ERR_ARG;
  const int bs = closed ? closed_block() : kBlock;
  // F_SPOT: one block per (pair, chunk) of seg_len rays
  int64_t blocks = (feat & F_SPOT) != 0 ? (int64_t)a_in.n_seg * a_in.spot_chunks
                                        : (a_in.n_rays + bs - 1) / bs;
  // a verify-and-re-trace round (statistics to check, or a run_if flag) of a kernel with a
  // grid-stride form (F_STRIDE): at most kVerifyGrid workgroups
  if (!closed && (feat & F_IA) == 0 && (a_in.vstats || a_in.run_if) && blocks > kVerifyGrid) {
    if (KernelFn fs = select_trace((feat | F_STRIDE) & ~F_AXIAL)) {
      fn = fs;
      blocks = kVerifyGrid;
    }
  }
  if (blocks > 0x7fffffff) return ORT_ERR_ARG;
  KArgs a = a_in;
  // Newton kernels on generated rays whose segments share one pupil: chunk-major block
  // order (pair_major_ray), where it is a bijection over whole blocks
  a.block_remap = (feat & F_KM) != 0 && (feat & F_IA) == 0 && (feat & F_GEN) != 0 &&
                  !a.pupil_per_ray && a.seg && a.n_seg > 1 && a.seg_len % kBlock == 0 &&
                  a.n_rays == (int64_t)a.n_seg * a.seg_len;
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(bs), 0, stream, a);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

int init_outputs(const KArgs& a, hipStream_t stream) {
  if (a.no_init) return ORT_OK;  // ORT_OPT_NO_INIT: ort_newton_fixup initialised them
  if (a.stats) {
    const int64_t groups = (a.n_rays + a.group_len - 1) / a.group_len;
    // conv_mask = {~0, ~0}, last_bad = -1, max_updates = -1 (all 0xFF bytes)
    if (hipMemsetAsync(a.stats, 0xFF, (size_t)(groups > 0 ? groups : 1) * a.n_surf *
                                          sizeof(ort_newton_stat),
                       stream) != hipSuccess)
      return ORT_ERR_LAUNCH;
  }
  if (a.status && hipMemsetAsync(a.status, 0, sizeof(int32_t), stream) != hipSuccess)
    return ORT_ERR_LAUNCH;
  return ORT_OK;
}

}  // namespace ortk

using namespace ortk;

extern "C" {

int ort_abi_version(void) { return ORT_ABI_VERSION; }

int ort_material_nk(const ort_lens* lens, int32_t mat, const double* w, int64_t n,
                    double* n_out, double* k_out, void* stream) {
  if (!lens || !lens->materials || !lens->coef || n < 0) return ORT_ERR_ARG;
  if (mat < 0 || mat >= lens->n_mat) return ORT_ERR_ARG;
  if (n == 0) return ORT_OK;
  if (!w || (n + kBlock - 1) / kBlock > 0x7fffffff) return ORT_ERR_ARG;
  launch_material_nk(lens->materials, lens->coef, mat, w, n, n_out, k_out,
                     (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

int ort_trace_sequential(const ort_lens* lens, const ort_rays* rays_in, ort_rays* rays_out,
                         const ort_batch* batch, const ort_options* opt, double* rec,
                         ort_newton_stat* newton_stat, int32_t* status, void* stream) {
  if (!rays_in || !rays_out || !batch) return ORT_ERR_ARG;
  if (batch->n_rays == 0) return ORT_OK;
  if (opt && (opt->tape || opt->rms_part)) return ORT_ERR_ARG;  // ort_trace_pupil's
  KArgs a{};
  uint32_t feat = 0;
  int rc = fill_args(a, lens, batch, opt, rec, newton_stat, status, feat);
  if (rc) return rc;
  a.in = *rays_in;
  a.out = *rays_out;
  hipStream_t s = (hipStream_t)stream;
  if ((rc = init_outputs(a, s))) return rc;
  return launch(a, feat, s);
}

int ort_trace_pupil(const ort_lens* lens, const double* px, const double* py,
                    ort_rays* rays_out, const ort_batch* batch, const ort_options* opt,
                    double* rec, ort_newton_stat* newton_stat, int32_t* status,
                    void* stream) {
  return trace_pupil_impl(lens, px, py, rays_out, batch, opt, rec, newton_stat, status, stream,
                          nullptr);
}

}  // extern "C"

namespace ortk {

int trace_pupil_impl(const ort_lens* lens, const double* px, const double* py,
                     ort_rays* rays_out, const ort_batch* batch, const ort_options* opt,
                     double* rec, ort_newton_stat* newton_stat, int32_t* status, void* stream,
                     SpotFuse* fuse) {
  if (fuse) fuse->fused = false;
  if (!rays_out || !batch) return ORT_ERR_ARG;
  if (batch->n_rays == 0) return ORT_OK;
  if (!px || !py || !batch->seg || batch->w) return ORT_ERR_ARG;
  KArgs a{};
  uint32_t feat = 0;
  int rc = fill_args(a, lens, batch, opt, rec, newton_stat, status, feat);
  if (rc) return rc;
  a.px = px;
  a.py = py;
  a.out = *rays_out;
  feat |= F_GEN;
  if (opt->tape) {  // the adjoint tape of a differentiable trace (Newton lenses)
    if ((feat & F_KM) == 0 || (feat & (F_REC | F_IA | F_WRAY)) != 0 ||
        opt->newton_mode != ORT_NEWTON_SCHEDULE || opt->start_surface != 0)
      return ORT_ERR_ARG;
    feat |= F_TAPE;
  }
  if (opt->rms_part) {  // the rms spot size's workgroup rows in the taped kernel's epilogue
    if ((feat & F_TAPE) == 0 || (feat & F_MONO) == 0 || fuse) return ORT_ERR_ARG;
    feat |= F_RMS;
  }
  // ort_trace_spot: spot pass 1 in the closed-form kernel's epilogue when its blocks can be
  // the spot chunks (one ray per thread, each (field, lambda) segment one pair)
  if (fuse && (feat & F_KM) != 0) return ORT_ERR_ARG;  // no schedule protocol here
  if (fuse && (feat & (F_KM | F_IA | F_REC | F_WRAY)) == 0 && closed_block() == 256 &&
      !a.pupil_per_ray && a.n_seg == fuse->pairs && a.n_rays == fuse->pairs * a.seg_len &&
      fuse->chunks * (int64_t)256 >= a.seg_len && (fuse->chunks - 1) * (int64_t)256 < a.seg_len) {
    a.spot_part1 = fuse->part1;
    a.spot_ops = fuse->ops;
    a.spot_n_ops = fuse->n_ops;
    a.spot_chunks = fuse->chunks;
    feat |= F_SPOT;
    fuse->fused = true;
  }
  hipStream_t s = (hipStream_t)stream;
  if ((rc = init_outputs(a, s))) return rc;
  return launch(a, feat, s);
}

}  // namespace ortk

extern "C" {

// ORT_VJP_ADJOINT workspace: tape [rows <= S kTapeRows][n_rays], partial [n_slot][n_wave],
// slot_sum [n_slot], need [n_slot] (each 256-byte aligned).
// ORT_VJP_UNROLLED workspace: the block partials [n_block][4] of one tangent chunk.
struct AdjLayout {
  int32_t n_slot;
  int64_t n_wave, tape, partial, slot_sum, need, total;
};

static bool adj_layout(const ort_lens* lens, const ort_batch* batch,
                       const ort_vjp_params* params, AdjLayout& L) {
  if (!lens || !batch || !params || params->n_zern < 0 || batch->n_rays < 0) return false;
  if (params->zern_param && params->n_zern == 0) return false;
  auto al = [](int64_t v) { return (v + 255) & ~(int64_t)255; };
  const int64_t S = lens->n_surfaces, n = batch->n_rays;
  if (params->mode == ORT_VJP_UNROLLED) {
    L.n_slot = 0;
    L.n_wave = (n + kBlock - 1) / kBlock;  // blocks
    L.tape = L.partial = L.slot_sum = L.need = 0;
    L.total = al(L.n_wave * 4 * (int64_t)sizeof(double));
    return true;
  }
  if (params->n_mono < 0 || (params->n_mono > 0 && !params->zern_param)) return false;
  L.n_slot = (int32_t)(3 * S + params->n_zern + 1 + params->n_mono);
  // partial columns: one per block (its waves combined in LDS, ort_adjoint.h)
  if (L.n_slot > kBlockSlots) return false;  // the forward-mode VJP serves such lenses
  L.n_wave = (n + kBlock - 1) / kBlock;
  L.tape = 0;
  // a tape the primal wrote (params->tape) lives outside the workspace
  const int64_t tape_bytes = params->tape ? 0 : S * kTapeRows * n * (int64_t)sizeof(double);
  L.partial = al(L.tape + tape_bytes);
  L.slot_sum = al(L.partial + (int64_t)L.n_slot * L.n_wave * (int64_t)sizeof(double));
  L.need = al(L.slot_sum + (int64_t)L.n_slot * (int64_t)sizeof(double));
  L.total = al(L.need + (int64_t)L.n_slot * (int64_t)sizeof(int32_t));
  return true;
}

int64_t ort_vjp_tape_size(const ort_lens* lens, const ort_batch* batch) {
  if (!lens || !batch || batch->n_rays < 0 || lens->n_surfaces < 0) return ORT_ERR_ARG;
  return (int64_t)lens->n_surfaces * kTapeRows * batch->n_rays * (int64_t)sizeof(double);
}

int64_t ort_vjp_workspace_size(const ort_lens* lens, const ort_batch* batch,
                               const ort_vjp_params* params) {
  AdjLayout L;
  if (!adj_layout(lens, batch, params, L)) return ORT_ERR_ARG;
  return L.total;
}

// Shared body of the two VJP entry points: generated rays (px, py) or resident rays
// (rays_in, resident = true).
static int vjp_run(const ort_lens* lens, const double* px, const double* py,
                   const ort_rays* rays_in, bool resident, const ort_batch* batch,
                   const ort_options* opt, const ort_vjp_params* params,
                   const ort_rays* cotangent, const double* rec_cotangent, const double* rec,
                   double* grad, const ort_rays* grad_in, void* stream) {
  if (!batch || !cotangent || !params || params->n_param < 0) return ORT_ERR_ARG;
  const int32_t n_param = params->n_param;
  const bool want_in = grad_in && (grad_in->x || grad_in->y || grad_in->z || grad_in->L ||
                                   grad_in->M || grad_in->N || grad_in->i || grad_in->opd);
  if (n_param > 0 && !grad) return ORT_ERR_ARG;
  if (batch->n_rays == 0 || (n_param == 0 && !want_in)) {
    // nothing to trace: an overwritten gradient is zero
    if (params->grad_init && n_param > 0 &&
        hipMemsetAsync(grad, 0, (size_t)n_param * sizeof(double), (hipStream_t)stream) !=
            hipSuccess)
      return ORT_ERR_LAUNCH;
    return ORT_OK;
  }
  if (rec_cotangent && !rec) return ORT_ERR_ARG;  // intensity rows weight the absorption
  if (resident) {
    if (!rays_in) return ORT_ERR_ARG;
  } else if (!px || !py || !batch->seg || batch->w) {
    return ORT_ERR_ARG;
  }
  KArgs a{};
  uint32_t feat = 0;
  if (opt && opt->verify_stats) return ORT_ERR_ARG;  // trace launches only
  int rc = fill_args(a, lens, batch, opt, nullptr, nullptr, nullptr, feat);
  if (rc) return rc;
  if (opt->newton_mode != ORT_NEWTON_SCHEDULE) return ORT_ERR_ARG;
  if (params->zern_param && (feat & ort::KM_ZERN) == 0) return ORT_ERR_ARG;
  // thin-lens / phase / grating surfaces: the forward-mode VJP only (vjp_ray's all-kinds
  // instantiation carries their interactions in duals; the adjoint has no reverse for them)
  if ((feat & F_IA) && params->mode != ORT_VJP_UNROLLED) return ORT_ERR_ARG;
  if (lens->geometry_mask & ((1u << ORT_GEOM_GRID_SAG) | (1u << ORT_GEOM_NURBS)))
    return ORT_ERR_ARG;  // nor grid sags / NURBS (no derivative kernels)
  if (resident) {
    a.in = *rays_in;
  } else {
    a.px = px;
    a.py = py;
  }
  const int64_t blocks = (a.n_rays + kBlock - 1) / kBlock;
  if (blocks > 0x7fffffff) return ORT_ERR_ARG;
  const uint32_t km = (feat & F_IA) ? 15u : (feat & F_KM);  // (F_IA: every kind, vjp_ray)
  hipStream_t s = (hipStream_t)stream;
  if (params->mode == ORT_VJP_ADJOINT) {
    AdjLayout L;
    if (!adj_layout(lens, batch, params, L)) return ORT_ERR_ARG;
    if (!params->workspace || params->workspace_size < L.total) return ORT_ERR_ARG;
    char* w = (char*)params->workspace;
    AArgs aj{};
    aj.zparam = params->zern_param;
    aj.tan_surf = params->surf_tangent;
    aj.tan_final = params->final_tangent;
    aj.n_param = n_param;
    aj.n_zern = params->n_zern;
    aj.n_slot = L.n_slot;
    aj.n_surf = lens->n_surfaces;
    aj.n_wave = L.n_wave;
    aj.cot = *cotangent;
    aj.rec_cot = rec_cotangent;
    aj.rec = rec;
    if (want_in) aj.gin = *grad_in;
    aj.tape = (double*)(w + L.tape);
    if (params->tape) {  // the primal wrote the tape: reverse sweep only
      if (resident || !params->primal.L || !params->primal.M || !params->primal.N ||
          !params->primal.i)
        return ORT_ERR_ARG;
      aj.tape = (double*)params->tape;
      aj.tape_ready = 1;
      aj.primal = params->primal;
    }
    aj.partial = (double*)(w + L.partial);
    aj.slot_sum = (double*)(w + L.slot_sum);
    aj.need = params->slot_need;  // NULL: adj_run derives it into the workspace
    aj.zero_partials = opt->start_surface > 0;
    aj.grad = grad;
    aj.grad_store = params->grad_init != 0;
    aj.n_mono = params->n_mono;
    aj.surf = lens->surfaces;
    aj.zern = lens->zern;
    aj.coef = lens->coef;
    // an rms spot size's cotangent folded into the x, y cotangent load
    if ((params->rms_stats != nullptr) != (params->rms_grad != nullptr)) return ORT_ERR_ARG;
    if (params->rms_stats && aj.tape_ready && (!params->primal.x || !params->primal.y))
      return ORT_ERR_ARG;
    aj.rms_stats = params->rms_stats;
    aj.rms_grad = params->rms_grad;
    // radius / conic tangents need duals seeded on them too
    return adj_run(a, aj, (int32_t*)(w + L.need), params->surf_tangent ? 4 : 2, km, resident,
                   blocks, s);
  }
  if (params->mode != ORT_VJP_UNROLLED) return ORT_ERR_ARG;
  if (want_in) return ORT_ERR_ARG;  // forward mode carries parameter tangents only
  if (params->rms_stats || params->rms_grad) return ORT_ERR_ARG;  // the adjoint's fold only
  AdjLayout L;
  if (!adj_layout(lens, batch, params, L)) return ORT_ERR_ARG;
  if (!params->workspace || params->workspace_size < L.total) return ORT_ERR_ARG;
  JArgs j{};
  j.zparam = params->zern_param;
  j.tan_surf = params->surf_tangent;
  j.tan_final = params->final_tangent;
  j.n_param = n_param;
  j.cot = *cotangent;
  j.rec_cot = rec_cotangent;
  j.grad = grad;
  j.partial = (double*)params->workspace;
  if (params->grad_init &&
      hipMemsetAsync(grad, 0, (size_t)n_param * sizeof(double), s) != hipSuccess)
    return ORT_ERR_LAUNCH;
  for (int p0 = 0; p0 < n_param;) {
    const int left = n_param - p0;
    // tangents per launch: ORT_VJP_TANGENTS overrides (A/B timing)
    const char* e = getenv("ORT_VJP_TANGENTS");
    const int pref = e ? atoi(e) : 4;
    const int P = left >= 4 && pref >= 4 ? 4 : (left >= 2 && pref >= 2 ? 2 : 1);
    VjpFn fn = select_vjp(P, km);
    VjpReduceFn red = select_vjp_reduce(P);
    if (!fn || !red) return ORT_ERR_ARG;
    j.p0 = p0;
    // the chunk's block partials, then their fixed-order sums into grad (the next chunk's
    // launch reuses the partials after this reduction on the same stream)
    hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kBlock), 0, s, a, j);
    hipLaunchKernelGGL(red, dim3((unsigned)P), dim3(kBlock), 0, s, j, blocks);
    if (hipGetLastError() != hipSuccess) return ORT_ERR_LAUNCH;
    p0 += P;
  }
  return ORT_OK;
}

int ort_trace_pupil_vjp(const ort_lens* lens, const double* px, const double* py,
                        const ort_batch* batch, const ort_options* opt,
                        const ort_vjp_params* params, const ort_rays* cotangent,
                        double* grad, void* stream) {
  return vjp_run(lens, px, py, nullptr, false, batch, opt, params, cotangent, nullptr, nullptr,
                 grad, nullptr, stream);
}

int ort_trace_sequential_vjp(const ort_lens* lens, const ort_rays* rays_in,
                             const ort_batch* batch, const ort_options* opt,
                             const ort_vjp_params* params, const ort_rays* cotangent,
                             const double* rec_cotangent, const double* rec, double* grad,
                             const ort_rays* grad_in, void* stream) {
  return vjp_run(lens, nullptr, nullptr, rays_in, true, batch, opt, params, cotangent,
                 rec_cotangent, rec, grad, grad_in, stream);
}

int ort_generate_pupil(const ort_pupil* pupil, double* px, double* py, void* stream) {
  if (!pupil || pupil->n_points < 0) return ORT_ERR_ARG;
  if (pupil->n_points == 0) return ORT_OK;
  if (!px || !py || pupil->kind < ORT_PUPIL_UNIFORM || pupil->kind > ORT_PUPIL_CROSS)
    return ORT_ERR_ARG;
  if (pupil->kind == ORT_PUPIL_UNIFORM && (pupil->n_rows <= 0 || !pupil->row_start ||
                                           !pupil->row_col))
    return ORT_ERR_ARG;
  if (pupil->kind == ORT_PUPIL_RANDOM && (!pupil->rng_chunk || !pupil->rng_lane))
    return ORT_ERR_ARG;
  return launch_pupil(*pupil, px, py, (hipStream_t)stream);
}

int ort_surface_sag_normal(const ort_lens* lens, int32_t surface, const double* x,
                           const double* y, int64_t n, double* sag, double* nx, double* ny,
                           double* nz, int32_t* status, void* stream) {
  if (n > 0 && (!x || !y)) return ORT_ERR_ARG;
  GArgs g{};
  g.mode = 0;
  g.x = x;
  g.y = y;
  g.sag = sag;
  g.nx = nx;
  g.ny = ny;
  g.nz = nz;
  return launch_geom(lens, surface, n, nullptr, g, nullptr, nullptr, status,
                     (hipStream_t)stream);
}

int ort_surface_distance(const ort_lens* lens, int32_t surface, const ort_rays* rays,
                         int64_t n, const ort_options* opt, double* t,
                         ort_newton_stat* newton_stat, int32_t* status, void* stream) {
  if (n > 0 && (!rays || !t)) return ORT_ERR_ARG;
  GArgs g{};
  g.mode = 1;
  g.t = t;
  return launch_geom(lens, surface, n, rays, g, opt, newton_stat, status,
                     (hipStream_t)stream);
}

int ort_generate_rays(const double* px, const double* py, ort_rays* rays_out,
                      const ort_batch* batch, void* stream) {
  if (!rays_out || !batch) return ORT_ERR_ARG;
  if (batch->n_rays == 0) return ORT_OK;
  if (!px || !py || !batch->seg || batch->seg_len < 1) return ORT_ERR_ARG;
  KArgs a{};
  a.px = px;
  a.py = py;
  a.out = *rays_out;
  a.n_rays = batch->n_rays;
  a.seg_len = batch->seg_len;
  a.seg = batch->seg;
  a.pupil_per_ray = batch->pupil_per_ray;
  a.apod = batch->apod;
  if (a.n_rays == 0) return ORT_OK;
  const int64_t blocks = (a.n_rays + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(select_generate(), dim3((unsigned)blocks), dim3(kBlock), 0,
                     (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

}  // extern "C"
