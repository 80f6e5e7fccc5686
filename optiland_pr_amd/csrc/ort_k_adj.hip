// ort_k_adj.hip -- adjoint VJP: slot flags, wave-partial reduction, contraction with the
// tangent tables, and the launch sequence (kernel templates: ort_adjoint.h)

#include "ort_adjoint.h"
#include "ort_reduce.h"

namespace ortk {

// need[slot]: some parameter depends on the slot (skips its wave sums); used when the
// caller passes no ort_vjp_params.slot_need
__global__ void adj_need_kernel(const AArgs j0, int32_t* need) {
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= j0.n_slot) return;
  AArgs j = j0;
  j.mono_on = mono_enabled(j0);
  int nd = 0;
  for (int p = 0; p < j.n_param && !nd; ++p) nd = slot_weight(j, slot, p) != 0.0;
  need[slot] = nd;
}

// The parameter reduction in two launches (round 5: with the monomial-basis slots a
// parameter depends on a few dozen slots, and one block per parameter re-reading every
// slot's partials cost 46 us per launch for the TMA's 30 parameters x 30 slots each):
//   adj_slot_reduce_kernel  one block per SLOT: slot_sum[slot] = its per-block partials
//                           summed in index order (each partial read once);
//   adj_grad_kernel         one block per PARAMETER: grad[p] (+)= sum over the slots of
//                           d slot / d p * slot_sum[slot], slots in index order.
// Deterministic (fixed orders, no atomics). The slot weights come from the tangent tables
// and, for the monomial slots, the lens's term matrices (slot_weight / mono_weight).
__global__ __launch_bounds__(kBlock) void adj_slot_reduce_kernel(const AArgs j) {
  const int slot = blockIdx.x;
  __shared__ double ws[kBlock / 64];
  if (!cst(j.need)[slot]) {  // uniform: the launch did not sum this slot
    if (threadIdx.x == 0) j.slot_sum[slot] = 0.0;
    return;
  }
  const double* src = j.partial + (int64_t)slot * j.n_wave;
  double v = 0.0;
  int64_t k = threadIdx.x;
  for (; k + 7 * kBlock < j.n_wave; k += 8 * kBlock) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = src[k + u * kBlock];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += x[u];
  }
  for (; k < j.n_wave; k += kBlock) v += src[k];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double sum = 0.0;
    for (int q = 0; q < kBlock / 64; ++q) sum += ws[q];
    j.slot_sum[slot] = sum;
  }
}

__global__ __launch_bounds__(kBlock) void adj_grad_kernel(const AArgs j0) {
  const int p = blockIdx.x;
  AArgs j = j0;
  j.mono_on = mono_enabled(j0);
  __shared__ double ws[kBlock / 64];
  double v = 0.0;
  for (int slot = threadIdx.x; slot < j.n_slot; slot += kBlock) {
    if (!cst(j.need)[slot]) continue;
    const double w = slot_weight(j, slot, p);
    if (w != 0.0) v += w * j.slot_sum[slot];
  }
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double g = 0.0;
    for (int q = 0; q < kBlock / 64; ++q) g += ws[q];
    if (j.grad_store)
      j.grad[p] = g;
    else
      j.grad[p] += g;
  }
}

int adj_run(const KArgs& a, AArgs j, int32_t* need_ws, int tangents, uint32_t km,
            bool resident, int64_t blocks, hipStream_t stream) {
  AdjFn fn = resident ? (tangents == 4 ? select_adj4r(km) : select_adj2r(km))
                      : (tangents == 4 ? select_adj4(km) : select_adj2(km));
  if (!fn) return ORT_ERR_ARG;
  if (j.zero_partials &&
      hipMemsetAsync(j.partial, 0, (size_t)j.n_slot * (size_t)j.n_wave * sizeof(double),
                     stream) != hipSuccess)
    return ORT_ERR_LAUNCH;
  if (!j.need) {
    hipLaunchKernelGGL(adj_need_kernel, dim3((unsigned)((j.n_slot + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, stream, j, need_ws);
    j.need = need_ws;
  }
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kBlock), 0, stream, a, j);
  if (j.n_param > 0) {
    hipLaunchKernelGGL(adj_slot_reduce_kernel, dim3((unsigned)j.n_slot), dim3(kBlock), 0,
                       stream, j);
    hipLaunchKernelGGL(adj_grad_kernel, dim3((unsigned)j.n_param), dim3(kBlock), 0, stream, j);
  }
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

// ---- device-side Newton schedule check (ort_newton_fixup) ---------------------------
// One workgroup: newton_decide (ort_kernels.h) on the global schedule, the code to *flag,
// and for a re-launch the next launch's statistics and status initialised here (instead of
// two memsets).
__global__ __launch_bounds__(kBlock) void newton_fixup_kernel(
    const ort_surface* surf, int32_t n_surf, int64_t n_groups, const ort_newton_stat* stats,
    int32_t conv_base, int32_t* sched, const int32_t* prev_flag, int32_t* flag,
    ort_newton_stat* next_stats, int32_t* next_status) {
  __shared__ int32_t codes[kBlock / 64];
  if (prev_flag && *prev_flag != 1) {  // the launch these stats belong to did not run:
    if (threadIdx.x == 0) *flag = *prev_flag;  // settled (0) or undecidable (2) stays so
    return;
  }
  const int c = newton_decide(surf, n_surf, n_groups, stats, conv_base, sched, codes);
  if (threadIdx.x == 0) *flag = c;
  // a re-launch follows: initialise its statistics (conv_mask all ones, last_bad and
  // max_updates -1: every byte 0xFF) and status word here, instead of two memsets
  if (c == 1) {
    if (next_stats) {
      const int64_t words = n_groups * n_surf * (int64_t)(sizeof(ort_newton_stat) / 8);
      uint64_t* w = reinterpret_cast<uint64_t*>(next_stats);
      for (int64_t k = threadIdx.x; k < words; k += kBlock) w[k] = ~0ull;
    }
    if (next_status && threadIdx.x == 0) *next_status = 0;
  }
}

// The last launch of the device-verified rounds (ort_newton_finish): the final fixup's
// check, then the per-call state reset for the next call on the same buffers -- the
// status of the last round that ran into *status_out, every round's status word zeroed and
// statistics set to 0xFF bytes, the settled schedule copied out -- in place of two fills
// and a copy per call.
// ort_newton_finish_rms: a second workgroup finishes the rms spot size from the F_RMS rows
// beside the check (one launch for both; the rows are final once the rounds are)
struct RmsFinish {
  const double* part;
  int32_t n_rows;
  double* stats;
  double* rms;
};

__global__ __launch_bounds__(kBlock) void newton_finish_kernel(
    const ort_surface* surf, int32_t n_surf, int64_t n_groups, ort_newton_stat* stats,
    int32_t rounds, int32_t conv_base, int32_t* sched, int32_t* flags, int32_t* statuses,
    int32_t* status_out, int32_t* sched_copy, const RmsFinish rf) {
  if (blockIdx.x == 1) {  // (launched with 2 workgroups only when rf.part is set)
    static_assert(kBlock == kRmsFinThreads, "ort_rms_finish's workgroup shape");
    __shared__ double lds[kBlock / 64 * 3];
    rms_finish_block<kRmsFinThreads, kRmsFinRows>(rf.part, rf.n_rows, rf.stats, rf.rms, lds);
    return;
  }
  __shared__ int32_t codes[kBlock / 64];
  __shared__ int32_t ran_last;
  const int64_t ngs = n_groups * n_surf;
  // the flags, the statuses and (the usual case: the last round did not run) the settled
  // schedule are loaded together up front: one memory round trip, not a chain of them
  const int t = threadIdx.x;
  const int32_t prev = flags[rounds - 1];
  const bool ran = t >= 1 && t <= rounds && flags[t - 1] == 1;  // round t ran
  const int32_t st_t = t <= rounds ? statuses[t] : 0;
  constexpr int kPre = 4;
  int32_t sc[kPre];
#pragma unroll
  for (int q = 0; q < kPre; ++q) {
    const int64_t k = t + (int64_t)q * kBlock;
    sc[q] = k < ngs ? sched[k] : 0;
  }
  if (t == 0) ran_last = 0;  // round 0 always runs
  __syncthreads();
  if (ran) atomicMax(&ran_last, t);  // the last round that ran (order-free: a max)
  if (prev == 1) {  // the last round ran: check its statistics (block-uniform branch)
    const int c = newton_decide(surf, n_surf, n_groups, stats + (int64_t)rounds * ngs,
                                conv_base, sched, codes);
    if (t == 0) flags[rounds] = c;
  } else if (t == 0) {
    flags[rounds] = prev;  // settled (0) or undecidable (2) stays so
  }
  __syncthreads();  // every read of stats / statuses / sched is done
  if (t == ran_last) *status_out = st_t;
  for (int r = t; r <= rounds; r += kBlock) statuses[r] = 0;
  const int64_t words = (int64_t)(rounds + 1) * ngs * (int64_t)(sizeof(ort_newton_stat) / 8);
  uint64_t* w = reinterpret_cast<uint64_t*>(stats);
  for (int64_t k = t; k < words; k += kBlock) w[k] = ~0ull;
  if (sched_copy) {
    if (prev != 1 && ngs <= kPre * kBlock) {  // the schedule was not changed here
#pragma unroll
      for (int q = 0; q < kPre; ++q) {
        const int64_t k = t + (int64_t)q * kBlock;
        if (k < ngs) sched_copy[k] = sc[q];
      }
    } else {
      for (int64_t k = t; k < ngs; k += kBlock) sched_copy[k] = sched[k];
    }
  }
}

}  // namespace ortk

static int newton_finish_launch(const ort_lens* lens, int64_t n_groups, ort_newton_stat* stats,
                                int32_t rounds, int32_t conv_base, int32_t* sched,
                                int32_t* flags, int32_t* statuses, int32_t* status_out,
                                int32_t* sched_copy, const ortk::RmsFinish& rf, void* stream) {
  using namespace ortk;
  if (!lens || !stats || !sched || !flags || !statuses || !status_out || n_groups < 1 ||
      rounds < 1 || conv_base < 0)
    return ORT_ERR_ARG;
  if (lens->n_surfaces < 1 || lens->n_surfaces > ORT_MAX_SURFACES || !lens->surfaces)
    return ORT_ERR_ARG;
  if (rounds >= kBlock) return ORT_ERR_ARG;  // one thread per round's flag and status
  hipLaunchKernelGGL(newton_finish_kernel, dim3(rf.part ? 2 : 1), dim3(kBlock), 0,
                     (hipStream_t)stream, lens->surfaces, lens->n_surfaces, n_groups, stats,
                     rounds, conv_base, sched, flags, statuses, status_out, sched_copy, rf);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

extern "C" int ort_newton_finish(const ort_lens* lens, int64_t n_groups, ort_newton_stat* stats,
                                 int32_t rounds, int32_t conv_base, int32_t* sched,
                                 int32_t* flags, int32_t* statuses, int32_t* status_out,
                                 int32_t* sched_copy, void* stream) {
  return newton_finish_launch(lens, n_groups, stats, rounds, conv_base, sched, flags, statuses,
                              status_out, sched_copy, ortk::RmsFinish{}, stream);
}

extern "C" int ort_newton_finish_rms(const ort_lens* lens, int64_t n_groups,
                                     ort_newton_stat* stats, int32_t rounds, int32_t conv_base,
                                     int32_t* sched, int32_t* flags, int32_t* statuses,
                                     int32_t* status_out, int32_t* sched_copy,
                                     const double* rms_part, int64_t rms_rows,
                                     double* rms_stats, double* rms, void* stream) {
  if (!rms_part || !rms_stats || rms_rows < 1 || rms_rows > ((int64_t)1 << 28))
    return ORT_ERR_ARG;
  return newton_finish_launch(lens, n_groups, stats, rounds, conv_base, sched, flags, statuses,
                              status_out, sched_copy,
                              ortk::RmsFinish{rms_part, (int32_t)rms_rows, rms_stats, rms},
                              stream);
}

extern "C" int ort_newton_fixup(const ort_lens* lens, int64_t n_groups,
                                const ort_newton_stat* stats, int32_t conv_base,
                                int32_t* sched, const int32_t* prev_flag, int32_t* flag,
                                ort_newton_stat* next_stats, int32_t* next_status,
                                void* stream) {
  using namespace ortk;
  if (!lens || !stats || !sched || !flag || n_groups < 1 || conv_base < 0) return ORT_ERR_ARG;
  if (lens->n_surfaces < 1 || lens->n_surfaces > ORT_MAX_SURFACES || !lens->surfaces)
    return ORT_ERR_ARG;
  hipLaunchKernelGGL(newton_fixup_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream,
                     lens->surfaces, lens->n_surfaces, n_groups, stats, conv_base, sched,
                     prev_flag, flag, next_stats, next_status);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

// ---- device-resident Zernike coefficients (ort_patch_zernike) ------------------------
// One workgroup per traced surface (the Zernike ones work, the others leave): the surface's
// coefficients gathered into LDS from the term table, the patched ones written over them
// (and into the table), then the surface's Cartesian block re-formed from LDS (As / An =
// sum_j c_j Ms[j] / Mn[j], term order, no FMA: the host's order in
// geometries.zernike_monomial_block, so a device-resident coefficient gives the same bits
// as the same value uploaded from the host). A surface of more than kPatchTerms terms
// gets its coefficients written into the table only (it has no block: radial order 6
// holds 28 terms).
namespace ortk {
constexpr int kPatchTerms = 1024;

__global__ __launch_bounds__(kBlock) void patch_zernike_kernel(const ort_surface* surf,
                                                               ort_zernike_term* zern,
                                                               double* coef, const double* c,
                                                               const double* const* cp,
                                                               const int64_t* rows, int64_t n) {
  __shared__ double cs[kPatchTerms];
  const ort_surface s = surf[blockIdx.x];
  if (s.geometry != ORT_GEOM_ZERNIKE) return;
  const int t0 = s.coef_off, nt = s.n_coef;
  for (int jt = threadIdx.x; jt < nt && jt < kPatchTerms; jt += kBlock) cs[jt] = zern[t0 + jt].c;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < n; i += kBlock) {
    const int64_t r = rows[i];
    if (r < t0 || r >= t0 + nt) continue;  // another surface's term
    const double v = cp ? *cp[i] : c[i];  // ort_patch_zernike_ptrs: through the pointers
    zern[r].c = v;
    if (r - t0 < kPatchTerms) cs[r - t0] = v;
  }
  __syncthreads();
  if (s.zm_deg < 0 || nt > kPatchTerms) return;
  const int K = (s.zm_deg + 1) * (s.zm_deg + 2) / 2;
  const double* Ms = coef + s.zm_off + 2 * K;
  const double* Mn = Ms + (int64_t)nt * K;
  for (int k = threadIdx.x; k < 2 * K; k += kBlock) {
    const double* M = k < K ? Ms : Mn;
    const int kk = k < K ? k : k - K;
    double acc = 0.0;
    for (int jt = 0; jt < nt; ++jt) acc = acc + cs[jt] * M[(int64_t)jt * K + kk];
    coef[s.zm_off + k] = acc;
  }
}
}  // namespace ortk

extern "C" int ort_patch_zernike(const ort_lens* lens, const double* c, const int64_t* rows,
                                 int64_t n, void* stream) {
  using namespace ortk;
  if (!lens || n < 0 || (n > 0 && (!c || !rows))) return ORT_ERR_ARG;
  if (lens->n_surfaces < 1 || lens->n_surfaces > ORT_MAX_SURFACES || !lens->surfaces ||
      !lens->zern || !lens->coef)
    return ORT_ERR_ARG;
  hipLaunchKernelGGL(patch_zernike_kernel, dim3((unsigned)lens->n_surfaces), dim3(kBlock), 0,
                     (hipStream_t)stream, lens->surfaces,
                     const_cast<ort_zernike_term*>(lens->zern), const_cast<double*>(lens->coef),
                     c, nullptr, rows, n);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

extern "C" int ort_patch_zernike_ptrs(const ort_lens* lens, const double* const* c_ptrs,
                                      const int64_t* rows, int64_t n, void* stream) {
  using namespace ortk;
  if (!lens || n < 0 || (n > 0 && (!c_ptrs || !rows))) return ORT_ERR_ARG;
  if (lens->n_surfaces < 1 || lens->n_surfaces > ORT_MAX_SURFACES || !lens->surfaces ||
      !lens->zern || !lens->coef)
    return ORT_ERR_ARG;
  hipLaunchKernelGGL(patch_zernike_kernel, dim3((unsigned)lens->n_surfaces), dim3(kBlock), 0,
                     (hipStream_t)stream, lens->surfaces,
                     const_cast<ort_zernike_term*>(lens->zern), const_cast<double*>(lens->coef),
                     nullptr, c_ptrs, rows, n);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

// ---- fused Adam step + coefficient patch (ort_adam_patch_zernike) --------------------
// One workgroup per traced surface, as patch_zernike_kernel: the surface's coefficients in
// LDS, the Adam update of those that are parameters (torch.optim.Adam's fused kernel math
// for doubles, FusedAdamKernel / fused_adam_utils: exp_avg = beta1 exp_avg + (1 - beta1) g,
// exp_avg_sq = beta2 exp_avg_sq + (1 - beta2) g g, step_size = lr / (1 - beta1^t),
// denom = sqrt(exp_avg_sq) / sqrt(1 - beta2^t) + eps, param -= step_size exp_avg / denom;
// compiled with the same contraction as that kernel's build, hipcc's default), the new
// value into the term table and LDS, then the surface's Cartesian blocks re-formed in term
// order (patch_zernike_kernel's loop). Each parameter tensor's rows lie within one surface,
// so one workgroup updates it and its step count (no cross-workgroup race).
namespace ortk {
__device__ inline void adam_update(const ort_adam_params& p, double t, double& param, double g,
                                   double& m, double& v) {
#pragma clang fp contract(fast)
  if (p.weight_decay != 0.0) g = g + param * p.weight_decay;
  m = p.beta1 * m + (1 - p.beta1) * g;
  v = p.beta2 * v + (1 - p.beta2) * g * g;
  const double bias_correction1 = 1 - ::pow(p.beta1, t);
  const double bias_correction2 = 1 - ::pow(p.beta2, t);
  const double bias_correction2_sqrt = ::sqrt(bias_correction2);
  const double step_size = p.lr / bias_correction1;
  const double denom = (::sqrt(v) / bias_correction2_sqrt) + p.eps;
  param -= step_size * m / denom;
}

__global__ __launch_bounds__(kBlock) void adam_patch_zernike_kernel(const ort_surface* surf,
                                                                    ort_zernike_term* zern,
                                                                    double* coef,
                                                                    const ort_adam_params p) {
  __shared__ double cs[kPatchTerms];
  const ort_surface s = surf[blockIdx.x];
  if (s.geometry != ORT_GEOM_ZERNIKE) return;
  const int t0 = s.coef_off, nt = s.n_coef;
  for (int jt = threadIdx.x; jt < nt && jt < kPatchTerms; jt += kBlock) cs[jt] = zern[t0 + jt].c;
  __syncthreads();
  uint32_t mine = 0;  // the tensors with rows on this surface (uniform)
  for (int k = 0; k < p.n_tensors; ++k) {
    const int64_t lo = p.row0[k] > t0 ? p.row0[k] : t0;
    const int64_t hi = (p.row0[k] + p.count[k] < t0 + nt) ? p.row0[k] + p.count[k] : t0 + nt;
    if (lo >= hi) continue;
    mine |= 1u << k;
    // the tensor's step count, incremented before the update (torch: step += 1 first)
    const double t = *p.step[k] + 1.0;
    for (int64_t r = lo + threadIdx.x; r < hi; r += kBlock) {
      const int64_t e = r - p.row0[k];
      double param = p.param[k][e], m = p.exp_avg[k][e], v = p.exp_avg_sq[k][e];
      adam_update(p, t, param, p.grad[k][e], m, v);
      p.param[k][e] = param;
      p.exp_avg[k][e] = m;
      p.exp_avg_sq[k][e] = v;
      zern[r].c = param;
      if (r - t0 < kPatchTerms) cs[r - t0] = param;
    }
  }
  __syncthreads();  // (every thread has read the step counts)
  if (!mine) return;
  if (threadIdx.x == 0)
    for (int k = 0; k < p.n_tensors; ++k)
      if (mine & (1u << k)) *p.step[k] = *p.step[k] + 1.0;
  if (s.zm_deg < 0 || nt > kPatchTerms) return;
  const int K = (s.zm_deg + 1) * (s.zm_deg + 2) / 2;
  const double* Ms = coef + s.zm_off + 2 * K;
  const double* Mn = Ms + (int64_t)nt * K;
  for (int k = threadIdx.x; k < 2 * K; k += kBlock) {
    const double* M = k < K ? Ms : Mn;
    const int kk = k < K ? k : k - K;
    double acc = 0.0;
    for (int jt = 0; jt < nt; ++jt) acc = acc + cs[jt] * M[(int64_t)jt * K + kk];
    coef[s.zm_off + k] = acc;
  }
}
}  // namespace ortk

extern "C" int ort_adam_patch_zernike(const ort_lens* lens, const ort_adam_params* p,
                                      void* stream) {
  using namespace ortk;
  if (!lens || !p || p->n_tensors < 0 || p->n_tensors > ORT_ADAM_MAX_TENSORS) return ORT_ERR_ARG;
  if (lens->n_surfaces < 1 || lens->n_surfaces > ORT_MAX_SURFACES || !lens->surfaces ||
      !lens->zern || !lens->coef)
    return ORT_ERR_ARG;
  for (int k = 0; k < p->n_tensors; ++k)
    if (!p->param[k] || !p->grad[k] || !p->exp_avg[k] || !p->exp_avg_sq[k] || !p->step[k] ||
        p->row0[k] < 0 || p->count[k] < 0)
      return ORT_ERR_ARG;
  hipLaunchKernelGGL(adam_patch_zernike_kernel, dim3((unsigned)lens->n_surfaces), dim3(kBlock), 0,
                     (hipStream_t)stream, lens->surfaces,
                     const_cast<ort_zernike_term*>(lens->zern), const_cast<double*>(lens->coef),
                     *p);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}
