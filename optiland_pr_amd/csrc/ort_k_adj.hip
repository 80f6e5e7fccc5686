// ort_k_adj.hip -- adjoint VJP: slot flags, wave-partial reduction, contraction with the
// tangent tables, and the launch sequence (kernel templates: ort_adjoint.h)

#include "ort_adjoint.h"

namespace ortk {

// need[slot]: some parameter depends on the slot (skips its wave sums); used when the
// caller passes no ort_vjp_params.slot_need
__global__ void adj_need_kernel(const AArgs j, int32_t* need) {
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= j.n_slot) return;
  int nd = 0;
  for (int p = 0; p < j.n_param && !nd; ++p) nd = slot_weight(j, slot, p) != 0.0;
  need[slot] = nd;
}

// One block per PARAMETER: grad[p] += sum over the slots p depends on of
// d slot / d p * (the slot's wave partials summed in index order) -- the reduction and
// the contraction with the tangent tables in one launch, deterministic (a fixed order,
// no atomics; a slot shared by several parameters is summed once per parameter). The
// slot weights are read by all threads at once (256 slots per pass into LDS) rather than
// one dependent table load per slot, and each thread's strided partial loads are issued
// eight at a time ahead of their (in-order) additions: 27 -> see DESIGN for the TMA's 43
// slots x 30 parameters.
__global__ __launch_bounds__(kBlock) void adj_param_reduce_kernel(const AArgs j) {
  const int p = blockIdx.x;
  __shared__ double ws[kBlock / 64];
  __shared__ double wt[kBlock];
  double g = 0.0;  // meaningful in thread 0
  for (int base = 0; base < j.n_slot; base += kBlock) {
    const int my = base + threadIdx.x;
    __syncthreads();  // the previous pass's wt reads are done
    wt[threadIdx.x] = my < j.n_slot ? slot_weight(j, my, p) : 0.0;
    __syncthreads();
    const int end = min(kBlock, j.n_slot - base);
    for (int c = 0; c < end; ++c) {
      const double w = wt[c];  // uniform
      if (w == 0.0) continue;
      const double* src = j.partial + (int64_t)(base + c) * j.n_wave;
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
        double s = 0.0;
        for (int q = 0; q < kBlock / 64; ++q) s += ws[q];
        g += s * w;
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) j.grad[p] += g;
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
  if (j.n_param > 0)
    hipLaunchKernelGGL(adj_param_reduce_kernel, dim3((unsigned)j.n_param), dim3(kBlock), 0,
                       stream, j);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

// ---- device-side Newton schedule check (ort_newton_fixup) ---------------------------
// The host's DeviceLens.verify (raytrace.py) per (group, Newton surface), one thread per
// group: the stop rule of newton_raphson.py:140-149 (grid_sag.py:108-140: index >= 1)
// read from the conv_mask window and last_bad of the launch that ran `sched`. Only the
// first wrong surface of a group is corrected (the later surfaces' statistics depend on
// it). code: 0 right, 1 corrected (re-run), 2 the window cannot decide (host).
__global__ __launch_bounds__(kBlock) void newton_fixup_kernel(
    const ort_surface* surf, int32_t n_surf, int64_t n_groups, const ort_newton_stat* stats,
    int32_t conv_base, int32_t* sched, const int32_t* prev_flag, int32_t* flag,
    ort_newton_stat* next_stats, int32_t* next_status) {
  __shared__ int32_t codes[kBlock / 64];
  __shared__ int32_t final_code;
  if (prev_flag && *prev_flag != 1) {  // the launch these stats belong to did not run:
    if (threadIdx.x == 0) *flag = *prev_flag;  // settled (0) or undecidable (2) stays so
    return;
  }
  constexpr int W = 128;  // stop indices per conv_mask window
  int code = 0;
  for (int64_t g = threadIdx.x; g < n_groups; g += kBlock) {
    for (int s = 0; s < n_surf; ++s) {
      const ort_surface sf = surf[s];
      if (sf.geometry == ORT_GEOM_PLANE || sf.geometry == ORT_GEOM_STANDARD) continue;
      int32_t* U_p = sched + g * n_surf + s;
      const int U = *U_p;
      const int max_iter = sf.max_iter;
      const int k_min = sf.geometry == ORT_GEOM_GRID_SAG ? 1 : 0;
      if (U < k_min) {  // grid_sag.py:111-129 always makes the first update
        *U_p = k_min;
        code = max(code, 1);
        break;
      }
      const ort_newton_stat st = stats[g * n_surf + s];
      // first stop index k in [k_min, U) every ray passed, from the window
      int k = -1;
      bool undecided = false;
      for (int i = k_min; i < U; ++i) {
        const int b = i - conv_base;
        if (b < 0 || b >= W) {
          undecided = true;
          break;
        }
        const uint64_t word = b < 64 ? st.conv_mask[0] : st.conv_mask[1];
        if ((word >> (b & 63)) & 1ull) {
          k = i;
          break;
        }
      }
      if (undecided) {
        code = 2;
        break;
      }
      if (k >= 0) {  // every ray passed before update U: the reference stops there
        *U_p = k;
        code = max(code, 1);
        break;
      }
      if (U < max_iter && st.last_bad >= U) {  // not all passed at U: it goes on
        *U_p = U >= 8 ? max_iter : min(max_iter, max(2 * U + 2, 8));
        code = max(code, 1);
        break;
      }
    }
  }
  // block max of the codes (fixed order, LDS)
  for (int o = 32; o > 0; o >>= 1) code = max(code, __shfl_xor(code, o, 64));
  if ((threadIdx.x & 63) == 0) codes[threadIdx.x >> 6] = code;
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0;
    for (int w = 0; w < kBlock / 64; ++w) c = max(c, codes[w]);
    *flag = c;
    final_code = c;
  }
  __syncthreads();
  // a re-launch follows: initialise its statistics (conv_mask all ones, last_bad and
  // max_updates -1: every byte 0xFF) and status word here, instead of two memsets
  if (final_code == 1) {
    if (next_stats) {
      const int64_t words = n_groups * n_surf * (int64_t)(sizeof(ort_newton_stat) / 8);
      uint64_t* w = reinterpret_cast<uint64_t*>(next_stats);
      for (int64_t k = threadIdx.x; k < words; k += kBlock) w[k] = ~0ull;
    }
    if (next_status && threadIdx.x == 0) *next_status = 0;
  }
}

}  // namespace ortk

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
