// ort_adjoint.h -- the reverse-mode (adjoint) VJP kernels of the fused trace.
//
// The per-ray sweep (forward replay with a tape, then the adjoint of every step of
// Surface.trace from the image back to the first surface) is adj_ray in ort_sweep.h,
// shared with the host build (ort_host.cpp). This file holds its GPU side: one ray per
// lane, each parameter-slot contribution summed over the wave into partial[slot][wave]
// (every needed (slot, wave) entry written by the launch: no memset), then
// adj_param_reduce_kernel sums, per parameter, the waves of its slots in a fixed order
// (deterministic) weighted by the tangent tables.
#pragma once

#include "ort_kernels.h"  // (and ort_sweep.h: adj_ray, AArgs)

namespace ortk {

// P = 2: duals seeded on the point (x, y); P = 4: also on the radius and conic.
//
// Occupancy of the Zernike kernels without freeform kinds (KM 4-7, P = 2; TMA 1M rays,
// rocprofv3 A/B per adjoint launch on the MI355X, round 4, with the plain-double Zernike
// jet): 2 waves per SIMD (184 VGPRs, no scratch) 755-757 us, 3 waves (168 VGPRs, 56 B of
// scratch) 582-588 us, 4 waves (128 VGPRs, 216 B) 591-595 us -- the compiler's choice is
// the slowest. Re-measured after the Cartesian Zernike form (177 VGPRs uncapped): 3 waves
// (168, 24 B) 437 us, 4 waves (128, 164 B) 446-452 us per ort_trace_pupil_vjp sequence.
// Other kernels keep the compiler's choice. ORT_ADJ_WAVES overrides the target for A/B
// builds.
template <uint32_t KM, int P>
struct AdjWaves {
  static constexpr int value = (P == 2 && (KM & ort::KM_ZERN) != 0 && KM < ort::KM_FREE) ? 3 : 1;
};
#ifdef ORT_ADJ_WAVES
#define ORT_ADJ_OCC __attribute__((amdgpu_waves_per_eu(ORT_ADJ_WAVES)))
#else
#define ORT_ADJ_OCC __attribute__((amdgpu_waves_per_eu(AdjWaves<KM, P>::value)))
#endif

// adj_ray's lane policy on the GPU (ort_sweep.h): one ray per lane; a slot contribution is
// summed over the wave and stored by lane 0 into partial[slot][wave] (one writer per slot
// and wave; `first`: a plain store instead of a read-modify-write whose load the wave
// would wait for -- the same value, 0 + w == w); the tape rows of the ray in HBM
// ([S][kTapeRows][n_rays], coalesced). (Round 3 parked the adjoint state in LDS across the
// Newton replay's dual-number Zernike evaluation; with the plain-double jet that costs
// more than it saves: 657 vs 591 us at 4 waves, rocprofv3 A/B, so the state stays in
// registers.)
// Zernike coefficient contributions: the first kZAcc terms of a surface are added per lane
// in LDS over the hit point and the (up to kHist) replayed Newton iterates, and summed over
// the wave once per surface -- one DPP wave sum per term and surface instead of one per
// term and evaluation (32 KB of LDS per block; TMA 1M rays: 582 -> 551 us per adjoint
// launch, rocprofv3 A/B). ORT_ADJ_ZACC=0 (A/B builds): a wave sum per evaluation.
#ifndef ORT_ADJ_ZACC
#define ORT_ADJ_ZACC 16
#endif
constexpr int kZAcc = ORT_ADJ_ZACC;
// Block partials: a wave's slot sums are added into bpart[slot][wave of the block] in LDS and
// the block's four waves combined in a fixed order at the end of the launch --
// partial[slot][block], a quarter of the columns the parameter reduce reads, no global
// read-modify-write per emit, and fewer registers than a per-wave global store path (the
// TMA adjoint's scratch 24 -> 20 B). n_slot <= kBlockSlots (16 KB of LDS per block); the
// host takes the forward-mode VJP above that (autodiff.vjp_mode).
constexpr int kBlockSlots = ORT_VJP_ADJOINT_MAX_SLOTS;

struct DevLane {
  const AArgs& j;
  int64_t r_ld;                // this lane's ray (0 for the idle tail lanes)
  int64_t n_rays;
  int64_t wave;
  bool active;
  double (*zacc)[kBlock];      // __shared__ [kZAcc][kBlock] (kZAcc > 0)
  double (*bpart)[kBlock / 64];  // __shared__ [kBlockSlots][4], zeroed at the kernel start

  __device__ inline void emit(int slot, double v, bool first) {
    if (!cst(j.need)[slot]) return;  // uniform
    const double w = wave_sum(active ? v : 0.0);
    (void)first;  // the LDS entries start at zero: 0 + w == w
    if ((threadIdx.x & 63) == 0) bpart[slot][threadIdx.x >> 6] += w;
  }
  __device__ inline double* tape(int si) const {
    return j.tape + (int64_t)si * kTapeRows * n_rays + r_ld;
  }
  __device__ inline int64_t tape_stride() const { return n_rays; }
  __device__ inline int uniform_max(int v) const { return wave_max_i32(v); }
  // Zernike coefficient contributions of one surface (term j of the surface, slot `slot`):
  // with kZAcc > 0 the surface's terms j < kZAcc are added per lane in LDS over the hit
  // point and the replayed Newton iterates and summed over the wave once, at zflush
  __device__ inline void zemit(int slot, int jt, double v, bool first) {
    if constexpr (kZAcc > 0) {
      if (jt < kZAcc) {
        if (!cst(j.need)[slot]) return;  // uniform
        if (first)
          zacc[jt][threadIdx.x] = v;
        else
          zacc[jt][threadIdx.x] += v;
        return;
      }
    }
    emit(slot, v, first);
  }
  __device__ inline void zflush(int slot0, int nt) {
    if constexpr (kZAcc > 0) {
      const int m = nt < kZAcc ? nt : kZAcc;
      for (int jt = 0; jt < m; ++jt)
        if (cst(j.need)[slot0 + jt]) emit(slot0 + jt, zacc[jt][threadIdx.x], true);
    }
  }
};

// RES = false: rays generated from pupil samples (ort_trace_pupil_vjp);
// RES = true: resident input rays (ort_trace_sequential_vjp). The per-ray sweep is
// adj_ray (ort_sweep.h).
template <uint32_t KM, int P, bool RES>
__global__ __launch_bounds__(kBlock) ORT_ADJ_OCC void adj_kernel(const KArgs a, const AArgs j) {
  const int64_t rid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool active = rid < a.n_rays;
  __shared__ double bpart_s[kBlockSlots][kBlock / 64];
  for (int k = threadIdx.x; k < j.n_slot * (kBlock / 64); k += kBlock)
    bpart_s[k / (kBlock / 64)][k % (kBlock / 64)] = 0.0;
  __syncthreads();
  if constexpr (kZAcc > 0 && (KM & ort::KM_ZERN) != 0) {
    __shared__ double zacc[kZAcc > 0 ? kZAcc : 1][kBlock];
    DevLane ln{j, active ? rid : 0, a.n_rays, rid >> 6, active, zacc, bpart_s};
    adj_ray<KM, P, RES>(a, j, ln, rid, active);
  } else {
    DevLane ln{j, active ? rid : 0, a.n_rays, rid >> 6, active, nullptr, bpart_s};
    adj_ray<KM, P, RES>(a, j, ln, rid, active);
  }
  __syncthreads();  // the block's waves combined in index order
  for (int slot = threadIdx.x; slot < j.n_slot; slot += kBlock) {
    if (!cst(j.need)[slot]) continue;
    double v = bpart_s[slot][0];
    for (int w = 1; w < kBlock / 64; ++w) v += bpart_s[slot][w];
    j.partial[(int64_t)slot * j.n_wave + blockIdx.x] = v;
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
