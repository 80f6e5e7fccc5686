// ort_adjoint.h -- the reverse-mode (adjoint) VJP kernels of the fused trace.
//
// The per-ray sweep (forward replay with a tape, then the adjoint of every step of
// Surface.trace from the image back to the first surface) is adj_ray in ort_sweep.h,
// shared with the host build (ort_host.cpp). This file holds its GPU side: one ray per
// lane, each parameter-slot contribution summed over the wave into partial[slot][wave]
// (every needed (slot, wave) entry written by the launch: no memset), then
// adj_slot_reduce_kernel / adj_grad_kernel sum each slot's partials, then per parameter the
// slot sums weighted by the tangent tables, in fixed orders (deterministic).
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
// ([rows][n_rays], coalesced). (Round 3 parked the adjoint state in LDS across the
// Newton replay's dual-number Zernike evaluation; with the plain-double jet that costs
// more than it saves: 657 vs 591 us at 4 waves, rocprofv3 A/B, so the state stays in
// registers.)
// Zernike coefficient contributions: the first kZAcc terms of a surface are added per lane
// in LDS over the hit point and the (up to kHist) replayed Newton iterates, and summed over
// the wave once per surface -- one DPP wave sum per term and surface instead of one per
// term and evaluation (32 KB of LDS per block; TMA 1M rays: 582 -> 551 us per adjoint
// launch, rocprofv3 A/B). ORT_ADJ_ZACC=0 (A/B builds): a wave sum per evaluation.
// Round 5: surfaces with a Cartesian block take the monomial-basis slots (mono_put below)
// and need no per-lane term accumulators; the LDS they took (32 KB per block) held the
// kernel at 3 blocks per CU, so the per-evaluation wave sums serve the polar surfaces
// (radial order > 6) by default.
#ifndef ORT_ADJ_ZACC
#define ORT_ADJ_ZACC 0
#endif
constexpr int kZAcc = ORT_ADJ_ZACC;
// Block partials: a wave's slot sums are added into bpart[slot][wave of the block] in LDS and
// the block's four waves combined in a fixed order at the end of the launch --
// partial[slot][block], a quarter of the columns the parameter reduce reads, no global
// read-modify-write per emit, and fewer registers than a per-wave global store path (the
// TMA adjoint's scratch 24 -> 20 B). n_slot <= kBlockSlots (16 KB of LDS per block); the
// host takes the forward-mode VJP above that (autodiff.vjp_mode).
constexpr int kBlockSlots = ORT_VJP_ADJOINT_MAX_SLOTS;

// Monomial-basis slots (AArgs.n_mono): one evaluation's 2 K values per lane are summed over
// the wave eight slots at a time through a per-wave LDS transpose -- lane l writes its
// value for slot row r to scr[r][l]; lane l then adds up row l / 8's entries l % 8,
// l % 8 + 8, ... (eight of them) and the eight lanes of a row combine by DPP (quad xor 1, 2,
// row_half_mirror) -- so a chunk of eight slots costs 8 LDS writes, 8 reads and ~16 VALU
// per lane instead of eight full wave sums (~20 VALU each). The row stride of 72 doubles
// puts the eight rows' reads on different LDS banks (2-way at most for 64-bit reads).
constexpr int kMonoStride = 72;

__device__ inline double group8_sum(double v) {
  if (__builtin_amdgcn_read_exec() == ~0ull) {
    v += dpp_step<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
    v += dpp_step<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
    v += dpp_step<0x141, 0xf>(v);  // row_half_mirror: lane i <- lane 7 - i of its 8
    return v;
  }
  for (int o = 1; o < 8; o <<= 1) v += __shfl_xor(v, o, 64);  // the same sums, same order
  return v;
}

struct DevLane {
  const AArgs& j;
  int64_t r_ld;                // this lane's ray (0 for the idle tail lanes)
  int64_t n_rays;
  int64_t wave;
  bool active;
  double (*zacc)[kBlock];      // __shared__ [kZAcc][kBlock] (kZAcc > 0)
  double (*bpart)[kBlock / 64];  // __shared__ [kBlockSlots][4], zeroed at the kernel start
  double (*mscr)[kMonoStride];   // __shared__ this wave's [8][kMonoStride] transpose rows

  // slot base + i of one evaluation's monomial values (i counts from 0: the chunk of eight
  // rows is reduced when its last row is written, i known at compile time after unrolling)
  __device__ inline void mono_put(int base, int i, double v) {
    mscr[i & 7][threadIdx.x & 63] = active ? v : 0.0;
    if ((i & 7) == 7) mono_chunk(base + (i & ~7), 8);
  }
  __device__ inline void mono_flush(int base, int n) {
    if (n & 7) mono_chunk(base + (n & ~7), n & 7);
  }
  __device__ inline void mono_chunk(int slot, int rows) {
    const int lane = threadIdx.x & 63, row = lane >> 3, c0 = lane & 7;
    __builtin_amdgcn_wave_barrier();  // (LDS operations of a wave complete in order)
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) v += mscr[row][c0 + 8 * k];
    v = group8_sum(v);
    if (c0 == 0 && row < rows) bpart[slot + row][threadIdx.x >> 6] += v;
    __builtin_amdgcn_wave_barrier();
  }

  __device__ inline void emit(int slot, double v, bool first) {
    if (!cst(j.need)[slot]) return;  // uniform
    const double w = wave_sum(active ? v : 0.0);
    (void)first;  // the LDS entries start at zero: 0 + w == w
    if ((threadIdx.x & 63) == 0) bpart[slot][threadIdx.x >> 6] += w;
  }
  __device__ inline double* tape_at(int64_t row) const { return j.tape + row * n_rays + r_ld; }
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
  AArgs jm = j;
  jm.mono_on = mono_enabled(j);
  if constexpr ((KM & ort::KM_ZERN) != 0) {
    __shared__ double mscr[kBlock / 64][8][kMonoStride];
    if constexpr (kZAcc > 0) {
      __shared__ double zacc[kZAcc > 0 ? kZAcc : 1][kBlock];
      DevLane ln{jm, active ? rid : 0, a.n_rays, rid >> 6, active, zacc, bpart_s,
                 mscr[threadIdx.x >> 6]};
      adj_ray<KM, P, RES>(a, jm, ln, rid, active);
    } else {
      DevLane ln{jm, active ? rid : 0, a.n_rays, rid >> 6, active, nullptr, bpart_s,
                 mscr[threadIdx.x >> 6]};
      adj_ray<KM, P, RES>(a, jm, ln, rid, active);
    }
  } else {
    DevLane ln{jm, active ? rid : 0, a.n_rays, rid >> 6, active, nullptr, bpart_s, nullptr};
    adj_ray<KM, P, RES>(a, jm, ln, rid, active);
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
