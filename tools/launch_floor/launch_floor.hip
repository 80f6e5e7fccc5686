// Launch-floor experiment (measurement tooling, not product): the device time of a
// dependent launch that returns at once, as a function of one property at a time -- the
// grid (64 .. 3,907 workgroups of 256), the kernel-argument size (8 B vs a 512 B struct by
// value), a 4 KB static LDS array with a 4-entry-per-thread prefetch into it, and the
// register allocation (a large body behind a branch that is never taken). Every variant
// runs N dependent launches captured in one hipGraph (as config 5's step is), replayed R
// times; per launch = replay time / N. VERDICT r05 item 3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

struct Big {  // ~ the trace kernel's KArgs (a few hundred bytes by value)
  const int* flag;
  int* out;
  double pad[62];
};

__global__ __launch_bounds__(256) void k_empty(const int* flag) { (void)flag; }

__global__ __launch_bounds__(256) void k_flag(const int* flag, int* out) {
  if (*flag != 1) return;
  out[blockIdx.x * 256 + threadIdx.x] = 1;
}

__global__ __launch_bounds__(256) void k_big(const Big a) {
  if (*a.flag != 1) return;
  a.out[blockIdx.x * 256 + threadIdx.x] = (int)a.pad[threadIdx.x & 31];
}

// the verify round's prologue: 4 schedule entries per thread loaded with the flag
__global__ __launch_bounds__(256) void k_lds(const int* flag, const int* sched, int* out) {
  __shared__ int vs[1024];
  int pre[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pre[q] = sched[threadIdx.x + q * 256];
  if (*flag != 1) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) vs[threadIdx.x + q * 256] = pre[q];
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = vs[(threadIdx.x * 7) & 1023];
}

// the flag test in front of a register-hungry body (never run: flag != 1)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void k_heavy(const int* flag, const double* in, double* out) {
  if (*flag != 1) return;
  double acc[96];
  const int t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 96; ++k) acc[k] = in[t + k * 4096];
#pragma unroll
  for (int it = 0; it < 8; ++it)
#pragma unroll
    for (int k = 0; k < 96; ++k) acc[k] = acc[k] * acc[(k + 17) % 96] + acc[(k + 5) % 96];
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 96; ++k) s += acc[k];
  out[t] = s;
}

// a chain of launches in which each reads what the previous one wrote (the verify
// rounds' protocol: round r reads round r - 1's flag, its schedule copy): the flag word of
// launch i - 1 and (sched_words > 0) a 4 KB schedule block 0 of launch i - 1 wrote
__global__ __launch_bounds__(256) void k_chain(const int* prev_flag, int* my_flag,
                                               const int* prev_sched, int* my_sched,
                                               int sched_words) {
  int pre[4] = {0, 0, 0, 0};
  if (sched_words > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) pre[q] = prev_sched[threadIdx.x + q * 256];
  }
  const int f = *prev_flag;
  if (blockIdx.x == 0) {
    if (sched_words > 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) my_sched[threadIdx.x + q * 256] = pre[q];
    }
    if (threadIdx.x == 0) *my_flag = f;
  }
}

// the flag test in front of a LARGE body (~10K instructions, as the trace kernels'): does
// the code size of a kernel cost its no-op launches anything (instruction fetch)?
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void k_huge(const int* flag, const double* in, double* out) {
  if (*flag != 1) return;
  double acc[32];
  const int t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 32; ++k) acc[k] = in[t + k * 4096];
#pragma unroll
  for (int it = 0; it < 300; ++it)
#pragma unroll
    for (int k = 0; k < 32; ++k) acc[k] = acc[k] * acc[(k + it) % 32] + in[(it * 32 + k) & 4095];
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 32; ++k) s += acc[k];
  out[t] = s;
}

template <class F>
static double per_launch_us(F launch, int N, int R, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < N; ++i) launch(st);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < R; ++i) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1e3 / ((double)N * R);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int *flag, *sched, *out;
  double *din, *dout;
  const size_t nmax = 4096 * 256;
  CK(hipMalloc(&flag, sizeof(int)));
  CK(hipMemset(flag, 0, sizeof(int)));  // never 1: every variant returns at once
  CK(hipMalloc(&sched, 1024 * sizeof(int)));
  CK(hipMemset(sched, 0, 1024 * sizeof(int)));
  CK(hipMalloc(&out, nmax * sizeof(int)));
  CK(hipMalloc(&din, (nmax + 96 * 4096) * sizeof(double)));
  CK(hipMalloc(&dout, nmax * sizeof(double)));
  Big big;
  std::memset(&big, 0, sizeof big);
  big.flag = flag;
  big.out = out;
  const int N = 100, R = 20;
  const unsigned grids[] = {64, 256, 1024, 3907};
  std::printf("{\"N\": %d, \"R\": %d, \"sizeof_big\": %zu, \"rows\": [\n", N, R, sizeof(Big));
  bool first = true;
  for (unsigned G : grids) {
    struct V { const char* name; double us; };
    V v[6];
    v[0] = {"empty", per_launch_us([&](hipStream_t s) { hipLaunchKernelGGL(k_empty, dim3(G), dim3(256), 0, s, flag); }, N, R, st)};
    v[1] = {"flag", per_launch_us([&](hipStream_t s) { hipLaunchKernelGGL(k_flag, dim3(G), dim3(256), 0, s, flag, out); }, N, R, st)};
    v[2] = {"big_args", per_launch_us([&](hipStream_t s) { hipLaunchKernelGGL(k_big, dim3(G), dim3(256), 0, s, big); }, N, R, st)};
    v[3] = {"lds_prefetch", per_launch_us([&](hipStream_t s) { hipLaunchKernelGGL(k_lds, dim3(G), dim3(256), 0, s, flag, sched, out); }, N, R, st)};
    v[4] = {"heavy_regs", per_launch_us([&](hipStream_t s) { hipLaunchKernelGGL(k_heavy, dim3(G), dim3(256), 0, s, flag, din, dout); }, N, R, st)};
    v[5] = {"huge_code", per_launch_us([&](hipStream_t s) { hipLaunchKernelGGL(k_huge, dim3(G), dim3(256), 0, s, flag, din, dout); }, N, R, st)};
    for (auto& x : v) {
      std::printf("%s {\"grid\": %u, \"kernel\": \"%s\", \"us_per_launch\": %.3f}", first ? " " : ",\n ", G, x.name, x.us);
      first = false;
    }
  }
  // the chains: N launches, launch i reading slot i - 1 and writing slot i
  int *flags, *scheds;
  CK(hipMalloc(&flags, (N + 1) * 64 * sizeof(int)));  // one 256 B line per flag
  CK(hipMemset(flags, 0, (N + 1) * 64 * sizeof(int)));
  CK(hipMalloc(&scheds, (size_t)(N + 1) * 1024 * sizeof(int)));
  CK(hipMemset(scheds, 0, (size_t)(N + 1) * 1024 * sizeof(int)));
  for (unsigned G : grids) {
    for (int sw : {0, 1024}) {
      const double us = per_launch_us([&](hipStream_t s) {
        static int i = 0;
        const int k = i++ % N;
        hipLaunchKernelGGL(k_chain, dim3(G), dim3(256), 0, s, flags + k * 64, flags + (k + 1) * 64,
                           scheds + (size_t)k * 1024, scheds + (size_t)(k + 1) * 1024, sw);
      }, N, R, st);
      std::printf(",\n {\"grid\": %u, \"kernel\": \"%s\", \"us_per_launch\": %.3f}", G,
                  sw ? "chain_flag_sched" : "chain_flag", us);
    }
  }
  std::printf("\n]}\n");
  return 0;
}
