/*
 * optiland_host.h -- C ABI of the host (CPU) build of the trace core: the CPU dispatch key
 * of the torch custom op torch.ops.ort.trace_sequential and of its VJP (SURVEY.md 8b:
 * "registered for the CUDA(HIP) and CPU dispatch keys").
 *
 * It replaces the same reference interfaces as ort_trace_sequential / ort_trace_pupil /
 * ort_rms_spot (optiland_rt.h):
 *   optiland/surfaces/surface_group.py:232-244      SurfaceGroup.trace(rays, skip)
 *   optiland/surfaces/standard_surface.py:186-233   Surface.trace (real-ray branch)
 * for rays held in HOST memory -- the reference's own default (backend/torch_backend.py:
 * 66-77 device "cpu"; its test fixture tests/conftest.py:5-19 runs the torch backend on the
 * CPU), and its backward under autograd (optimization/optimizer/torch/base.py:116-131).
 *
 * Same structs as optiland_rt.h, every pointer a HOST pointer. The per-ray arithmetic is
 * the GPU kernels' own source (csrc/ort_core.h, ort_interact.h, ort_material.h, and the
 * derivative sweeps of csrc/ort_sweep.h) compiled with g++ -ffp-contract=off, so a trace
 * gives the GPU's bits. Newton surfaces follow the reference's global stop rule
 * (newton_raphson.py:137-166: stop when max |f| < tol over the rays of one trace call)
 * directly: every Newton group (batch->group_len rays) is stepped in lockstep, as the
 * reference evaluates it, and the update counts it made are written to `updates`. Calls
 * are synchronous; OpenMP threads split the rays (results do not depend on the thread
 * count: every reduction runs in a fixed order).
 */
#ifndef OPTILAND_HOST_H
#define OPTILAND_HOST_H

#include "optiland_rt.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORT_HOST_ABI_VERSION 2

int ort_host_abi_version(void);

/* ort_trace_sequential on host memory. updates (nullable): int32 [n_groups][n_surfaces],
 * the Newton updates the reference's stop rule made per (group, surface) (0 for closed-form
 * surfaces) -- the schedule ort_host_trace_sequential_vjp replays. opt->sched and
 * opt->newton_mode are ignored (the stop rule is evaluated exactly); opt->start_surface is
 * the SurfaceGroup.trace skip. status (nullable): ort_status bits (Zernike / Chebyshev
 * range errors, unknown geometry). rays_out may alias rays_in. Returns 0 or an ort_error. */
int ort_host_trace_sequential(const ort_lens* lens, const ort_rays* rays_in,
                              ort_rays* rays_out, const ort_batch* batch,
                              const ort_options* opt, double* rec, int32_t* updates,
                              int32_t* status);

/* ort_trace_sequential_vjp on host memory, with the same parameters (ADJOINT or UNROLLED
 * mode; params->workspace unused: the host allocates its own scratch; params->slot_need
 * nullable). opt->sched: the `updates` the primal host trace reported. */
int ort_host_trace_sequential_vjp(const ort_lens* lens, const ort_rays* rays_in,
                                  const ort_batch* batch, const ort_options* opt,
                                  const ort_vjp_params* params, const ort_rays* cotangent,
                                  const double* rec_cotangent, const double* rec,
                                  double* grad, const ort_rays* grad_in);

/* ort_trace_pupil on host memory (v2): rays generated from the pupil samples px, py by the
 * batch's segments (ray r of segment r / seg_len; pupil sample r with pupil_per_ray, else
 * r - segment * seg_len; ray_generator.py:28-106 through the GPU's generate_ray), then
 * traced in Newton groups of batch->group_len rays with the reference's stop rule as in
 * ort_host_trace_sequential (updates: [n_groups][n_surfaces]). No records, no start surface,
 * no per-ray wavelengths; n_rays must be n_seg * seg_len. Replaces RealRayTracer.trace
 * (raytrace/real_ray_tracer.py:37-97) for host tensors. */
int ort_host_trace_pupil(const ort_lens* lens, const double* px, const double* py,
                         ort_rays* rays_out, const ort_batch* batch, const ort_options* opt,
                         int32_t* updates, int32_t* status);

/* ort_trace_pupil_vjp on host memory (v2): the adjoint / forward-mode sweeps of the pupil
 * trace (generation included, not differentiated), opt->sched = the primal's updates. */
int ort_host_trace_pupil_vjp(const ort_lens* lens, const double* px, const double* py,
                             const ort_batch* batch, const ort_options* opt,
                             const ort_vjp_params* params, const ort_rays* cotangent,
                             double* grad);

/* ort_rms_spot / ort_rms_spot_vjp on host memory (v2): RayOperand.rms_spot_size
 * (optimization/operand/ray.py:300-340), stats = n, mean x, mean y, rms, max radius; sums in
 * index order. */
int ort_host_rms_spot(const double* x, const double* y, int64_t n, double* stats, double* rms);
int ort_host_rms_spot_vjp(const double* x, const double* y, int64_t n, const double* stats,
                          const double* grad_out, double* gx, double* gy);

/* threads used by the calls (OpenMP; <= 0: the OpenMP default) */
void ort_host_set_threads(int32_t n);

#ifdef __cplusplus
}
#endif
#endif /* OPTILAND_HOST_H */
