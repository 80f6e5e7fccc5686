"""Launch-overhead experiment (measurement tooling): DoubleGauss 1M-ray trace, K steps
back to back (a) plain, (b) with per-step HIP events, (c) captured in a HIP graph; plus
the host cost of one trace_pupil call."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from optiland_pr_amd import _native
from optiland_pr_amd.lowering import segment_params
from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil, upload_segments
from optiland_pr_amd.samples import DoubleGauss
from optiland_pr_amd.distribution import RandomDistribution

_native.load()
dev = torch.device("cuda", 0)
lens = DoubleGauss()
dl = lens_for(lens, [0.5876])
R = 1_000_000
d = RandomDistribution(seed=0); d.generate_points(R)
px = torch.as_tensor(np.ascontiguousarray(d.x), device=dev)
py = torch.as_tensor(np.ascontiguousarray(d.y), device=dev)
seg_dev = upload_segments(np.stack([segment_params(lens, 0.0, 1.0, 0)]), dev)
out = RealRays.empty(R, 0.5876, device=dev)
step = lambda: trace_pupil(dl, seg_dev, px, py, out, R, R, R)
for _ in range(10): step()
torch.cuda.synchronize()
K = 200
# host cost per call (the GPU queue absorbs it)
t0 = time.perf_counter()
for _ in range(K): step()
t_host = (time.perf_counter() - t0) / K
torch.cuda.synchronize()
def timed(fn):
    torch.cuda.synchronize(); t0 = time.perf_counter(); fn(); torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e6
a = timed(lambda: [step() for _ in range(K)])
s = torch.cuda.current_stream()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
def with_events():
    for k in range(K):
        ev[k][0].record(s); step(); ev[k][1].record(s)
b = timed(with_events)
kern = np.mean([x.elapsed_time(y) for x, y in ev]) * 1e3
g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    step()
torch.cuda.current_stream().wait_stream(side)
with torch.cuda.graph(g):
    for _ in range(20): step()
torch.cuda.synchronize()
c = timed(lambda: [g.replay() for _ in range(K // 20)])
print(f"host per call {t_host*1e6:.1f} us | plain {a:.1f} us/step | events {b:.1f} us/step "
      f"(kernel {kern:.1f} us) | graph {c:.1f} us/step")
