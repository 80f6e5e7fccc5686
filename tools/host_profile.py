"""cProfile of a bench config's host side on the GPU box (which Python calls fill the gaps
between kernels): python tools/host_profile.py --config 5 --steps 20."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import argparse  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rays", type=int, default=1_000_000)
    ap.add_argument("--out", default="gpurun_out/host_profile.txt")
    a = ap.parse_args()
    args = argparse.Namespace(rays=a.rays, newton_mode="reference", gpus=1)
    dev = torch.device("cuda:0")
    wl = bench.CONFIGS[a.config](args, dev, 0, 1, torch)
    for _ in range(3):
        wl.step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        wl.step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(60)
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(40)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        f.write(s.getvalue())
    print("steps", a.steps, "written", a.out)


if __name__ == "__main__":
    main()
