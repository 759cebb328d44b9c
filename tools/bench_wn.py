"""WaveNet denoiser forward timing on the GPU (bf16 residual-layer kernel variants).

    python tools/bench_wn.py [--batch 8] [--frames 861] [--layer 0|1|2|3] [--iters 20] [--cyc 1]

Random-init WaveNet 20x256 (M=80, H=256).  Prints one JSON line: ms per forward and the
per-tag HIP-event table of one profiled forward.  Run under `rocprofv3 --kernel-trace --stats`
for exact per-kernel durations."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from prodiff_amd import WaveNet, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--frames", type=int, default=861)
    ap.add_argument("--layer", type=int, default=2)
    ap.add_argument("--cyc", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    net = WaveNet(80, 256, 20, 256, a.cyc)
    net = net.cuda().set_compute_dtype("bf16").set_options(layer=a.layer)
    B, T = a.batch, a.frames
    spec = torch.randn(B, 1, 80, T, device="cuda")
    cond = torch.randn(B, 256, T, device="cuda")
    steps = torch.full((B,), 3.0, device="cuda")
    for _ in range(3):
        net(spec, steps, cond)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        net(spec, steps, cond)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.iters
    _lib.profile_enable(True)
    net(spec, steps, cond)
    torch.cuda.synchronize()
    prof = _lib.profile_summary()
    _lib.profile_enable(False)
    print(json.dumps({"batch": B, "frames": T, "layer": a.layer, "ms_per_forward": round(ms, 3),
                      "kernels": {k: {"launches": n, "avg_us": round(t * 1e3 / n, 2)} for k, (n, t) in prof.items()}}))


if __name__ == "__main__":
    main()
