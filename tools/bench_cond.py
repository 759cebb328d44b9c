"""Timing of the condition stage (pd_cond_forward) on the GPU, per launch tag.

    python tools/bench_cond.py [--batch B] [--tokens N] [--dtype fp32|bf16] [--iters K]

Synthetic handler-config teacher (H=256, 4 FFT layers, 2 heads, k=9), N tokens per
utterance with durations 1..12 frames.  Prints one JSON line: ms per call, the
per-tag HIP-event table, algorithmic FLOPs and weight bytes per call."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from prodiff_amd import _lib, synth  # noqa: E402
from prodiff_amd.teacher import ProDiffTeacher  # noqa: E402


def cond_flops(B, Tt, Tm, H=256, L=4, k=9):
    rows = B * Tt
    per_layer = 2 * rows * H * 3 * H + 2 * 2 * B * Tt * Tt * H + 2 * rows * H * H + 2 * rows * H * 4 * H * k \
        + 2 * rows * 4 * H * H
    return L * per_layer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--tokens", type=int, default=120)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    hp = dict(synth.COND_DEFAULTS, num_spk=4, num_langs=3)
    V = 64
    rhp = dict(hp, audio_num_mel_bins=128, languages=["zh", "jp"], residual_layers=1, residual_channels=64,
               dilation_cycle_length=1, timesteps=4, timescale=1000, schedule_type="vpsde", max_beta=40.0,
               spec_min=[-12], spec_max=[0])
    t = ProDiffTeacher(V, rhp)
    P = synth.synth_cond_params(synth.cond_param_shapes(V, **hp), 0)
    t.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()}, strict=False)
    t = t.cuda().set_compute_dtype(a.dtype)
    x = synth.synth_cond_inputs(7, [a.tokens] * a.batch, V, 4, 3)
    # equal mel length per batch (the denoiser's constraint): trim to the shortest utterance
    Tm = int((x["mel2ph"] > 0).sum(1).min())
    for k in ("mel2ph", "f0", "voicing", "breath"):
        x[k] = x[k][:, :Tm]
    g = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in x.items()}
    args = (g.pop("txt_tokens"), g.pop("mel2ph"), g.pop("f0"))
    for _ in range(3):
        t.forward_condition(*args, **g)
    torch.cuda.synchronize()
    _lib.profile_enable(True)
    t.forward_condition(*args, **g)
    torch.cuda.synchronize()
    prof = _lib.profile_summary()
    _lib.profile_enable(False)
    t0 = time.perf_counter()
    for _ in range(a.iters):
        t.forward_condition(*args, **g)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.iters * 1e3
    fl = cond_flops(a.batch, a.tokens, Tm)
    wbytes = sum(v.size for v in P.values()) * (2 if a.dtype == "bf16" else 4)
    print(json.dumps({"what": "pd_cond_forward", "dtype": a.dtype, "batch": a.batch, "tokens": a.tokens,
                      "mel_frames": Tm, "ms_per_call": round(ms, 4), "gflop": round(fl / 1e9, 3),
                      "tflops": round(fl / ms / 1e9, 2), "weight_MB": round(wbytes / 1e6, 2),
                      "kernels_us": {k: round(v[1] * 1e3 / v[0], 2) for k, v in prof.items()},
                      "launches": {k: v[0] for k, v in prof.items()}}), flush=True)


if __name__ == "__main__":
    main()
