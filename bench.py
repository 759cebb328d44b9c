#!/usr/bin/env python
"""ProDiff 2-iter + FastDiff 4-iter end-to-end synthesis throughput on MI355X.

One step = one pass of the hot path over one batch per GPU: the ProDiff x0-predict
sampler (WaveNet 20x256, M=80, 2 reverse steps) turns cond [B,861,256] into mel
[B,861,80], the FastDiff sampler (base.yaml, 4 reverse steps) turns that into
wav [B,220416] (10 s at 22.05 kHz, hop 256).  For N>1 every rank runs its own
shard (weak scaling, no data-path collective) and the step ends with the
point-to-point gather of mel+wav to rank 0 (RCCL over xGMI).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--frames T]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.  Synthetic inputs and random-init weights of the
reference architectures (no checkpoints or datasets offline).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "mel-frames/sec + audio RTF, 2-iter ProDiff + 4-iter FastDiff @1/2/4/8 GPU"
FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, dense
BF16_PEAK_TFLOPS = 2500.0    # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (no sparsity)
HBM_PEAK_GBS = 8000.0


def flops_per_launch(B, T, hops=(8, 64, 256), M=80, C=256, H=256):
    """Algorithmic FLOPs (2 x MAC) of ONE launch of each tagged kernel.
    Tags used by several block sizes report the mean over their launches in one call."""
    F = B * T
    rows = [F * h for h in hops]
    d_rows = [F * 64, F * 8, F]                       # DBlock output rates (L/4, L/32, L/256)
    dblock = sum(2 * r * 32 * 96 * 2 + 2 * r * 32 * 128 for r in d_rows) / 9.0
    return {
        "wn_inproj": 2 * F * M * C,
        "wn_gate": 2 * F * 2 * C * (3 * C + H),
        "wn_resskip": 2 * F * 2 * C * C,
        "wn_layer": 2 * F * 2 * C * (3 * C + H) + 2 * F * 2 * C * C,     # fused gate + res/skip (bf16)
        "wn_skiphead": 2 * F * C * C,
        "wn_outproj_posterior": 2 * F * M * C,
        "fd_first_conv": 2 * F * 256 * 32 * 7,
        "fd_dblock": dblock,
        "fd_dblock_fused": dblock * 3.0,                    # all 3 convs + residual of one DBlock
        "fd_kp_in": 2 * F * 64 * 80 * 5,
        "fd_kp_res": 2 * F * 64 * 64 * 3,
        "fd_kp_bias": 2 * F * 256 * 64 * 3,
        "fd_kp_kernel": 2 * F * 6144 * 64 * 3,
        "fd_upsample": sum(2 * r * 32 * 64 for r in rows) / 3.0,
        "fd_lvc_preconv": sum(2 * r * 32 * 96 for r in rows) / 3.0,
        "fd_lvc": sum(2 * r * 64 * 96 for r in rows) / 3.0,
        # fused pre-conv + LVC, launched for the hop >= 64 blocks only (bf16 path)
        "fd_lvc_fused": sum(2 * r * 32 * 96 + 2 * r * 64 * 96 for r in rows[1:]) / 2.0,
        # whole LVC block (4 layers of pre-conv + LVC), hop >= 64 blocks (bf16 path)
        "fd_lvc_block": sum(4 * (2 * r * 32 * 96 + 2 * r * 64 * 96) for r in rows[1:]) / 2.0,
        "fd_final_update": 2 * F * 256 * 32 * 7,
        # whole LVC block with the upsample fused (hop-64 block, r = 8)
        "fd_lvc_block_ups": rows[1] * (4 * (2 * 32 * 96 + 2 * 64 * 96) + 2 * 2 * 32 * 32),
        # hop-8 block (several frames per 32-row tile), upsample fused (r = 8)
        "fd_lvc_block_sub": rows[0] * (4 * (2 * 32 * 96 + 2 * 64 * 96) + 2 * 2 * 32 * 32),
        # hop-256 block with upsample (r = 4), first conv and final conv + update fused
        "fd_lvc_block_final": rows[2] * (4 * (2 * 32 * 96 + 2 * 64 * 96) + 2 * 2 * 32 * 32 + 2 * 2 * 7 * 32),
    }


def bytes_per_launch(B, T, dtype, hops=(8, 64, 256), M=80, C=256, H=256):
    """Compulsory HBM bytes of ONE launch of each tagged kernel with the layouts the
    kernels use (activations fp32 time-major; weights and LVC kernels bf16 in the
    bf16 path, fp32 otherwise).  Mean over launches where the block size varies."""
    F = B * T
    wb = 2 if dtype == "bf16" else 4
    rows = [F * h for h in hops]
    per_row_io = 32 * 4
    kf_frame = 6144 * wb + 256 * 4
    # fused LVC (hop >= 64): x read+write, audio_down read, this layer's kernels+biases
    lvc_f = [r * 3 * per_row_io + F * kf_frame for r in rows[1:]]
    lvc_v = [r * 4 * per_row_io + F * kf_frame for r in rows]          # unfused: x r/w, a, y
    return {
        "wn_inproj": F * (M + C) * 4 + C * M * wb,
        "wn_gate": F * (C + H + C) * 4 + 2 * C * (3 * C + H) * wb,
        "wn_resskip": F * (C + 2 * C + 2 * C) * 4 + 2 * C * C * wb,
        "wn_layer": F * (C + H + C + 2 * C) * 4 + 2 * C * (4 * C + H) * wb,
        "wn_skiphead": F * 2 * C * 4 + C * C * wb,
        "wn_outproj_posterior": F * (C + 3 * M) * 4 + M * C * wb,
        "fd_first_conv": F * 256 * (1 + 32) * 4,
        # fused DBlock: strided input rows (32 ch) read once + output written once
        "fd_dblock_fused": sum(r * 2 * per_row_io for r in (F * 64, F * 8, F)) / 3.0,
        "fd_kp_kernel": F * (64 * 4 + 6144 * wb) + 6144 * 192 * wb,
        "fd_kp_hidden": F * (80 + 64 + 256) * 4 + (64 * 480 + 6 * 64 * 192 + 256 * 192) * wb,
        "fd_lvc_fused": sum(lvc_f) / 2.0,
        # x in + a in + x out once per block, plus all 4 layers' kernels and biases
        "fd_lvc_block": sum(r * 3 * per_row_io + F * 4 * kf_frame for r in rows[1:]) / 2.0,
        "fd_lvc": sum(lvc_v) / 3.0,
        "fd_upsample": sum(r * (1 + 1.0 / h) * per_row_io for r, h in zip(rows, (8, 8, 4))) / 3.0,
        "fd_final_update": F * 256 * (32 + 3) * 4,
        # x_prev (r = 8 fewer rows) + audio_down in, x out, the 4 layers' kernels + biases
        "fd_lvc_block_ups": rows[1] / 8 * per_row_io + rows[1] * 2 * per_row_io + F * 4 * kf_frame,
        "fd_lvc_block_sub": rows[0] / 8 * per_row_io + rows[0] * 2 * per_row_io + F * 4 * kf_frame,
        # x_prev (r = 4 fewer rows) + audio sample in + new audio sample out, kernels + biases
        "fd_lvc_block_final": rows[2] / 4 * per_row_io + rows[2] * 2 * 4 + F * 4 * kf_frame,
    }


# bench tag -> kernel symbol (the default tile sizes) for the PMC traffic lookup
TAG_KERNEL = {
    "fd_lvc_block_final": "lvc_block_bf16_kernel<384, true, true, true, true, false>",
    "fd_lvc_block_ups": "lvc_block_bf16_kernel<384, true, false, false, true, false>",
    "fd_lvc_block_sub": "lvc_block_bf16_kernel<128, true, false, false, false, true>",
    "fd_kp_kernel": "kp_kernel_bf16_kernel",
    "wn_layer": "wn_layer_bf16_kernel",
}


def pmc_traffic(tag, path=None):
    """HBM bytes per launch of `tag`'s kernel from the newest committed PMC summary
    (profiles/rNN_vMM_traffic.json, written by tools/pmc_traffic.py from separate
    FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this bench command).  None if absent."""
    import glob
    import re
    if path is None:
        def ver(f):
            m = re.search(r"r(\d+)_v(\d+)_traffic\.json$", f)
            return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_v*_traffic.json")), key=ver)
        if not files:
            return None, None
        path = files[-1]
    sym = TAG_KERNEL.get(tag)
    if sym is None or not os.path.exists(path):
        return None, None
    with open(path) as f:
        kern = json.load(f)["kernels"]
    for name, v in kern.items():
        if sym in name:
            return float(v["traffic_bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


def step_flops(B, T):
    """Whole-step algorithmic FLOPs: 2 x 26.43 + 4 x 56.98 MFLOP per frame."""
    f = flops_per_launch(B, T)
    per_prodiff_step = f["wn_inproj"] + 20 * (f["wn_gate"] + f["wn_resskip"]) + f["wn_skiphead"] + \
        f["wn_outproj_posterior"]
    per_fd_call = f["fd_first_conv"] + 9 * f["fd_dblock"] + 3 * (f["fd_kp_in"] + 6 * f["fd_kp_res"] +
                                                             f["fd_kp_bias"] + 4 * f["fd_kp_kernel"] +
                                                             f["fd_upsample"] + 4 * f["fd_lvc_preconv"] +
                                                             4 * f["fd_lvc"]) + f["fd_final_update"]
    return 2 * per_prodiff_step + 4 * per_fd_call


def cpu_baseline(frames=200):
    """The numpy oracle (a CPU port of the reference math, float64) on a bounded
    sample: ONE utterance of `frames` mel frames through the same 2+4-iter pipeline."""
    from oracle import oracle_fastdiff as OF
    from oracle import oracle_prodiff as OP
    from prodiff_amd import schedules as S
    from prodiff_amd import synth
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
    except Exception:
        cores = int(os.environ.get("OMP_NUM_THREADS", "1"))
    p = synth.synth_params(synth.wavenet_param_shapes(80, 256, 20, 256), 0)
    bufs = OP.diffusion_buffers(OP.vpsde_betas(2, 40.0))
    bufs["timesteps"] = 2
    fp = OF.fold_weight_norm(synth.synth_params(synth.fastdiff_param_shapes(), 1))
    b, a, s, st = S.fastdiff_infer_params(S.fastdiff_reverse_schedule(4), S.fastdiff_train_alpha())
    cond = synth.synth_inputs(0, (1, frames, 256))
    t0 = time.perf_counter()
    mel = OP.prodiff_sample(p, bufs, cond, synth.synth_inputs(1, (1, 1, 80, frames), kind="uniform"),
                            synth.synth_inputs(2, (2, 1, 1, 80, frames)))
    OF.fastdiff_sample(fp, np.transpose(mel, (0, 2, 1)), synth.synth_inputs(3, (1, 1, frames * 256)),
                       synth.synth_inputs(4, (3, 1, 1, frames * 256)), b, a, s, st)
    dt = time.perf_counter() - t0
    return {"value": round(frames / dt, 3), "unit": "mel-frames/s", "cores": int(cores), "kind": "port",
            "sample": f"numpy float64 oracle, 1 utterance x {frames} frames ({frames * 256 / 22050:.2f} s audio), "
                      f"2-iter ProDiff + 4-iter FastDiff, {dt:.1f} s wall",
            "rtf": round(dt / (frames * 256 / 22050), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=8, help="utterances per GPU (C3: 8)")
    ap.add_argument("--frames", type=int, default=861, help="mel frames per utterance (10 s @ 22.05 kHz/256)")
    ap.add_argument("--cpu-frames", type=int, default=200, help="cpu_baseline sample length (0 = skip)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="compute dtype (C3 is specified in bf16; fp32 is the exact parity path)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--prof-steps", type=int, default=2,
                    help="untimed steps with every launch bracketed by HIP events (the `kernels` table)")
    ap.add_argument("--traffic", default=None, help="PMC traffic summary (default: newest profiles/r*_v*_traffic.json)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from prodiff_amd import _lib
    from prodiff_amd.pipeline import HOP, SAMPLE_RATE, Synthesizer, gather_to_root

    B, T = args.batch, args.frames
    syn = Synthesizer.synthetic(dev, seed=0, dtype=args.dtype)
    cond = torch.from_numpy(np.random.default_rng(1000 + rank).standard_normal((B, T, 256), dtype=np.float32)).to(dev)

    def step(i):
        mel, wav = syn(cond, seed=10_000 * rank + i)
        if world > 1:
            gather_to_root(mel)
            gather_to_root(wav)
        return mel, wav

    fl = flops_per_launch(B, T)
    by = bytes_per_launch(B, T, args.dtype)
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    # Kernel timing.  An event pair costs GPU time at every launch it brackets (about
    # 0.7 ms per step over all ~100 launches), so the per-kernel table comes from an
    # untimed pass with every launch recorded, and the timed region records only the
    # dominant kernel (the roofline's `avg_launch_us`, measured live in the timed steps).
    timing = not args.no_kernel_timing
    kern_all, dom, nprof = {}, None, 0
    if timing:
        nprof = max(1, args.prof_steps)
        _lib.profile_filter(None)
        _lib.profile_enable(True)
        for i in range(nprof):
            step(args.warmup + i)
        torch.cuda.synchronize()
        kern_all = _lib.profile_summary()
        _lib.profile_enable(False)
        known = {k: v for k, v in kern_all.items() if k in fl and k in by}
        dom = max(known.items(), key=lambda kv: kv[1][1])[0]
        _lib.profile_filter([dom])
        _lib.profile_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        mel, wav = step(args.warmup + nprof + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern = _lib.profile_summary() if timing else {}
    _lib.profile_enable(False)
    _lib.profile_filter(None)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    assert torch.isfinite(wav).all() and torch.isfinite(mel).all()

    frames = B * T * world * args.steps
    audio_s = frames * HOP / SAMPLE_RATE
    ms_step = dt / args.steps * 1e3
    peak_tf = BF16_PEAK_TFLOPS if args.dtype == "bf16" else FP32_PEAK_TFLOPS
    ridge = peak_tf * 1e12 / (HBM_PEAK_GBS * 1e9)          # FLOP/B where MFMA and HBM bounds meet
    roofline, kernels = None, {}
    if kern:
        for tag, (cnt, ms) in sorted(kern_all.items(), key=lambda kv: -kv[1][1]):
            sec = ms * 1e-3
            kernels[tag] = {"launches": cnt, "ms_total": round(ms, 3), "avg_us": round(ms / cnt * 1e3, 2),
                            "tflops": round(fl.get(tag, 0.0) * cnt / sec / 1e12, 2) if ms > 0 else 0.0,
                            "gbs": round(by.get(tag, 0.0) * cnt / sec / 1e9, 1) if ms > 0 else 0.0}
        cnt, ms = kern[dom]
        sec = ms * 1e-3
        intensity = fl[dom] / by[dom] if by.get(dom) else float("inf")
        if intensity < ridge:      # HBM-bound at its compulsory bytes
            ach = by[dom] * cnt / sec / 1e9
            roofline = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4)}
        else:
            ach = fl[dom] * cnt / sec / 1e12
            roofline = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak_tf, "unit": "TFLOP/s",
                        "frac": round(ach / peak_tf, 4)}
        traffic, tsrc = pmc_traffic(dom, args.traffic)
        roofline.update({"traffic": round(traffic) if traffic else None, "traffic_source": tsrc, "kernel": dom, "flop_per_launch": fl[dom],
                         "bytes_per_launch": by.get(dom), "intensity_flop_per_byte": round(intensity, 1),
                         "ridge_flop_per_byte": round(ridge, 1), "avg_launch_us": round(ms / cnt * 1e3, 2),
                         "launches": cnt, "share_of_step": round(ms / (dt * 1e3), 3),
                         "timing": "HIP events around this kernel only, over the timed steps"})
    out = {
        "metric": METRIC,
        "value": round(frames / dt, 1),
        "unit": "mel-frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (cond ~ N(0,1)); random-init weights of the reference architectures; on-device Philox draws",
        "config": {"workload": f"C3: ProDiff 2-iter (WaveNet 20x256, M=80, vpsde max_beta 40) + FastDiff 4-iter "
                               f"(base.yaml, hop 256), {B} x {T}-frame utterances per GPU",
                   "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world} (utterance shards, "
                                                                           f"RCCL gather to rank 0)"},
        "rtf": round(dt / audio_s, 6),
        "x_realtime": round(audio_s / dt, 1),
        "model_tflops": round(step_flops(B, T) * world * args.steps / dt / 1e12, 2),
        "roofline": roofline,
        "kernels": kernels,
        "kernels_source": f"untimed pass of {nprof} steps, every launch bracketed by HIP events",
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.cpu_frames > 0:
        out["cpu_baseline"] = cpu_baseline(args.cpu_frames)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
