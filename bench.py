#!/usr/bin/env python
"""ProDiff 2-iter + FastDiff 4-iter end-to-end synthesis throughput on MI355X.

One step = one pass of the hot path over one batch: the ProDiff x0-predict
sampler (WaveNet 20x256, M=80, 2 reverse steps) turns cond [B,861,256] into mel
[B,861,80], the FastDiff sampler (base.yaml, 4 reverse steps) turns that into
wav [B,220416] (10 s at 22.05 kHz, hop 256).  Configurations (BASELINE.json):

  C3   (default at N=1)  8 utterances per GPU, bf16                   weak scaling
  C4   (default at N>1)  32 utterances per GPU (256 at N=8), bf16     weak scaling
  C4S                    256 utterances over all N GPUs, bf16         strong scaling
  C2                     ProDiff 2-iter only, B=1, T=1000, fp32, mel-only (hipGraph replay)
  C5                     SVS path: teacher condition (FFT encoder) + ProDiff 4-iter (M=128) +
                         NSF-HiFiGAN (44.1 kHz, hop 512), 8 segments per GPU (64 at N=8), bf16
  PITCH                  SURVEY §8(f)1: the pitch predictor's sampler (PitchRectifiedFlow, 20 Euler
                         steps of WaveNet 20x256, M=64 repeat bins, dilation cycle 5) + denorm,
                         8 segments x 861 frames, bf16, one GPU

For N>1 every rank runs its LPT shard (pipeline.distributed_synthesize: no
data-path collective) and the step ends with the ragged point-to-point gather of
mel+wav to rank 0 (RCCL over xGMI).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3|C4|C4S|C2]
    torchrun --nproc-per-node N bench.py --gpus N ...

Without torchrun, ``--gpus N`` (N>1) re-launches itself as N ranks under
torch.distributed.run before anything touches the GPU.  ``--dry-run`` runs the
launcher, sharding and gather on CPU/gloo with a stub synthesizer (no GPU).
Rank 0 prints ONE JSON line.  Synthetic inputs and random-init weights of the
reference architectures (no checkpoints or datasets offline).
"""
import argparse
import contextlib
import json
import os
import socket
import subprocess
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
HOP, SAMPLE_RATE = 256, 22050

CONFIGS = {
    # name: (utterances per GPU or global, global?, frames, dtype, vocoder, description)
    "C3": dict(batch=8, strong=False, frames=861, dtype="bf16", vocoder=True, timesteps=2,
               desc="C3: ProDiff 2-iter (WaveNet 20x256, M=80, vpsde max_beta 40) + FastDiff 4-iter "
                    "(base.yaml, hop 256), {b} x {t}-frame utterances per GPU"),
    "C4": dict(batch=32, strong=False, frames=861, dtype="bf16", vocoder=True, timesteps=2,
               desc="C4: 32 x {t}-frame utterances per GPU (256 at N=8), ProDiff 2-iter + FastDiff 4-iter, "
                    "LPT utterance shards + RCCL gather to rank 0"),
    "C4S": dict(batch=256, strong=True, frames=861, dtype="bf16", vocoder=True, timesteps=2,
                desc="C4 strong scaling: {b} x {t}-frame utterances in total over all GPUs, ProDiff 2-iter + "
                     "FastDiff 4-iter, LPT shards + RCCL gather"),
    "C2": dict(batch=1, strong=False, frames=1000, dtype="fp32", vocoder=False, timesteps=2,
               desc="C2: ProDiff 2-iter mel denoiser (WaveNet 20x256, M=80), B={b}, T={t}, fp32, mel only"),
    "C5": dict(batch=8, strong=False, frames=861, dtype="bf16", vocoder=True, timesteps=4, svs=True, tokens=120,
               desc="C5: SVS path (modules/svs) -- ProDiffTeacher condition (FFT encoder, {n} phonemes, speaker mix, "
                    "zh/jp lang ids, voicing/breath) + ProDiff 4-iter (WaveNet 20x256, M=128) + NSF-HiFiGAN "
                    "(44.1 kHz, hop 512), {b} x {t}-frame segments per GPU (64 at N=8)"),
    # the pitch predictor's diffusion (handler/base_config.yaml:135-149 f0_prediction_args: repeat_bins 64,
    # residual_layers 20, residual_channels 256, dilation_cycle_length 5; sampling_algorithm euler :204;
    # infer_step 20, pitch_predictor.py:63,120; reflow.py:86-144)
    "PITCH": dict(batch=8, strong=False, frames=861, dtype="bf16", vocoder=False, timesteps=20, pitch=True, mels=64,
                  cyc=5,
                  desc="PITCH: pitch predictor sampler -- PitchRectifiedFlow, 20 Euler steps of WaveNet 20x256 "
                       "(M = 64 repeat bins, dilation cycle 5) + denorm_spec (mean over the bins, clamp), "
                       "{b} x {t}-frame segments per GPU"),
}


WN_LAYERS, WN_STACK_NL = 20, 10          # residual layers; layers per wn_stack_bf16_kernel launch
WN_STACK_HMAX = 16                        # wavenet.hip WST_HMAX: a launch's dilations sum to at most this
FD_STEPS, FD_BLOCKS = 4, 3                # FastDiff sampler passes per call; LVC blocks (hop 8, 64, 256)


def wn_stack_launches(cyc=1, L=WN_LAYERS, nl_max=WN_STACK_NL, hmax=WN_STACK_HMAX):
    """The stack launches of one denoiser call, as wavenet.hip groups the layers: at most nl_max
    layers per launch whose dilations 2^(l % cyc) sum to at most hmax (cycle 1: 2 launches of 10;
    cycle 5: {1,2,4,8}, {16} four times -- 8 launches)."""
    n, l0 = 0, 0
    while l0 < L:
        nl, s = 0, 0
        while l0 + nl < L and nl < nl_max:
            d = 1 << ((l0 + nl) % cyc)
            if nl > 0 and s + d > hmax:
                break
            s += d
            nl += 1
        l0 += nl
        n += 1
    return n


def flops_per_launch(B, T, dtype="bf16", hops=(8, 64, 256), M=80, C=256, H=256, cyc=1):
    """Algorithmic FLOPs (2 x MAC) of ONE launch of each tagged kernel.
    Tags used by several block sizes report the mean over their launches in one call."""
    F = B * T
    rows = [F * h for h in hops]
    d_rows = [F * 64, F * 8, F]                       # DBlock output rates (L/4, L/32, L/256)
    dblock = sum(2 * r * 32 * 96 * 2 + 2 * r * 32 * 128 for r in d_rows) / 9.0
    kp_layers = 4 if dtype == "bf16" else 1           # bf16: one launch computes all 4 layers' kernels
    gate, resskip = 2 * F * 2 * C * (3 * C + H), 2 * F * 2 * C * C
    nstack = wn_stack_launches(cyc)
    return {
        "wn_inproj": 2 * F * M * C,
        "wn_gate": gate,
        "wn_resskip": resskip,
        # one sampler pass = nstack launches: the first also computes the input projection, the
        # last the skip head + output projection (+ posterior); mean over the pass's launches
        "wn_stack": (WN_LAYERS * (gate + resskip) + 2 * F * M * C + 2 * F * C * C + 2 * F * M * C) / nstack,
        "wn_condb": 0.0,
        # kernel-predictor hidden stacks of every (step, block) of one sampler call in one launch:
        # conv5 80 -> 64, 6 x conv3 64 -> 64, bias conv3 64 -> 256
        "fd_kp_hidden": FD_STEPS * FD_BLOCKS * 2 * F * (64 * 80 * 5 + 6 * 64 * 64 * 3 + 256 * 64 * 3),
        "wn_layer": 2 * F * 2 * C * (3 * C + H) + 2 * F * 2 * C * C,     # fused gate + res/skip (bf16)
        "wn_gate2": 2 * F * 2 * C * (3 * C + H),                            # two-kernel layer (bf16)
        "wn_resskip2": 2 * F * 2 * C * C * 39 / 40,                          # last of 20 layers: skip half only
        "wn_skiphead": 2 * F * C * C,
        "wn_outproj_posterior": 2 * F * M * C,
        "fd_first_conv": 2 * F * 256 * 32 * 7,
        "fd_dblock": dblock,
        "fd_dblock_fused": dblock * 3.0,                    # all 3 convs + residual of one DBlock
        "fd_kp_in": 2 * F * 64 * 80 * 5,
        "fd_kp_res": 2 * F * 64 * 64 * 3,
        "fd_kp_bias": 2 * F * 256 * 64 * 3,
        "fd_kp_kernel": kp_layers * 2 * F * 6144 * 64 * 3,
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


def bytes_per_launch(B, T, dtype, hops=(8, 64, 256), M=80, C=256, H=256, cyc=1):
    """Compulsory HBM bytes of ONE launch of each tagged kernel with the layouts the
    kernels use (activations fp32 time-major; weights and LVC kernels bf16 in the
    bf16 path, fp32 otherwise).  Mean over launches where the block size varies."""
    F = B * T
    wb = 2 if dtype == "bf16" else 4
    rows = [F * h for h in hops]
    per_row_io = 32 * 4
    kf_frame = 6144 * wb + 256 * 4
    kp_layers = 4 if dtype == "bf16" else 1
    # fused LVC (hop >= 64): x read+write, audio_down read, this layer's kernels+biases
    lvc_f = [r * 3 * per_row_io + F * kf_frame for r in rows[1:]]
    lvc_v = [r * 4 * per_row_io + F * kf_frame for r in rows]          # unfused: x r/w, a, y
    layer_w = 2 * C * (4 * C + H) * wb
    nstack = wn_stack_launches(cyc)
    return {
        "wn_inproj": F * (M + C) * 4 + C * M * wb,
        # first launch: spec in, bf16 cond in, x and skip out; last: x and skip in, bf16 cond in,
        # mel read + written (posterior); inner launches (none at 20 layers / 10): x, skip in + out.
        # Plus each launch's layers' weights once (the compulsory HBM bytes; blocks re-read them from L2)
        "wn_stack": (F * (M * 4 + H * 2 + 2 * C * 4) + F * (2 * C * 4 + H * 2 + 2 * M * 4) +
                     max(nstack - 2, 0) * F * (4 * C * 4 + H * 2)) / nstack + WN_LAYERS / nstack * layer_w,
        "wn_condb": F * H * (4 + 2),
        "wn_gate": F * (C + H + C) * 4 + 2 * C * (3 * C + H) * wb,
        "wn_resskip": F * (C + 2 * C + 2 * C) * 4 + 2 * C * C * wb,
        "wn_layer": F * (C + H + C + 2 * C) * 4 + 2 * C * (4 * C + H) * wb,
        # bf16 activations in (xa = x + dp, cond), g out, weights once
        "wn_gate2": F * (C + H + C) * 2 + 2 * C * (3 * C + H) * wb,
        # g in; x read + written, skip read + written (fp32), xa' written
        "wn_resskip2": F * (C * 2 + C * 4 * 2 + C * 4 * 2 + C * 2) + 2 * C * C * wb,
        "wn_skiphead": F * 2 * C * 4 + C * C * wb,
        # two-kernel layer path, once per denoiser call: x + dp and cond (fp32) -> bf16 copies
        "wn_xa": F * (C + H) * (4 + 2),
        "wn_outproj_posterior": F * (C + 3 * M) * 4 + M * C * wb,
        "fd_first_conv": F * 256 * (1 + 32) * 4,
        # fused DBlock: strided input rows (32 ch) read once + output written once
        "fd_dblock_fused": sum(r * 2 * per_row_io for r in (F * 64, F * 8, F)) / 3.0,
        # h in (bf16 / fp32), every layer's 6144 kernel values per frame out, weights once
        "fd_kp_kernel": F * (64 * wb + kp_layers * 6144 * wb) + kp_layers * 6144 * 192 * wb,
        # per (step, block) job: mel in, bf16 h out, fp32 LVC biases out, the block's weights
        "fd_kp_hidden": FD_STEPS * FD_BLOCKS * (F * (80 * 4 + 64 * 2 + 256 * 4) +
                                                (64 * 480 + 6 * 64 * 192 + 256 * 192) * wb),
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


# bench tag -> kernel symbols that can serve it (the default kernel first) for the PMC
# traffic lookup; the first one present in a summary is used.  The LVC prefixes stop before
# the last template arguments (r04 added the tiles-per-wave argument).
TAG_KERNEL = {
    # the default (two tiles per wave) instantiation first: a summary may hold both
    # (r06: the persistent kernels, FD_OPT_LVC_PS, are the default; the one-tile kernel with lvc_ps=0)
    "fd_lvc_block_final": ("lvc_ps_kernel<true>", "lvc_final_ps_kernel", "lvc_block_bf16_kernel<384, true, true, true, true, false, 2>",
                           "lvc_block_bf16_kernel<384, true, true, true, true, false,"),
    "fd_lvc_block_ups": ("lvc_ps_kernel<false>", "lvc_block_bf16_kernel<384, true, false, false, true, false, 2>",
                         "lvc_block_bf16_kernel<384, true, false, false, true, false,"),
    "fd_lvc_block_sub": ("lvc_block_bf16_kernel<256, true, false, false, false, true,",
                         "lvc_block_bf16_kernel<128, true, false, false, false, true,"),
    "fd_kp_kernel": ("kp_kernel_bf16_kernel",),
    "fd_kp_hidden": ("kp_hidden_bf16_kernel",),
    "fd_dblock_fused": ("dblock_bf16_kernel",),
    "wn_stack": ("wn_stack_bf16_kernel",),
    "wn_layer": ("wn_layer_bf16_kernel",),
    "wn_gate2": ("wn_gate_bf16_kernel",),
    "wn_resskip2": ("wn_resskip_bf16_kernel",),
    "nsf_pair": ("nsf_pair_kernel<",),
    "nsf_pair16": ("nsf_pair16_kernel<",),
    "nsf_rb16": ("nsf_rb16_kernel<",),
    "nsf_rb32": ("nsf_rb_kernel<32,",),
    "nsf_res": ("nsf_wconv_kernel<",),
    "nsf_ups": ("nsf_ups_kernel<",),
}
DENOISER_TAGS = ("wn_stack", "wn_condb", "wn_layer", "wn_gate", "wn_resskip", "wn_gate2", "wn_resskip2", "wn_xa",
                 "wn_inproj", "wn_skiphead", "wn_outproj", "wn_outproj_posterior", "wn_f32_tail")


def dominant_kernel(kern_all, fl, by):
    """The tag with the most GPU time in the all-launch profile.  Every tag that can be the slowest
    must be in the FLOP and byte tables: an untagged slowest kernel is an error, not a reason to
    report the roofline of a smaller one."""
    dom = max(kern_all.items(), key=lambda kv: kv[1][1])[0]
    if dom not in fl or dom not in by:
        raise SystemExit(f"bench.py: the slowest kernel tag {dom!r} has no FLOP/byte entry "
                         f"(flops_per_launch / bytes_per_launch / svs_tables)")
    return dom


def lib_sha16(path=None):
    """First 16 hex digits of the loaded library's sha256 (profile summaries record the one they
    were measured on)."""
    import hashlib
    if path is None:
        from prodiff_amd import _lib
        path = _lib.LIB_PATH
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def traffic_workload(d, fname):
    """(config, per-GPU batch, frames) a PMC summary was measured on.  Summaries written
    before round 3 carry no workload: they are C5 (file name *c5*) or C3, 8 x 861."""
    if "config" in d:
        return d["config"], int(d["batch"]), int(d["frames"])
    return ("C5" if "c5" in os.path.basename(fname) else "C3"), 8, 861


def sq_utilisation(config):
    """Per-kernel MFMA-busy / VALU-busy fractions of the SQ-counter summary of this config (one of the
    running library if there is one, else the newest round's)
    (profiles/rNN_*/<config>_sq.json, written by tools/sq_summary.py from separate rocprofv3 SQ
    passes over a short bench of the same workload).  None when no summary covers the config."""
    import glob
    import re
    best = None
    for f in glob.glob(os.path.join(ROOT, "profiles", "r*", "*_sq.json")):
        m = re.search(r"profiles/r(\d+)_", f.replace(os.sep, "/"))
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config") != config or not m:
            continue
        # a summary of the running library first, then the newest round
        key = (d.get("lib_sha16") == lib_sha16(), int(m.group(1)), os.path.getmtime(f))
        if best is None or key > best[0]:
            best = (key, f, d)
    if best is None:
        return None
    _, f, d = best
    ks = [{k: r.get(k) for k in ("kernel", "avg_us_profiled", "mfma_busy", "valu_busy", "wait_any", "wait_inst")}
          for r in d["kernels"]]
    src_lib = d.get("lib_sha16")
    return {"source": os.path.relpath(f, ROOT), "kernels": ks,
            "source_lib_sha16": src_lib, "running_lib_sha16": lib_sha16(),
            "same_library": bool(src_lib) and src_lib == lib_sha16(),
            "note": "rocprofv3 SQ counters, separate passes: mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x cycles), "
                    "valu_busy = 4 SQ_ACTIVE_INST_VALU / (SIMDs x cycles), wait_* = fractions of SQ_WAVE_CYCLES"}


def pmc_traffic(tag, config, batch, frames, path=None):
    """HBM bytes per launch of `tag`'s kernel(s) from the newest committed PMC summary
    measured on the SAME workload (config, per-GPU batch, frames) -- profiles/rNN_vMM_traffic.json,
    written by tools/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes
    of the bench command.  A tag served by several template instantiations (nsf_res) gets the
    launch-weighted mean.  Returns (bytes per launch, summary path, the library sha16 the summary
    records); (None, None, None) when no summary of this workload holds the kernel."""
    import glob
    import re
    syms = TAG_KERNEL.get(tag)
    if syms is None:
        return None, None, None
    if path is None:
        def ver(f):
            m = re.search(r"r(\d+)_v(\d+)[a-z0-9_]*_traffic\.json$", f)
            return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_v*_traffic.json")), key=ver, reverse=True)
    else:
        files = [path]
    for fpath in files:
        if not os.path.exists(fpath):
            continue
        with open(fpath) as f:
            d = json.load(f)
        if traffic_workload(d, fpath) != (config, batch, frames):
            continue
        kern = d["kernels"]
        for sym in syms:
            hits = [v for name, v in kern.items() if sym in name]
            if hits:
                n = sum(v["launches"] for v in hits)
                tb = sum(v["traffic_bytes_per_launch"] * v["launches"] for v in hits) / n
                return float(tb), os.path.relpath(fpath, ROOT), d.get("lib_sha16")
    return None, None, None


def nsf_stage_dims(h=None):
    """(samples per mel frame, channels) after each NSF-HiFiGAN upsample (handler/base_config.yaml)."""
    rates, ch0 = (8, 8, 2, 2, 2), 512
    out, r = [], 1
    for i, u in enumerate(rates):
        r *= u
        out.append((r, ch0 // 2 ** (i + 1)))
    return out


NSF_PAIR_C = (32, 64, 128)     # ResBlock1 conv pairs fused into one nsf_pair launch (bf16, NSF_OPT_PAIR)
NSF_PAIR16_C = (16,)           # ... and into one nsf_pair16 launch (bf16, NSF_OPT_PAIR16, r05; rb16 = 0)
NSF_RB16_C = (16,)             # r06: a whole 16-channel ResBlock1 (3 pairs) per nsf_rb16 launch (NSF_OPT_RB16)
NSF_RB32_KS = (3,)             # r06: the 32-channel ResBlock1s of these kernel sizes per nsf_rb32 launch (NSF_OPT_RB32 1)
NSF_KS = (3, 7, 11)            # resblock kernel sizes; 3 dilation pairs each (ResBlock1)
NSF_HOP, NSF_MELS, NSF_C0, NSF_HARM = 512, 128, 512, 9


def _mean(xs):
    return sum(xs) / len(xs) if xs else 0.0


def svs_tables(B, T, Tt, dtype, small_max=16, H=256, k_ffn=9):
    """(FLOPs, compulsory HBM bytes) of ONE launch of each condition-encoder / NSF-HiFiGAN tag;
    a tag launched at several stages reports the mean over its launches in one forward.
    NSF stage s (nsf_stage_dims) runs at r_s samples per mel frame with C_s channels: its 3
    ResBlock1s (k = 3, 7, 11) hold 3 (c1, c2) conv pairs each; pairs with C in NSF_PAIR_C run as
    one nsf_pair launch (bf16), the other stages' convs as single launches (nsf_res for
    C > small_max, nsf_res_small otherwise)."""
    wb = 2 if dtype == "bf16" else 4
    F = B * T
    rows = B * Tt
    st = nsf_stage_dims()
    paired = [(r, c) for r, c in st if dtype == "bf16" and c in NSF_PAIR_C]
    paired16 = [(r, c) for r, c in st if dtype == "bf16" and c in NSF_PAIR16_C]
    single = [(r, c) for r, c in st if (r, c) not in paired and (r, c) not in paired16]
    fl, by = {}, {}
    # pair (k, d): c1 (k, dil d) and c2 (k, dil 1) over F r rows; x read once (fp32), the pair's
    # output written once (fp32), the last pair of resblocks 1, 2 also reads + writes the ResBlock sum
    # r06: the C = 16 ResBlock1 whole (three pairs) per launch: x read once, the ResBlock sum written
    # (first ResBlock) or read + written (the other two) once
    rf, rb_ = [], []
    for r, c in paired16:
        if c not in NSF_RB16_C:
            continue
        for j, k in enumerate(NSF_KS):
            rf.append(3 * 2 * 2 * F * r * c * c * k)
            rb_.append(F * r * c * 4 * (2 if j == 0 else 3) + 6 * c * c * k * wb)
    fl["nsf_rb16"], by["nsf_rb16"] = _mean(rf), _mean(rb_)
    rf, rb_ = [], []
    for r, c in paired:
        if c != 32:
            continue
        for j, k in enumerate(NSF_KS):
            if k in NSF_RB32_KS:
                rf.append(3 * 2 * 2 * F * r * c * c * k)
                rb_.append(F * r * c * 4 * (2 if j == 0 else 3) + 6 * c * c * k * wb)
    fl["nsf_rb32"], by["nsf_rb32"] = _mean(rf), _mean(rb_)
    for tag, stages in (("nsf_pair", paired), ("nsf_pair16", paired16)):
        pf, pb = [], []
        for r, c in stages:
            for k in NSF_KS:
                if tag == "nsf_pair" and c == 32 and k in NSF_RB32_KS:
                    continue        # a whole-ResBlock nsf_rb32 launch (r06)
                for q in range(3):
                    pf.append(2 * 2 * F * r * c * c * k)
                    acc = q == 2 and k != NSF_KS[0]
                    pb.append(F * r * c * 4 * (2 + (1 if acc else 0)) + 2 * c * c * k * wb)
        fl[tag], by[tag] = _mean(pf), _mean(pb)
    for tag, sel in (("nsf_res", lambda c: c > small_max), ("nsf_res_small", lambda c: c <= small_max)):
        cf, cb = [], []
        for r, c in single:
            if not sel(c):
                continue
            for k in NSF_KS:
                for _ in range(6):          # 3 pairs x (c1, c2), one launch each
                    cf.append(2 * F * r * c * c * k)
                    cb.append(F * r * c * 4 * 2.5 + c * c * k * wb)     # in, out, half of them a residual
        fl[tag], by[tag] = _mean(cf), _mean(cb)
    # ConvTranspose1d (k = 2u: 2 taps per output row) + the noise-conv add
    uf, ub, nf, nb_ = [], [], [], []
    r_in, c_in = 1, NSF_C0
    for r, c in st:
        uf.append(2 * F * r * c_in * c * 2)
        ub.append(F * r_in * c_in * 4 + 2 * F * r * c * 4 + c_in * c * 2 * (r // r_in) * wb)
        sf = NSF_HOP // r
        K = 2 * sf if sf > 1 else 1
        nf.append(2 * F * r * c * K)
        nb_.append(F * NSF_HOP * 4 + F * r * c * 4)
        r_in, c_in = r, c
    fl["nsf_ups"], by["nsf_ups"] = _mean(uf), _mean(ub)
    fl["nsf_noise_conv"], by["nsf_noise_conv"] = _mean(nf), _mean(nb_)
    rl, cl = st[-1]
    fl["nsf_post"], by["nsf_post"] = 2 * F * rl * cl * 7, F * rl * (cl + 1) * 4
    fl["nsf_conv_pre"], by["nsf_conv_pre"] = 2 * F * NSF_MELS * NSF_C0 * 7, F * (NSF_MELS + NSF_C0) * 4
    # SineGen + SourceModule: 9 harmonics per sample (sin on the VALU), har written once
    fl["nsf_source"], by["nsf_source"] = 2 * F * NSF_HOP * NSF_HARM * 2, F * NSF_HOP * 4 + F * 8
    fl.update({"enc_qkv": 2 * rows * H * 3 * H, "enc_outproj": 2 * rows * H * H,
               "enc_ffn1": 2 * rows * H * 4 * H * k_ffn, "enc_ffn2": 2 * rows * 4 * H * H,
               "enc_attn": 2 * 2 * B * Tt * Tt * H, "enc_ln": 0.0, "enc_embed": 0.0, "enc_cond": 0.0})
    by.update({"enc_qkv": rows * 4 * H * 4 + 3 * H * H * wb, "enc_outproj": rows * 3 * H * 4 + H * H * wb,
               "enc_ffn1": rows * 5 * H * 4 + 4 * H * H * 9 * wb, "enc_ffn2": rows * 6 * H * 4 + 4 * H * H * wb,
               "enc_attn": rows * 4 * H * 4, "enc_ln": rows * H * 8, "enc_embed": rows * H * 4,
               "enc_cond": F * H * 4})
    return fl, by


def svs_step_flops(B, T, Tt):
    f, _ = svs_tables(B, T, Tt, "fp32", small_max=0)
    enc = 4 * (f["enc_qkv"] + f["enc_outproj"] + f["enc_ffn1"] + f["enc_ffn2"] + f["enc_attn"])
    nsf = 18 * 5 * f["nsf_res"]
    ups = 0
    F = B * T
    r_in, c_in = 1, 512
    for (r, c), k in zip(nsf_stage_dims(), (16, 16, 4, 4, 4)):
        ups += 2 * F * r_in * c_in * c * k
        r_in, c_in = r, c
    pre_post = 2 * F * 512 * 128 * 7 + 2 * F * 512 * 16 * 7
    return enc + 4 * prodiff_step_flops(B, T, M=128) + nsf + ups + pre_post


def prodiff_step_flops(B, T, M=80, C=256, H=256):
    """One denoiser call: 26.43 MFLOP per frame at M=80."""
    f = flops_per_launch(B, T, M=M, C=C, H=H)
    return f["wn_inproj"] + 20 * (f["wn_gate"] + f["wn_resskip"]) + f["wn_skiphead"] + f["wn_outproj_posterior"]


def fastdiff_step_flops(B, T):
    """One FastDiff eps-network call: 56.98 MFLOP per frame."""
    f = flops_per_launch(B, T, dtype="fp32")          # per-layer kernel_conv entry
    return (f["fd_first_conv"] + 9 * f["fd_dblock"] + f["fd_final_update"] +
            3 * (f["fd_kp_in"] + 6 * f["fd_kp_res"] + f["fd_kp_bias"] + 4 * f["fd_kp_kernel"] +
                 f["fd_upsample"] + 4 * f["fd_lvc_preconv"] + 4 * f["fd_lvc"]))


def ref_cpu_baseline(config):
    """The reference's own CPU path, timed by tools/ref_cpu_bench.py where
    /root/reference exists (profiles/r02_ref_cpu.json; the GPU box has no reference)."""
    path = os.path.join(ROOT, "profiles", "r02_ref_cpu.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    key = config if config in ("C2", "C5", "PITCH") else "C3"
    e = d.get("configs", {}).get(key)
    if not e:
        return None
    return {"value": e["mel_frames_per_s"], "unit": "mel-frames/s", "cores": d["threads"], "kind": "reference",
            "sample": e["sample"], "rtf": e.get("rtf"), "host": d["host"],
            "timing": f"median of {e.get('repeats', d['repeats'])} after 1 warm-up, fp32, torch.no_grad",
            "source": os.path.relpath(path, ROOT)}


def port_cpu_baseline(frames, batch=1, vocoder=True):
    """The torch-fp32 CPU restatement (oracle/oracle_torch.py, a port of the
    reference math) timed on THIS host's cores on a bounded sample of the workload: `batch`
    utterances of `frames` mel frames through the same 2-iter ProDiff (+ 4-iter FastDiff).
    r06: by default the workload's own batch (C3: 8 x 861, ~8 s on the box's 16 cores), timed once
    after a 200-frame warm-up (r05 timed one 200-frame utterance: 34x smaller than C3's batch)."""
    from oracle import oracle_torch as OT
    from prodiff_amd import synth
    threads = torch.get_num_threads()
    model = OT.PortModels(synth, seed=0)

    def run(b, t):
        cond = torch.from_numpy(synth.synth_inputs(0, (b, t, 256)))
        mel = model.prodiff(cond, seed=1)
        if vocoder:
            model.fastdiff(mel, seed=2)

    run(1, min(frames, 200))                  # warm-up (thread pool, allocator)
    t0 = time.perf_counter()
    run(batch, frames)
    dt = time.perf_counter() - t0
    audio_s = batch * frames * HOP / SAMPLE_RATE
    return {"value": round(batch * frames / dt, 2), "unit": "mel-frames/s", "cores": threads, "kind": "port",
            "sample": f"torch fp32 CPU restatement (oracle/oracle_torch.py), {batch} utterance(s) x {frames} frames "
                      f"({audio_s:.2f} s audio), 2-iter ProDiff" + (" + 4-iter FastDiff" if vocoder else "") +
                      f", one timed run after a 200-frame warm-up: {dt:.2f} s",
            "rtf": round(dt / audio_s, 4)}


def denoiser_roofline(kern_all, nprof, B, T, cfg, dtype, peak_tf, cfg_name, pmc_key=None):
    """The north star's denoiser figure: the WaveNet residual stack (every launch of the ProDiff
    sampler's denoiser, tags DENOISER_TAGS) against the MFMA roof at its algorithmic FLOPs
    (26.43 MFLOP per mel frame per pass at M = 80), and -- where a PMC summary of
    this workload holds the stack kernel -- its measured HBM bytes against the 8 TB/s roof."""
    M = cfg.get("mels", 128 if cfg.get("svs") else 80)
    tags = [t for t in kern_all if t in DENOISER_TAGS]
    if not tags:
        return None
    ms = sum(kern_all[t][1] for t in tags)
    passes = cfg["timesteps"]
    flop = passes * prodiff_step_flops(B, T, M=M) * nprof
    ach = flop / (ms * 1e-3) / 1e12
    out = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak_tf, "unit": "TFLOP/s",
           "frac": round(ach / peak_tf, 4), "kernels": sorted(tags), "ms_per_step": round(ms / nprof, 3),
           "flop_per_step": passes * prodiff_step_flops(B, T, M=M),
           "timing": "the untimed all-launch pass (HIP events around every launch)"}
    if "wn_stack" in kern_all:
        # pmc_key: the (per-launch batch, frames) the PMC summaries are keyed by (B, T here are the
        # rank's totals, the FLOP count's basis)
        tb, src, tlib = pmc_traffic("wn_stack", cfg_name, *(pmc_key or (B, T)))
        if tb:
            cnt, sms = kern_all["wn_stack"]
            gbs = tb * cnt / (sms * 1e-3) / 1e9
            out["hbm"] = {"kernel": "wn_stack", "traffic_bytes_per_launch": round(tb), "achieved": round(gbs, 1),
                          "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                          "source": src, "same_library": bool(tlib) and tlib == lib_sha16()}
    return out


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def stub_synth(cond, seed, utt_ids=None, lens=None):
    """--dry-run stand-in for the Synthesizer (CPU, no compute worth timing)."""
    B, T, _ = cond.shape
    return cond[..., :80].clone(), torch.zeros(B, T * HOP)


stub_synth.mel_bins = 80


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="auto", choices=["auto"] + list(CONFIGS),
                    help="auto: C3 at N=1, C4 (32 utterances per GPU) at N>1")
    ap.add_argument("--batch", type=int, default=None, help="utterances per GPU (global for C4S)")
    ap.add_argument("--frames", type=int, default=None, help="mel frames per utterance")
    ap.add_argument("--lengths", default="fixed", choices=["fixed", "ds"],
                    help="ds: the reference song's 30 segment lengths (and phoneme counts) per GPU "
                         "(tests/golden/ds_lengths.json, from samples/00_*.ds), run as ragged batches")
    ap.add_argument("--cpu-frames", type=int, default=-1,
                    help="cpu_baseline_port sample: -1 = the workload's batch (at most 8 x 861 frames' worth), "
                         "N > 0 = one utterance of N frames, 0 = skip")
    ap.add_argument("--overlap", type=int, default=None,
                    help="jobs in flight: step i runs on HIP stream i %% N, so consecutive jobs overlap "
                         "(default: 2 for C3 / C5 on one GPU, else 1)")
    ap.add_argument("--max-frames", type=int, default=0,
                    help="cap on a ragged batch's padded frames (0 = none): a rank's utterances then run as "
                         "several batches on concurrent HIP streams")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"],
                    help="compute dtype (default: the config's; fp32 is the exact parity path)")
    ap.add_argument("--no-graph", action="store_true", help="C2: launch eagerly instead of replaying a hipGraph")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--prof-steps", type=int, default=2,
                    help="untimed steps with every launch bracketed by HIP events (the `kernels` table)")
    ap.add_argument("--traffic", default=None, help="PMC traffic summary (default: newest profiles/r*_v*_traffic.json)")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo launcher + sharding + gather check, no GPU")
    ap.add_argument("--fd-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="FastDiff kernel-variant option for A/B runs (fd_set_option, e.g. kp_chunk=4)")
    ap.add_argument("--wn-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="WaveNet kernel-variant option for A/B runs (pd_wavenet_set_option, e.g. layer=0)")
    ap.add_argument("--nsf-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="NSF-HiFiGAN kernel-variant option for A/B runs (nsf_set_option, e.g. pair=0)")
    args = ap.parse_args()

    # ---- N ranks: re-launch under torch.distributed.run BEFORE anything touches the GPU
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    cfg_name = args.config if args.config != "auto" else ("C3" if world == 1 else "C4")
    cfg = CONFIGS[cfg_name]
    svs = cfg.get("svs", False)
    # (the pitch predictor runs at the SVS frame rate, handler/base_config.yaml: hop 512 at 44.1 kHz)
    hop, sample_rate = (512, 44100) if (svs or cfg.get("pitch")) else (HOP, SAMPLE_RATE)
    dtype = args.dtype or cfg["dtype"]
    nb = args.batch or cfg["batch"]
    T = args.frames or cfg["frames"]
    dry = args.dry_run
    if cfg_name in ("C2", "PITCH") and world > 1:
        raise SystemExit(f"{cfg_name} is a single-GPU config")
    pitch = cfg.get("pitch", False)
    if world > 1:
        dist.init_process_group("gloo" if dry else "nccl", init_method="env://")
        assert dist.get_world_size() == args.gpus
    if dry:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)

    from prodiff_amd.pipeline import JobStreams, distributed_synthesize, lpt_shards

    # utterance list (all ranks know every length; only the own shard is resident)
    from prodiff_amd.pipeline import ragged_batches
    if args.lengths == "ds":   # the song's segments, once per GPU (weak scaling), ragged batches
        ds = json.load(open(os.path.join(ROOT, "tests", "golden", "ds_lengths.json")))
        per = len(ds["frames"])
        n_total = per if cfg["strong"] else per * world
        lengths = [ds["frames"][i % per] for i in range(n_total)]
        tokens = [min(ds["phonemes"][i % per], lengths[i]) for i in range(n_total)]
        nb = per
    else:
        n_total = nb if cfg["strong"] else nb * world
        lengths = [T] * n_total
        tokens = [cfg.get("tokens", 0)] * n_total
    shards = lpt_shards(lengths, world)
    mine = shards[rank]
    B = len(mine)                                           # utterances this rank runs per step
    F_rank = sum(lengths[i] for i in mine)
    n_batches = max(1, len(ragged_batches(lengths, mine, max_frames=args.max_frames or None)))
    rng = np.random.default_rng(1000 + rank)
    conds = [(L_, None) for L_ in lengths]
    from prodiff_amd import synth as _synth
    for i in mine:
        if svs:      # one SVS segment: phonemes + durations summing to T frames, f0, voicing, breath
            from prodiff_amd.pipeline import SVS_VOCAB
            u = {k: torch.from_numpy(v).to(dev) for k, v in
                 _synth.synth_svs_utterance(100 + i, lengths[i], tokens[i], SVS_VOCAB).items()}
            conds[i] = (lengths[i], (lambda u=u: u))
        else:
            conds[i] = torch.from_numpy(rng.standard_normal((lengths[i], 256), dtype=np.float32)).to(dev)

    _lib = None
    if dry:
        synth_fn = stub_synth
        if svs or pitch:
            raise SystemExit("--dry-run covers the C3/C4 launcher; C5 / PITCH need the GPU")
    elif svs:
        from prodiff_amd import _lib
        from prodiff_amd.pipeline import SvsSynthesizer
        syn = SvsSynthesizer.synthetic(dev, seed=0, dtype=dtype)
        if args.wn_opt:
            syn.diffusion.denoise_fn.set_options(**{k: int(v) for k, v in (o.split("=") for o in args.wn_opt)})
        if args.nsf_opt:
            syn.generator.set_options(**{k: int(v) for k, v in (o.split("=") for o in args.nsf_opt)})
        synth_fn = syn
    elif pitch:
        # the pitch predictor's sampler alone (its note / phoneme encoders are out of scope, SURVEY §2
        # row 15): PitchRectifiedFlow over a WaveNet(64, 256, 20, 256, cycle 5) with random-init weights
        from prodiff_amd import PitchRectifiedFlow, WaveNet, _lib
        M_p = cfg["mels"]
        net = WaveNet(M_p, 256, 20, 256, cfg["cyc"])
        net.load_state_dict({k: torch.from_numpy(v) for k, v in
                             _synth.synth_params(_synth.wavenet_param_shapes(M_p, 256, 20, 256), 0).items()})
        rf = PitchRectifiedFlow(M_p, net, time_scale=1000, sampling_algorithm="euler").to(dev).eval()
        rf.set_compute_dtype(dtype)
        if args.wn_opt:
            net.set_options(**{k: int(v) for k, v in (o.split("=") for o in args.wn_opt)})
        synth_fn = None
    else:
        from prodiff_amd import _lib
        from prodiff_amd.pipeline import Synthesizer
        syn = Synthesizer.synthetic(dev, seed=0, dtype=dtype)
        if args.fd_opt:
            syn.vocoder.model.set_options(**{k: int(v) for k, v in (o.split("=") for o in args.fd_opt)})
        if args.wn_opt:
            syn.diffusion.denoise_fn.set_options(**{k: int(v) for k, v in (o.split("=") for o in args.wn_opt)})
        synth_fn = syn

    phase_marks = []    # N > 1: per timed step, where it went (event marks, read after the timed region)
    ovl = None      # JobStreams when --overlap > 1
    if args.overlap is None:
        # jobs in flight (measured on one GPU, profiles/r05_ab/job_overlap*_ab.txt): C3 2 (3: the same),
        # C5 3 (2 on the .ds lengths, whose ragged batches already run on 4 streams), C4 2 (-1.4%).
        # N > 1 ranks (r06): 2, so job i's RCCL gather to rank 0 runs beside job i + 1's compute
        args.overlap = 1
        if cfg["vocoder"]:
            args.overlap = 2
            if world == 1 and cfg_name == "C5" and args.lengths != "ds":
                args.overlap = 3

    if cfg["vocoder"]:
        if args.overlap > 1:
            # consecutive jobs on alternating HIP streams (pipeline.JobStreams): one job's
            # low-occupancy launches (the ProDiff WaveNet stack fills 157 of 256 CUs at C3) overlap
            # the previous job's vocoder.  Handles are packed first (stream-ordered packing).
            # N > 1: a job's gathers are issued from its own stream; torch's process group runs every
            # collective on ONE collective stream per device in host issue order -- the same on every
            # rank -- which waits for the issuing job's stream, and the job's stream waits for the
            # gathers (no host wait).  So job i's gather overlaps job i + 1's compute on the other stream.
            if getattr(synth_fn, "prepare", None) and not dry:
                synth_fn.prepare()
            if not dry:
                torch.cuda.synchronize()
            ovl = JobStreams(args.overlap, dev)     # (a CPU device: a no-op, same schedule on the host)

        def step(i, timed=False, iso=False):
            st = {} if (timed and not iso and world > 1) else None
            ctx = ovl.next() if (ovl and not iso) else contextlib.nullcontext()
            with ctx:
                out = distributed_synthesize(synth_fn, conds, seed=10_000 * i, device=dev, hop=hop, stats=st,
                                             max_frames=args.max_frames or None)
            if st is not None:
                phase_marks.append(st)
            return out
    elif pitch:
        # PITCH: 20 Euler steps (every velocity evaluation the fused WaveNet stack, x += v dt in its
        # last launch) then denorm_spec: mean over the 64 repeat bins, clamp -> pitch [B, T]
        cond_b = torch.stack([conds[i] for i in mine])

        def step(i, timed=False, iso=False):
            return rf.denorm_spec(rf.sample(cond_b, infer_step=cfg["timesteps"], seed=10_000 * i))
    else:
        # C2: the ProDiff sampler alone on one utterance (B=1), mel only
        gd = syn.diffusion
        cond_b = torch.stack([conds[i] for i in mine])
        graph = None
        if not args.no_graph:
            graph = gd.capture(cond_b, seed=1)             # hipGraph of the whole 2-step sampler

        def step(i, timed=False, iso=False):
            if graph is not None:
                return graph.replay()
            return gd.sample(cond_b, seed=10_000 * i)

    # per-launch tables: a launch covers one batch; with ragged batches (--lengths ds) the mean
    # batch, F_rank / n_batches real frames (padding is not algorithmic work)
    ds_mode = args.lengths == "ds"
    wl_name = cfg_name + ("DS" if ds_mode else "")        # workload key of the PMC / SQ summaries
    Bl = B / n_batches
    Tl = F_rank / B if ds_mode else T
    if svs:
        fl = flops_per_launch(Bl, Tl, dtype, M=128)
        by = bytes_per_launch(Bl, Tl, dtype, M=128)
        sf, sb = svs_tables(Bl, Tl, sum(tokens[i] for i in mine) / max(B, 1), dtype)
        fl.update(sf)
        by.update(sb)
    else:
        fl = flops_per_launch(Bl, Tl, dtype, M=cfg.get("mels", 80), cyc=cfg.get("cyc", 1))
        by = bytes_per_launch(Bl, Tl, dtype, M=cfg.get("mels", 80), cyc=cfg.get("cyc", 1))
    for i in range(args.warmup):
        step(i)
    if ovl is not None:
        # the isolated passes below run on the current stream, whose workspaces the overlapped
        # warm-up never touched: one untimed job there first (fresh allocations run cold)
        step(args.warmup, iso=True)
    if not dry:
        torch.cuda.synchronize()
    # Kernel timing.  An event pair costs GPU time at every launch it brackets, so the
    # per-kernel table comes from an untimed pass with every launch recorded, and the
    # timed region records only the dominant kernel (the roofline's avg_launch_us).
    timing = not (args.no_kernel_timing or dry or (cfg_name == "C2" and not args.no_graph))
    kern_all, dom, nprof = {}, None, 0
    if timing:
        nprof = max(1, args.prof_steps)
        _lib.profile_filter(None)
        _lib.profile_enable(True)
        for i in range(nprof):
            step(args.warmup + i, iso=True)      # one job at a time: per-kernel times unshared
        torch.cuda.synchronize()
        kern_all = _lib.profile_summary()
        _lib.profile_enable(False)
        dom = dominant_kernel(kern_all, fl, by)
        if ovl is None:
            _lib.profile_filter([dom])
            _lib.profile_enable(True)
    if not dry:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if not dry:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = step(args.warmup + nprof + i, timed=True)
    if not dry:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt_iso = None
    if timing and ovl is not None:
        # jobs in flight share the GPU, so a kernel's launch time in the timed region is not its own:
        # the roofline's launch time comes from K more steps run one job at a time, HIP events
        # around the dominant kernel only (and their wall time is reported beside `value`)
        _lib.profile_filter([dom])
        _lib.profile_enable(True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(args.steps):
            step(args.warmup + nprof + args.steps + i, timed=True, iso=True)
        torch.cuda.synchronize()
        dt_iso = time.perf_counter() - t1
    kern = _lib.profile_summary() if timing else {}
    if timing:
        _lib.profile_enable(False)
        _lib.profile_filter(None)
    graph_prof = (cfg_name == "C2" and not args.no_graph and not args.no_kernel_timing and not dry)
    if graph_prof:
        # the timed steps replayed a hipGraph, whose kernels HIP events cannot bracket: take the
        # kernel table and the roofline's launch time from untimed EAGER runs of the same sampler
        # (the same launches, one host launch each; first all tags, then the dominant one alone)
        nprof = max(1, args.prof_steps)
        _lib.profile_filter(None)
        _lib.profile_enable(True)
        for i in range(nprof):
            gd.sample(cond_b, seed=10_000 * i)
        torch.cuda.synchronize()
        kern_all = _lib.profile_summary()
        dom = dominant_kernel(kern_all, fl, by)
        _lib.profile_filter([dom])
        _lib.profile_enable(True)
        for i in range(args.steps):
            gd.sample(cond_b, seed=10_000 * i)
        torch.cuda.synchronize()
        kern = _lib.profile_summary()
        _lib.profile_enable(False)
        _lib.profile_filter(None)
    phases = None
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        if phase_marks:
            # per-step compute (own shard) and gather of every rank, from the HIP events each timed
            # job recorded on its stream (no synchronisation inside the timed steps)
            from prodiff_amd.pipeline import phase_ms
            pm = [phase_ms(st) for st in phase_marks]
            v = torch.tensor([sum(c for c, _ in pm) / len(pm), sum(g for _, g in pm) / len(pm)],
                             device=dev, dtype=torch.float64)
            allv = [torch.empty_like(v) for _ in range(world)]
            dist.all_gather(allv, v)
            c = [float(x[0]) for x in allv]
            g = [float(x[1]) for x in allv]
            phases = {"compute_ms_per_step_slowest_rank": round(max(c), 3),
                      "compute_ms_per_step_fastest_rank": round(min(c), 3),
                      "gather_ms_per_step_max": round(max(g), 3),
                      "gather_ms_per_step_rank0": round(g[0], 3),
                      "note": "per rank, from HIP events on each timed job's stream: its shard's synthesis, then "
                              "the ragged RCCL gather to rank 0 (with jobs in flight the gather overlaps the next "
                              "job's compute on the other job stream)"}
    if rank == 0 and not dry:
        if cfg["vocoder"]:
            mels, wavs = out
            assert len(mels) == n_total and all(torch.isfinite(m).all() for m in mels)
            assert all(torch.isfinite(w).all() for w in wavs)
        else:
            assert torch.isfinite(out).all()
            if pitch:
                assert out.shape == (B, T) and float(out.abs().max()) <= 12.0   # clamp_min / clamp_max

    frames = sum(lengths) * args.steps
    audio_s = frames * hop / sample_rate
    ms_step = dt / args.steps * 1e3
    peak_tf = BF16_PEAK_TFLOPS if dtype == "bf16" else FP32_PEAK_TFLOPS
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
        # keyed by a launch's batch (a split batch's launches cover B / n_batches utterances)
        traffic, tsrc, tlib = pmc_traffic(dom, wl_name, B if ds_mode else int(Bl), T, args.traffic)
        roofline.update({"bound_basis": "model estimate: algorithmic intensity vs the ridge; the measured limiter "
                                        "is in `utilisation` (MFMA / VALU busy, wait fractions)",
                         "traffic": round(traffic) if traffic else None, "traffic_source": tsrc,
                         "traffic_same_library": bool(tlib) and tlib == lib_sha16(), "kernel": dom,
                         "flop_per_launch": fl[dom], "bytes_per_launch": by.get(dom),
                         "intensity_flop_per_byte": round(intensity, 1), "ridge_flop_per_byte": round(ridge, 1),
                         "avg_launch_us": round(ms / cnt * 1e3, 2), "launches": cnt,
                         "share_of_step": round(ms / ((dt_iso or dt) * 1e3), 3),
                         "timing": ("HIP events around this kernel only, over untimed eager runs of the same "
                                    "sampler (the timed steps replay a hipGraph)") if graph_prof else
                                   ("HIP events around this kernel only, over K steps run one job at a time right "
                                    f"after the timed region (which keeps {args.overlap} jobs in flight on "
                                    f"{args.overlap} HIP streams: their kernels share the GPU)") if dt_iso else
                                   "HIP events around this kernel only, over the timed steps"})
        roofline["denoiser"] = denoiser_roofline(kern_all, nprof, 1, F_rank, cfg, dtype, peak_tf, wl_name,
                                                 pmc_key=(B if ds_mode else int(Bl), T))
    if svs:
        step_fl = svs_step_flops(n_total, sum(lengths) / n_total, sum(tokens) / n_total)
    elif pitch:
        step_fl = cfg["timesteps"] * prodiff_step_flops(1, sum(lengths), M=cfg["mels"])
    else:
        Fa = sum(lengths)
        step_fl = 2 * prodiff_step_flops(1, Fa) + (4 * fastdiff_step_flops(1, Fa) if cfg["vocoder"] else 0)
    out_line = {
        "metric": METRIC,
        "value": round(frames / dt, 1),
        "unit": "mel-frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if cfg["strong"] else "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": ("synthetic SVS segments (phonemes, durations summing to T, f0 with unvoiced gaps, voicing/breath, "
                 "speaker mix)" if svs else "synthetic (cond ~ N(0,1): the pitch predictor's encoder output)" if pitch
                 else "synthetic (cond ~ N(0,1))") +
                "; random-init weights of the reference architectures; on-device Philox draws",
        "config": {"workload": cfg["desc"].format(b=nb, t=T if not ds_mode else f"{min(lengths)}..{max(lengths)}",
                                                  n=cfg.get("tokens") if not ds_mode else "the .ds file's"),
                   "name": cfg_name + (" --lengths ds" if ds_mode else ""),
                   "global_batch": n_total,
                   "per_gpu_batch": B, "seq_len": T if not ds_mode else max(lengths),
                   "lengths": None if not ds_mode else
                   f"ragged: the reference song's {nb} segments per GPU ({min(lengths)}..{max(lengths)} frames, "
                   f"{sum(lengths[i] for i in mine)} per GPU; samples/00_*.ds via tests/golden/ds_lengths.json), "
                   f"{n_batches} padded batches per GPU (ragged_batches, <= 15% padding)",
                   "batches_per_gpu": n_batches,
                   "jobs_in_flight": ovl.depth if ovl is not None else 1,
                   "schedule": None if ovl is None or ovl.depth == 1 else
                   (f"job i on HIP stream i % {ovl.depth}" + (
                       "; its ragged RCCL gather to rank 0 on the process group's collective stream (host issue "
                       "order, the same on every rank), overlapping job i + 1's compute" if world > 1 else "")),
                   "one_job_in_flight": None if dt_iso is None else
                   {"value": round(frames / dt_iso, 1), "ms_per_step": round(dt_iso / args.steps * 1e3, 3),
                    "note": "the same K steps run one after the other right after the timed region"},
                   "parallelism": f"dp{world} (utterance shards, RCCL gather to rank 0)" if cfg["vocoder"]
                   else "single GPU" + ("" if (args.no_graph or pitch) else ", hipGraph replay")},
        "rtf": round(dt / audio_s, 6),
        "x_realtime": round(audio_s / dt, 1),
        "model_tflops": round(step_fl * args.steps / dt / 1e12, 2),
        "roofline": roofline,
        "utilisation": sq_utilisation(wl_name) if not dry else None,
        "kernels": kernels,
        "phases": phases,
        "kernels_source": (f"untimed {'eager ' if graph_prof else ''}pass of {nprof} steps, every launch bracketed by "
                           f"HIP events") if kernels else None,
        "cpu_baseline": None,
        "cpu_baseline_port": None,
        "build": None if dry else {"pd_build_config": _lib.lib().pd_build_config().decode(), "lib_sha16": lib_sha16()},
        "dry_run": dry,
    }
    if rank == 0 and world == 1 and not dry:
        out_line["cpu_baseline"] = ref_cpu_baseline(cfg_name)
        if args.cpu_frames != 0 and not svs and not pitch:
            if args.cpu_frames > 0:
                pb, pt = 1, args.cpu_frames
            else:                                # the workload's own batch, bounded to C3's 6 888 frames
                pb, pt = max(1, min(B, 8 * 861 // T)), T
            out_line["cpu_baseline_port"] = port_cpu_baseline(pt, batch=pb, vocoder=cfg["vocoder"])
    if rank == 0:
        print(json.dumps(out_line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
