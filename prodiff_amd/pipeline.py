"""End-to-end mel -> waveform synthesis and utterance sharding across GPUs.

``Synthesizer`` chains the two fused samplers the way the reference chains
``ProDiffTeacher.forward(infer=True)`` (prodiff_teacher.py:148-168) and the
vocoder's ``spec2wav`` (component/vocoder/fastdiff.py:117-126); the ProDiff
output is already the time-major mel the FastDiff sampler consumes, so nothing
is transposed or copied between them.

Multi-GPU: utterances are independent, so a batch is split into
per-rank shards with no data-path collective (``lpt_shards``); the only
exchange is the final point-to-point gather of each shard's outputs to the root
rank (``gather_to_root``, RCCL over xGMI under the ``nccl`` backend).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import synth
from .fastdiff import FastDiff
from .prodiff import GaussianDiffusion, WaveNet
from .vocoder import FastDiff as FastDiffVocoder

# handler/base_config.yaml:195-211 (diffusion/decoder), modules/FastDiff/config/base.yaml:4-42
PRODIFF_DEFAULTS = dict(in_dims=80, hidden_size=256, residual_layers=20, residual_channels=256,
                        dilation_cycle_length=1, timesteps=2, max_beta=40.0)
HOP = 256
SAMPLE_RATE = 22050


class Synthesizer:
    """cond [B,T,H] -> (mel [B,T,M], wav [B,T*hop])."""

    def __init__(self, diffusion: GaussianDiffusion, vocoder: FastDiffVocoder):
        self.diffusion = diffusion
        self.vocoder = vocoder

    @classmethod
    def synthetic(cls, device, seed=0, dtype="fp32", **over):
        """Random-init weights of the reference architectures (no checkpoints offline)."""
        cfg = dict(PRODIFF_DEFAULTS, **over)
        net = WaveNet(cfg["in_dims"], cfg["hidden_size"], cfg["residual_layers"], cfg["residual_channels"],
                      cfg["dilation_cycle_length"])
        shapes = synth.wavenet_param_shapes(cfg["in_dims"], cfg["hidden_size"], cfg["residual_layers"],
                                            cfg["residual_channels"])
        net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_params(shapes, seed).items()})
        gd = GaussianDiffusion(cfg["in_dims"], net, timesteps=cfg["timesteps"], time_scale=1000,
                               max_beta=cfg["max_beta"]).to(device).eval()
        fd = FastDiff()
        fd.load_state_dict({k: torch.from_numpy(v)
                            for k, v in synth.synth_params(synth.fastdiff_param_shapes(), seed + 1).items()})
        fd.remove_weight_norm()
        gd.set_compute_dtype(dtype)
        fd.set_compute_dtype(dtype)
        voc = FastDiffVocoder({"hop_size": HOP}, model=fd.to(device), reverse_step=4, device=device)
        return cls(gd, voc)

    @torch.no_grad()
    def __call__(self, cond, seed=None):
        g = None if seed is None else 2 * seed
        mel = self.diffusion.sample(cond, seed=g)
        wav = self.vocoder.spec2wav_torch(mel, seed=None if seed is None else g + 1)
        return mel, wav


def lpt_shards(lengths, world):
    """Longest-processing-time partition of utterances over ranks (sorted by length,
    each to the currently lightest rank).  Returns a list of index lists."""
    order = np.argsort(-np.asarray(lengths), kind="stable")
    load = np.zeros(world, np.int64)
    shards = [[] for _ in range(world)]
    for i in order:
        r = int(np.argmin(load))
        shards[r].append(int(i))
        load[r] += int(lengths[i])
    return [sorted(s) for s in shards]


def gather_to_root(t, root=0):
    """Point-to-point gather of equally shaped per-rank tensors to `root`
    (torch NCCL/RCCL implements gather as sends to the root).  Returns the
    stacked tensor on root, None elsewhere."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return t[None]
    world = dist.get_world_size()
    if dist.get_rank() == root:
        bufs = [torch.empty_like(t) for _ in range(world)]
        dist.gather(t.contiguous(), gather_list=bufs, dst=root)
        return torch.stack(bufs)
    dist.gather(t.contiguous(), dst=root)
    return None
