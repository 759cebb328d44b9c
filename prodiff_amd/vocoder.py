"""Vocoder plugin registry + the FastDiff vocoder (drop-in for the reference's).

Mirrors component/vocoder/base_vocoder.py:1-34 (``BaseVocoder``,
``register_vocoder``, ``get_vocoder_cls``) and component/vocoder/fastdiff.py:
17-126 (``load_fastdiff_model``, ``FastDiff`` with ``spec2wav``), and adds the
``to_device`` / ``spec2wav_torch`` pair that ``InferHandler`` calls
(handler/infer/handler.py:151-158) but the reference FastDiff lacks.
"""
from __future__ import annotations

import glob
import os
import re

import numpy as np
import torch
import yaml

from .fastdiff import FastDiff as FastDiffModel
from .schedules import fastdiff_infer_params, fastdiff_reverse_schedule, fastdiff_train_alpha


class BaseVocoder:
    def __init__(self, hparams):
        self.hparams = hparams

    def spec2wav(self, mel):
        """:param mel: [T, 80]  :return: wav [T']"""
        raise NotImplementedError

    @staticmethod
    def wav2spec(wav_fn, hparams):
        raise NotImplementedError


VOCODERS = {}


def register_vocoder(cls):
    VOCODERS[cls.__name__.lower()] = cls
    VOCODERS[cls.__name__] = cls
    return cls


def get_vocoder_cls(vocoder):
    cls_name = vocoder.lower()
    if cls_name not in VOCODERS:
        raise ValueError(f"Vocoder {cls_name} not found in VOCODERS")
    return VOCODERS[cls_name]


MODEL_KEYS = ("audio_channels", "inner_channels", "cond_channels", "upsample_ratios", "lvc_layers_each_block",
              "lvc_kernel_size", "kpnet_hidden_channels", "kpnet_conv_size", "dropout",
              "diffusion_step_embed_dim_in", "diffusion_step_embed_dim_mid", "diffusion_step_embed_dim_out",
              "use_weight_norm")


def build_fastdiff_model(config):
    return FastDiffModel(**{k: config[k] for k in MODEL_KEYS if k in config})


def load_fastdiff_model(config_path, checkpoint_path, reverse_step=4, device=None):
    """fastdiff.py:17-86.  Checkpoints load with weights_only=True (no unpickling)."""
    with open(config_path) as f:
        config = yaml.safe_load(f)
    model = build_fastdiff_model(config)
    state = torch.load(checkpoint_path, map_location="cpu", weights_only=True)["state_dict"]["model"]
    model.load_state_dict(state, strict=True)
    sched = fastdiff_reverse_schedule(reverse_step, config.get("noise_schedule") or None)
    model.remove_weight_norm()
    device = device or torch.device("cuda")
    model = model.eval().to(device)
    dh = {"T": int(config["T"]),
          "alpha": fastdiff_train_alpha(int(config["T"]), float(config["beta_0"]), float(config["beta_T"]))}
    return model, dh, sched, config, device


@register_vocoder
class FastDiff(BaseVocoder):
    """``hparams['vocoder_ckpt']`` names a directory with config.yaml +
    model_ckpt_steps_*.ckpt (fastdiff.py:92-115).  A ready model can be passed
    instead (``model=``/``config=``), e.g. for synthetic-weight benchmarks."""

    def __init__(self, hparams, model=None, config=None, reverse_step=4, device=None):
        super().__init__(hparams)
        if model is None:
            base_dir = hparams.get("vocoder_ckpt") or "checkpoint/FastDiff"
            ckpts = glob.glob(f"{base_dir}/model_ckpt_steps_*.ckpt")
            if not ckpts:
                raise FileNotFoundError(f"no FastDiff checkpoint under {base_dir}")
            ckpt = sorted(ckpts, key=lambda x: int(re.findall(r"model_ckpt_steps_(\d+)\.ckpt", x)[0]))[-1]
            self.model, self.dh, self.noise_schedule, self.config, self.device = load_fastdiff_model(
                os.path.join(base_dir, "config.yaml"), ckpt, reverse_step, device)
        else:
            self.config = dict(config or {"T": 1000, "beta_0": 1e-6, "beta_T": 0.01})
            self.device = device or next(model.parameters()).device
            self.model = model.eval().to(self.device)
            self.noise_schedule = fastdiff_reverse_schedule(reverse_step, self.config.get("noise_schedule") or None)
            self.dh = {"T": int(self.config.get("T", 1000)),
                       "alpha": fastdiff_train_alpha(int(self.config.get("T", 1000)),
                                                     float(self.config.get("beta_0", 1e-6)),
                                                     float(self.config.get("beta_T", 0.01)))}
        b, a, s, st = fastdiff_infer_params(self.noise_schedule, self.dh["alpha"])
        n = len(st)
        self.sched = (b[:n], a[:n], s[:n], st)
        self.scaler = None

    def to_device(self, device):
        self.device = torch.device(device)
        self.model = self.model.to(self.device)
        return self

    @torch.no_grad()
    def spec2wav_batch(self, mel, x_T=None, noise=None, seed=None, utt_ids=None, lens=None):
        """mel [B,T,80] on the device -> wav [B, T*hop], one row per utterance (``lens``: ragged
        batch, each row's length in frames; samples past lens[b] * hop are unspecified)."""
        b, a, s, st = self.sched
        return self.model.sample(mel.to(self.device), b, a, s, st, x_T=x_T, noise=noise, seed=seed,
                                 utt_ids=utt_ids, lens=lens)[:, 0]

    @torch.no_grad()
    def spec2wav_torch(self, mel, f0=None, x_T=None, noise=None, seed=None, **kwargs):
        """mel [B,T,80] (or [T,80]) on the device -> wav flattened to [B*T*hop], the vocoder
        contract InferHandler consumes (component/vocoder/nsf_hifigan.py:55-57 `view(-1)`,
        handler/infer/handler.py:157,351); f0 is unused (FastDiff is not NSF).  Batched
        callers that want one row per utterance use ``spec2wav_batch``."""
        if mel.dim() == 2:
            mel = mel[None]
        return self.spec2wav_batch(mel, x_T=x_T, noise=noise, seed=seed, utt_ids=kwargs.get("utt_ids")).reshape(-1)

    def spec2wav(self, mel, **kwargs):
        """fastdiff.py:117-126: mel np [T,80] -> np [1,1,T*hop]."""
        c = torch.as_tensor(np.asarray(mel), dtype=torch.float32, device=self.device)[None]
        wav = self.spec2wav_batch(c, x_T=kwargs.get("x_T"), noise=kwargs.get("noise"), seed=kwargs.get("seed"))
        return wav[:, None].cpu().numpy()
