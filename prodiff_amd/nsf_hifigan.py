"""NSF-HiFiGAN vocoder on the HIP kernels of ``nsf_hifigan.hip``.

Drop-in for the reference's
  * ``Generator`` -- modules/nsf_hifigan/models.py:222-293: same constructor
    (an ``AttrDict``/dict of the vocoder's config.json), same parameter names as the
    state dict after ``remove_weight_norm`` (weight-norm ``weight_g``/``weight_v``
    pairs are folded on load), ``forward(c [B,M,T], f0 [B,T]) -> [B,1,T*hop]``;
  * ``load_model`` -- models.py:21-33 (config.json beside the checkpoint,
    ``['generator']`` state dict), loaded with ``torch.load(weights_only=True)``;
  * ``NsfHifiGAN`` -- component/vocoder/nsf_hifigan.py:10-56, registered under
    ``nsfhifigan`` (handler/base_config.yaml:218), ``spec2wav_torch(mel, f0=...)``.

The nn.Conv1d / ConvTranspose1d children only hold parameters; every forward goes
through ``nsf_forward`` in libprodiff_hip.so (there is no CPU fallback).  Unlike
the reference SineGen (batch 1 only, models.py:162-163) a batch holds independent
utterances.
"""
from __future__ import annotations

import json
import pathlib

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .vocoder import BaseVocoder, register_vocoder

LOG10_TO_LN = 2.30259     # component/vocoder/nsf_hifigan.py:53


def _get(h, k, default=None):
    return h[k] if k in h else default


class _ResBlock1(nn.Module):
    """Parameter holder with ResBlock1's names (models.py:36-70)."""

    def __init__(self, ch, k, dil):
        super().__init__()
        self.convs1 = nn.ModuleList([nn.Conv1d(ch, ch, k, 1, dilation=d, padding=d * (k - 1) // 2) for d in dil])
        self.convs2 = nn.ModuleList([nn.Conv1d(ch, ch, k, 1, dilation=1, padding=(k - 1) // 2) for _ in dil])


class _ResBlock2(nn.Module):
    """Parameter holder with ResBlock2's names (models.py:73-97)."""

    def __init__(self, ch, k, dil):
        super().__init__()
        self.convs = nn.ModuleList([nn.Conv1d(ch, ch, k, 1, dilation=d, padding=d * (k - 1) // 2) for d in dil])


class _Source(nn.Module):
    def __init__(self, harmonic_num):
        super().__init__()
        self.l_linear = nn.Linear(harmonic_num + 1, 1)


class Generator(nn.Module):
    def __init__(self, h):
        super().__init__()
        self.h = h
        self.harmonic_num = 8                                 # models.py:229
        rates = list(_get(h, "upsample_rates"))
        ks = list(_get(h, "upsample_kernel_sizes"))
        self.num_kernels = len(_get(h, "resblock_kernel_sizes"))
        self.num_upsamples = len(rates)
        self.upp = int(np.prod(rates))
        ch0 = int(_get(h, "upsample_initial_channel"))
        self.m_source = _Source(self.harmonic_num)
        self.noise_convs = nn.ModuleList()
        self.conv_pre = nn.Conv1d(int(_get(h, "num_mels")), ch0, 7, 1, padding=3)
        self.ups = nn.ModuleList()
        for i, (u, k) in enumerate(zip(rates, ks)):
            c = ch0 // 2 ** (i + 1)
            self.ups.append(nn.ConvTranspose1d(ch0 // 2 ** i, c, k, u, padding=(k - u) // 2))
            if i + 1 < len(rates):
                sf = int(np.prod(rates[i + 1:]))
                self.noise_convs.append(nn.Conv1d(1, c, kernel_size=sf * 2, stride=sf, padding=sf // 2))
            else:
                self.noise_convs.append(nn.Conv1d(1, c, kernel_size=1))
        rb = _ResBlock1 if str(_get(h, "resblock")) == "1" else _ResBlock2
        self.resblocks = nn.ModuleList()
        for i in range(len(rates)):
            c = ch0 // 2 ** (i + 1)
            for k, d in zip(_get(h, "resblock_kernel_sizes"), _get(h, "resblock_dilation_sizes")):
                self.resblocks.append(rb(c, k, d))
        self.conv_post = nn.Conv1d(ch0 // 2 ** len(rates), 1, 7, 1, padding=3)
        self._h = None
        self._sig = None
        self._ws = _lib.Workspace()
        self.compute_dtype = "fp32"
        self._options = {}

    def set_options(self, **opts):
        """Kernel-variant options (nsf_set_option, include/prodiff_hip.h NSF_OPT_*): small_max."""
        for k, v in opts.items():
            if k not in _lib.NSF_OPTIONS:
                raise ValueError(f"unknown NSF-HiFiGAN option {k!r}")
            self._options[k] = int(v)
        self._release()
        return self

    def set_compute_dtype(self, dtype):
        """"fp32" (exact parity path) or "bf16" (bf16 MFMA GEMMs, fp32 accumulate)."""
        if dtype not in ("fp32", "bf16"):
            raise ValueError(dtype)
        if dtype != self.compute_dtype:
            self._release()
            self.compute_dtype = dtype
        return self

    # ------------------------------------------------------------------ weights
    def load_state_dict(self, state_dict, strict=True):
        """Accepts the plain state dict or the weight-norm one (``weight_g``/``weight_v``,
        folded here: w = g * v / ||v|| over every dim but 0, torch weight_norm dim=0)."""
        sd = {}
        for k, v in state_dict.items():
            if k.endswith(".weight_v"):
                continue
            if k.endswith(".weight_g"):
                base = k[:-len(".weight_g")]
                vv = state_dict[base + ".weight_v"]
                n = vv.float().pow(2).sum(dim=tuple(range(1, vv.dim())), keepdim=True).sqrt()
                sd[base + ".weight"] = (v.float() * vv.float() / n).to(vv.dtype)
            else:
                sd[k] = v
        self._release()
        return super().load_state_dict(sd, strict=strict)

    def remove_weight_norm(self):
        """Weights are stored folded already (models.py:285-293 is a no-op here)."""
        return self

    def _dims(self):
        h = self.h
        d = _lib.nsf_dims()
        d.num_mels = int(_get(h, "num_mels"))
        d.upsample_initial_channel = int(_get(h, "upsample_initial_channel"))
        rates, ks = list(_get(h, "upsample_rates")), list(_get(h, "upsample_kernel_sizes"))
        d.num_upsamples = len(rates)
        for i, (u, k) in enumerate(zip(rates, ks)):
            d.upsample_rates[i] = int(u)
            d.upsample_kernel_sizes[i] = int(k)
        d.resblock = int(_get(h, "resblock"))
        rk, rd = list(_get(h, "resblock_kernel_sizes")), list(_get(h, "resblock_dilation_sizes"))
        d.num_kernels = len(rk)
        d.num_dilations = len(rd[0])
        for j, (k, dl) in enumerate(zip(rk, rd)):
            if len(dl) != d.num_dilations:
                raise _lib.HipError("every resblock needs the same number of dilations")
            d.resblock_kernel_sizes[j] = int(k)
            for q, v in enumerate(dl):
                d.resblock_dilation_sizes[j][q] = int(v)
        d.sampling_rate = int(_get(h, "sampling_rate"))
        d.harmonic_num = self.harmonic_num
        return d

    def _param_sig(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def handle(self):
        sig = self._param_sig()
        if self._h is not None and self._sig == sig:
            return self._h
        self._release()
        L = _lib.lib()
        dev = self.conv_pre.weight.device
        if dev.type != "cuda":
            raise _lib.HipError("NSF-HiFiGAN parameters must live on the GPU (call .cuda())")
        dims = self._dims()
        params = [v.detach().float().contiguous() for v in self.state_dict().values()]
        if len(params) != L.nsf_num_params(C_byref(dims)):
            raise _lib.HipError("parameter count does not match nsf_dims")
        self._keep = params
        arr = (_lib.C.c_void_p * len(params))(*[p.data_ptr() for p in params])
        h = _lib.C.c_void_p()
        dt = _lib.PD_DTYPE_BF16 if self.compute_dtype == "bf16" else _lib.PD_DTYPE_F32
        _lib.check(L.nsf_create(C_byref(dims), arr, dt, _lib.stream_ptr(dev), _lib.C.byref(h)))
        for k, v in self._options.items():
            rc = L.nsf_set_option(h, _lib.NSF_OPTIONS[k], v)
            if rc != 0:
                L.nsf_destroy(h)
                _lib.check(rc)
        self._h, self._sig = h, sig
        return h

    def _release(self):
        if getattr(self, "_h", None) is not None:
            torch.cuda.synchronize()
            _lib.lib().nsf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def synthesize(self, mel, f0, mel_scale=1.0, rand_ini=None, noise=None, seed=None, utt_ids=None, lens=None):
        """mel [B,T,M] time-major, f0 [B,T] -> wav [B, T*hop].  rand_ini [dim] / noise
        [B, T*hop, dim] replay the reference's torch.rand / randn_like draws
        (models.py:139,182); None draws them on the device (Philox, `seed` and each row's
        ``utt_ids``).  ``lens``: ragged batch, each row's length in frames (samples past
        lens[b] * hop are unspecified; the rest equal the utterance run alone)."""
        h = self.handle()
        dev = mel.device
        mel = mel.float().contiguous()
        f0 = f0.to(dev).float().contiguous()
        B, T, _ = mel.shape
        if f0.shape != (B, T):
            raise _lib.HipError(f"f0 must be [B,T] = {(B, T)}, got {tuple(f0.shape)}")
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        ri = None if rand_ini is None else rand_ini.to(dev).float().contiguous().reshape(-1)
        nz = None if noise is None else noise.to(dev).float().contiguous()
        wav = torch.empty(B, T * self.upp, device=dev, dtype=torch.float32)
        uid = _lib.utt_ids(utt_ids, B, dev)
        ln = _lib.lens(lens, B, T, dev)
        L = _lib.lib()
        ws, wsb = self._ws.get(L.nsf_workspace_size(h, B, T), dev)
        _lib.check(L.nsf_forward(h, _lib.fptr(mel), float(mel_scale), _lib.fptr(f0), _lib.fptr(ri), _lib.fptr(nz),
                                 int(seed), _lib.iptr(uid), _lib.iptr(ln), _lib.fptr(wav), B, T, ws, wsb,
                                 _lib.stream_ptr(dev)))
        return wav

    def forward(self, x, f0, **kw):
        """Reference signature: x [B, num_mels, T] (natural-log mel), f0 [B,T] -> [B,1,T*hop]."""
        return self.synthesize(x.transpose(1, 2).contiguous(), f0, 1.0, **kw)[:, None, :]


def C_byref(x):
    return _lib.C.byref(x)


class AttrDict(dict):
    def __getattr__(self, k):
        return self[k]


def load_model(model_path, device="cuda"):
    """models.py:21-33: config.json beside the checkpoint, ``cp_dict['generator']``."""
    model_path = pathlib.Path(model_path)
    with open(model_path.with_name("config.json")) as f:
        h = AttrDict(json.load(f))
    g = Generator(h)
    cp = torch.load(model_path, map_location="cpu", weights_only=True)
    g.load_state_dict(cp["generator"])
    g.eval()
    g.remove_weight_norm()
    return g.to(device), h


@register_vocoder
class NsfHifiGAN(BaseVocoder):
    """component/vocoder/nsf_hifigan.py:10-110 (spec2wav_torch / spec2wav)."""

    def __init__(self, hparams, model=None, h=None, device="cuda"):
        super().__init__(hparams)
        if model is None:
            model_path = pathlib.Path(hparams["vocoder_ckpt"])
            assert model_path.exists(), "HifiGAN model file is not found!"
            model, h = load_model(model_path, device)
        self.model, self.h = model, (h if h is not None else model.h)

    @property
    def device(self):
        return next(self.model.parameters()).device

    def to_device(self, device):
        self.model.to(device)

    def get_device(self):
        return self.device

    def spec2wav_torch(self, mel, **kwargs):
        """mel [B,T,bins] log10 mel, f0 [B,T] -> wav [B*T*hop] (nsf_hifigan.py:29-56)."""
        f0 = kwargs.get("f0")
        if f0 is None:
            raise TypeError("NSF-HiFiGAN needs f0 (Generator.forward(x, f0), models.py:265)")
        wav = self.model.synthesize(mel, f0, LOG10_TO_LN, rand_ini=kwargs.get("rand_ini"),
                                    noise=kwargs.get("noise"), seed=kwargs.get("seed"),
                                    utt_ids=kwargs.get("utt_ids"))
        return wav.view(-1)

    def spec2wav(self, mel, **kwargs):
        """mel [T,bins] numpy, f0 [T] -> wav numpy (nsf_hifigan.py:58-87)."""
        dev = self.device
        c = torch.as_tensor(np.asarray(mel, np.float32), device=dev)[None]
        f0 = kwargs.get("f0")
        f0 = None if f0 is None else torch.as_tensor(np.asarray(f0, np.float32), device=dev)[None]
        return self.spec2wav_torch(c, f0=f0).cpu().numpy()
