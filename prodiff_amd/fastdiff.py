"""FastDiff eps-network and sampler, drop-in for the reference.

``FastDiff`` mirrors modules/FastDiff/module/FastDiff_model.py:10-123 (same
constructor, same children and state-dict keys, including the weight-norm
``weight_g``/``weight_v`` form the checkpoints store, fastdiff.py:41), and
``sampling_given_noise_schedule`` mirrors util.py:158-232.  The torch children
are parameter containers: all compute runs in libprodiff_hip (fd_forward /
fd_sample), which raises when it is unavailable.
"""
from __future__ import annotations

import logging
import warnings

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .schedules import fastdiff_infer_params


def _weight_norm(m):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return torch.nn.utils.weight_norm(m)


class DiffusionDBlock(nn.Module):
    """modules.py:116-129 (parameters)."""

    def __init__(self, input_size, hidden_size, factor):
        super().__init__()
        self.factor = factor
        self.residual_dense = nn.Conv1d(input_size, hidden_size, 1)
        self.conv = nn.ModuleList([
            nn.Conv1d(input_size, hidden_size, 3, dilation=1, padding=1),
            nn.Conv1d(hidden_size, hidden_size, 3, dilation=2, padding=2),
            nn.Conv1d(hidden_size, hidden_size, 3, dilation=4, padding=4),
        ])


class KernelPredictor(nn.Module):
    """modules.py:257-318 (parameters; Sequential indices match the reference)."""

    def __init__(self, cond_channels, conv_in_channels, conv_out_channels, conv_layers,
                 conv_kernel_size=3, kpnet_hidden_channels=64, kpnet_conv_size=3, kpnet_dropout=0.0):
        super().__init__()
        self.conv_in_channels = conv_in_channels
        self.conv_out_channels = conv_out_channels
        self.conv_kernel_size = conv_kernel_size
        self.conv_layers = conv_layers
        l_w = conv_in_channels * conv_out_channels * conv_kernel_size * conv_layers
        l_b = conv_out_channels * conv_layers
        pad = (kpnet_conv_size - 1) // 2
        Hk = kpnet_hidden_channels
        act = lambda: nn.LeakyReLU(0.1)
        self.input_conv = nn.Sequential(nn.Conv1d(cond_channels, Hk, 5, padding=2, bias=True), act())
        self.residual_conv = nn.Sequential(
            nn.Dropout(kpnet_dropout), nn.Conv1d(Hk, Hk, kpnet_conv_size, padding=pad), act(),
            nn.Conv1d(Hk, Hk, kpnet_conv_size, padding=pad), act(),
            nn.Dropout(kpnet_dropout), nn.Conv1d(Hk, Hk, kpnet_conv_size, padding=pad), act(),
            nn.Conv1d(Hk, Hk, kpnet_conv_size, padding=pad), act(),
            nn.Dropout(kpnet_dropout), nn.Conv1d(Hk, Hk, kpnet_conv_size, padding=pad), act(),
            nn.Conv1d(Hk, Hk, kpnet_conv_size, padding=pad), act(),
        )
        self.kernel_conv = nn.Conv1d(Hk, l_w, kpnet_conv_size, padding=pad, bias=True)
        self.bias_conv = nn.Conv1d(Hk, l_b, kpnet_conv_size, padding=pad, bias=True)


class TimeAware_LVCBlock(nn.Module):
    """modules.py:141-188 (parameters)."""

    def __init__(self, in_channels, cond_channels, upsample_ratio, conv_layers=4, conv_kernel_size=3,
                 cond_hop_length=256, kpnet_hidden_channels=64, kpnet_conv_size=3, kpnet_dropout=0.0,
                 noise_scale_embed_dim_out=512):
        super().__init__()
        self.cond_hop_length = cond_hop_length
        self.conv_layers = conv_layers
        self.conv_kernel_size = conv_kernel_size
        self.upsample_ratio = upsample_ratio
        self.convs = nn.ModuleList()
        self.upsample = nn.ConvTranspose1d(in_channels, in_channels, kernel_size=upsample_ratio * 2,
                                           stride=upsample_ratio,
                                           padding=upsample_ratio // 2 + upsample_ratio % 2,
                                           output_padding=upsample_ratio % 2)
        self.kernel_predictor = KernelPredictor(cond_channels, in_channels, 2 * in_channels, conv_layers,
                                                conv_kernel_size, kpnet_hidden_channels, kpnet_conv_size,
                                                kpnet_dropout)
        self.fc_t = nn.Linear(noise_scale_embed_dim_out, cond_channels)
        for i in range(conv_layers):
            padding = (3 ** i) * int((conv_kernel_size - 1) / 2)
            self.convs.append(nn.Conv1d(in_channels, in_channels, kernel_size=conv_kernel_size,
                                        padding=padding, dilation=3 ** i))


class FastDiff(nn.Module):
    """FastDiff_model.py:10-123.  forward((audio[B,1,L], c[B,80,T'], steps[B,1])) -> eps[B,1,L]."""

    def __init__(self, audio_channels=1, inner_channels=32, cond_channels=80, upsample_ratios=(8, 8, 4),
                 lvc_layers_each_block=4, lvc_kernel_size=3, kpnet_hidden_channels=64, kpnet_conv_size=3,
                 dropout=0.0, diffusion_step_embed_dim_in=128, diffusion_step_embed_dim_mid=512,
                 diffusion_step_embed_dim_out=512, use_weight_norm=True):
        super().__init__()
        self.diffusion_step_embed_dim_in = diffusion_step_embed_dim_in
        self.audio_channels = audio_channels
        self.cond_channels = cond_channels
        self.upsample_ratios = list(upsample_ratios)
        self.lvc_block_nums = len(upsample_ratios)
        self._dims = dict(audio_channels=audio_channels, inner_channels=inner_channels,
                          cond_channels=cond_channels, lvc_layers_each_block=lvc_layers_each_block,
                          lvc_kernel_size=lvc_kernel_size, kpnet_hidden_channels=kpnet_hidden_channels,
                          kpnet_conv_size=kpnet_conv_size, step_embed_in=diffusion_step_embed_dim_in,
                          step_embed_mid=diffusion_step_embed_dim_mid,
                          step_embed_out=diffusion_step_embed_dim_out)
        self.first_audio_conv = nn.Conv1d(1, inner_channels, kernel_size=7, padding=3, dilation=1, bias=True)
        self.lvc_blocks = nn.ModuleList()
        self.downsample = nn.ModuleList()
        self.fc_t = nn.ModuleList()
        self.fc_t1 = nn.Linear(diffusion_step_embed_dim_in, diffusion_step_embed_dim_mid)
        self.fc_t2 = nn.Linear(diffusion_step_embed_dim_mid, diffusion_step_embed_dim_out)
        hop = 1
        for n in range(self.lvc_block_nums):
            hop *= upsample_ratios[n]
            self.lvc_blocks.append(TimeAware_LVCBlock(
                inner_channels, cond_channels, upsample_ratios[n], lvc_layers_each_block, lvc_kernel_size,
                hop, kpnet_hidden_channels, kpnet_conv_size, dropout, diffusion_step_embed_dim_out))
            self.downsample.append(DiffusionDBlock(inner_channels, inner_channels,
                                                   upsample_ratios[self.lvc_block_nums - n - 1]))
        self.hop_length = hop
        self.final_conv = nn.Sequential(nn.Conv1d(inner_channels, audio_channels, kernel_size=7, padding=3,
                                                  dilation=1, bias=True))
        if use_weight_norm:
            self.apply_weight_norm()
        self.compute_dtype = "fp32"
        self._options = {}
        self._h = None
        self._sig = None
        self._ws = _lib.Workspace()

    def set_compute_dtype(self, dtype):
        """'fp32' (exact, the parity path) or 'bf16' (bf16 MFMA, bf16 LVC kernels)."""
        if dtype not in ("fp32", "bf16"):
            raise ValueError(dtype)
        self.compute_dtype = dtype
        return self

    def set_options(self, **opts):
        """Kernel-variant options (fd_set_option, include/prodiff_hip.h FD_OPT_*): lvc_ts,
        lvc_ts_sub, lvc_fuse, lvc_pf, lvc_sub, kp_side.  Unset ones keep the measured defaults."""
        for k, v in opts.items():
            if k not in _lib.FD_OPTIONS:
                raise ValueError(f"unknown FastDiff option {k!r}")
            self._options[k] = int(v)
        return self

    # ------------------------------------------------------- weight norm
    def apply_weight_norm(self):
        """FastDiff_model.py:115-122 (Conv1d only; ConvTranspose1d/Linear keep plain weights)."""
        for m in self.modules():
            if type(m) is nn.Conv1d:
                _weight_norm(m)

    def remove_weight_norm(self):
        """FastDiff_model.py:104-113."""
        for m in self.modules():
            try:
                torch.nn.utils.remove_weight_norm(m)
            except ValueError:
                pass

    # ------------------------------------------------------- packing
    def _convs_in_order(self):
        """(module, kind) in the include/prodiff_hip.h FD parameter order."""
        seq = [self.first_audio_conv, self.fc_t1, self.fc_t2]
        for blk in self.lvc_blocks:
            kp = blk.kernel_predictor
            seq += [blk.upsample, kp.input_conv[0]]
            seq += [kp.residual_conv[j] for j in (1, 3, 6, 8, 11, 13)]
            seq += [kp.kernel_conv, kp.bias_conv, blk.fc_t]
            seq += list(blk.convs)
        for dn in self.downsample:
            seq += [dn.residual_dense] + list(dn.conv)
        seq += [self.final_conv[0]]
        return seq

    def _param_sig(self):
        return (self.compute_dtype, tuple(sorted(self._options.items()))) + \
            tuple((p.data_ptr(), p._version) for p in self.parameters())

    def handle(self):
        sig = self._param_sig()
        if self._h is not None and sig == self._sig:
            return self._h
        L = _lib.lib()
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise _lib.HipError("FastDiff parameters must live on the GPU (call .cuda())")
        st = _lib.stream_ptr(dev)
        keep, ptrs = [], []
        for m in self._convs_in_order():
            if hasattr(m, "weight_g"):
                g = m.weight_g.detach().float().contiguous()
                v = m.weight_v.detach().float().contiguous()
                w = torch.empty_like(v)
                _lib.check(L.fd_fold_weight_norm(_lib.fptr(w), _lib.fptr(g), _lib.fptr(v), v.shape[0],
                                                 v[0].numel(), st))
            else:
                w = m.weight.detach().float().contiguous()
            b = m.bias.detach().float().contiguous()
            keep += [w, b]
            ptrs += [w.data_ptr(), b.data_ptr()]
        arr = (_lib.C.c_void_p * len(ptrs))(*ptrs)
        d = self._dims
        ratios = (_lib.C.c_int * 4)(*(self.upsample_ratios + [0] * (4 - len(self.upsample_ratios))))
        dims = _lib.fd_dims(d["audio_channels"], d["inner_channels"], d["cond_channels"], self.lvc_block_nums,
                            ratios, d["lvc_layers_each_block"], d["lvc_kernel_size"],
                            d["kpnet_hidden_channels"], d["kpnet_conv_size"], d["step_embed_in"],
                            d["step_embed_mid"], d["step_embed_out"])
        h = _lib.C.c_void_p()
        dt = _lib.PD_DTYPE_BF16 if self.compute_dtype == "bf16" else _lib.PD_DTYPE_F32
        _lib.check(L.fd_create(_lib.C.byref(dims), arr, dt, st, _lib.C.byref(h)))
        for k, v in self._options.items():
            rc = L.fd_set_option(h, _lib.FD_OPTIONS[k], v)
            if rc != 0:
                L.fd_destroy(h)
                _lib.check(rc)
        self._release()
        self._h, self._sig, self._keep = h, sig, keep
        return h

    def _release(self):
        if self._h is not None:
            torch.cuda.synchronize()
            _lib.lib().fd_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            if self._h is not None:
                _lib.lib().fd_destroy(self._h)
        except Exception:
            pass

    # ------------------------------------------------------- forward
    @torch.no_grad()
    def forward(self, data):
        audio, c, diffusion_steps = data
        h = self.handle()
        B, _, L = audio.shape
        Tc = c.shape[-1]
        assert L == Tc * self.hop_length, "length of (x, kernel) is not matched"
        audio = audio.float().contiguous()
        c = c.float().contiguous()
        steps = diffusion_steps.reshape(B).float().contiguous()
        eps = torch.empty_like(audio)
        lib = _lib.lib()
        ws, wsb = self._ws.get(lib.fd_workspace_size(h, B, Tc, 1), audio.device)
        _lib.check(lib.fd_forward(h, _lib.fptr(audio), _lib.fptr(c), _lib.fptr(steps), _lib.fptr(eps), B, Tc,
                                  ws, wsb, _lib.stream_ptr(audio.device)))
        return eps

    @torch.no_grad()
    def draw_x_T(self, B, Tc, seed, utt_ids=None, device=None):
        """The samplers' x_T ~ N(0,1) draw (util.py:208) for (seed, utt_ids): [B,1,L]."""
        h = self.handle()
        dev = device if device is not None else next(self.parameters()).device
        x = torch.empty(B, 1, Tc * self.hop_length, device=dev, dtype=torch.float32)
        uid = _lib.utt_ids(utt_ids, B, dev)
        _lib.check(_lib.lib().fd_draw_x_T(h, _lib.fptr(x), B, Tc, int(seed), _lib.iptr(uid), _lib.stream_ptr(dev)))
        return x

    @torch.no_grad()
    def sample_coefs(self, mel, ce, den, sg, steps, x_T=None, noise=None, seed=None, utt_ids=None, draw0=0,
                     lens=None):
        """The reverse loop with explicit per-pass coefficients (fd_sample_coefs): pass j
        evaluates eps at steps[j] and sets x = (x - ce[j] eps) / den[j] + sg[j] z.  ``lens``: ragged
        batch, each row's utterance length in mel frames (``sample``)."""
        h = self.handle()
        B, Tc, _ = mel.shape
        N = len(steps)
        L = Tc * self.hop_length
        dev = mel.device
        mel = mel.float().contiguous()
        xT = None if x_T is None else x_T.float().reshape(B, L).contiguous()
        nz = None if noise is None else noise.float().reshape(-1, B, L).contiguous()
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        wav = torch.empty(B, 1, L, device=dev, dtype=torch.float32)
        uid = _lib.utt_ids(utt_ids, B, dev)
        ln = _lib.lens(lens, B, Tc, dev)
        lib = _lib.lib()
        ws, wsb = self._ws.get(lib.fd_workspace_size(h, B, Tc, N), dev)
        _lib.check(lib.fd_sample_coefs(h, _lib.fptr(mel), _lib.farr(ce), _lib.farr(den), _lib.farr(sg),
                                       _lib.farr(steps), N, _lib.fptr(xT), _lib.fptr(nz), seed, _lib.iptr(uid),
                                       _lib.iptr(ln), int(draw0), _lib.fptr(wav), B, Tc, ws, wsb,
                                       _lib.stream_ptr(dev)))
        return wav

    @torch.no_grad()
    def sample(self, mel, beta, alpha, sigma, steps, x_T=None, noise=None, seed=None, utt_ids=None, lens=None):
        """Fused reverse process.  mel [B,T',80] TIME-major (the ProDiff output);
        beta/alpha/sigma/steps: float32 arrays of the reverse schedule;
        x_T [B,1,L] / noise [N-1,B,1,L] optional explicit draws -> wav [B,1,L].
        Missing draws: on-device Philox keyed by ``seed`` and each row's ``utt_ids``.
        lens: ragged batch -- each row's utterance length in mel frames (<= T'); row b's first
        lens[b] * hop samples equal a run of that utterance alone (include/prodiff_hip.h)."""
        h = self.handle()
        B, Tc, _ = mel.shape
        N = len(steps)
        L = Tc * self.hop_length
        dev = mel.device
        mel = mel.float().contiguous()
        xT = None if x_T is None else x_T.float().reshape(B, L).contiguous()
        nz = None if noise is None else noise.float().reshape(-1, B, L).contiguous()
        if nz is not None and nz.shape[0] < N - 1:
            raise ValueError(f"noise holds {nz.shape[0]} draws, sampler needs {N - 1}")
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        wav = torch.empty(B, 1, L, device=dev, dtype=torch.float32)
        uid = _lib.utt_ids(utt_ids, B, dev)
        ln = _lib.lens(lens, B, Tc, dev)
        lib = _lib.lib()
        ws, wsb = self._ws.get(lib.fd_workspace_size(h, B, Tc, N), dev)
        _lib.check(lib.fd_sample(h, _lib.fptr(mel), _lib.farr(beta), _lib.farr(alpha), _lib.farr(sigma),
                                 _lib.farr(steps), N, _lib.fptr(xT), _lib.fptr(nz), seed, _lib.iptr(uid),
                                 _lib.iptr(ln), _lib.fptr(wav), B, Tc, ws, wsb, _lib.stream_ptr(dev)))
        return wav


def _pass_coefs(b, a, s, steps, ddim):
    """Per-pass (ce, den, sg, step) of the reverse loop (util.py:211-226), pass j = schedule
    index n = N-1-j, in float32 as the reference forms them (torch float tensors):
    DDPM  x = (x - b/sqrt(1-a^2) eps) / sqrt(1-b) + [n>0] s z
    DDIM  x = c1 x + (c2 + c3) eps,  a' = a/sqrt(1-b), c1 = a'/a, c2 = -sqrt(1-a^2) c1,
          c3 = sqrt(1-a'^2), as (x - ce eps) / den with ce = -(c2 + c3)/c1, den = 1/c1."""
    N = len(steps)
    f = np.float32
    ce, den, sg, st = (np.zeros(N, f) for _ in range(4))
    for j in range(N):
        n = N - 1 - j
        bn, an = f(b[n]), f(a[n])
        st[j] = steps[n]
        if ddim:
            anext = f(an / f(np.sqrt(f(1) - bn)))
            c1 = f(anext / an)
            c2 = f(-f(np.sqrt(f(1) - f(an * an))) * c1)
            c3 = f(np.sqrt(f(1) - f(anext * anext)))
            ce[j] = f(-(c2 + c3) / c1)
            den[j] = f(f(1) / c1)
        else:
            ce[j] = f(bn / f(np.sqrt(f(1) - f(an * an))))
            den[j] = f(np.sqrt(f(1) - bn))
            sg[j] = f(s[n]) if n > 0 else f(0)
    return ce, den, sg, st


def sampling_given_noise_schedule(net, size, diffusion_hyperparams, inference_noise_schedule, condition=None,
                                  ddim=False, return_sequence=False, x_T=None, noise=None, seed=None):
    """util.py:158-232 on the fused GPU path.  ``condition`` is [B,80,T'] as in the
    reference; ``diffusion_hyperparams['alpha']`` is the training alpha table.
    ddim=True takes the deterministic update (util.py:215-220); return_sequence=True returns
    [x_T, x after pass 1, ..., x_0] (util.py:209-210,228-231), running the passes one call
    each with the fused run's draw keys."""
    if not isinstance(net, FastDiff):
        raise TypeError("net must be a prodiff_amd.FastDiff")
    alpha_train = np.asarray(torch.as_tensor(diffusion_hyperparams["alpha"]).cpu().numpy(), np.float32)
    sched = torch.as_tensor(inference_noise_schedule).detach().cpu().numpy().astype(np.float32)
    b, a, s, steps = fastdiff_infer_params(sched, alpha_train)
    B, _, L = size
    mel = condition.float().transpose(1, 2).contiguous()
    assert L == mel.shape[1] * net.hop_length
    N = len(steps)
    if not ddim and not return_sequence:
        return net.sample(mel, b[:N], a[:N], s[:N], steps, x_T=x_T, noise=noise, seed=seed)
    ce, den, sg, st = _pass_coefs(b[:N], a[:N], s[:N], steps, ddim)
    if not return_sequence:
        return net.sample_coefs(mel, ce, den, sg, st, x_T=x_T, noise=noise, seed=seed)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    if x_T is None:   # the fused run's x_T draw (fd_draw_x_T: fd_sample_coefs' draw with x_T NULL)
        x = net.draw_x_T(B, mel.shape[1], seed, device=mel.device)
    else:
        x = x_T.float().reshape(B, 1, L).clone()
    xs = [x.clone()]
    nz = None if noise is None else noise.float().reshape(-1, B, 1, L)
    for j in range(N):
        x = net.sample_coefs(mel, ce[j:j + 1], den[j:j + 1], sg[j:j + 1], st[j:j + 1], x_T=x,
                             noise=None if nz is None or sg[j] == 0 else nz[j:j + 1], seed=seed, draw0=j)
        xs.append(x.clone())
    return xs
