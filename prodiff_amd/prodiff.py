"""ProDiff denoiser + reverse sampler, drop-in for the reference classes.

``WaveNet`` replaces modules/decoder/wavenet.py:74-123 and ``GaussianDiffusion``
replaces modules/diffusion/prodiff.py:48-159.  Constructor signatures, parameter
and buffer names equal the reference's, so ``load_ckpt(model, ..., strict=False)``
(utils/ckpt_utils.py:28-68) fills them and ``ProDiffTeacher`` can hold them
unchanged (modules/svs/prodiff_teacher.py:49-66).  The nn.Conv1d/nn.Linear
children are parameter containers only: every forward runs the HIP library
(include/prodiff_hip.h) and raises if it is unavailable.
"""
from __future__ import annotations

from functools import partial

import numpy as np
import torch
from torch import nn

from . import _lib
from .schedules import diffusion_buffers, get_noise_schedule_list, posterior_step_scalars


class ResidualBlock(nn.Module):
    """Parameter container of wavenet.py:52-58 (compute lives in the fused kernels)."""

    def __init__(self, encoder_hidden, residual_channels, dilation):
        super().__init__()
        self.dilation = dilation
        self.dilated_conv = nn.Conv1d(residual_channels, 2 * residual_channels, 3, padding=dilation,
                                      dilation=dilation)
        self.diffusion_projection = nn.Linear(residual_channels, residual_channels)
        self.conditioner_projection = nn.Conv1d(encoder_hidden, 2 * residual_channels, 1)
        self.output_projection = nn.Conv1d(residual_channels, 2 * residual_channels, 1)


class Mish(nn.Module):
    """Marker module at mlp.1 (wavenet.py:22-24); applied inside the step-MLP kernel."""


class WaveNet(nn.Module):
    """Denoiser ``x0 = WaveNet(spec[B,1,M,T], step[B], cond[B,H,T])`` (wavenet.py:74-123)."""

    def __init__(self, in_dims, hidden_size, residual_layers, residual_channels, dilation_cycle_length):
        super().__init__()
        self.in_dims = in_dims
        self.hidden_size = hidden_size
        self.n_layers = residual_layers
        self.residual_channels = residual_channels
        self.dilation_cycle_length = dilation_cycle_length
        C = residual_channels
        self.input_projection = nn.Conv1d(in_dims, C, 1)
        self.mlp = nn.Sequential(nn.Linear(C, C * 4), Mish(), nn.Linear(C * 4, C))
        self.residual_layers = nn.ModuleList([
            ResidualBlock(hidden_size, C, 2 ** (i % dilation_cycle_length)) for i in range(residual_layers)
        ])
        self.skip_projection = nn.Conv1d(C, C, 1)
        self.output_projection = nn.Conv1d(C, in_dims, 1)
        nn.init.zeros_(self.output_projection.weight)
        self.compute_dtype = "fp32"
        self._options = {}
        self._h = None
        self._sig = None
        self._ws = _lib.Workspace()

    def set_compute_dtype(self, dtype):
        """'fp32' (exact, the parity path) or 'bf16' (bf16 MFMA, fp32 accumulate)."""
        if dtype not in ("fp32", "bf16"):
            raise ValueError(dtype)
        self.compute_dtype = dtype
        return self

    def set_options(self, **opts):
        """Kernel-variant options (pd_wavenet_set_option, include/prodiff_hip.h PD_WN_OPT_*): layer."""
        for k, v in opts.items():
            if k not in _lib.WN_OPTIONS:
                raise ValueError(f"unknown WaveNet option {k!r}")
            self._options[k] = int(v)
        return self

    # ----------------------------------------------------------- packing
    def ordered_params(self):
        """Tensors in the include/prodiff_hip.h order (== reference state-dict order)."""
        out = [self.input_projection.weight, self.input_projection.bias,
               self.mlp[0].weight, self.mlp[0].bias, self.mlp[2].weight, self.mlp[2].bias]
        for rl in self.residual_layers:
            out += [rl.dilated_conv.weight, rl.dilated_conv.bias,
                    rl.diffusion_projection.weight, rl.diffusion_projection.bias,
                    rl.conditioner_projection.weight, rl.conditioner_projection.bias,
                    rl.output_projection.weight, rl.output_projection.bias]
        out += [self.skip_projection.weight, self.skip_projection.bias,
                self.output_projection.weight, self.output_projection.bias]
        return out

    def param_signature(self):
        """What the packed handle depends on: dtype, options and every parameter's storage
        and version (load_state_dict / in-place updates change it)."""
        ps = self.ordered_params()
        return (self.compute_dtype, tuple(sorted(self._options.items()))) + tuple((p.data_ptr(), p._version) for p in ps)

    def handle(self):
        """The packed C handle; re-packed whenever a parameter is replaced or modified."""
        ps = self.ordered_params()
        sig = self.param_signature()
        if self._h is not None and sig == self._sig:
            return self._h
        L = _lib.lib()
        dev = ps[0].device
        if dev.type != "cuda":
            raise _lib.HipError("WaveNet parameters must live on the GPU (call .cuda())")
        tensors = [p.detach().float().contiguous() for p in ps]
        arr = (_lib.C.c_void_p * len(tensors))(*[t.data_ptr() for t in tensors])
        dims = _lib.pd_wavenet_dims(self.in_dims, self.hidden_size, self.n_layers,
                                    self.residual_channels, self.dilation_cycle_length)
        h = _lib.C.c_void_p()
        dt = _lib.PD_DTYPE_BF16 if self.compute_dtype == "bf16" else _lib.PD_DTYPE_F32
        _lib.check(L.pd_wavenet_create(_lib.C.byref(dims), arr, dt,
                                       _lib.stream_ptr(dev), _lib.C.byref(h)))
        for k, v in self._options.items():
            rc = L.pd_wavenet_set_option(h, _lib.WN_OPTIONS[k], v)
            if rc != 0:
                L.pd_wavenet_destroy(h)
                _lib.check(rc)
        self._release()
        self._h, self._sig = h, sig
        self._keep = tensors   # the pack is stream-ordered; keep sources alive
        return h

    def _release(self):
        if self._h is not None:
            torch.cuda.synchronize()
            _lib.lib().pd_wavenet_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            if self._h is not None:
                _lib.lib().pd_wavenet_destroy(self._h)
        except Exception:
            pass

    # ----------------------------------------------------------- forward
    @torch.no_grad()
    def forward(self, spec, diffusion_step, cond):
        """spec [B,1,M,T], diffusion_step [B] (long or float), cond [B,H,T] -> [B,1,M,T]."""
        h = self.handle()
        B, _, M, T = spec.shape
        assert M == self.in_dims and cond.shape == (B, self.hidden_size, T)
        spec = spec.float().contiguous()
        cond = cond.float().contiguous()
        steps = diffusion_step.reshape(B).float().contiguous()
        out = torch.empty_like(spec)
        L = _lib.lib()
        nbytes = L.pd_wavenet_workspace_size(h, B, T, 1)
        ws, wsb = self._ws.get(nbytes, spec.device)
        _lib.check(L.pd_wavenet_forward(h, _lib.fptr(spec), _lib.fptr(steps), _lib.fptr(cond),
                                        _lib.fptr(out), B, T, ws, wsb, _lib.stream_ptr(spec.device)))
        return out


class SampleGraph:
    """A captured sampler (``GaussianDiffusion.capture``): static input, static output.

    The graph bakes in device addresses: its own workspace and the draw buffers (held
    here), and the WaveNet handle's packed weight pool.  The handle is owned by the
    denoiser and re-packed (the old pool freed) when its parameters, dtype or options
    change, so ``replay`` refuses to run once the denoiser no longer matches the capture."""

    def __init__(self, graph, cond, mel, denoiser, keep=()):
        self.graph, self.cond, self.mel = graph, cond, mel
        self._denoiser = denoiser
        self._handle = denoiser._h.value
        self._sig = denoiser.param_signature()
        self._keep = keep        # workspace and captured draw buffers stay alive with the graph

    def replay(self):
        d = self._denoiser
        if d._h is None or d._h.value != self._handle or d.param_signature() != self._sig:
            raise RuntimeError("SampleGraph: the denoiser was re-packed or its parameters changed "
                               "since capture; capture again")
        self.graph.replay()
        return self.mel


class GaussianDiffusion(nn.Module):
    """x0-predict DDPM sampler (prodiff.py:48-159), fused on the GPU.

    Buffers (and their checkpoint override) are the reference's; inference runs
    every reverse step through ``pd_prodiff_sample``.
    """

    def __init__(self, out_dims, denoise_fn, timesteps=1000, time_scale=1, betas=None,
                 schedule_type="vpsde", max_beta=0.02, spec_min=None, spec_max=None):
        super().__init__()
        self.denoise_fn = denoise_fn
        self.mel_bins = out_dims
        if betas is not None:
            betas = betas.detach().cpu().numpy() if isinstance(betas, torch.Tensor) else betas
        else:
            betas = get_noise_schedule_list(schedule_mode=schedule_type, timesteps=timesteps + 1,
                                            min_beta=0.1, max_beta=max_beta, s=0.008)
        self.time_scale = time_scale
        self.num_timesteps = int(timesteps)
        to_torch = partial(torch.tensor, dtype=torch.float32)
        self.register_buffer("timesteps", to_torch(self.num_timesteps))
        self.register_buffer("timescale", to_torch(self.time_scale))
        for k, v in diffusion_buffers(betas).items():
            self.register_buffer(k, to_torch(v))
        spec_min = [-12] if spec_min is None else spec_min
        spec_max = [0] if spec_max is None else spec_max
        self.register_buffer("spec_min", torch.FloatTensor(spec_min)[None, None, :out_dims].transpose(-3, -2),
                             persistent=False)
        self.register_buffer("spec_max", torch.FloatTensor(spec_max)[None, None, :out_dims].transpose(-3, -2),
                             persistent=False)
        self._ws = _lib.Workspace()
        self._coef_cache = None

    def set_compute_dtype(self, dtype):
        self.denoise_fn.set_compute_dtype(dtype)
        return self

    def _step_scalars(self):
        key = tuple(b._version for b in (self.posterior_mean_coef1, self.posterior_mean_coef2,
                                         self.posterior_log_variance_clipped))
        if self._coef_cache is None or self._coef_cache[0] != key:
            c1, c2, sg = posterior_step_scalars(self.posterior_mean_coef1.detach().cpu().numpy(),
                                                self.posterior_mean_coef2.detach().cpu().numpy(),
                                                self.posterior_log_variance_clipped.detach().cpu().numpy())
            self._coef_cache = (key, c1, c2, sg)
        return self._coef_cache[1:]

    @torch.no_grad()
    def sample(self, cond, infer_step=4, x_T=None, noise=None, seed=None, workspace=None, utt_ids=None,
               lens=None):
        """cond [B,T,H] -> mel [B,T,M].

        lens: ragged batch -- each row's utterance length in frames (B ints <= T, or a device
        int32 tensor); row b's first lens[b] frames equal a run of that utterance alone (B = 1,
        T = lens[b]), the frames after it are unspecified (include/prodiff_hip.h).

        x_T: [B,1,M,T] draw (reference layout, prodiff.py:147) or None;
        noise: [S,B,1,M,T] per-step draws in sampling order, or None.
        Missing draws come from the on-device Philox generator keyed by ``seed``
        (default: drawn from torch's CPU generator, so torch.manual_seed applies) and
        by each row's utterance id (``utt_ids``, default 0..B-1): a row's draws do not
        depend on the rest of the batch.
        ``workspace``: a ``_lib.Workspace`` to use instead of the module's own (capture)."""
        if not isinstance(self.denoise_fn, WaveNet):
            raise TypeError("GaussianDiffusion needs a prodiff_amd.WaveNet denoise_fn")
        B, T, H = cond.shape
        M = self.mel_bins
        S = int(np.clip(infer_step, 1, self.num_timesteps))
        h = self.denoise_fn.handle()
        cond = cond.float().contiguous()
        dev = cond.device
        xT = None if x_T is None else x_T.float()[:, 0].transpose(1, 2).contiguous()
        nz = None if noise is None else noise.float()[:, :, 0].transpose(2, 3).contiguous()
        if nz is not None and nz.shape[0] < S:
            raise ValueError(f"noise holds {nz.shape[0]} steps, sampler needs {S}")
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        c1, c2, sg = self._step_scalars()
        mel = torch.empty(B, T, M, device=dev, dtype=torch.float32)
        uid = _lib.utt_ids(utt_ids, B, dev)
        ln = _lib.lens(lens, B, T, dev)
        L = _lib.lib()
        nbytes = L.pd_wavenet_workspace_size(h, B, T, S)
        ws, wsb = (workspace or self._ws).get(nbytes, dev)
        _lib.check(L.pd_prodiff_sample(h, _lib.fptr(cond), _lib.farr(c1), _lib.farr(c2), _lib.farr(sg), S,
                                       _lib.fptr(xT), _lib.fptr(nz), seed, _lib.iptr(uid), _lib.iptr(ln), _lib.fptr(mel),
                                       B, T, ws, wsb, _lib.stream_ptr(dev)))
        return mel

    @torch.no_grad()
    def capture(self, cond, infer_step=4, seed=0, x_T=None, noise=None, utt_ids=None):
        """Record the whole reverse process for cond's shape as ONE hipGraph.

        The library's calls are stream-ordered and allocation-free, so
        torch.cuda.CUDAGraph (hipGraph on ROCm) captures every launch of
        ``pd_prodiff_sample``; a replay costs one graph launch instead of one
        host launch per kernel -- the B=1 regime of the reference's per-step
        loop (prodiff.py:148-150).  The draws are keyed by the captured ``seed``
        (fixed across replays), or explicit ``x_T``/``noise`` draws are captured
        by address (parity mode).  Returns a ``SampleGraph``: copy new conditions
        into ``.cond`` and ``.replay()`` returns the static mel [B,T,M]."""
        cond = cond.float().contiguous()
        xT = None if x_T is None else x_T.float().contiguous().clone()
        nz = None if noise is None else noise.float().contiguous().clone()
        # the graph's own workspace, one buffer for every stream: the warm-up call below sizes it on
        # the current stream and the capture (on torch's capture stream) reuses it instead of
        # allocating a second full-size buffer from the graph pool; later eager calls may grow
        # (reallocate) self._ws without touching it
        ws = _lib.Workspace(per_stream=False)
        uid = _lib.utt_ids(utt_ids, cond.shape[0], cond.device)
        self.sample(cond, infer_step=infer_step, seed=seed, x_T=xT, noise=nz, workspace=ws, utt_ids=uid)   # packs, sizes ws
        torch.cuda.synchronize()
        static_cond = cond.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            mel = self.sample(static_cond, infer_step=infer_step, seed=seed, x_T=xT, noise=nz, workspace=ws,
                              utt_ids=uid)
        return SampleGraph(g, static_cond, mel, self.denoise_fn, keep=(ws, xT, nz, uid))

    def forward(self, cond, src_spec=None, gt_spec=None, infer_step=4, infer=False):
        if not infer:
            raise NotImplementedError("training (infer=False, prodiff.py:139-144) is out of scope")
        return self.denorm_spec(self.sample(cond, infer_step=infer_step))

    def norm_spec(self, x):
        return x

    def denorm_spec(self, x):
        return x
