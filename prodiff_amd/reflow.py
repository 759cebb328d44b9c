"""Rectified-flow sampler with the WaveNet velocity field, drop-in for the reference.

``RectifiedFlow`` replaces modules/diffusion/reflow.py:5-107 (the SVS teacher's
``diff_type: reflow``, modules/svs/prodiff_teacher.py:67-82) and
``PitchRectifiedFlow`` replaces reflow.py:110-144 (the pitch predictor's sampler,
modules/variance_predictor/pitch_predictor.py:40-55).  Constructor arguments,
``velocity_fn`` and the ``spec_min``/``spec_max`` buffers are the reference's.
The whole Euler / RK2 / RK4 / RK5 integration runs in ``pd_reflow_sample`` (every
velocity evaluation is the fused WaveNet), denormalisation in ``pd_reflow_denorm``;
both raise if the HIP library is unavailable.
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib
from .prodiff import WaveNet


class RectifiedFlow(nn.Module):
    def __init__(self, out_dims, denoise_fn, time_scale=1000, num_features=1, sampling_algorithm="euler",
                 spec_min=None, spec_max=None):
        super().__init__()
        self.velocity_fn = denoise_fn
        self.out_dims = out_dims
        self.num_features = num_features
        self.sampling_algorithm = sampling_algorithm
        self.t_start = 0.
        self.time_scale = time_scale
        spec_min = torch.FloatTensor(spec_min)[None, None, :out_dims].transpose(-3, -2)
        spec_max = torch.FloatTensor(spec_max)[None, None, :out_dims].transpose(-3, -2)
        self.register_buffer("spec_min", spec_min, persistent=False)
        self.register_buffer("spec_max", spec_max, persistent=False)
        self._ws = _lib.Workspace()

    def set_compute_dtype(self, dtype):
        self.velocity_fn.set_compute_dtype(dtype)
        return self

    def _algo(self):
        # reflow.py:90-95: unknown names fall back to Euler
        return _lib.PD_REFLOW.get(self.sampling_algorithm, _lib.PD_REFLOW["euler"])

    @torch.no_grad()
    def sample(self, cond, infer_step=20, x_T=None, seed=None, utt_ids=None, lens=None):
        """cond [B,T,H] (time-major, as the teacher hands it) -> x [B,T,M] before denorm_spec.

        x_T: [B,1,M,T] draw (reference layout, reflow.py:88) or None -> on-device Philox
        N(0,1) keyed by ``seed`` (default: drawn from torch's CPU generator) and each row's
        utterance id (``utt_ids``, default 0..B-1).  ``lens``: ragged batch (GaussianDiffusion.sample)."""
        if not isinstance(self.velocity_fn, WaveNet):
            raise TypeError("RectifiedFlow needs a prodiff_amd.WaveNet velocity_fn")
        if self.num_features != 1:
            raise NotImplementedError("num_features > 1 (the WaveNet velocity field takes one feature)")
        h = self.velocity_fn.handle()
        B, T, H = cond.shape
        M = self.out_dims
        S = max(1, int(infer_step))
        cond = cond.float().contiguous()
        dev = cond.device
        xT = None if x_T is None else x_T.float()[:, 0].transpose(1, 2).contiguous()
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        algo = self._algo()
        L = _lib.lib()
        nbytes = L.pd_reflow_workspace_size(h, B, T, S, algo)
        if nbytes == 0:
            raise ValueError(f"infer_step={S} with {self.sampling_algorithm} exceeds 128 velocity evaluations")
        ws, wsb = self._ws.get(nbytes, dev)
        x = torch.empty(B, T, M, device=dev, dtype=torch.float32)
        uid = _lib.utt_ids(utt_ids, B, dev)
        ln = _lib.lens(lens, B, T, dev)
        _lib.check(L.pd_reflow_sample(h, _lib.fptr(cond), S, algo, float(self.time_scale), _lib.fptr(xT), seed,
                                      _lib.iptr(uid), _lib.iptr(ln), _lib.fptr(x), B, T, ws, wsb,
                                      _lib.stream_ptr(dev)))
        return x

    def inference(self, cond, b=1, infer_step=20, device=None):
        """reflow.py:86-101: cond [B,H,T] (already transposed, :33) -> x [B,T,M]."""
        return self.sample(cond.transpose(1, 2), infer_step=infer_step)

    def forward(self, cond, gt_spec=None, infer_step=20, infer=True):
        if not infer:
            raise NotImplementedError("training (infer=False, reflow.py:36-43) is out of scope")
        return self.denorm_spec(self.sample(cond, infer_step=infer_step))

    def _denorm(self, x, mean_clamp, cmin=0.0, cmax=0.0):
        x = x.float().contiguous()
        M = x.shape[-1]
        smin = self.spec_min.reshape(-1).float().contiguous().to(x.device)
        smax = self.spec_max.reshape(-1).float().contiguous().to(x.device)
        rows = x.numel() // M
        out = torch.empty(x.shape[:-1] if mean_clamp else x.shape, device=x.device, dtype=torch.float32)
        _lib.check(_lib.lib().pd_reflow_denorm(_lib.fptr(x), _lib.fptr(smin), _lib.fptr(smax), smin.numel(), M, rows,
                                               1 if mean_clamp else 0, float(cmin), float(cmax), _lib.fptr(out),
                                               _lib.stream_ptr(x.device)))
        return out

    def norm_spec(self, x):
        raise NotImplementedError("norm_spec is used by training only (reflow.py:38)")

    def denorm_spec(self, x):
        """reflow.py:106-107: (x + 1) / 2 * (spec_max - spec_min) + spec_min."""
        return self._denorm(x, False)


class PitchRectifiedFlow(RectifiedFlow):
    def __init__(self, repeat_bins, denoise_fn, time_scale=1000, sampling_algorithm="euler", spec_min=-8.0,
                 spec_max=8.0, clamp_min=-12.0, clamp_max=12.0):
        self.clamp_min = clamp_min
        self.clamp_max = clamp_max
        self.repeat_bins = repeat_bins
        super().__init__(out_dims=repeat_bins, denoise_fn=denoise_fn, time_scale=time_scale, num_features=1,
                         sampling_algorithm=sampling_algorithm, spec_min=[spec_min], spec_max=[spec_max])

    def denorm_spec(self, x):
        """reflow.py:138-144: [B,T,R] -> mean over the R repeat bins, clamped -> [B,T]."""
        return self._denorm(x, True, self.clamp_min, self.clamp_max)
