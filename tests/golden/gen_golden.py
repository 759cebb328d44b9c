"""Generate the golden parity vectors from the REFERENCE PyTorch code.

Runs only in the survey container, where ``/root/reference`` exists:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

The reference is imported read-only with the shims SURVEY.md §8(c) lists
(lower-case ``modules.fastdiff`` alias for FastDiff_model.py:4-5, and
``Tensor.cuda`` as identity for the hard-coded ``.cuda()`` in util.py:68,214,424).
Weights are drawn by ``prodiff_amd.synth`` (keyed by parameter name), so only
inputs/outputs are stored; the GPU box regenerates the same weights.
Every random draw the reference makes (``torch.rand``/``torch.randn`` in
prodiff.py:118,147, ``std_normal`` in util.py:208,226) is replaced by a seeded
draw and recorded (cloned: util.py:223-224 mutates x in place).
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

from prodiff_amd import synth  # noqa: E402

torch.Tensor.cuda = lambda self, *a, **k: self          # shim (util.py:68,214,424)
sys.modules.setdefault("chardet", types.ModuleType("chardet"))   # utils/__init__.py:6
torch.set_num_threads(8)

from modules.decoder.wavenet import WaveNet            # noqa: E402
from modules.diffusion.prodiff import GaussianDiffusion  # noqa: E402
import modules.FastDiff                                # noqa: E402
import modules.FastDiff.module                         # noqa: E402
import modules.FastDiff.module.modules as fd_modules   # noqa: E402
import modules.FastDiff.module.util as fd_util         # noqa: E402
sys.modules["modules.fastdiff"] = modules.FastDiff
sys.modules["modules.fastdiff.module"] = modules.FastDiff.module
sys.modules["modules.fastdiff.module.modules"] = fd_modules
sys.modules["modules.fastdiff.module.util"] = fd_util
from modules.FastDiff.module.FastDiff_model import FastDiff  # noqa: E402

OUT = HERE
FASTDIFF_SCHEDULES = {   # component/vocoder/fastdiff.py:62-73
    3: [9.0000e-05, 9.0000e-03, 6.0000e-01],
    4: [3.2176e-04, 2.5743e-03, 2.5376e-02, 7.0414e-01],
    6: [1.7838445955931093e-06, 2.7984189728158526e-05, 0.00043231004383414984,
        0.006634317338466644, 0.09357017278671265, 0.6000000238418579],
    8: [6.689325005027058e-07, 1.0033881153503899e-05, 0.00015496854030061513,
        0.002387222135439515, 0.035597629845142365, 0.3681158423423767, 0.4735414385795593, 0.5],
}


def load_synth(model, shapes, seed):
    sd = model.state_dict()
    params = synth.synth_params(shapes, seed)
    assert set(params) <= set(sd), set(params) - set(sd)
    missing = [k for k in sd if k not in params]
    assert all(k in ("spec_min", "spec_max") or "timesteps" in k or "timescale" in k
               or k.startswith(("betas", "alphas", "sqrt", "log_", "posterior"))
               for k in missing), missing
    for k, v in params.items():
        assert tuple(sd[k].shape) == tuple(v.shape), (k, sd[k].shape, v.shape)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    return params


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"  wrote {name}.npz  ({os.path.getsize(path) / 1024:.0f} KiB)")


# --------------------------------------------------------------------------
# WaveNet denoiser (wavenet.py:74-123)
# --------------------------------------------------------------------------
WAVENET_CASES = {
    # name: (in_dims, hidden, layers, channels, cycle, B, T, seed, steps)
    "wavenet_m80_c256_l20_cyc1": (80, 256, 20, 256, 1, 2, 48, 11, [0, 1]),
    "wavenet_m80_c256_l20_float": (80, 256, 20, 256, 1, 2, 48, 11, [537.5, 12.25]),
    "wavenet_m64_c256_l20_cyc5": (64, 256, 20, 256, 5, 2, 64, 12, [3, 900]),
    "wavenet_m128_c256_l20_cyc1": (128, 256, 20, 256, 1, 1, 37, 13, [2]),
    "wavenet_m80_c64_l4_cyc2": (80, 32, 4, 64, 2, 3, 29, 14, [0, 1, 3]),
}


def gen_wavenet():
    for name, (M, H, L, C, cyc, B, T, seed, steps) in WAVENET_CASES.items():
        net = WaveNet(M, H, L, C, cyc).eval()
        load_synth(net, synth.wavenet_param_shapes(M, H, L, C), seed)
        spec = synth.synth_inputs(seed + 100, (B, 1, M, T))
        cond = synth.synth_inputs(seed + 200, (B, H, T))
        is_float = any(isinstance(s, float) for s in steps)
        st = torch.tensor(steps, dtype=torch.float32 if is_float else torch.long)
        with torch.no_grad():
            out = net(torch.from_numpy(spec), st, torch.from_numpy(cond)).numpy()
        save(name, dims=np.array([M, H, L, C, cyc]), seed=seed, spec=spec, cond=cond,
             steps=np.array(steps, dtype=np.float32), out=out)


# --------------------------------------------------------------------------
# ProDiff sampler (prodiff.py:48-153)
# --------------------------------------------------------------------------
class Recorder:
    """Replace torch.rand / torch.randn with seeded draws and record them."""

    def __init__(self, seed):
        self.seed = seed
        self.n = 0
        self.rand = []
        self.randn = []

    def __enter__(self):
        self._r, self._rn = torch.rand, torch.randn

        def rand(*size, device=None, **kw):
            a = synth.synth_inputs(self.seed * 1000 + self.n, tuple(size), kind="uniform")
            self.n += 1
            self.rand.append(a.copy())
            return torch.from_numpy(a)

        def randn(size, device=None, **kw):
            a = synth.synth_inputs(self.seed * 1000 + self.n, tuple(size))
            self.n += 1
            self.randn.append(a.copy())
            return torch.from_numpy(a)

        torch.rand, torch.randn = rand, randn
        return self

    def __exit__(self, *a):
        torch.rand, torch.randn = self._r, self._rn


PRODIFF_CASES = {
    # name: (timesteps, max_beta, M, B, T, seed)
    "prodiff_t2_m80": (2, 40.0, 80, 2, 40, 21),     # C2-shape sampler (2-iter)
    "prodiff_t4_m80": (4, 40.0, 80, 1, 33, 22),     # C1-shape teacher (4-iter)
    "prodiff_t4_m128": (4, 40.0, 128, 2, 24, 23),   # C5-shape (SVS, 128 mel bins)
}


def gen_prodiff():
    for name, (ts, mb, M, B, T, seed) in PRODIFF_CASES.items():
        H, L, C = 256, 20, 256
        net = WaveNet(M, H, L, C, 1)
        gd = GaussianDiffusion(out_dims=M, denoise_fn=net, timesteps=ts, time_scale=1000,
                               schedule_type="vpsde", max_beta=mb,
                               spec_min=[-12], spec_max=[0]).eval()
        load_synth(net, synth.wavenet_param_shapes(M, H, L, C), seed)
        cond = synth.synth_inputs(seed + 300, (B, T, H))
        with torch.no_grad(), Recorder(seed) as rec:
            mel = gd(torch.from_numpy(cond), infer=True).numpy()
        assert len(rec.rand) == 1 and len(rec.randn) == min(4, ts)
        bufs = {k: v.numpy() for k, v in gd.state_dict().items() if not k.startswith("denoise_fn")}
        save(name, timesteps=ts, max_beta=mb, seed=seed, cond=cond, x_T=rec.rand[0],
             noise=np.stack(rec.randn), mel=mel, **{"buf_" + k: v for k, v in bufs.items()})


def gen_schedules():
    out = {}
    for ts in (1, 2, 4, 8, 100):
        for mb in (40.0, 0.06):
            gd = GaussianDiffusion(out_dims=4, denoise_fn=None, timesteps=ts, max_beta=mb,
                                   spec_min=[-12], spec_max=[0])
            for k, v in gd.state_dict().items():
                out[f"t{ts}_mb{mb}_{k}"] = v.numpy()
    # the other ProDiff schedule types (prodiff.py:27-46); logsnr yields betas outside
    # (0, 1) and NaN buffers in the reference -- recorded as they are
    for st in ("linear", "cosine", "logsnr"):
        for ts in (4, 100):
            gd = GaussianDiffusion(out_dims=4, denoise_fn=None, timesteps=ts, max_beta=0.06,
                                   schedule_type=st, spec_min=[-12], spec_max=[0])
            for k, v in gd.state_dict().items():
                out[f"{st}_t{ts}_{k}"] = v.numpy()
    # FastDiff: training linear schedule (fastdiff.py:44-51) and the reverse
    # schedules (fastdiff.py:62-73) mapped to fractional steps (util.py:187-206)
    beta = torch.linspace(1e-6, 0.01, 1000)
    dh = fd_util.compute_hyperparams_given_schedule(beta)
    out["fd_train_alpha"] = dh["alpha"].numpy()
    out["fd_train_sigma"] = dh["sigma"].numpy()
    long_scheds = {1000: torch.linspace(0.000001, 0.01, 1000),   # fastdiff.py:60-63 (torch, float32)
                   200: torch.linspace(0.0001, 0.02, 200)}
    for n, sched in list(FASTDIFF_SCHEDULES.items()) + list(long_scheds.items()):
        b = torch.FloatTensor(sched) if isinstance(sched, list) else sched.clone()
        a = 1 - b
        sg = b + 0
        for i in range(1, len(b)):
            a[i] *= a[i - 1]
            sg[i] *= (1 - a[i - 1]) / (1 - a[i])
        a, sg = torch.sqrt(a), torch.sqrt(sg)
        steps = [fd_util.map_noise_scale_to_time_step(a[i], dh["alpha"]) for i in range(len(b))]
        out[f"fd_n{n}_beta"] = b.numpy()
        out[f"fd_n{n}_alpha"] = a.numpy()
        out[f"fd_n{n}_sigma"] = sg.numpy()
        out[f"fd_n{n}_steps"] = np.array(steps, dtype=np.float32)
    save("schedules", **out)


# --------------------------------------------------------------------------
# FastDiff network (FastDiff_model.py:74-102) and sampler (util.py:158-232)
# --------------------------------------------------------------------------
def build_fastdiff(seed):
    m = FastDiff()           # base.yaml defaults, weight norm on (FastDiff_model.py:70-71)
    params = load_synth(m, synth.fastdiff_param_shapes(), seed)
    m.remove_weight_norm()   # fastdiff.py:82
    return m.eval(), params


def gen_fastdiff():
    seed = 31
    m, _ = build_fastdiff(seed)
    B, Tc = 2, 8
    L = Tc * 256
    audio = synth.synth_inputs(seed + 1, (B, 1, L))
    c = synth.synth_inputs(seed + 2, (B, 80, Tc), loc=-5.0, scale=2.0)
    steps = np.array([[7.41324], [498.054]], dtype=np.float32)
    caps = {}

    def hook(name):
        def f(mod, inp, out):
            if isinstance(out, tuple):
                for i, o in enumerate(out):
                    caps[f"{name}.out{i}"] = o.detach().numpy().copy()
            else:
                caps[name] = out.detach().numpy().copy()
        return f

    hs = [m.first_audio_conv.register_forward_hook(hook("first_audio_conv"))]
    for n in range(3):
        hs.append(m.downsample[n].register_forward_hook(hook(f"downsample{n}")))
        hs.append(m.lvc_blocks[n].register_forward_hook(hook(f"lvc{n}")))
        hs.append(m.lvc_blocks[n].upsample.register_forward_hook(hook(f"upsample{n}")))
        hs.append(m.lvc_blocks[n].kernel_predictor.register_forward_hook(hook(f"kp{n}")))
    with torch.no_grad():
        eps = m((torch.from_numpy(audio), torch.from_numpy(c), torch.from_numpy(steps))).numpy()
    for h in hs:
        h.remove()
    keep = {k: v for k, v in caps.items() if not k.startswith("kp")}
    keep["kp0_kernels_b0"] = caps["kp0.out0"][0]          # [4,32,64,3,T'] of batch 0
    keep["kp2_bias"] = caps["kp2.out1"]
    keep["kp1_kernels_b1_f3"] = caps["kp1.out0"][1, ..., 3]
    save("fastdiff_fwd", seed=seed, audio=audio, c=c, steps=steps, eps=eps,
         **{"cap_" + k: v for k, v in keep.items()})

    gen_fastdiff_samples({4: (2, 6, 41), 3: (1, 5, 42)})


def gen_fastdiff_samples(cases=None):
    """Sampler goldens.  Default (`gen_golden.py fastdiff_samples`): the 6- and 8-step
    noise-predictor tables (fastdiff.py:64-70) and the 200-step linspace schedule
    and the 1000-step one (fastdiff.py:60-63), which run through fd_sample's 16-step chunk loop."""
    seed = 31
    m, _ = build_fastdiff(seed)
    cases = cases or {6: (2, 3, 43), 8: (1, 4, 44), 200: (1, 2, 45), 1000: (1, 1, 46)}
    for n_iter, (B, Tc, seed_s) in cases.items():
        L = Tc * 256
        c = synth.synth_inputs(seed_s + 2, (B, 80, Tc), loc=-5.0, scale=2.0)
        dh = fd_util.compute_hyperparams_given_schedule(torch.linspace(1e-6, 0.01, 1000))
        sched = (torch.FloatTensor(FASTDIFF_SCHEDULES[n_iter]) if n_iter in FASTDIFF_SCHEDULES
                 else torch.linspace(0.0001, 0.02, 200) if n_iter == 200
                 else torch.linspace(0.000001, 0.01, 1000))
        draws, seen_steps = [], []
        cnt = [0]

        def std_normal(size):
            a = synth.synth_inputs(seed_s * 1000 + cnt[0], tuple(size))
            cnt[0] += 1
            draws.append(a.copy())
            return torch.from_numpy(a)

        class Spy(torch.nn.Module):
            def forward(self, data):
                seen_steps.append(data[2][0, 0].item())
                return m(data)

        orig = fd_util.std_normal
        fd_util.std_normal = std_normal
        try:
            with torch.no_grad():
                wav = fd_util.sampling_given_noise_schedule(
                    Spy(), (B, 1, L), dh, sched, condition=torch.from_numpy(c)).numpy()
        finally:
            fd_util.std_normal = orig
        assert len(draws) == n_iter
        save(f"fastdiff_sample_n{n_iter}", seed=seed, c=c, x_T=draws[0],
             noise=np.stack(draws[1:]), steps_seen=np.array(seen_steps, dtype=np.float32),
             wav=wav)


def gen_fastdiff_variants():
    """sampling_given_noise_schedule with ddim=True (4-step table) and return_sequence=True
    (3-step table), util.py:209-231."""
    seed = 31
    m, _ = build_fastdiff(seed)
    for name, n_iter, (B, Tc, seed_s), kw in (("fastdiff_sample_ddim_n4", 4, (2, 3, 47), dict(ddim=True)),
                                              ("fastdiff_sample_seq_n3", 3, (1, 2, 48), dict(return_sequence=True))):
        L = Tc * 256
        c = synth.synth_inputs(seed_s + 2, (B, 80, Tc), loc=-5.0, scale=2.0)
        dh = fd_util.compute_hyperparams_given_schedule(torch.linspace(1e-6, 0.01, 1000))
        sched = torch.FloatTensor(FASTDIFF_SCHEDULES[n_iter])
        draws = []
        cnt = [0]

        def std_normal(size):
            a = synth.synth_inputs(seed_s * 1000 + cnt[0], tuple(size))
            cnt[0] += 1
            draws.append(a.copy())
            return torch.from_numpy(a)

        orig = fd_util.std_normal
        fd_util.std_normal = std_normal
        try:
            with torch.no_grad():
                out = fd_util.sampling_given_noise_schedule(m, (B, 1, L), dh, sched, condition=torch.from_numpy(c),
                                                            **kw)
        finally:
            fd_util.std_normal = orig
        if kw.get("ddim"):
            assert len(draws) == 1
            save(name, seed=seed, c=c, x_T=draws[0], wav=out.numpy())
        else:
            assert len(draws) == n_iter
            save(name, seed=seed, c=c, x_T=draws[0], noise=np.stack(draws[1:]),
                 seq=np.stack([x.numpy() for x in out]))


# --------------------------------------------------------------------------
# Rectified flow (reflow.py:5-144): the teacher's "reflow" sampler and the pitch
# predictor's PitchRectifiedFlow, every algorithm; x_T = the torch.randn at :88.
# --------------------------------------------------------------------------
REFLOW_CASES = {
    # name: (kind, M, cycle, algorithm, infer_step, B, T, seed)
    "reflow_euler_m80": ("mel", 80, 1, "euler", 4, 2, 24, 51),
    "reflow_rk2_m128": ("mel", 128, 1, "rk2", 3, 1, 19, 52),
    "reflow_rk4_m80": ("mel", 80, 1, "rk4", 2, 2, 17, 53),
    "reflow_rk5_m80": ("mel", 80, 1, "rk5", 2, 1, 21, 54),
    "pitch_reflow_rk2_r64": ("pitch", 64, 5, "rk2", 3, 2, 30, 55),
}


def gen_reflow():
    from modules.diffusion.reflow import PitchRectifiedFlow, RectifiedFlow
    for name, (kind, M, cyc, algo, S, B, T, seed) in REFLOW_CASES.items():
        H, L, C = 256, 20, 256
        net = WaveNet(M, H, L, C, cyc)
        if kind == "mel":
            rf = RectifiedFlow(out_dims=M, denoise_fn=net, time_scale=1000, num_features=1,
                               sampling_algorithm=algo, spec_min=[-12], spec_max=[0]).eval()
        else:
            rf = PitchRectifiedFlow(repeat_bins=M, denoise_fn=net, time_scale=1000, sampling_algorithm=algo,
                                    spec_min=-8.0, spec_max=8.0, clamp_min=-12.0, clamp_max=12.0).eval()
        load_synth(net, synth.wavenet_param_shapes(M, H, L, C), seed)
        cond = synth.synth_inputs(seed + 400, (B, T, H))
        x_T = synth.synth_inputs(seed + 500, (B, 1, M, T))
        seen = []
        orig = torch.randn

        def randn(*size, device=None, **kw):
            seen.append(tuple(size))
            return torch.from_numpy(x_T.copy())

        torch.randn = randn
        try:
            with torch.no_grad():
                out = rf(torch.from_numpy(cond), infer_step=S, infer=True).numpy()
                x = rf.inference(torch.from_numpy(cond).transpose(1, 2), b=B, infer_step=S).numpy()
        finally:
            torch.randn = orig
        assert seen[0] == (B, 1, M, T), seen
        save(name, kind=np.array(kind), dims=np.array([M, H, L, C, cyc]), seed=seed, algo=np.array(algo),
             infer_step=S, cond=cond, x_T=x_T, x=x, out=out)


# --------------------------------------------------------------------------
# Full-size fixtures (SURVEY §8(c) fixture (vi)): C2 (ProDiff 2-iter, B=1, T=1000)
# and a C3 slice (B=2 x 861 frames: ProDiff 2-iter -> FastDiff 4-iter).  Every
# input and draw is regenerated from its seed by prodiff_amd.synth (see
# FULLSIZE_CASES), so only outputs are stored: the full mel, the whole waveform (fp32,
# 2 x 220,416 samples for C3) and per-utterance statistics of it.
# --------------------------------------------------------------------------
FULLSIZE_CASES = {
    # name: (B, T, prodiff weight seed, fastdiff weight seed or None, draw seed for FastDiff)
    "fullsize_c2": (1, 1000, 61, None, None),
    "fullsize_c3_b2": (2, 861, 62, 63, 64),
}


def gen_fullsize():
    for name, (B, T, ps, fs, ds) in FULLSIZE_CASES.items():
        M, H, L, C = 80, 256, 20, 256
        net = WaveNet(M, H, L, C, 1)
        gd = GaussianDiffusion(out_dims=M, denoise_fn=net, timesteps=2, time_scale=1000,
                               schedule_type="vpsde", max_beta=40.0, spec_min=[-12], spec_max=[0]).eval()
        load_synth(net, synth.wavenet_param_shapes(M, H, L, C), ps)
        cond = synth.synth_inputs(ps + 300, (B, T, H))
        with torch.no_grad(), Recorder(ps) as rec:
            mel = gd(torch.from_numpy(cond), infer=True).numpy()
        assert len(rec.rand) == 1 and len(rec.randn) == 2
        out = dict(B=B, T=T, prodiff_seed=ps, mel=mel)
        if fs is not None:
            m, _ = build_fastdiff(fs)
            dh = fd_util.compute_hyperparams_given_schedule(torch.linspace(1e-6, 0.01, 1000))
            cnt = [0]

            def std_normal(size):
                a = synth.synth_inputs(ds * 1000 + cnt[0], tuple(size))
                cnt[0] += 1
                return torch.from_numpy(a)

            orig = fd_util.std_normal
            fd_util.std_normal = std_normal
            try:
                with torch.no_grad():
                    wav = fd_util.sampling_given_noise_schedule(
                        m, (B, 1, T * 256), dh, torch.FloatTensor(FASTDIFF_SCHEDULES[4]),
                        condition=torch.from_numpy(mel).transpose(1, 2).contiguous()).numpy()[:, 0]
            finally:
                fd_util.std_normal = orig
            assert cnt[0] == 4
            w64 = wav.astype(np.float64)
            out.update(fastdiff_seed=fs, draw_seed=ds, wav=wav.astype(np.float32),
                       wav_l2=np.linalg.norm(w64, axis=1), wav_mean=w64.mean(1), wav_absmax=np.abs(w64).max(1))
        save(name, **out)


# --------------------------------------------------------------------------
# SVS teacher condition stage (modules/svs/prodiff_teacher.py:103-146)
# --------------------------------------------------------------------------
COND_CASES = {
    # name: (hparam overrides, vocab, lengths, pad_tokens, param seed, input seed, spk mode)
    "cond_small": (dict(num_spk=3, num_langs=3), 40, [17, 9, 23], 2, 41, 141, "id"),
    # handler/config.yaml flags: single speaker, voicing/breath embeds off
    "cond_handler": (dict(num_spk=1, num_langs=2, use_voicing_embed=False, use_breath_embed=False),
                     64, [120], 0, 42, 142, "id"),
    # 4 heads (head dim 64), 2 layers, time-varying speaker mix, gender ids (looked up in lang_embed)
    "cond_mix_gender": (dict(num_spk=4, num_langs=4, num_heads=4, enc_layers=2, use_gender_id=True),
                        50, [30, 11], 1, 43, 143, "mix_t"),
    # 1 head (head dim 256), long utterances: many query / key blocks, T_mel ~ 2000
    "cond_long": (dict(num_spk=2, num_langs=3, num_heads=1, enc_layers=2, use_breath_embed=False),
                  80, [300, 257], 0, 44, 144, "mix_1"),
    # RelPositionalEncoding (tts_modules.py:299-300,324-325), padded batch
    "cond_relpos": (dict(num_spk=2, num_langs=3, enc_layers=2, rel_pos=True), 40, [21, 13], 1, 45, 145, "id"),
    # the same after the module's table grew to 5,010 rows (extend_pe, espnet_positional_embedding.py:24-45,
    # as a 5,010-token batch leaves it): later batches count reversed positions from 5,010
    "cond_relpos_grown": (dict(num_spk=2, num_langs=3, enc_layers=2, rel_pos=True), 40, [21, 13], 1, 45, 145, "id",
                          5010),
}


def cond_hparams(over):
    hp = dict(synth.COND_DEFAULTS)
    hp.update(over)
    return hp


def gen_cond():
    from modules.svs.prodiff_teacher import ProDiffTeacher
    for name, case in COND_CASES.items():
        (over, V, lengths, padt, ps, xs, spk_mode), grow = case[:7], (case[7] if len(case) > 7 else 0)
        hp = cond_hparams(over)
        rhp = dict(hp, audio_num_mel_bins=128, dropout=0.1, languages=["l%d" % i for i in range(hp["num_langs"] - 1)],
                   residual_layers=1, residual_channels=64, dilation_cycle_length=1, timesteps=4, timescale=1000,
                   schedule_type="vpsde", max_beta=40.0, spec_min=[-12], spec_max=[0])
        m = ProDiffTeacher(V, rhp).eval()
        shapes = synth.cond_param_shapes(V, **hp)
        P = synth.synth_cond_params(shapes, ps)
        sd = m.state_dict()
        assert [k for k in sd if not k.startswith("diffusion") and k in shapes] == list(shapes), "state-dict order"
        for k, v in P.items():
            assert tuple(sd[k].shape) == v.shape, (k, sd[k].shape, v.shape)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()}, strict=False)
        x = synth.synth_cond_inputs(xs, lengths, V, hp["num_spk"], hp["num_langs"], pad_tokens=padt)
        B, Tm = x["mel2ph"].shape
        kw = dict(lang_seq=torch.from_numpy(x["lang_seq"]))
        extra = {}
        if spk_mode == "id":
            kw["spk_embed_id"] = torch.from_numpy(x["spk_embed_id"])
        else:
            frames = Tm if spk_mode == "mix_t" else 1
            mix = synth.synth_inputs(xs + 7, (B, frames, hp["hidden_size"]), scale=0.3)
            kw["spk_mix_embed"] = torch.from_numpy(mix)
            extra["spk_mix_embed"] = mix
        if hp["use_gender_id"]:
            gid = np.arange(B, dtype=np.int64) % 2
            kw["gender_embed_id"] = torch.from_numpy(gid)
            extra["gender_embed_id"] = gid
        if hp["use_voicing_embed"]:
            kw["voicing"] = torch.from_numpy(x["voicing"])
        if hp["use_breath_embed"]:
            kw["breath"] = torch.from_numpy(x["breath"])
        if grow:
            m.encoder.embed_positions.extend_pe(torch.zeros(1, grow))
            assert m.encoder.embed_positions.pe.shape[1] == grow
        enc_out = {}
        hook = m.encoder.register_forward_hook(lambda mod, inp, out: enc_out.setdefault("enc", out.detach().clone()))
        with torch.no_grad():
            cond = m.forward_condition(torch.from_numpy(x["txt_tokens"]), torch.from_numpy(x["mel2ph"]),
                                       torch.from_numpy(x["f0"]), **kw).numpy()
        hook.remove()
        save(name, vocab=V, lengths=np.array(lengths), pad_tokens=padt, param_seed=ps, input_seed=xs,
             spk_mode=spk_mode, hp_keys=np.array(list(over)), hp_vals=np.array([int(v) for v in over.values()]),
             cond=cond, enc=enc_out["enc"].numpy(), grow=grow, **{k: v for k, v in x.items()}, **extra)


# --------------------------------------------------------------------------
# Full-size SVS chain (C5's shapes at real segment lengths): the reference teacher's
# forward_condition (prodiff_teacher.py:103-146) -> GaussianDiffusion 4-iter at M=128
# (prodiff.py:136-153) -> NSF-HiFiGAN spec2wav_torch (component/vocoder/nsf_hifigan.py:29-58,
# models.py:21-297), each segment alone (B=1: the reference SineGen is batch-1 only,
# models.py:162-163, and the handler runs one segment at a time, handler/infer/handler.py:373-388).
# Lengths and phoneme counts are two real segments of the reference's sample song
# (tests/golden/ds_lengths.json: segment 21, 286 frames / 6 phonemes; segment 0, 504 / 24).
# Weights are SvsSynthesizer.synthetic(seed)'s (cond seed, WaveNet seed + 1, NSF seed + 2);
# inputs come from synth.synth_svs_utterance; every draw from synth.synth_inputs keyed by
# (draw seed * 1000 + draw index) -- torch.rand (x_T) and 4 x torch.randn for the sampler,
# torch.rand(1, 9) and torch.randn_like for the SineGen -- so only outputs are stored.
# --------------------------------------------------------------------------
FULLSIZE_C5 = {
    # name: (ds segment, frames, phonemes, utterance seed, prodiff draw seed, nsf draw seed)
    "fullsize_c5_s21": (21, 286, 6, 171, 173, 175),
    "fullsize_c5_s0": (0, 504, 24, 172, 174, 176),
}
C5_WEIGHT_SEED = 71


def gen_fullsize_c5():
    import json
    from modules.nsf_hifigan.env import AttrDict
    from modules.nsf_hifigan.models import Generator
    from modules.svs.prodiff_teacher import ProDiffTeacher
    from prodiff_amd.pipeline import SVS_TEACHER, SVS_VOCAB
    ds = json.load(open(os.path.join(HERE, "ds_lengths.json")))
    hp = dict(SVS_TEACHER)
    t = ProDiffTeacher(SVS_VOCAB, hp).eval()
    cp = synth.synth_cond_params(synth.cond_param_shapes(SVS_VOCAB, num_langs=len(hp["languages"]) + 1,
                                                         **{k: v for k, v in hp.items() if k != "num_langs"}),
                                 C5_WEIGHT_SEED)
    wn = synth.synth_params(synth.wavenet_param_shapes(hp["audio_num_mel_bins"], hp["hidden_size"],
                                                       hp["residual_layers"], hp["residual_channels"]),
                            C5_WEIGHT_SEED + 1)
    sd = t.state_dict()
    full = {k: torch.from_numpy(v) for k, v in cp.items()}
    full.update({"diffusion.denoise_fn." + k: torch.from_numpy(v) for k, v in wn.items()})
    for k, v in full.items():
        assert tuple(sd[k].shape) == tuple(v.shape), (k, sd[k].shape, v.shape)
    t.load_state_dict(full, strict=False)
    h = dict(synth.NSF_DEFAULTS)
    g = Generator(AttrDict(num_mels=h["num_mels"], upsample_initial_channel=h["upsample_initial_channel"],
                           upsample_rates=list(h["upsample_rates"]),
                           upsample_kernel_sizes=list(h["upsample_kernel_sizes"]), resblock=h["resblock"],
                           resblock_kernel_sizes=list(h["resblock_kernel_sizes"]),
                           resblock_dilation_sizes=[list(d) for d in h["resblock_dilation_sizes"]],
                           sampling_rate=h["sampling_rate"]))
    g.remove_weight_norm()
    g.load_state_dict({k: torch.from_numpy(v)
                       for k, v in synth.synth_params(synth.nsf_param_shapes(**h), C5_WEIGHT_SEED + 2).items()},
                      strict=True)
    g.eval()
    for name, (seg, T, ntok, us, ps, ns) in FULLSIZE_C5.items():
        assert ds["frames"][seg] == T and ds["phonemes"][seg] == ntok, (seg, T, ntok)
        u = synth.synth_svs_utterance(us, T, ntok, SVS_VOCAB)
        ins = {k: torch.from_numpy(v)[None] for k, v in u.items()}
        conds = {}
        hk = t.diffusion.register_forward_pre_hook(lambda mod, a: conds.setdefault("cond", a[0].detach().clone()))
        with torch.no_grad(), Recorder(ps) as rec:
            mel = t(ins["txt_tokens"], ins["mel2ph"], ins["f0"], lang_seq=ins["lang_seq"],
                    spk_mix_embed=ins["spk_mix_embed"], voicing=ins["voicing"], breath=ins["breath"],
                    infer=True)
        hk.remove()
        assert len(rec.rand) == 1 and len(rec.randn) == 4
        # spec2wav_torch (nsf_hifigan.py:50-56) with the SineGen draws replayed from synth
        cnt = [0]
        r0, rl = torch.rand, torch.randn_like

        def rand(*size, device=None, **kw):
            assert cnt[0] == 0 and tuple(size) == (1, 9), size
            cnt[0] += 1
            return torch.from_numpy(synth.synth_inputs(ns * 1000, (1, 9), kind="uniform"))

        def randn_like(x, **kw):
            assert cnt[0] == 1
            cnt[0] += 1
            return torch.from_numpy(synth.synth_inputs(ns * 1000 + 1, tuple(x.shape)))

        torch.rand, torch.randn_like = rand, randn_like
        try:
            with torch.no_grad():
                c = 2.30259 * mel.transpose(2, 1)
                wav = g(c, ins["f0"]).view(-1).numpy()
        finally:
            torch.rand, torch.randn_like = r0, rl
        assert cnt[0] == 2 and wav.shape == (T * 512,)
        w64 = wav.astype(np.float64)
        save(name, segment=seg, T=T, ntok=ntok, weight_seed=C5_WEIGHT_SEED, utt_seed=us, prodiff_seed=ps,
             nsf_seed=ns, cond=conds["cond"].numpy()[0], mel=mel.numpy()[0], wav=wav.astype(np.float32),
             wav_l2=np.linalg.norm(w64), wav_mean=w64.mean(), wav_absmax=np.abs(w64).max())


if __name__ == "__main__":
    if len(sys.argv) > 1:          # e.g. `gen_golden.py reflow` regenerates one family
        globals()["gen_" + sys.argv[1]]()
        sys.exit(0)
    gen_schedules()
    gen_wavenet()
    gen_prodiff()
    gen_fastdiff()
    gen_reflow()
    gen_fullsize()
