"""HIP path vs the reference's golden vectors and the (pinned) oracle.

Tolerance (north star, BASELINE.json): max |delta| <= 1e-4 in fp32 on identical
inputs and identical random draws.  Quantities whose magnitude exceeds ~10
(FastDiff LVC-block outputs, sampler waveforms) are compared at 1e-5 x max|ref|,
which is at the reference's own fp32 drift (tests/test_oracle.py).
"""
import numpy as np
import pytest
import torch

from oracle import oracle_fastdiff as OF
from oracle import oracle_prodiff as OP
from prodiff_amd import FastDiff, GaussianDiffusion, WaveNet, synth
from prodiff_amd.fastdiff import sampling_given_noise_schedule
from tests import golden_io as G

pytestmark = pytest.mark.gpu
TOL = 1e-4
DEV = torch.device("cuda:0")


def tt(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def wavenet_from(dims, params):
    M, H, L, C, cyc = [int(v) for v in dims]
    net = WaveNet(M, H, L, C, cyc)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    return net.to(DEV)


def assert_close(got, ref, tol=TOL, rel=None):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.isfinite(got).all()
    lim = tol if rel is None else max(tol, rel * np.abs(ref).max())
    err = np.abs(got - ref).max()
    assert err <= lim, f"max|d|={err:.3e} > {lim:.3e}"


# ------------------------------------------------------------------ WaveNet
@pytest.mark.parametrize("name", ["wavenet_m80_c256_l20_cyc1", "wavenet_m80_c256_l20_float",
                                  "wavenet_m64_c256_l20_cyc5", "wavenet_m128_c256_l20_cyc1",
                                  "wavenet_m80_c64_l4_cyc2"])
def test_wavenet_golden(name):
    d = G.load(name)
    net = wavenet_from(d["dims"], G.wavenet_params(d["dims"], d["seed"]))
    out = net(tt(d["spec"]), tt(d["steps"]), tt(d["cond"])).cpu().numpy()
    assert_close(out, d["out"])


@pytest.mark.parametrize("B,T,seed", [(1, 1, 1), (3, 67, 2), (2, 130, 3)])
def test_wavenet_oracle_shapes(B, T, seed):
    """Ragged/edge lengths (T=1: every tap is padding) against the oracle."""
    dims = (80, 256, 20, 256, 1)
    p = synth.synth_params(synth.wavenet_param_shapes(80, 256, 20, 256), seed)
    net = wavenet_from(dims, p)
    spec = synth.synth_inputs(seed + 1, (B, 1, 80, T))
    cond = synth.synth_inputs(seed + 2, (B, 256, T))
    steps = np.arange(B, dtype=np.float32)
    out = net(tt(spec), tt(steps), tt(cond)).cpu().numpy()
    assert_close(out, OP.wavenet_forward(p, spec, steps, cond, 20, 1))


# ------------------------------------------------------------------ ProDiff sampler
@pytest.mark.parametrize("name", ["prodiff_t2_m80", "prodiff_t4_m80", "prodiff_t4_m128"])
def test_prodiff_sample_golden(name):
    d = G.load(name)
    M = int(d["mel"].shape[-1])
    net = WaveNet(M, 256, 20, 256, 1)
    gd = GaussianDiffusion(M, net, timesteps=int(d["timesteps"]), time_scale=1000, max_beta=float(d["max_beta"]))
    sd = {"denoise_fn." + k: torch.from_numpy(v) for k, v in G.prodiff_params(name).items()}
    sd.update({k: torch.from_numpy(v) for k, v in G.prodiff_buffers(d).items()})
    gd.load_state_dict(sd, strict=True)
    gd = gd.to(DEV)
    mel = gd.sample(tt(d["cond"]), x_T=tt(d["x_T"]), noise=tt(d["noise"])).cpu().numpy()
    assert_close(mel, d["mel"])


def test_prodiff_forward_infer_api():
    """forward(cond, infer=True) -- the teacher's call (prodiff_teacher.py:167) -- on-device draws."""
    net = WaveNet(80, 256, 20, 256, 1)
    p = synth.synth_params(synth.wavenet_param_shapes(80, 256, 20, 256), 4)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})   # (reference zero-inits output_projection)
    gd = GaussianDiffusion(80, net, timesteps=2, max_beta=40.0).to(DEV)
    cond = tt(synth.synth_inputs(7, (2, 50, 256)))
    torch.manual_seed(0)
    a = gd(cond, infer=True)
    torch.manual_seed(0)
    b = gd(cond, infer=True)
    c = gd(cond, infer=True)
    assert a.shape == (2, 50, 80) and torch.isfinite(a).all()
    assert torch.equal(a, b) and not torch.equal(a, c)


def test_prodiff_batch_independence():
    """Utterances never mix: sampling a batch == sampling each utterance alone."""
    net = WaveNet(80, 256, 20, 256, 1)
    gd = GaussianDiffusion(80, net, timesteps=2, max_beta=40.0)
    p = synth.synth_params(synth.wavenet_param_shapes(80, 256, 20, 256), 3)
    gd.denoise_fn.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    gd = gd.to(DEV)
    B, T = 3, 41
    cond = tt(synth.synth_inputs(1, (B, T, 256)))
    xT = tt(synth.synth_inputs(2, (B, 1, 80, T), kind="uniform"))
    nz = tt(synth.synth_inputs(3, (2, B, 1, 80, T)))
    full = gd.sample(cond, x_T=xT, noise=nz)
    for b in range(B):
        one = gd.sample(cond[b:b + 1].contiguous(), x_T=xT[b:b + 1].contiguous(),
                        noise=nz[:, b:b + 1].contiguous())
        assert torch.allclose(one, full[b:b + 1], atol=1e-6, rtol=0)


# ------------------------------------------------------------------ FastDiff
@pytest.fixture(scope="module")
def fdnet():
    p = G.fastdiff_params(31)
    m = FastDiff()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    return m.to(DEV), OF.fold_weight_norm(p)


def test_fastdiff_forward_golden(fdnet):
    m, _ = fdnet
    d = G.load("fastdiff_fwd")
    eps = m((tt(d["audio"]), tt(d["c"]), tt(d["steps"]))).cpu().numpy()
    assert_close(eps, d["eps"])


def test_fastdiff_forward_after_remove_weight_norm(fdnet):
    """Folding in torch (reference remove_weight_norm) or on device gives the same eps."""
    m, _ = fdnet
    d = G.load("fastdiff_fwd")
    m2 = FastDiff()
    m2.load_state_dict({k: torch.from_numpy(v) for k, v in G.fastdiff_params(31).items()})
    m2.remove_weight_norm()
    m2 = m2.to(DEV)
    eps = m2((tt(d["audio"]), tt(d["c"]), tt(d["steps"]))).cpu().numpy()
    assert_close(eps, d["eps"])


@pytest.mark.parametrize("B,Tc,step", [(1, 1, 0.0), (3, 5, 74.9923), (2, 9, 999.0)])
def test_fastdiff_forward_oracle_shapes(fdnet, B, Tc, step):
    m, pf = fdnet
    audio = synth.synth_inputs(B * 10 + Tc, (B, 1, Tc * 256))
    c = synth.synth_inputs(B * 10 + Tc + 1, (B, 80, Tc), loc=-5.0, scale=2.0)
    st = np.full((B, 1), step, np.float32)
    eps = m((tt(audio), tt(c), tt(st))).cpu().numpy()
    assert_close(eps, OF.fastdiff_forward(pf, audio, c, st))


@pytest.mark.parametrize("n_iter", [4, 3, 6, 8, 200, 1000])
def test_fastdiff_sample_golden(fdnet, n_iter):
    """Every reverse schedule of component/vocoder/fastdiff.py:58-73 against the reference
    sampler (util.py:158-232) with its recorded draws.  200 and 1000 steps run through
    fd_sample's 16-step chunk loop (13 and 63 chunks: step-embedding / kernel-predictor
    batching per chunk, workspace reuse)."""
    m, _ = fdnet
    d = G.load(f"fastdiff_sample_n{n_iter}")
    s = G.load("schedules")
    dh = {"alpha": torch.from_numpy(s["fd_train_alpha"])}
    sched = torch.from_numpy(s[f"fd_n{n_iter}_beta"])
    B, _, Tc = d["c"].shape
    wav = sampling_given_noise_schedule(m, (B, 1, Tc * 256), dh, sched, condition=tt(d["c"]),
                                        x_T=tt(d["x_T"]), noise=tt(d["noise"])).cpu().numpy()
    assert_close(wav, d["wav"], rel=1e-5)


def _fd_golden_args(d, n_iter):
    s = G.load("schedules")
    dh = {"alpha": torch.from_numpy(s["fd_train_alpha"])}
    sched = torch.from_numpy(s[f"fd_n{n_iter}_beta"])
    B, _, Tc = d["c"].shape
    return (B, 1, Tc * 256), dh, sched


def test_fastdiff_sample_ddim_golden(fdnet):
    """ddim=True (util.py:215-220): deterministic update, only x_T is drawn."""
    m, _ = fdnet
    d = G.load("fastdiff_sample_ddim_n4")
    size, dh, sched = _fd_golden_args(d, 4)
    wav = sampling_given_noise_schedule(m, size, dh, sched, condition=tt(d["c"]), ddim=True,
                                        x_T=tt(d["x_T"])).cpu().numpy()
    assert_close(wav, d["wav"], rel=1e-5)


def test_fastdiff_sample_return_sequence_golden(fdnet):
    """return_sequence=True (util.py:209-210,228-231): [x_T, x after each pass]."""
    m, _ = fdnet
    d = G.load("fastdiff_sample_seq_n3")
    size, dh, sched = _fd_golden_args(d, 3)
    xs = sampling_given_noise_schedule(m, size, dh, sched, condition=tt(d["c"]), return_sequence=True,
                                       x_T=tt(d["x_T"]), noise=tt(d["noise"]))
    assert len(xs) == d["seq"].shape[0] == 4
    for x, ref in zip(xs, d["seq"]):
        assert_close(x.cpu().numpy(), ref, rel=1e-5)


def test_fastdiff_return_sequence_keeps_fused_draws(fdnet):
    """Pass-by-pass (return_sequence) with on-device draws ends where the fused sampler does."""
    m, _ = fdnet
    from prodiff_amd.schedules import fastdiff_reverse_schedule, fastdiff_train_alpha
    B, Tc = 2, 3
    c = tt(synth.synth_inputs(12, (B, 80, Tc), loc=-5.0, scale=2.0))
    dh = {"alpha": torch.from_numpy(fastdiff_train_alpha())}
    sched = torch.from_numpy(fastdiff_reverse_schedule(4))
    fused = sampling_given_noise_schedule(m, (B, 1, Tc * 256), dh, sched, condition=c, seed=77)
    xs = sampling_given_noise_schedule(m, (B, 1, Tc * 256), dh, sched, condition=c, seed=77, return_sequence=True)
    assert len(xs) == 5
    assert_close(xs[-1].cpu().numpy(), fused.cpu().numpy(), rel=1e-5)


def test_fastdiff_sample_batch_independence(fdnet):
    m, _ = fdnet
    from prodiff_amd.schedules import fastdiff_infer_params, fastdiff_reverse_schedule, fastdiff_train_alpha
    b, a, s, st = fastdiff_infer_params(fastdiff_reverse_schedule(4), fastdiff_train_alpha())
    B, Tc = 3, 7
    mel = tt(synth.synth_inputs(9, (B, Tc, 80), loc=-5.0, scale=2.0))
    xT = tt(synth.synth_inputs(10, (B, 1, Tc * 256)))
    nz = tt(synth.synth_inputs(11, (3, B, 1, Tc * 256)))
    full = m.sample(mel, b, a, s, st, x_T=xT, noise=nz)
    for i in range(B):
        one = m.sample(mel[i:i + 1].contiguous(), b, a, s, st, x_T=xT[i:i + 1].contiguous(),
                       noise=nz[:, i:i + 1].contiguous())
        assert torch.allclose(one, full[i:i + 1], atol=1e-5, rtol=0)


def test_onchip_rng_moments(fdnet):
    """Philox draws used when no explicit noise is given: U[0,1) x_T and N(0,1) steps."""
    net = WaveNet(80, 32, 2, 64, 1)
    gd = GaussianDiffusion(80, net, timesteps=1, max_beta=40.0).to(DEV)
    with torch.no_grad():
        for p in gd.denoise_fn.parameters():
            p.zero_()
    # with zero weights x0 == 0, so mel = c2[0] * x_T  (c2[0] = 0 at t=0 would hide it -> check c1/c2)
    gd.posterior_mean_coef2.fill_(1.0)
    mel = gd.sample(tt(np.zeros((4, 4096, 32), np.float32)), seed=1234)
    x = mel.cpu().numpy()
    assert abs(x.mean() - 0.5) < 0.01 and abs(x.var() - 1 / 12) < 0.01 and x.min() >= 0 and x.max() < 1


# ------------------------------------------------------------------ rectified flow
REFLOW = ["reflow_euler_m80", "reflow_rk2_m128", "reflow_rk4_m80", "reflow_rk5_m80", "pitch_reflow_rk2_r64"]


def reflow_from(d):
    from prodiff_amd import PitchRectifiedFlow, RectifiedFlow
    M, H, L, C, cyc = [int(v) for v in d["dims"]]
    net = wavenet_from(d["dims"], G.wavenet_params(d["dims"], d["seed"]))
    if str(d["kind"]) == "pitch":
        return PitchRectifiedFlow(M, net, time_scale=1000, sampling_algorithm=str(d["algo"])).to(DEV)
    return RectifiedFlow(M, net, time_scale=1000, sampling_algorithm=str(d["algo"]), spec_min=[-12],
                         spec_max=[0]).to(DEV)


@pytest.mark.parametrize("name", REFLOW)
def test_reflow_golden(name):
    """Euler / RK2 / RK4 / RK5 integration and denorm_spec against the reference's outputs."""
    d = G.load(name)
    rf = reflow_from(d)
    x = rf.sample(tt(d["cond"]), infer_step=int(d["infer_step"]), x_T=tt(d["x_T"]))
    assert_close(x.cpu().numpy(), d["x"])
    assert_close(rf.denorm_spec(x).cpu().numpy(), d["out"])


@pytest.mark.parametrize("B,T,S", [(3, 33, 20), (1, 1, 5)])
def test_reflow_euler_oracle_shapes(B, T, S):
    """The teacher's default (20 Euler steps) on ragged shapes against the oracle."""
    from oracle import oracle_reflow as OR
    from prodiff_amd import RectifiedFlow
    p = synth.synth_params(synth.wavenet_param_shapes(80, 256, 20, 256), 61)
    rf = RectifiedFlow(80, wavenet_from((80, 256, 20, 256, 1), p), spec_min=[-12], spec_max=[0]).to(DEV)
    cond = synth.synth_inputs(62, (B, T, 256))
    xT = synth.synth_inputs(63, (B, 1, 80, T))
    x = rf.sample(tt(cond), infer_step=S, x_T=tt(xT)).cpu().numpy()
    assert_close(x, OR.reflow_sample(p, cond, xT, S, "euler", 1000, 20, 1))


def test_reflow_forward_api():
    """forward(cond, infer=True) -- the teacher's call (prodiff_teacher.py:167) -- Philox draws."""
    from prodiff_amd import RectifiedFlow
    p = synth.synth_params(synth.wavenet_param_shapes(80, 256, 20, 256), 64)
    rf = RectifiedFlow(80, wavenet_from((80, 256, 20, 256, 1), p), spec_min=[-12], spec_max=[0]).to(DEV)
    cond = tt(synth.synth_inputs(65, (2, 40, 256)))
    torch.manual_seed(0)
    a = rf(cond, infer=True)
    torch.manual_seed(0)
    b = rf(cond, infer=True)
    assert a.shape == (2, 40, 80) and torch.isfinite(a).all() and torch.equal(a, b)


@pytest.mark.parametrize("cyc,B,T", [(1, 1, 1000), (5, 3, 101), (1, 2, 37), (2, 2, 1)])
def test_wavenet_fp32_layer_kernel(cyc, B, T):
    """PD_WN_OPT_F32_LAYER: the fp32 residual layers as wn_f32_layer_kernel launches (GATE: four
    K segments -- the three dilated taps of x + dp and cond -- summed per wave, then in segment
    order; RESSKIP) against the split-K GEMM engine, at C2's shape (B=1 x 1000), a dilation cycle
    of 5 (taps crossing utterance edges at d = 1..16), ragged lengths and T = 1.  Different fp32
    summation order, so the bar is the north-star 1e-4."""
    torch.manual_seed(22)
    net = WaveNet(80, 256, 20, 256, cyc)
    spec = torch.randn(B, 1, 80, T, device=DEV)
    cond = torch.randn(B, 256, T, device=DEV)
    steps = torch.tensor([7.0, 250.0, 99.0][:B], device=DEV)
    outs = []
    for mode in (0, 2):
        m = WaveNet(80, 256, 20, 256, cyc)
        m.load_state_dict(net.state_dict())
        m = m.to(DEV).set_options(f32_layer=mode)
        outs.append(m(spec, steps, cond).float().cpu().numpy())
    assert_close(outs[1], outs[0])


@pytest.mark.parametrize("B,T,S", [(1, 1000, 4), (3, 101, 2)])
def test_prodiff_fp32_small_batch_kernels(B, T, S):
    """The fp32 sampler at small batches on wn_f32_layer_kernel + wn_f32_tail_kernel (skip head,
    output projection and posterior in one launch; PD_WN_OPT_F32_LAYER=2 forces them) against
    the split-K GEMM engine path (=0), Philox draws: within the north-star 1e-4."""
    torch.manual_seed(23)
    gd = GaussianDiffusion(80, WaveNet(80, 256, 20, 256, 1), timesteps=4, time_scale=1000, max_beta=0.7)
    sd = gd.state_dict()
    cond = torch.randn(B, T, 256, device=DEV)
    outs = []
    for mode in (0, 2):
        g = GaussianDiffusion(80, WaveNet(80, 256, 20, 256, 1), timesteps=4, time_scale=1000, max_beta=0.7)
        g.load_state_dict(sd)
        g = g.to(DEV)
        g.denoise_fn.set_options(f32_layer=mode)
        outs.append(g.sample(cond, infer_step=S, seed=99).cpu().numpy())
    assert_close(outs[1], outs[0])
