"""bf16 throughput path (C3) against the fp32 golden vectors / oracle.

The stated tolerance lives in tests/bf16_bar.py (rel-L2 and max-relative bars set
just above the measured errors; every test prints its "BF16ERR" line).
"""
import numpy as np
import pytest
import torch

from oracle import oracle_fastdiff as OF
from prodiff_amd import FastDiff, GaussianDiffusion, WaveNet, synth
from prodiff_amd.fastdiff import sampling_given_noise_schedule
from tests import golden_io as G

from tests.bf16_bar import EPS_REL_L2, EPS_REL_MAX, assert_bf16_close

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def tt(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("layer", [3, 0, 1])
@pytest.mark.parametrize("name", ["wavenet_m80_c256_l20_cyc1", "wavenet_m64_c256_l20_cyc5",
                                  "wavenet_m80_c64_l4_cyc2"])
def test_wavenet_bf16(name, layer):
    """Every bf16 residual-layer kernel (PD_WN_OPT_LAYER: 3 = fused, 64 frames per block; 0 =
    fused, 32 frames; 1 = GATE + RESSKIP kernels, 128-frame GATE tiles; the default 2 picks 3 or 0
    by grid size) against the reference goldens.  cyc5 runs the 16-row-halo
    GATE variant (dilations 1..16); the C=64 net has no fused kernel (engine path)."""
    d = G.load(name)
    M, H, L, C, cyc = [int(v) for v in d["dims"]]
    net = WaveNet(M, H, L, C, cyc)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in G.wavenet_params(d["dims"], d["seed"]).items()})
    net = net.to(DEV).set_compute_dtype("bf16").set_options(layer=layer)
    out = net(tt(d["spec"]), tt(d["steps"]), tt(d["cond"])).cpu().numpy()
    assert_bf16_close(out, d["out"], f"{name} layer={layer}")


@pytest.mark.parametrize("name", ["prodiff_t2_m80", "prodiff_t4_m128"])
def test_prodiff_sample_bf16(name):
    d = G.load(name)
    M = int(d["mel"].shape[-1])
    gd = GaussianDiffusion(M, WaveNet(M, 256, 20, 256, 1), timesteps=int(d["timesteps"]), time_scale=1000,
                           max_beta=float(d["max_beta"]))
    sd = {"denoise_fn." + k: torch.from_numpy(v) for k, v in G.prodiff_params(name).items()}
    sd.update({k: torch.from_numpy(v) for k, v in G.prodiff_buffers(d).items()})
    gd.load_state_dict(sd)
    gd = gd.to(DEV).set_compute_dtype("bf16")
    mel = gd.sample(tt(d["cond"]), x_T=tt(d["x_T"]), noise=tt(d["noise"])).cpu().numpy()
    assert_bf16_close(mel, d["mel"], name)


@pytest.fixture(scope="module")
def fd16():
    p = G.fastdiff_params(31)
    m = FastDiff()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    return m.to(DEV).set_compute_dtype("bf16"), OF.fold_weight_norm(p)


def test_fastdiff_forward_bf16(fd16):
    m, _ = fd16
    d = G.load("fastdiff_fwd")
    eps = m((tt(d["audio"]), tt(d["c"]), tt(d["steps"]))).cpu().numpy()
    assert_bf16_close(eps, d["eps"], "fastdiff_fwd", EPS_REL_L2, EPS_REL_MAX)


@pytest.mark.parametrize("B,Tc", [(1, 1), (3, 5)])
def test_fastdiff_forward_bf16_oracle(fd16, B, Tc):
    """Utterance edges inside fused-LVC blocks (1 frame = 2 blocks at hop 256)."""
    m, pf = fd16
    audio = synth.synth_inputs(B + 50 * Tc, (B, 1, Tc * 256))
    c = synth.synth_inputs(B + 50 * Tc + 1, (B, 80, Tc), loc=-5.0, scale=2.0)
    st = np.full((B, 1), 23.4676, np.float32)
    eps = m((tt(audio), tt(c), tt(st))).cpu().numpy()
    assert_bf16_close(eps, OF.fastdiff_forward(pf, audio, c, st), f"fastdiff_fwd B={B} Tc={Tc}", EPS_REL_L2,
                      EPS_REL_MAX)


def test_fastdiff_sample_bf16(fd16):
    m, _ = fd16
    d = G.load("fastdiff_sample_n4")
    s = G.load("schedules")
    B, _, Tc = d["c"].shape
    wav = sampling_given_noise_schedule(m, (B, 1, Tc * 256), {"alpha": torch.from_numpy(s["fd_train_alpha"])},
                                        torch.from_numpy(s["fd_n4_beta"]), condition=tt(d["c"]),
                                        x_T=tt(d["x_T"]), noise=tt(d["noise"])).cpu().numpy()
    assert_bf16_close(wav, d["wav"], "fastdiff_sample_n4")


def _lvc_opts(ts):
    """FD options selecting one LVC-block implementation: the whole-block kernel with tile
    `ts` (0 = one fused launch per layer)."""
    return dict(lvc_ts=ts)


@pytest.mark.parametrize("ts_sub", [128, 384])
@pytest.mark.parametrize("B,Tc", [(1, 1), (3, 5), (2, 9)])
def test_fastdiff_lvc_sub_tiles_bf16(ts_sub, B, Tc):
    """The hop-8 block's non-default tiles (FD_OPT_LVC_TS_SUB; 256 is the default, covered by
    every other FastDiff test) against the oracle."""
    p = G.fastdiff_params(31)
    m = FastDiff()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    m = m.to(DEV).set_compute_dtype("bf16").set_options(lvc_ts_sub=ts_sub)
    audio = synth.synth_inputs(5 * B + Tc, (B, 1, Tc * 256))
    c = synth.synth_inputs(5 * B + Tc + 1, (B, 80, Tc), loc=-5.0, scale=2.0)
    st = np.full((B, 1), 23.47, np.float32)
    eps = m((tt(audio), tt(c), tt(st))).cpu().numpy()
    assert_bf16_close(eps, OF.fastdiff_forward(OF.fold_weight_norm(p), audio, c, st),
                      f"lvc_sub ts={ts_sub} B={B} Tc={Tc}", EPS_REL_L2, EPS_REL_MAX)


@pytest.mark.parametrize("ts", [0, 128, 256, 384])
@pytest.mark.parametrize("B,Tc", [(1, 1), (3, 5), (2, 9), (1, 40)])
def test_fastdiff_lvc_block_bf16(ts, B, Tc):
    """LVC modes against the oracle, including utterances shorter than one block and the
    grid/halo edges: the whole-block kernel (FD_OPT_LVC_TS: 0 = one fused launch per layer,
    128/256/384 = whole block)."""
    p = G.fastdiff_params(31)
    m = FastDiff()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    opts = _lvc_opts(ts)
    m = m.to(DEV).set_compute_dtype("bf16").set_options(**opts)
    audio = synth.synth_inputs(7 * B + Tc, (B, 1, Tc * 256))
    c = synth.synth_inputs(7 * B + Tc + 1, (B, 80, Tc), loc=-5.0, scale=2.0)
    st = np.full((B, 1), 41.5, np.float32)
    eps = m((tt(audio), tt(c), tt(st))).cpu().numpy()
    assert_bf16_close(eps, OF.fastdiff_forward(OF.fold_weight_norm(p), audio, c, st),
                      f"lvc_block ts={ts} B={B} Tc={Tc}", EPS_REL_L2, EPS_REL_MAX)


@pytest.mark.parametrize("fuse,ts", [(0, 128), (0, 256), (0, 384), (1, 128), (1, 256), (1, 384)])
@pytest.mark.parametrize("B,Tc", [(1, 1), (3, 5), (2, 9)])
def test_fastdiff_sample_bf16_oracle(fuse, ts, B, Tc):
    """The 4-step sampler with the upsample / first conv / final update fused into the LVC
    block kernel (FD_OPT_LVC_FUSE=1: audio ping-pong between steps; FD_OPT_LVC_SUB=1: the hop-8
    block on the masked multi-frame whole-block kernel) and unfused, against
    the oracle sampler with the same explicit draws; ragged lengths put utterance edges
    inside blocks and halos."""
    from prodiff_amd.schedules import fastdiff_infer_params, fastdiff_reverse_schedule, fastdiff_train_alpha
    p = G.fastdiff_params(31)
    m = FastDiff()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    opts = _lvc_opts(ts)
    m = m.to(DEV).set_compute_dtype("bf16").set_options(lvc_fuse=fuse, lvc_sub=fuse, **opts)
    b, a, s, st = fastdiff_infer_params(fastdiff_reverse_schedule(4), fastdiff_train_alpha())
    mel = synth.synth_inputs(40 + B, (B, Tc, 80), loc=-5.0, scale=2.0)
    xT = synth.synth_inputs(41 + B, (B, 1, Tc * 256))
    nz = synth.synth_inputs(42 + B, (3, B, 1, Tc * 256))
    wav = m.sample(tt(mel), b, a, s, st, x_T=tt(xT), noise=tt(nz)).cpu().numpy()
    ref = OF.fastdiff_sample(OF.fold_weight_norm(p), np.transpose(mel, (0, 2, 1)), xT, nz, b, a, s, st)
    assert_bf16_close(wav.reshape(ref.shape), ref, f"sampler fuse={fuse} ts={ts} B={B} Tc={Tc}")


def test_reflow_euler_bf16():
    """bf16 velocity field over the teacher's 20 Euler steps, against the fp64 oracle."""
    from oracle import oracle_reflow as OR
    from prodiff_amd import RectifiedFlow
    p = synth.synth_params(synth.wavenet_param_shapes(80, 256, 20, 256), 71)
    net = WaveNet(80, 256, 20, 256, 1)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    rf = RectifiedFlow(80, net.to(DEV).set_compute_dtype("bf16"), spec_min=[-12], spec_max=[0]).to(DEV)
    cond = synth.synth_inputs(72, (2, 37, 256))
    xT = synth.synth_inputs(73, (2, 1, 80, 37))
    x = rf.sample(tt(cond), infer_step=20, x_T=tt(xT)).cpu().numpy()
    assert_bf16_close(x, OR.reflow_sample(p, cond, xT, 20, "euler", 1000, 20, 1), "reflow_euler_20")


@pytest.mark.parametrize("chunk", [1, 2])
def test_fastdiff_kp_chunk_bitexact(chunk):
    """FD_OPT_KP_CHUNK (kernel predictor + LVC block per chunk of utterances) changes only the
    launch order: the sample -- on-device Philox draws included -- is bit-identical."""
    p = G.fastdiff_params(31)
    s = G.load("schedules")
    B, Tc = 3, 7
    c = synth.synth_inputs(77, (B, 80, Tc), loc=-5.0, scale=2.0)
    outs = []
    for ch in (0, chunk):
        m = FastDiff()
        m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
        m = m.to(DEV).set_compute_dtype("bf16").set_options(kp_chunk=ch)
        wav = sampling_given_noise_schedule(m, (B, 1, Tc * 256), {"alpha": torch.from_numpy(s["fd_train_alpha"])},
                                            torch.from_numpy(s["fd_n4_beta"]), condition=tt(c), seed=1234)
        outs.append(wav.cpu().numpy())
    assert np.isfinite(outs[0]).all()
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("cyc", [1, 5])
def test_wavenet_two_kernel_vs_fused(cyc):
    """PD_WN_OPT_LAYER=1 (GATE + RESSKIP) against the fused layer at a ragged size: B=5 x 203
    frames puts utterance boundaries inside 128-frame GATE blocks (tap masks) and, with cyc=5,
    dilations up to 16 (the 16-row-halo GATE variant).  Same bf16 roundings, only the fp32
    summation order differs (measured: bit-identical outputs; the bf16 rounding of every layer's
    inputs absorbs the reordering).  The launch tags prove which path ran."""
    torch.manual_seed(3)
    net = WaveNet(80, 256, 20, 256, cyc)
    B, T = 5, 203
    spec = torch.randn(B, 1, 80, T, device=DEV)
    cond = torch.randn(B, 256, T, device=DEV)
    steps = torch.full((B,), 7.0, device=DEV)
    from prodiff_amd import _lib
    outs, tags = {}, {}
    for layer in (0, 1):
        m = WaveNet(80, 256, 20, 256, cyc)
        m.load_state_dict(net.state_dict())
        m = m.to(DEV).set_compute_dtype("bf16").set_options(layer=layer)
        m(spec, steps, cond)                      # pack the handle
        torch.cuda.synchronize()
        _lib.profile_enable(True)
        outs[layer] = m(spec, steps, cond).float().cpu().numpy()
        torch.cuda.synchronize()
        tags[layer] = set(_lib.profile_summary())
        _lib.profile_enable(False)
    assert "wn_gate2" in tags[1] and "wn_resskip2" in tags[1] and "wn_layer" not in tags[1], tags[1]
    assert "wn_layer" in tags[0], tags[0]
    a, b = outs[1], outs[0]
    rel = float(np.linalg.norm(a - b) / np.linalg.norm(b))
    print(f"BF16ERR two-kernel vs fused WaveNet cyc={cyc} B={B}x{T} rel-L2={rel:.3e}")
    assert np.isfinite(a).all() and rel <= 2e-3



@pytest.mark.parametrize("opts", [dict(lvc_pf=0, lvc_tpw=1), dict(lvc_pf=1, lvc_tpw=1), dict(lvc_pf=1, lvc_prio=1)])
@pytest.mark.parametrize("B,Tc", [(1, 1), (3, 5), (2, 9)])
def test_fastdiff_lvc_schedule_variants(opts, B, Tc):
    """LVC-block variants that change only the schedule, not the arithmetic of a tile:
    FD_OPT_LVC_TPW=1 (16 waves, one 32-row tile each; with and without the next-layer kernel
    prefetch), and FD_OPT_LVC_PRIO (static priority for half the waves).
    The sample is bit-identical to the default kernel with the same prefetch setting, and within
    the bf16 bar of the oracle."""
    from prodiff_amd.schedules import fastdiff_infer_params, fastdiff_reverse_schedule, fastdiff_train_alpha
    p = G.fastdiff_params(31)
    b, a, s, st = fastdiff_infer_params(fastdiff_reverse_schedule(4), fastdiff_train_alpha())
    mel = synth.synth_inputs(60 + B, (B, Tc, 80), loc=-5.0, scale=2.0)
    xT = synth.synth_inputs(61 + B, (B, 1, Tc * 256))
    nz = synth.synth_inputs(62 + B, (3, B, 1, Tc * 256))
    outs = []
    for o in (dict(lvc_pf=opts["lvc_pf"]), opts):
        m = FastDiff()
        m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
        m = m.to(DEV).set_compute_dtype("bf16").set_options(**o)
        outs.append(m.sample(tt(mel), b, a, s, st, x_T=tt(xT), noise=tt(nz)).cpu().numpy())
    np.testing.assert_array_equal(outs[1], outs[0])
    ref = OF.fastdiff_sample(OF.fold_weight_norm(p), np.transpose(mel, (0, 2, 1)), xT, nz, b, a, s, st)
    assert_bf16_close(outs[1].reshape(ref.shape), ref, f"sampler {opts} B={B} Tc={Tc}")


@pytest.mark.parametrize("stack", [1, 4, 7, 10, 16])
@pytest.mark.parametrize("B,T", [(2, 64), (3, 101), (1, 250)])
def test_wavenet_stack_bitexact(stack, B, T):
    """PD_WN_OPT_STACK (wn_stack_bf16_kernel: `stack` residual layers per launch on a resident
    64-frame window) against the one-layer fused kernel (PD_WN_OPT_LAYER=0): the same bf16
    roundings and MFMA order, so the output is bit-identical -- ragged lengths put utterance
    boundaries inside the windows (T = 64 is the smallest T the stack path takes), and 20 layers
    run as uneven launch groups (7: 7 + 7 + 6).  Then within the bf16 bar of the fp32 path."""
    torch.manual_seed(11)
    net = WaveNet(80, 256, 20, 256, 1)
    spec = torch.randn(B, 1, 80, T, device=DEV)
    cond = torch.randn(B, 256, T, device=DEV)
    steps = torch.tensor([3.0, 511.0, 77.0][:B], device=DEV)
    outs = {}
    for name, opts in (("layer", dict(layer=0, stack=0)), ("stack", dict(stack=stack))):
        m = WaveNet(80, 256, 20, 256, 1)
        m.load_state_dict(net.state_dict())
        m = m.to(DEV).set_compute_dtype("bf16").set_options(**opts)
        outs[name] = m(spec, steps, cond).float().cpu().numpy()
    np.testing.assert_array_equal(outs["stack"], outs["layer"])
    m32 = WaveNet(80, 256, 20, 256, 1)
    m32.load_state_dict(net.state_dict())
    ref = m32.to(DEV)(spec, steps, cond).float().cpu().numpy()
    assert_bf16_close(outs["stack"], ref, f"wavenet stack={stack} B={B} T={T}")


@pytest.mark.parametrize("ro", [16, 23, 32, 41, 44])
@pytest.mark.parametrize("B,T", [(3, 101), (2, 300)])
def test_wavenet_stack_rows_bitexact(ro, B, T):
    """PD_WN_OPT_STACK_RO: stack blocks writing `ro` of their 64 window rows (up to 44 = 64 - 2 x
    10 layers of halo, the default) compute every frame exactly as the one-layer kernel does (the
    block boundaries move): bit-identical."""
    torch.manual_seed(12)
    net = WaveNet(80, 256, 20, 256, 1)
    spec = torch.randn(B, 1, 80, T, device=DEV)
    cond = torch.randn(B, 256, T, device=DEV)
    steps = torch.tensor([5.0, 300.0, 17.0][:B], device=DEV)
    outs = {}
    for name, opts in (("layer", dict(layer=0, stack=0)), ("stack", dict(stack=10, stack_ro=ro))):
        m = WaveNet(80, 256, 20, 256, 1)
        m.load_state_dict(net.state_dict())
        m = m.to(DEV).set_compute_dtype("bf16").set_options(**opts)
        outs[name] = m(spec, steps, cond).float().cpu().numpy()
    np.testing.assert_array_equal(outs["stack"], outs["layer"])


@pytest.mark.parametrize("draws", ["explicit", "philox"])
@pytest.mark.parametrize("M,B,T,S", [(80, 2, 101, 2), (80, 3, 64, 4), (80, 1, 250, 3), (128, 2, 90, 4)])
def test_prodiff_stack_fuse_bitexact(draws, M, B, T, S):
    """PD_WN_OPT_STACK_FUSE: the input projection inside the first stack launch and the skip head +
    output projection + posterior update inside the last one (prodiff.py:106-126) use the separate
    launches' roundings and k order: the whole bf16 sample is bit-identical to stack_fuse=0, with
    explicit draws and with on-device Philox draws (utterance ids shuffled), at the C3 (M=80) and
    SVS (M=128) mel sizes; and a single forward (input projection fused, no posterior) matches too."""
    torch.manual_seed(41 + B)
    gd = GaussianDiffusion(M, WaveNet(M, 256, 20, 256, 1), timesteps=4, time_scale=1000, max_beta=0.7)
    sd = gd.state_dict()
    cond = torch.randn(B, T, 256, device=DEV)
    xT = torch.rand(B, 1, M, T, device=DEV) if draws == "explicit" else None
    nz = torch.randn(S, B, 1, M, T, device=DEV) if draws == "explicit" else None
    ids = list(range(7, 7 + B))[::-1]
    spec = torch.randn(B, 1, M, T, device=DEV)
    steps = torch.tensor([3.0, 1.0, 2.0][:B], device=DEV)
    outs, fwd = [], []
    for fuse in (0, 1):
        g = GaussianDiffusion(M, WaveNet(M, 256, 20, 256, 1), timesteps=4, time_scale=1000, max_beta=0.7)
        g.load_state_dict(sd)
        g = g.to(DEV).set_compute_dtype("bf16")
        g.denoise_fn.set_options(stack_fuse=fuse)
        outs.append(g.sample(cond, infer_step=S, x_T=xT, noise=nz, seed=1234, utt_ids=ids).cpu().numpy())
        fwd.append(g.denoise_fn(spec, steps, cond.transpose(1, 2)).float().cpu().numpy())
    assert np.isfinite(outs[1]).all()
    np.testing.assert_array_equal(outs[1], outs[0])
    np.testing.assert_array_equal(fwd[1], fwd[0])


@pytest.mark.parametrize("cyc,M", [(5, 64), (2, 80), (3, 128)])
@pytest.mark.parametrize("B,T", [(2, 64), (3, 101), (1, 300)])
def test_wavenet_stack_dilation_bitexact(cyc, M, B, T):
    """r06: the stack kernel at dilation cycles > 1 (the pitch predictor's WaveNet: cycle 5, M = 64,
    pitch_predictor.py:40-55) -- layers grouped so each launch's dilations sum to <= 16 (cycle 5:
    {1,2,4,8} and {16}), taps at -+2^(l % cyc) -- against the one-layer kernel: bit-identical (batch
    rows end inside the windows; the dilation-16 taps cross the whole halo).  Then within the bf16
    bar of the fp32 path."""
    torch.manual_seed(13 + cyc)
    net = WaveNet(M, 256, 20, 256, cyc)
    spec = torch.randn(B, 1, M, T, device=DEV)
    cond = torch.randn(B, 256, T, device=DEV)
    steps = torch.tensor([3.0, 511.0, 77.0][:B], device=DEV)
    outs = {}
    for name, opts in (("layer", dict(layer=0, stack=0)), ("stack", dict(stack=10))):
        m = WaveNet(M, 256, 20, 256, cyc)
        m.load_state_dict(net.state_dict())
        m = m.to(DEV).set_compute_dtype("bf16").set_options(**opts)
        outs[name] = m(spec, steps, cond).float().cpu().numpy()
    np.testing.assert_array_equal(outs["stack"], outs["layer"])
    m32 = WaveNet(M, 256, 20, 256, cyc)
    m32.load_state_dict(net.state_dict())
    ref = m32.to(DEV)(spec, steps, cond).float().cpu().numpy()
    assert_bf16_close(outs["stack"], ref, f"wavenet cyc={cyc} stack B={B} T={T}")


@pytest.mark.parametrize("algo", ["euler", "rk2"])
@pytest.mark.parametrize("ragged", [False, True])
def test_pitch_reflow_stack_bitexact(algo, ragged):
    """The pitch predictor's sampler (PitchRectifiedFlow, 20 steps, WaveNet cycle 5, M = 64) on the
    stack kernel -- with Euler's x += v dt fused into the last stack launch (the posterior epilogue
    with c1 = dt, c2 = 1) -- against the one-layer kernel with the separate skip-head and output
    launches: bit-identical, dense and ragged (per-row lens)."""
    from prodiff_amd import PitchRectifiedFlow
    torch.manual_seed(17)
    B, T = 3, 150
    net = WaveNet(64, 256, 20, 256, 5)
    cond = torch.randn(B, T, 256, device=DEV)
    xT = torch.randn(B, 1, 64, T, device=DEV)
    lens = [150, 97, 64] if ragged else None
    outs = {}
    for name, opts in (("layer", dict(layer=0, stack=0)), ("stack", dict(stack=10))):
        m = WaveNet(64, 256, 20, 256, 5)
        m.load_state_dict(net.state_dict())
        rf = PitchRectifiedFlow(64, m, time_scale=1000, sampling_algorithm=algo).to(DEV)
        rf.set_compute_dtype("bf16")
        m.set_options(**opts)
        outs[name] = rf.sample(cond, infer_step=20 if algo == "euler" else 4, x_T=xT, lens=lens).cpu().numpy()
    assert np.isfinite(outs["stack"]).all()
    if ragged:
        for r, n in enumerate(lens):
            np.testing.assert_array_equal(outs["stack"][r, :n], outs["layer"][r, :n])
    else:
        np.testing.assert_array_equal(outs["stack"], outs["layer"])


@pytest.mark.parametrize("B,Tc,lens,draws", [(1, 1, None, "explicit"), (3, 5, [5, 2, 4], "explicit"),
                                              (4, 100, None, "philox"), (8, 200, [200, 150, 199, 3, 200, 120, 77, 200],
                                                                          "philox")])
def test_fastdiff_lvc_persistent_bitexact(B, Tc, lens, draws):
    """FD_OPT_LVC_PS (r06: the final and the hop-64 LVC blocks as persistent kernels, one block per CU
    walking the tiles, the next tile's audio / x_prev / biases by LDS-DMA under the current tile's layers)
    against the one-tile-per-block kernels: the 4-step sample bit for bit -- one tile, ragged rows, and grids
    of 268 and 1 072 final-block tiles (several per block; 4x as many hop-64 tiles), explicit and on-device
    draws."""
    from prodiff_amd.schedules import fastdiff_infer_params, fastdiff_reverse_schedule, fastdiff_train_alpha
    from prodiff_amd import _lib
    p = G.fastdiff_params(31)
    b, a, s, st = fastdiff_infer_params(fastdiff_reverse_schedule(4), fastdiff_train_alpha())
    mel = synth.synth_inputs(80 + B, (B, Tc, 80), loc=-5.0, scale=2.0)
    kw = {}
    if draws == "explicit":
        kw = dict(x_T=tt(synth.synth_inputs(81 + B, (B, 1, Tc * 256))),
                  noise=tt(synth.synth_inputs(82 + B, (3, B, 1, Tc * 256))))
    else:
        kw = dict(seed=77)
    outs = []
    for ps in (0, 1):
        m = FastDiff()
        m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
        m = m.to(DEV).set_compute_dtype("bf16").set_options(lvc_ps=ps)
        _lib.profile_enable(True)
        outs.append(m.sample(tt(mel), b, a, s, st, lens=lens, **kw).cpu().numpy())
        torch.cuda.synchronize()
        assert "fd_lvc_block_final" in _lib.profile_summary()
        _lib.profile_enable(False)
    assert np.isfinite(outs[1]).all()
    if lens is None:
        np.testing.assert_array_equal(outs[1], outs[0])
    else:
        o0, o1 = outs[0].reshape(B, -1), outs[1].reshape(B, -1)
        for r, n in enumerate(lens):
            np.testing.assert_array_equal(o1[r, :n * 256], o0[r, :n * 256])
