"""The oracle (CPU restatement) against the reference's own outputs.

The golden vectors were produced by running the reference PyTorch code
(tests/golden/gen_golden.py); matching them pins the oracle before it is used
to check the HIP path at other sizes.
"""
import numpy as np
import pytest

from oracle import oracle_fastdiff as OF
from oracle import oracle_prodiff as OP
from tests import golden_io as G

WAVENET = ["wavenet_m80_c256_l20_cyc1", "wavenet_m80_c256_l20_float",
           "wavenet_m64_c256_l20_cyc5", "wavenet_m128_c256_l20_cyc1", "wavenet_m80_c64_l4_cyc2"]


@pytest.mark.parametrize("name", WAVENET)
def test_wavenet_oracle(name):
    d = G.load(name)
    p = G.wavenet_params(d["dims"], d["seed"])
    L, cyc = int(d["dims"][2]), int(d["dims"][4])
    out = OP.wavenet_forward(p, d["spec"], d["steps"], d["cond"], L, cyc)
    assert np.abs(out - d["out"]).max() < 2e-5


def test_prodiff_schedule():
    s = G.load("schedules")
    for ts in (1, 2, 4, 8, 100):
        for mb in (40.0, 0.06):
            bufs = OP.diffusion_buffers(OP.vpsde_betas(ts, mb))
            for k, v in bufs.items():
                ref = s[f"t{ts}_mb{mb}_{k}"]
                np.testing.assert_allclose(v, ref, rtol=1e-6, atol=0, err_msg=k)


@pytest.mark.parametrize("name", ["prodiff_t2_m80", "prodiff_t4_m80", "prodiff_t4_m128"])
def test_prodiff_sample_oracle(name):
    d = G.load(name)
    p = G.prodiff_params(name)
    bufs = G.prodiff_buffers(d)
    mel = OP.prodiff_sample(p, bufs, d["cond"], d["x_T"], d["noise"])
    assert mel.shape == d["mel"].shape
    assert np.abs(mel - d["mel"]).max() < 2e-5


def test_fastdiff_schedules():
    s = G.load("schedules")
    at = OF.train_alpha()
    np.testing.assert_allclose(at, s["fd_train_alpha"], rtol=0, atol=1e-7)
    for n in (3, 4, 6, 8):
        b, a, sg, st = OF.infer_schedule(s[f"fd_n{n}_beta"], s["fd_train_alpha"])
        np.testing.assert_allclose(a, s[f"fd_n{n}_alpha"], rtol=1e-6)
        np.testing.assert_allclose(sg, s[f"fd_n{n}_sigma"], rtol=1e-6)
        np.testing.assert_allclose(st, s[f"fd_n{n}_steps"], rtol=0, atol=1e-3)


@pytest.fixture(scope="module")
def fd():
    d = G.load("fastdiff_fwd")
    p = OF.fold_weight_norm(G.fastdiff_params(d["seed"]))
    return d, p


def test_fastdiff_forward_oracle(fd):
    d, p = fd
    cap = {}
    eps = OF.fastdiff_forward(p, d["audio"], d["c"], d["steps"], capture=cap)
    for n in range(3):
        np.testing.assert_allclose(cap[f"downsample{n}"], d[f"cap_downsample{n}"], atol=2e-5, rtol=0)
        # block outputs reach |x|~30; the fp32 reference itself drifts ~5e-6 relative there
        ref = d[f"cap_lvc{n}"]
        assert np.abs(cap[f"lvc{n}"] - ref).max() < 1e-5 * np.abs(ref).max()
    assert np.abs(eps - d["eps"]).max() < 2e-5


def test_fastdiff_ops_oracle(fd):
    d, p = fd
    e = OF.step_embedding(d["steps"])
    e = OF.swish(OF.linear(e, p["fc_t1.weight"], p["fc_t1.bias"]))
    e = OF.swish(OF.linear(e, p["fc_t2.weight"], p["fc_t2.bias"]))
    q = "lvc_blocks.0."
    noise = OF.linear(e, p[q + "fc_t.weight"], p[q + "fc_t.bias"])[:, :, None]
    k, b = OF.kernel_predictor(p, q + "kernel_predictor.", d["c"] + noise)
    np.testing.assert_allclose(k[0], d["cap_kp0_kernels_b0"], atol=2e-5, rtol=0)
    x = OF.lrelu(d["cap_downsample2"], 0.2)
    up = OF.conv_transpose1d(x, p[q + "upsample.weight"], p[q + "upsample.bias"], 8, 4, 0)
    np.testing.assert_allclose(up, d["cap_upsample0"], atol=2e-5, rtol=0)


@pytest.mark.parametrize("n_iter", [4, 3, 6, 8])
def test_fastdiff_sample_oracle(n_iter):
    d = G.load(f"fastdiff_sample_n{n_iter}")
    s = G.load("schedules")
    p = OF.fold_weight_norm(G.fastdiff_params(31))
    b, a, sg, st = OF.infer_schedule(s[f"fd_n{n_iter}_beta"], s["fd_train_alpha"])
    np.testing.assert_allclose(st[::-1], d["steps_seen"], atol=1e-4)
    wav = OF.fastdiff_sample(p, d["c"], d["x_T"], d["noise"], b, a, sg, st)
    assert np.abs(wav - d["wav"]).max() < 1e-4


REFLOW = ["reflow_euler_m80", "reflow_rk2_m128", "reflow_rk4_m80", "reflow_rk5_m80", "pitch_reflow_rk2_r64"]


@pytest.mark.parametrize("name", REFLOW)
def test_reflow_oracle(name):
    from oracle import oracle_reflow as OR
    d = G.load(name)
    p = G.wavenet_params(d["dims"], d["seed"])
    L, cyc = int(d["dims"][2]), int(d["dims"][4])
    x = OR.reflow_sample(p, d["cond"], d["x_T"], int(d["infer_step"]), str(d["algo"]), 1000, L, cyc)
    assert x.shape == d["x"].shape
    assert np.abs(x - d["x"]).max() < 2e-5
    if str(d["kind"]) == "pitch":
        out = OR.pitch_denorm(x, -8.0, 8.0, -12.0, 12.0)
    else:
        out = OR.denorm_spec(x, [-12.0], [0.0])
    assert np.abs(out - d["out"]).max() < 2e-5


# ---------------------------------------------------------------- torch fp32 port
# oracle_torch.py is the CPU line bench.py times on the GPU box (cpu_baseline_port);
# pin it to the same reference goldens.
def _tt(a):
    import torch
    return torch.as_tensor(np.asarray(a), dtype=torch.float32)


def test_torch_port_prodiff_sample():
    from oracle import oracle_torch as OT
    d = G.load("prodiff_t2_m80")
    p = {k: _tt(v) for k, v in G.prodiff_params("prodiff_t2_m80").items()}
    mel = OT.prodiff_sample(p, G.prodiff_buffers(d), _tt(d["cond"]), _tt(d["x_T"]),
                            [_tt(n) for n in d["noise"]]).numpy()
    assert np.abs(mel - d["mel"]).max() < 1e-4


def test_torch_port_fastdiff_sample():
    from oracle import oracle_torch as OT
    d = G.load("fastdiff_sample_n4")
    s = G.load("schedules")
    p = OT.fold_weight_norm(G.fastdiff_params(31))
    b, a, sg, st = OF.infer_schedule(s["fd_n4_beta"], s["fd_train_alpha"])
    wav = OT.fastdiff_sample(p, _tt(d["c"]), _tt(d["x_T"]), [_tt(n) for n in d["noise"]], b, a, sg, st).numpy()
    assert np.abs(wav - d["wav"]).max() < 1e-4


def test_torch_port_lvc_matches_numpy():
    import torch
    from oracle import oracle_torch as OT
    rng = np.random.default_rng(3)
    x = rng.standard_normal((2, 32, 5 * 8))
    k = rng.standard_normal((2, 32, 64, 3, 5))
    b = rng.standard_normal((2, 64, 5))
    ref = OF.lvc(x, k, b, 8)
    out = OT.lvc(_tt(x), _tt(k), _tt(b), 8).numpy()
    assert np.abs(out - ref).max() < 1e-4


# ---------------------------------------------------------------- condition stage
@pytest.mark.parametrize("name", G.COND_CASES)
def test_cond_oracle(name):
    """oracle_encoder.forward_condition vs the reference teacher's outputs (fp32 reference,
    float64 oracle: the gap is the reference's own rounding)."""
    from oracle import oracle_encoder as OE
    hp, P, ins, d = G.cond_case(name)
    cond, enc = OE.forward_condition(P, hp, return_encoder=True, **ins)
    assert np.abs(enc - d["enc"]).max() <= 5e-5
    assert np.abs(cond - d["cond"]).max() <= 5e-5
    # length-regulator invariants: padding frames are exactly zero; dur sums to the frame count
    assert np.all(cond[d["mel2ph"] == 0] == 0)
    dur = OE.mel2ph_to_dur(d["mel2ph"], d["txt_tokens"].shape[1])
    assert np.array_equal(dur.sum(1), (d["mel2ph"] > 0).sum(1))
