"""NSF-HiFiGAN on the GPU through the C-ABI (nsf_forward).

Bar: |wav - ref| <= 1e-4 absolute (fp32 compute; wav is tanh-bounded in [-1, 1]),
against the reference's own outputs (tests/golden/nsf_*.npz) and the fp64 oracle.
"""
import numpy as np
import pytest
import torch

from oracle import oracle_nsf as ON
from prodiff_amd import synth
from prodiff_amd.nsf_hifigan import Generator, NsfHifiGAN
from tests.nsf_cases import CASES, load

pytestmark = pytest.mark.gpu
TOL = 1e-4
DEV = "cuda"


def _gen(h, seed):
    p = synth.synth_params(synth.nsf_param_shapes(**h), seed)
    g = Generator(h)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    return g.to(DEV).eval(), p


@pytest.mark.parametrize("name", CASES)
def test_golden_spec2wav_torch(name):
    h, io, seed = load(name)
    g, _ = _gen(h, seed)
    voc = NsfHifiGAN({}, model=g)
    t = lambda a: torch.from_numpy(a).to(DEV)
    wav = voc.spec2wav_torch(t(io["mel"]), f0=t(io["f0"]), rand_ini=t(io["rand_ini"]), noise=t(io["noise"]))
    err = float(np.abs(wav.cpu().numpy() - io["wav"].reshape(-1)).max())
    assert err < TOL, err


def test_generator_forward_channel_major_vs_oracle():
    h, io, seed = load("nsf_c64_r8822")
    g, p = _gen(h, seed)
    c = 2.30259 * np.transpose(io["mel"], (0, 2, 1)).astype(np.float32)
    out = g(torch.from_numpy(c).to(DEV), torch.from_numpy(io["f0"]).to(DEV),
            rand_ini=torch.from_numpy(io["rand_ini"]), noise=torch.from_numpy(io["noise"]))
    ref = ON.generator_forward(p, h, c, io["f0"], io["rand_ini"], io["noise"])
    assert out.shape == (1, 1, io["wav"].shape[-1])
    assert float(np.abs(out.cpu().numpy() - ref).max()) < TOL


@pytest.mark.parametrize("T", [1, 3, 24])
def test_full_dims_batch_vs_oracle(T):
    """SVS dims (512 ch, hop 512), B=2 independent utterances, ragged voicing, T=1 edge."""
    h = dict(synth.NSF_DEFAULTS)
    g, p = _gen(h, 7)
    B, L = 2, T * 512
    rng = np.random.default_rng(T)
    mel = rng.normal(-2.0, 1.0, size=(B, T, 128)).astype(np.float32)
    f0 = rng.uniform(60.0, 1100.0, size=(B, T)).astype(np.float32)
    f0[0, ::2] = 0.0
    ri = rng.random(9, dtype=np.float32)
    nz = rng.standard_normal((B, L, 9), dtype=np.float32)
    wav = g.synthesize(torch.from_numpy(mel).to(DEV), torch.from_numpy(f0).to(DEV), 2.30259,
                       rand_ini=torch.from_numpy(ri), noise=torch.from_numpy(nz)).cpu().numpy()
    for b in range(B):
        ref = ON.spec2wav(p, h, mel[b:b + 1], f0[b:b + 1], ri, nz[b:b + 1])[0]
        assert float(np.abs(wav[b] - ref).max()) < TOL


def test_device_draws_deterministic_and_bounded():
    h, io, seed = load("nsf_c64_r8822")
    g, _ = _gen(h, seed)
    mel = torch.from_numpy(np.repeat(io["mel"], 2, 0)).to(DEV)
    f0 = torch.from_numpy(np.repeat(io["f0"], 2, 0)).to(DEV)
    a = g.synthesize(mel, f0, 2.30259, seed=5)
    b = g.synthesize(mel, f0, 2.30259, seed=5)
    c = g.synthesize(mel, f0, 2.30259, seed=6)
    assert torch.equal(a, b)
    assert not torch.equal(a, c)
    assert torch.isfinite(a).all() and a.abs().max() <= 1.0
    # utterances draw independent noise: identical inputs, different outputs
    assert not torch.equal(a[0], a[1])
    # the draws only perturb the source: output stays near the golden one
    assert float((a[0].cpu() - torch.from_numpy(io["wav"][0])).abs().mean()) < 0.1


@pytest.mark.parametrize("wconv,T,B", [(1, 24, 1), (0, 24, 1), (1, 37, 2), (1, 1, 3), (1, 70, 1)])
def test_bf16_full_dims_vs_oracle(wconv, T, B):
    """bf16 path (windowed MFMA ResBlock convs and ConvTranspose upsamples, or the implicit-GEMM
    engine with wconv=0) against the fp64 oracle with the shared bf16 bar (tests/bf16_bar.py);
    T=37/70 leave partial tiles at every stage (the 512-channel upsample's 64-row input tiles
    included), T=1 is all halo, B>1 checks utterances do not bleed into each other's windows."""
    h = dict(synth.NSF_DEFAULTS)
    g, p = _gen(h, 7)
    g.set_compute_dtype("bf16").set_options(wconv=wconv)
    L = T * 512
    rng = np.random.default_rng(11)
    mel = rng.normal(-2.0, 1.0, size=(B, T, 128)).astype(np.float32)
    f0 = rng.uniform(60.0, 900.0, size=(B, T)).astype(np.float32)
    ri = rng.random(9, dtype=np.float32)
    nz = rng.standard_normal((B, L, 9), dtype=np.float32)
    wav = g.synthesize(torch.from_numpy(mel).to(DEV), torch.from_numpy(f0).to(DEV), 2.30259,
                       rand_ini=torch.from_numpy(ri), noise=torch.from_numpy(nz)).cpu().numpy()
    from tests.bf16_bar import assert_bf16_close
    for b in range(B):
        ref = ON.spec2wav(p, h, mel[b:b + 1], f0[b:b + 1], ri, nz[b:b + 1])[0]
        assert_bf16_close(wav[b], ref, f"nsf full dims T={T} wconv={wconv} b={b}")


@pytest.mark.parametrize("T,B", [(24, 1), (37, 2), (1, 3)])
def test_bf16_resblock_pair_bitexact(T, B):
    """NSF_OPT_PAIR (one launch per ResBlock1 conv pair, the inner activation kept in LDS) against
    the two-launch path: same bf16 roundings and MFMA order, so the waveform is bit-identical --
    partial tiles at every stage (T = 37), T = 1 all halo, utterances side by side (B > 1)."""
    h = dict(synth.NSF_DEFAULTS)
    g, _ = _gen(h, 7)
    rng = np.random.default_rng(5)
    mel = torch.from_numpy(rng.normal(-2.0, 1.0, size=(B, T, 128)).astype(np.float32)).to(DEV)
    f0 = torch.from_numpy(rng.uniform(60.0, 900.0, size=(B, T)).astype(np.float32)).to(DEV)
    outs = []
    for pair in (0, 1):
        g.set_compute_dtype("bf16").set_options(pair=pair)
        outs.append(g.synthesize(mel, f0, 2.30259, seed=9).cpu().numpy())
    assert np.isfinite(outs[1]).all()
    np.testing.assert_array_equal(outs[1], outs[0])


@pytest.mark.parametrize("T,B,lens", [(24, 1, None), (37, 2, [37, 21]), (1, 3, None)])
def test_bf16_ups_noise_conv_fused_bitexact(T, B, lens):
    """NSF_OPT_UPS_NC (the k <= 8 noise convs computed in the upsample's epilogue from a source
    window in LDS) against the separate nsf_noise_conv_kernel launches: same fp32 tap order, so
    the waveform is bit-identical -- partial tiles, T = 1, and a ragged row (its source reads zero
    past its own end)."""
    h = dict(synth.NSF_DEFAULTS)
    g, _ = _gen(h, 7)
    rng = np.random.default_rng(6)
    mel = torch.from_numpy(rng.normal(-2.0, 1.0, size=(B, T, 128)).astype(np.float32)).to(DEV)
    f0 = torch.from_numpy(rng.uniform(60.0, 900.0, size=(B, T)).astype(np.float32)).to(DEV)
    outs = []
    for nc in (0, 1):
        g.set_compute_dtype("bf16").set_options(ups_nc=nc)
        outs.append(g.synthesize(mel, f0, 2.30259, seed=9, lens=lens).cpu().numpy())
    assert np.isfinite(outs[1]).all()
    if lens is None:
        np.testing.assert_array_equal(outs[1], outs[0])
    else:
        for r, n in enumerate(lens):
            np.testing.assert_array_equal(outs[1][r, :n * g.upp], outs[0][r, :n * g.upp])


@pytest.mark.parametrize("T,B,lens", [(24, 1, None), (37, 2, [37, 21]), (1, 3, None), (300, 2, [300, 251])])
def test_bf16_resblock16_fused_bitexact(T, B, lens):
    """NSF_OPT_RB16 (r06: each 16-channel ResBlock1 -- three conv pairs, dilations 1 / 3 / 5 -- as one
    launch with the residual in registers; geometry 1 = 32-tile windows, 2 = 64-tile windows) against
    one nsf_pair16 launch per pair: the transposed MFMA sums the same products in the same k order and
    the epilogues round and add as the pair launches do, so the waveform is bit-identical -- partial
    windows, T = 1 (all halo), utterances side by side, ragged rows (zero past each one's end) and
    T = 300 (several windows per utterance at the 512-sample stage)."""
    h = dict(synth.NSF_DEFAULTS)
    g, _ = _gen(h, 7)
    rng = np.random.default_rng(8)
    mel = torch.from_numpy(rng.normal(-2.0, 1.0, size=(B, T, 128)).astype(np.float32)).to(DEV)
    f0 = torch.from_numpy(rng.uniform(60.0, 900.0, size=(B, T)).astype(np.float32)).to(DEV)
    outs = []
    from prodiff_amd import _lib
    for rb in (0, 1, 2):
        g.set_compute_dtype("bf16").set_options(rb16=rb)
        _lib.profile_enable(True)
        outs.append(g.synthesize(mel, f0, 2.30259, seed=9, lens=lens).cpu().numpy())
        torch.cuda.synchronize()
        tags = set(_lib.profile_summary())
        _lib.profile_enable(False)
        assert ("nsf_rb16" in tags) == (rb > 0) and ("nsf_pair16" in tags) == (rb == 0), (rb, tags)
    g.set_options(rb16=1)
    assert np.isfinite(outs[1]).all()
    for rb in (1, 2):
        if lens is None:
            np.testing.assert_array_equal(outs[rb], outs[0])
        else:
            for r, n in enumerate(lens):
                np.testing.assert_array_equal(outs[rb][r, :n * g.upp], outs[0][r, :n * g.upp])


@pytest.mark.parametrize("opt", ["rb32", "rb64"])
@pytest.mark.parametrize("T,B,lens", [(24, 1, None), (37, 2, [37, 21]), (1, 3, None), (150, 2, [150, 97])])
def test_bf16_resblock_fused_bitexact(opt, T, B, lens):
    """NSF_OPT_RB32 / RB64 (r06: the 32- / 64-channel ResBlock1s as one launch each, every kernel
    size enabled) against one nsf_pair launch per pair: bit-identical, as the C = 16 variant."""
    h = dict(synth.NSF_DEFAULTS)
    g, _ = _gen(h, 7)
    rng = np.random.default_rng(11)
    mel = torch.from_numpy(rng.normal(-2.0, 1.0, size=(B, T, 128)).astype(np.float32)).to(DEV)
    f0 = torch.from_numpy(rng.uniform(60.0, 900.0, size=(B, T)).astype(np.float32)).to(DEV)
    from prodiff_amd import _lib
    outs = []
    tag = "nsf_rb32" if opt == "rb32" else "nsf_rb64"
    for v in (0, 7):
        g.set_compute_dtype("bf16").set_options(**{opt: v})
        _lib.profile_enable(True)
        outs.append(g.synthesize(mel, f0, 2.30259, seed=9, lens=lens).cpu().numpy())
        torch.cuda.synchronize()
        tags = _lib.profile_summary()
        _lib.profile_enable(False)
        assert (tag in tags) == (v > 0), (v, tags)
        if v:
            assert tags[tag][0] == 3, tags[tag]   # one launch per ResBlock of that stage
    g.set_options(**{opt: 0})
    assert np.isfinite(outs[1]).all()
    if lens is None:
        np.testing.assert_array_equal(outs[1], outs[0])
    else:
        for r, n in enumerate(lens):
            np.testing.assert_array_equal(outs[1][r, :n * g.upp], outs[0][r, :n * g.upp])


@pytest.mark.parametrize("T,B,lens", [(24, 1, None), (37, 2, [37, 21]), (1, 3, None)])
def test_bf16_c256_nc_mfma_bitexact(T, B, lens):
    """r06 launch shapes against the previous ones, the waveform bit for bit: NSF_OPT_C256 (the 256-channel
    windowed convs with 8 waves and all output channels per block) and NSF_OPT_NC_MFMA (the K = 128 / 16
    source convs as f32-MFMA chains from the bias, the VALU kernel's fmaf order)."""
    h = dict(synth.NSF_DEFAULTS)
    g, _ = _gen(h, 7)
    rng = np.random.default_rng(12)
    mel = torch.from_numpy(rng.normal(-2.0, 1.0, size=(B, T, 128)).astype(np.float32)).to(DEV)
    f0 = torch.from_numpy(rng.uniform(60.0, 900.0, size=(B, T)).astype(np.float32)).to(DEV)
    g.set_compute_dtype("bf16")
    outs = {}
    for name, o in (("base", dict(c256=0, nc_mfma=0)), ("c256", dict(c256=1, nc_mfma=0)),
                    ("nc_mfma", dict(c256=0, nc_mfma=2))):
        g.set_options(**o)
        outs[name] = g.synthesize(mel, f0, 2.30259, seed=9, lens=lens).cpu().numpy()
    g.set_options(c256=1, nc_mfma=2)
    for name in ("c256", "nc_mfma"):
        assert np.isfinite(outs[name]).all()
        if lens is None:
            np.testing.assert_array_equal(outs[name], outs["base"], err_msg=name)
        else:
            for r, n in enumerate(lens):
                np.testing.assert_array_equal(outs[name][r, :n * g.upp], outs["base"][r, :n * g.upp], err_msg=name)
