"""NSF-HiFiGAN, CPU side: the oracle against the reference's own
outputs (tests/golden/gen_golden_nsf.py ran modules/nsf_hifigan/models.py), the
mirrored module's state-dict names, the C-ABI parameter count and the registry."""
import numpy as np
import pytest

from oracle import oracle_nsf as ON
from prodiff_amd import _lib, synth
from prodiff_amd.nsf_hifigan import Generator, NsfHifiGAN
from prodiff_amd.vocoder import get_vocoder_cls
from tests.nsf_cases import CASES, load


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_golden(name):
    h, io, seed = load(name)
    p = synth.synth_params(synth.nsf_param_shapes(**h), seed)
    wav = ON.spec2wav(p, h, io["mel"], io["f0"], io["rand_ini"], io["noise"])
    # reference runs in fp32 (its phase cumsum in fp64): 2.7e-6 seen, bar 1e-5
    assert np.abs(wav - io["wav"]).max() < 1e-5


def test_oracle_sine_phase_shift_is_whole_cycles():
    """The restatement drops the reference's cumsum_shift (models.py:155-161): with
    f0 high enough to wrap inside every frame the golden still matches (above)."""
    h, io, _ = load("nsf_c64_r8822")
    rad = np.fmod(io["f0"][0] * 9 / h["sampling_rate"], 1.0)
    assert (rad * np.prod(h["upsample_rates"]) > 1.0).any()


@pytest.mark.parametrize("name", CASES)
def test_state_dict_names_and_param_count(name):
    h, _, _ = load(name)
    g = Generator(h)
    shapes = synth.nsf_param_shapes(**h)
    sd = g.state_dict()
    assert list(sd) == list(shapes)
    assert all(tuple(sd[k].shape) == tuple(v) for k, v in shapes.items())
    assert _lib.lib().nsf_num_params(_lib.C.byref(g._dims())) == len(sd)


def test_weight_norm_state_dict_is_folded():
    import torch
    h, _, _ = load("nsf_c32_r44_rb2")
    g = Generator(h)
    p = synth.synth_params(synth.nsf_param_shapes(**h), 3)
    sd = {k: torch.from_numpy(v) for k, v in p.items()}
    wn = dict(sd)
    v = torch.randn(32, 16, 8)       # ConvTranspose1d [Cin, Cout, k], weight_norm dim 0
    gg = torch.rand(32, 1, 1) + 0.5
    del wn["ups.0.weight"]
    wn["ups.0.weight_g"], wn["ups.0.weight_v"] = gg, v
    g.load_state_dict(wn)
    ref = gg * v / v.pow(2).sum(dim=(1, 2), keepdim=True).sqrt()
    assert torch.allclose(g.ups[0].weight, ref)


def test_registry_and_cpu_tensors_fail_loudly():
    import torch
    assert get_vocoder_cls("NsfHifiGAN") is NsfHifiGAN
    h, io, _ = load("nsf_c32_r44_rb2")
    voc = NsfHifiGAN({}, model=Generator(h))
    with pytest.raises((_lib.HipError, TypeError)):
        voc.spec2wav_torch(torch.from_numpy(io["mel"]), f0=torch.from_numpy(io["f0"]))
