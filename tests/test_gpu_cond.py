"""GPU parity of the condition stage (pd_cond_forward, prodiff_amd.teacher.ProDiffTeacher)
against the reference teacher's own outputs (tests/golden/cond_*.npz, made by
tests/golden/gen_golden.py:gen_cond from modules/svs/prodiff_teacher.py:103-146).

fp32: max|delta| <= 1e-4 (north star tolerance) on the encoder output and the condition.
bf16: the shared bf16 bar (tests/bf16_bar.py).
"""
import numpy as np
import pytest
import torch

from tests import golden_io as G
from tests.bf16_bar import assert_bf16_close

pytestmark = pytest.mark.gpu

TOL = 1e-4


def teacher_for(hp, P, vocab):
    from prodiff_amd.teacher import ProDiffTeacher
    rhp = dict(hp, audio_num_mel_bins=128, dropout=0.1, languages=["l%d" % i for i in range(hp["num_langs"] - 1)],
               residual_layers=2, residual_channels=256, dilation_cycle_length=1, timesteps=4, timescale=1000,
               schedule_type="vpsde", max_beta=40.0, spec_min=[-12], spec_max=[0])
    t = ProDiffTeacher(vocab, rhp)
    missing, unexpected = t.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()}, strict=False)
    assert not unexpected
    assert all(k.startswith("diffusion.") or k.endswith("_float_tensor") for k in missing), missing
    return t.cuda()


def cuda_inputs(ins):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in ins.items()}


@pytest.mark.parametrize("name", G.COND_CASES)
def test_cond_golden_fp32(name):
    hp, P, ins, d = G.cond_case(name)
    t = teacher_for(hp, P, int(d["vocab"]))
    if hp.get("rel_pos_len"):   # the state a longer batch leaves (forward_condition extends it the same way)
        t.encoder.embed_positions.extend(hp["rel_pos_len"])
    x = cuda_inputs(ins)
    cond, enc = t.forward_condition(x.pop("txt_tokens"), x.pop("mel2ph"), x.pop("f0"), return_encoder=True, **x)
    enc, cond = enc.cpu().numpy(), cond.cpu().numpy()
    e1, e2 = np.abs(enc - d["enc"]).max(), np.abs(cond - d["cond"]).max()
    print(f"COND {name} enc max|d|={e1:.3e} cond max|d|={e2:.3e}", flush=True)
    assert e1 <= TOL and e2 <= TOL
    assert np.all(cond[d["mel2ph"] == 0] == 0)


@pytest.mark.parametrize("name", ["cond_small", "cond_handler"])
def test_cond_golden_bf16(name):
    hp, P, ins, d = G.cond_case(name)
    t = teacher_for(hp, P, int(d["vocab"])).set_compute_dtype("bf16")
    x = cuda_inputs(ins)
    cond, enc = t.forward_condition(x.pop("txt_tokens"), x.pop("mel2ph"), x.pop("f0"), return_encoder=True, **x)
    assert_bf16_close(enc.cpu().numpy(), d["enc"], f"cond-encoder {name}")
    assert_bf16_close(cond.cpu().numpy(), d["cond"], f"cond {name}")


def test_cond_deterministic_and_encoder_only():
    hp, P, ins, d = G.cond_case("cond_small")
    t = teacher_for(hp, P, int(d["vocab"]))
    x = cuda_inputs(ins)
    args = (x.pop("txt_tokens"), x.pop("mel2ph"), x.pop("f0"))
    c1, e1 = t.forward_condition(*args, return_encoder=True, **x)
    c2 = t.forward_condition(*args, **x)
    assert torch.equal(c1, c2)
    # encoder-only call through the C-ABI (cond = NULL)
    from prodiff_amd import _lib
    L = _lib.lib()
    h = t.cond_handle()
    B, Tt = args[0].shape
    Tm = args[1].shape[1]   # mel2ph still feeds the duration embedding
    enc = torch.empty(B, Tt, hp["hidden_size"], device="cuda")
    vp = lambda v: None if v is None else v.data_ptr()
    ins_c = _lib.pd_cond_inputs(vp(args[0]), vp(args[1]), None, vp(x["lang_seq"]), None, None, 0, None, None, 0,
                                None, None)
    nb = L.pd_cond_workspace_size(h, B, Tt, Tm)
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    _lib.check(L.pd_cond_forward(h, _lib.C.byref(ins_c), None, _lib.fptr(enc), B, Tt, Tm, _lib.C.c_void_p(ws.data_ptr()),
                                 nb, _lib.stream_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(enc, e1)
    # missing required inputs fail loudly, before any launch
    ins_c.lang_seq = None
    assert L.pd_cond_forward(h, _lib.C.byref(ins_c), None, _lib.fptr(enc), B, Tt, Tm, _lib.C.c_void_p(ws.data_ptr()),
                             nb, _lib.stream_ptr()) == 1
    assert b"lang_seq" in L.pd_last_error()


def test_teacher_forward_infer_end_to_end():
    """ProDiffTeacher.forward(infer=True) == diffusion(forward_condition(...)) (prodiff_teacher.py:148-168)."""
    from prodiff_amd import synth
    hp, P, ins, d = G.cond_case("cond_small")
    t = teacher_for(hp, P, int(d["vocab"]))
    wn = synth.synth_params(synth.wavenet_param_shapes(128, 256, 2, 256), 5)
    t.diffusion.denoise_fn.load_state_dict({k: torch.from_numpy(v) for k, v in wn.items()})
    t.cuda()
    x = cuda_inputs(ins)
    args = (x.pop("txt_tokens"), x.pop("mel2ph"), x.pop("f0"))
    torch.manual_seed(3)
    mel = t(*args, infer=True, **x)
    torch.manual_seed(3)
    ref = t.diffusion(t.forward_condition(*args, **x), infer=True)
    assert mel.shape == (args[0].shape[0], args[1].shape[1], 128)
    assert torch.isfinite(mel).all() and torch.equal(mel, ref)


def test_svs_synthesizer_ragged_tokens_and_pipeline():
    """SvsSynthesizer (bench C5): a batch with different phoneme counts, encoded in ONE padded
    pass with each row's phoneme count as txt_lens, equals every segment encoded alone (B=1, the
    reference handler's way) within 1e-5 * max (the split-K choice of the small GEMMs depends on
    the row count); the whole path returns finite mel [B,T,128] and wav [B,T*512];
    distributed_synthesize un-permutes it."""
    from prodiff_amd import synth
    from prodiff_amd.pipeline import SVS_VOCAB, SvsSynthesizer, distributed_synthesize
    syn = SvsSynthesizer.synthetic(torch.device("cuda"), seed=0, dtype="fp32", residual_layers=2)
    T = 40
    utts = [{k: torch.from_numpy(v).cuda() for k, v in synth.synth_svs_utterance(s, T, n, SVS_VOCAB).items()}
            for s, n in ((1, 9), (2, 13), (3, 9))]
    batch = SvsSynthesizer.collate(utts)
    cond = syn.condition(batch)
    for i, u in enumerate(utts):
        alone = syn.condition(SvsSynthesizer.collate([u]))
        err = float((cond[i] - alone[0]).abs().max())
        assert err <= 1e-5 * float(alone[0].abs().max()), (i, err)
    mel, wav = syn(batch, seed=5)
    assert mel.shape == (3, T, 128) and wav.shape == (3, T * 512)
    assert torch.isfinite(mel).all() and torch.isfinite(wav).all() and wav.abs().max() <= 1.0
    mels, wavs = distributed_synthesize(syn, [(T, (lambda u=u: u)) for u in utts], seed=5, hop=512)
    assert len(mels) == 3 and all(m.shape == (T, 128) for m in mels) and all(w.shape == (T * 512,) for w in wavs)
