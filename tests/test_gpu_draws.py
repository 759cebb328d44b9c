"""Sharding-invariant random draws (on-device Philox, no explicit draws).

Every sampler keys its draws by (seed, utterance id, element within the utterance)
(include/prodiff_hip.h, common.h philox_*_u), so an utterance's mel and waveform do not
depend on its row in a batch, on the rest of the batch, or on how a job is sharded over
GPUs -- the property that makes a 1-GPU and an 8-GPU run of the same utterance list
comparable element by element.  The reference is random too (handler/infer/handler.py:
373-388 runs each segment alone with torch's global RNG); these tests pin the batching
semantics, not values of the reference.

Bar: a batch of 3 equals each utterance run alone (and a permuted batch), |delta| <= 1e-5
relative to max|x| (fp32: the batched kernels may sum in a different order at other B).
The bf16 path (the one bench.py and C4 run: the FIN epilogue of the last LVC block draws
each output sample's noise by Philox keyed with utt_id(uid, b + b_off)) is held to the same
bar: every bf16 kernel computes a row from that row's inputs only, in a fixed order.
"""
import numpy as np
import pytest
import torch

from prodiff_amd import synth
from prodiff_amd.pipeline import Synthesizer, distributed_synthesize

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def close(a, b, rel=1e-5):
    a, b = a.detach().float().cpu().numpy(), b.detach().float().cpu().numpy()
    tol = rel * max(1.0, float(np.abs(b).max()))
    err = float(np.abs(a - b).max())
    assert err <= tol, (err, tol)


@pytest.fixture(scope="module", params=["fp32", "bf16"])
def syn(request):
    # the full FastDiff vocoder; a 4-layer ProDiff WaveNet keeps the test short
    return Synthesizer.synthetic(DEV, seed=3, dtype=request.param, residual_layers=4)


def test_synthesizer_batch_equals_each_alone(syn):
    # 9 frames = 2,304 samples per utterance: several 384-sample LVC tiles per utterance
    B, T = 3, 9
    cond = torch.from_numpy(synth.synth_inputs(77, (B, T, 256))).to(DEV)
    ids = [5, 9, 2]
    mel, wav = syn(cond, seed=11, utt_ids=ids)
    for i in range(B):
        m1, w1 = syn(cond[i:i + 1].contiguous(), seed=11, utt_ids=[ids[i]])
        close(mel[i:i + 1], m1)
        close(wav[i:i + 1], w1)
    # permuted batch: rows follow their ids
    perm = [2, 0, 1]
    mp, wp = syn(cond[perm].contiguous(), seed=11, utt_ids=[ids[p] for p in perm])
    close(mp, mel[perm])
    close(wp, wav[perm])
    # different ids (same inputs) draw different noise
    m2, _ = syn(cond, seed=11, utt_ids=[6, 10, 3])
    assert float((m2 - mel).abs().max()) > 1e-3


def test_default_ids_are_rows(syn):
    cond = torch.from_numpy(synth.synth_inputs(78, (2, 7, 256))).to(DEV)
    a = syn(cond, seed=4)
    b = syn(cond, seed=4, utt_ids=[0, 1])
    close(a[0], b[0], rel=0)
    close(a[1], b[1], rel=0)


def test_distributed_synthesize_matches_batched(syn):
    """distributed_synthesize (one rank here) runs equal-length groups with their global
    indices as ids: every utterance equals the plain batched call with the same ids."""
    lengths = [7, 9, 7, 5]
    conds = [torch.from_numpy(synth.synth_inputs(80 + i, (T, 256))).to(DEV) for i, T in enumerate(lengths)]
    mels, wavs = distributed_synthesize(syn, conds, seed=21)
    for i, c in enumerate(conds):
        m1, w1 = syn(c[None], seed=21, utt_ids=[i])
        close(mels[i][None], m1)
        close(wavs[i][None], w1[:, :wavs[i].shape[0]])


def test_job_streams_overlap_equals_sequential(syn):
    """pipeline.JobStreams (bench.py --overlap): jobs with 2 in flight on their own HIP streams
    give exactly the outputs of the same jobs run one after the other (per-stream workspaces,
    draws keyed by seed and utterance id)."""
    from prodiff_amd.pipeline import JobStreams
    lengths = [9, 9, 7]
    conds = [torch.from_numpy(synth.synth_inputs(90 + i, (T, 256))).to(DEV) for i, T in enumerate(lengths)]
    seq = [distributed_synthesize(syn, conds, seed=30 + j) for j in range(4)]
    torch.cuda.synchronize()
    js = JobStreams(2, DEV)
    ovl = []
    for j in range(4):
        with js.next():
            ovl.append(distributed_synthesize(syn, conds, seed=30 + j))
    torch.cuda.synchronize()
    for (m0, w0), (m1, w1) in zip(seq, ovl):
        for i in range(len(lengths)):
            close(m1[i], m0[i], rel=0)
            close(w1[i], w0[i], rel=0)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_reflow_and_nsf_batch_equals_each_alone(dtype):
    from prodiff_amd import WaveNet
    from prodiff_amd.nsf_hifigan import Generator
    from prodiff_amd.reflow import RectifiedFlow
    M, H, L, C = 80, 32, 2, 64
    net = WaveNet(M, H, L, C, 1)
    net.load_state_dict({k: torch.from_numpy(v)
                         for k, v in synth.synth_params(synth.wavenet_param_shapes(M, H, L, C), 8).items()})
    rf = RectifiedFlow(out_dims=M, denoise_fn=net, spec_min=[-12.0], spec_max=[0.0]).to(DEV)
    rf.set_compute_dtype(dtype)
    cond = torch.from_numpy(synth.synth_inputs(81, (3, 11, H))).to(DEV)
    x = rf.sample(cond, infer_step=3, seed=5, utt_ids=[4, 1, 7])
    for i, u in enumerate([4, 1, 7]):
        close(x[i:i + 1], rf.sample(cond[i:i + 1].contiguous(), infer_step=3, seed=5, utt_ids=[u]))
    h = dict(synth.NSF_DEFAULTS, upsample_initial_channel=32, upsample_rates=(4, 4), upsample_kernel_sizes=(8, 8))
    g = Generator(h)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_params(synth.nsf_param_shapes(**h), 9).items()})
    g = g.to(DEV).eval().set_compute_dtype(dtype)
    mel = torch.from_numpy(synth.synth_inputs(82, (3, 6, 128), loc=-2.0)).to(DEV)
    f0 = torch.full((3, 6), 220.0, device=DEV)
    f0[1, 2:] = 0.0
    w = g.synthesize(mel, f0, 2.30259, seed=3, utt_ids=[8, 0, 5])
    for i, u in enumerate([8, 0, 5]):
        close(w[i:i + 1], g.synthesize(mel[i:i + 1].contiguous(), f0[i:i + 1].contiguous(), 2.30259, seed=3,
                                       utt_ids=[u]))
