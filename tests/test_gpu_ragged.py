"""Ragged batches (include/prodiff_hip.h `lens`): a padded batch of utterances of different
lengths equals each utterance synthesized alone -- the reference's one-segment-at-a-time
inference (handler/infer/handler.py:373-388: every segment is its own B=1 call).

Each test runs the batch with each row's length as ``lens`` and every utterance alone (B = 1,
T = its length), with the same seed and the utterance's id (on-device Philox draws are keyed by
(seed, utterance id, element), so the draws agree), and compares the utterance's frames /
samples.  Bar: |padded - alone| <= 1e-5 * max|alone|, fp32 and bf16.  The kernels
compute each row in the same order in both runs, so most cases are bit-identical; the bar
leaves room for the fp32 layer kernels' split choice, which depends on the batch's row count.
Plus the C5 path on the reference song's 30 segment lengths (tests/golden/ds_lengths.json).
"""
import json
import os

import numpy as np
import pytest
import torch

from prodiff_amd import FastDiff, GaussianDiffusion, WaveNet, synth
from prodiff_amd.nsf_hifigan import Generator
from prodiff_amd.schedules import fastdiff_infer_params, fastdiff_reverse_schedule, fastdiff_train_alpha
from tests.bf16_bar import assert_bf16_close

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
REL = 1e-5
SCHED = fastdiff_infer_params(fastdiff_reverse_schedule(4), fastdiff_train_alpha())
HERE = os.path.dirname(os.path.abspath(__file__))


def close(a, b, what):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err, ref = float(np.abs(a - b).max()), float(np.abs(b).max())
    print(f"{what}: max|d| = {err:.3e} (max|ref| {ref:.3f})")
    assert np.isfinite(a).all() and err <= REL * max(ref, 1e-30), (what, err, ref)


def prodiff(seed, dtype, M=80, cyc=1):
    net = WaveNet(M, 256, 20, 256, cyc)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in
                         synth.synth_params(synth.wavenet_param_shapes(M, 256, 20, 256), seed).items()})
    return GaussianDiffusion(M, net, timesteps=2, time_scale=1000, max_beta=40.0).to(DEV).set_compute_dtype(dtype)


def fastdiff(seed, dtype):
    m = FastDiff()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_params(synth.fastdiff_param_shapes(),
                                                                             seed).items()})
    return m.to(DEV).set_compute_dtype(dtype)


def padded(arrs, T):
    return torch.stack([torch.nn.functional.pad(a, (0, 0) * (a.dim() - 1) + (0, T - a.shape[0])) for a in arrs])


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("lengths", [[70, 130, 64, 97], [5, 33, 12], [200, 1]])
def test_prodiff_ragged_equals_alone(dtype, lengths):
    """ProDiff 2-iter sampler: the stack kernel (T >= 64), the one-layer kernels (T < 64) and
    the fp32 layer kernels, each utterance's frames against its own B=1 run."""
    gd = prodiff(0, dtype)
    g = torch.Generator(device=DEV).manual_seed(len(lengths))
    conds = [torch.randn(T, 256, device=DEV, generator=g) for T in lengths]
    T = max(lengths)
    ids = [10 + i for i in range(len(lengths))]
    mel = gd.sample(padded(conds, T), seed=7, utt_ids=ids, lens=lengths)
    for i, c in enumerate(conds):
        alone = gd.sample(c[None], seed=7, utt_ids=[ids[i]])
        close(mel[i, :lengths[i]].cpu(), alone[0].cpu(), f"ProDiff {dtype} utt {i} ({lengths[i]} of {T})")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_reflow_pitch_ragged_equals_alone(dtype):
    """The pitch predictor's rectified-flow sampler (dilation cycle 5: the one-layer kernels'
    dilated taps) on a ragged batch."""
    from prodiff_amd import RectifiedFlow
    M, lengths = 64, [40, 23, 57]
    net = WaveNet(M, 256, 20, 256, 5)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in
                         synth.synth_params(synth.wavenet_param_shapes(M, 256, 20, 256), 3).items()})
    rf = RectifiedFlow(M, net, time_scale=1000, spec_min=[-12], spec_max=[0]).to(DEV)
    net.set_compute_dtype(dtype)
    g = torch.Generator(device=DEV).manual_seed(3)
    conds = [torch.randn(T, 256, device=DEV, generator=g) for T in lengths]
    T = max(lengths)
    x = rf.sample(padded(conds, T), infer_step=4, seed=5, utt_ids=[0, 1, 2], lens=lengths)
    for i, c in enumerate(conds):
        alone = rf.sample(c[None], infer_step=4, seed=5, utt_ids=[i])
        close(x[i, :lengths[i]].cpu(), alone[0].cpu(), f"reflow {dtype} utt {i}")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("lengths", [[12, 7, 20], [3, 9]])
def test_fastdiff_ragged_equals_alone(dtype, lengths):
    """FastDiff 4-iter sampler: DBlocks, kernel predictor, the three LVC blocks (hop 8 / 64 /
    256, the upsample, first conv and final conv + update fused) on a ragged batch."""
    m = fastdiff(1, dtype)
    b, a, s, st = SCHED
    g = torch.Generator(device=DEV).manual_seed(11)
    mels = [torch.randn(T, 80, device=DEV, generator=g) - 5.0 for T in lengths]
    T = max(lengths)
    ids = [3 * i + 1 for i in range(len(lengths))]
    wav = m.sample(padded(mels, T), b, a, s, st, seed=9, utt_ids=ids, lens=lengths)[:, 0]
    for i, mel in enumerate(mels):
        alone = m.sample(mel[None], b, a, s, st, seed=9, utt_ids=[ids[i]])[0, 0]
        close(wav[i, :lengths[i] * 256].cpu(), alone.cpu(), f"FastDiff {dtype} utt {i} ({lengths[i]} of {T} frames)")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_nsf_ragged_equals_alone(dtype):
    """NSF-HiFiGAN at the SVS dims: source module, noise convs, windowed upsample, the ResBlock
    pair / windowed / small-channel convs and conv_post on a ragged batch."""
    h = dict(synth.NSF_DEFAULTS)
    gen = Generator(h)
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_params(synth.nsf_param_shapes(**h),
                                                                               4).items()})
    gen = gen.to(DEV).eval().set_compute_dtype(dtype)
    lengths = [20, 13, 31]
    rng = np.random.default_rng(5)
    mels = [torch.from_numpy(rng.normal(-2.0, 1.0, (T, 128)).astype(np.float32)).to(DEV) for T in lengths]
    f0s = [torch.from_numpy(np.where(rng.random(T) < 0.2, 0.0, rng.uniform(80, 900, T)).astype(np.float32)).to(DEV)
           for T in lengths]
    T = max(lengths)
    f0p = torch.stack([torch.nn.functional.pad(f, (0, T - f.shape[0])) for f in f0s])
    wav = gen.synthesize(padded(mels, T), f0p, 2.30259, seed=4, utt_ids=[0, 1, 2], lens=lengths)
    for i in range(len(lengths)):
        alone = gen.synthesize(mels[i][None], f0s[i][None], 2.30259, seed=4, utt_ids=[i])
        close(wav[i, :lengths[i] * 512].cpu(), alone[0].cpu(), f"NSF {dtype} utt {i}")


def test_pipeline_ragged_batch_equals_alone():
    """distributed_synthesize (one rank) plans a ragged batch for similar lengths; every
    utterance's mel and waveform equal its own B=1 Synthesizer call (bf16, the bench path)."""
    from prodiff_amd.pipeline import Synthesizer, distributed_synthesize, ragged_batches
    syn = Synthesizer.synthetic(DEV, seed=0, dtype="bf16")
    lengths = [72, 80, 69, 75]
    assert len(ragged_batches(lengths, range(4))) == 1          # one padded batch
    g = torch.Generator(device=DEV).manual_seed(2)
    conds = [torch.randn(T, 256, device=DEV, generator=g) for T in lengths]
    mels, wavs = distributed_synthesize(syn, conds, seed=13)
    for i, c in enumerate(conds):
        m1, w1 = syn(c[None], 13, utt_ids=[i])
        close(mels[i].cpu(), m1[0].cpu(), f"pipeline mel {i}")
        close(wavs[i].cpu(), w1[0].cpu(), f"pipeline wav {i}")


def ds_lengths():
    return json.load(open(os.path.join(HERE, "golden", "ds_lengths.json")))


def svs_items(lengths, phonemes, dev):
    from prodiff_amd.pipeline import SVS_VOCAB
    return [{k: torch.from_numpy(v).to(dev) for k, v in synth.synth_svs_utterance(200 + i, T, min(n, T), SVS_VOCAB).items()}
            for i, (T, n) in enumerate(zip(lengths, phonemes))]


def test_svs_ragged_equals_alone():
    """C5 (SvsSynthesizer, bf16): three of the song's segments in one padded batch (different
    frame and phoneme counts) against each segment alone."""
    from prodiff_amd.pipeline import SvsSynthesizer
    d = ds_lengths()
    pick = [0, 1, 2]                 # 504, 522, 539 frames
    lengths = [d["frames"][i] for i in pick]
    items = svs_items(lengths, [d["phonemes"][i] for i in pick], DEV)
    syn = SvsSynthesizer.synthetic(DEV, seed=0, dtype="bf16")
    mel, wav = syn(SvsSynthesizer.collate(items), seed=3, utt_ids=pick)
    for r, i in enumerate(pick):
        m1, w1 = syn(SvsSynthesizer.collate([items[r]]), seed=3, utt_ids=[i])
        close(mel[r, :lengths[r]].cpu(), m1[0].cpu(), f"SVS mel seg {i}")
        close(wav[r, :lengths[r] * 512].cpu(), w1[0].cpu(), f"SVS wav seg {i}")


def test_c5_ds_lengths_bf16_vs_fp32():
    """C5 on the reference song's real segment lengths (30 segments, 286 .. 1917 frames, the
    .ds file's own phoneme counts) through distributed_synthesize's ragged plan: bf16 vs the
    exact fp32 pipeline (same weights, same on-device draws) at the shared bf16 bar, on every
    third segment plus the longest and shortest (the fp32 NSF at 18k frames is slow)."""
    from prodiff_amd.pipeline import SvsSynthesizer, distributed_synthesize
    d = ds_lengths()
    assert len(d["frames"]) == 30 and min(d["frames"]) == 286 and max(d["frames"]) == 1917
    pick = sorted(set(range(0, 30, 3)) | {d["frames"].index(1917), d["frames"].index(286)})
    lengths = [d["frames"][i] for i in pick]
    items = svs_items(lengths, [d["phonemes"][i] for i in pick], DEV)
    outs = {}
    for dt in ("fp32", "bf16"):
        syn = SvsSynthesizer.synthetic(DEV, seed=0, dtype=dt)
        mels, wavs = distributed_synthesize(syn, [(T, (lambda it=it: it)) for T, it in zip(lengths, items)], seed=21,
                                            hop=512, device=DEV)
        outs[dt] = ([m.cpu().numpy() for m in mels], [w.cpu().numpy() for w in wavs])
        del syn
    for k, (m16, m32, w16, w32) in enumerate(zip(outs["bf16"][0], outs["fp32"][0], outs["bf16"][1], outs["fp32"][1])):
        assert m16.shape == (lengths[k], 128) and w16.shape == (lengths[k] * 512,)
        assert np.isfinite(w32).all() and np.abs(w32).max() <= 1.0
        assert_bf16_close(m16, m32, f"C5 .ds segment {pick[k]} mel ({lengths[k]} frames)")
        assert_bf16_close(w16, w32, f"C5 .ds segment {pick[k]} wav")


def test_lens_validation():
    """Host lengths outside [1, T] are refused before any launch; all-equal lengths take the
    dense path (lens = NULL)."""
    from prodiff_amd import _lib
    gd = prodiff(0, "fp32")
    cond = torch.zeros(2, 16, 256, device=DEV)
    with pytest.raises(_lib.HipError):
        gd.sample(cond, seed=1, lens=[16, 17])
    with pytest.raises(_lib.HipError):
        gd.sample(cond, seed=1, lens=[0, 5])
    assert _lib.lens([16, 16], 2, 16, DEV) is None
    a = gd.sample(cond, seed=1, lens=[16, 16])
    b = gd.sample(cond, seed=1)
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())


def test_pipeline_multibatch_streams_bitexact():
    """a shard that splits into several ragged batches (max_frames) runs them on side
    streams, and JobStreams keeps two such jobs in flight: every utterance's mel and waveform equal
    the same plan run on one stream (streams=1, one job at a time) bit for bit, over repeated jobs
    (the side streams and their workspaces are reused, not re-created), and each utterance equals
    its own B = 1 call within the ragged bar."""
    from prodiff_amd.pipeline import JobStreams, Synthesizer, distributed_synthesize, ragged_batches
    syn = Synthesizer.synthetic(DEV, seed=0, dtype="bf16")
    lengths = [72, 80, 69, 75, 140, 151, 66]
    assert len(ragged_batches(lengths, range(len(lengths)), max_frames=240)) >= 3
    g = torch.Generator(device=DEV).manual_seed(3)
    conds = [torch.randn(T, 256, device=DEV, generator=g) for T in lengths]
    seeds = [31, 32, 33]
    ref = [distributed_synthesize(syn, conds, seed=s, max_frames=240, streams=1) for s in seeds]
    torch.cuda.synchronize()
    nws = None
    js = JobStreams(2, DEV)
    for rep in range(2):
        got = []
        for s in seeds:
            with js.next():
                got.append(distributed_synthesize(syn, conds, seed=s, max_frames=240, streams=4))
        torch.cuda.synchronize()
        for (m0, w0), (m1, w1) in zip(ref, got):
            for i in range(len(lengths)):
                assert torch.equal(m1[i], m0[i]) and torch.equal(w1[i], w0[i]), (rep, i)
        n = len(syn.diffusion._ws.bufs) + len(syn.vocoder.model._ws.bufs)
        assert nws is None or n == nws, "workspaces grew over repeated jobs"
        nws = n
    for i in (0, 5):
        m1, w1 = syn(conds[i][None], seeds[0], utt_ids=[i])
        close(ref[0][0][i].cpu(), m1[0].cpu(), f"multibatch mel {i}")
        close(ref[0][1][i].cpu(), w1[0].cpu(), f"multibatch wav {i}")


def test_device_rows_cache_cross_stream():
    """the lens / utt_ids device cache fills a new entry with a non-blocking copy on
    the current stream; a hit on ANOTHER stream must wait for that copy.  Stream A is held busy,
    a new key is created there, then read on stream B at once: B sees the values."""
    from prodiff_amd import _lib
    a, b = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    vals = [int(v) for v in np.random.default_rng(7).integers(1, 1 << 20, 64)]
    with torch.cuda.stream(a):
        torch.cuda._sleep(200_000_000)            # ~0.1 s of GPU time ahead of the copy
        _lib.utt_ids(vals, len(vals), DEV)
    with torch.cuda.stream(b):
        d = _lib.utt_ids(vals, len(vals), DEV)    # cache hit on another stream
        out = d.clone()
    torch.cuda.synchronize()
    assert out.cpu().tolist() == vals
