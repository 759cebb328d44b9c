"""End-to-end mel -> waveform synthesis and utterance sharding across GPUs.

``Synthesizer`` chains the two fused samplers the way the reference chains
``ProDiffTeacher.forward(infer=True)`` (prodiff_teacher.py:148-168) and the
vocoder's ``spec2wav`` (component/vocoder/fastdiff.py:117-126); the ProDiff
output is already the time-major mel the FastDiff sampler consumes, so nothing
is transposed or copied between them.

Multi-GPU: utterances are independent, so a batch is split into
per-rank shards with no data-path collective (``lpt_shards``); the only
exchange is the final point-to-point gather of each shard's outputs to the root
rank (``gather_to_root``, RCCL over xGMI under the ``nccl`` backend).
"""
from __future__ import annotations

import contextlib
import time

import numpy as np
import torch
import torch.distributed as dist

from . import synth
from .fastdiff import FastDiff
from .prodiff import GaussianDiffusion, WaveNet
from .vocoder import FastDiff as FastDiffVocoder
from .nsf_hifigan import LOG10_TO_LN, Generator as NsfGenerator
from .teacher import ProDiffTeacher

# handler/base_config.yaml:195-211 (diffusion/decoder), modules/FastDiff/config/base.yaml:4-42
PRODIFF_DEFAULTS = dict(in_dims=80, hidden_size=256, residual_layers=20, residual_channels=256,
                        dilation_cycle_length=1, timesteps=2, max_beta=40.0)
HOP = 256
SAMPLE_RATE = 22050


class Synthesizer:
    """cond [B,T,H] -> (mel [B,T,M], wav [B,T*hop])."""

    def __init__(self, diffusion: GaussianDiffusion, vocoder: FastDiffVocoder):
        self.diffusion = diffusion
        self.vocoder = vocoder
        self.mel_bins = diffusion.mel_bins

    def prepare(self):
        """Pack every handle now (stream-ordered packing must finish before batches run on other
        streams: distributed_synthesize calls this, then synchronizes)."""
        self.diffusion.denoise_fn.handle()
        self.vocoder.model.handle()

    @staticmethod
    def collate(conds):
        """[T_i,H] conditions -> one [B, max T_i, H] batch, zero-padded (a ragged batch: the
        samplers take each row's length as ``lens``)."""
        return _pad_stack(conds)

    @classmethod
    def synthetic(cls, device, seed=0, dtype="fp32", **over):
        """Random-init weights of the reference architectures (no checkpoints offline)."""
        cfg = dict(PRODIFF_DEFAULTS, **over)
        net = WaveNet(cfg["in_dims"], cfg["hidden_size"], cfg["residual_layers"], cfg["residual_channels"],
                      cfg["dilation_cycle_length"])
        shapes = synth.wavenet_param_shapes(cfg["in_dims"], cfg["hidden_size"], cfg["residual_layers"],
                                            cfg["residual_channels"])
        net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_params(shapes, seed).items()})
        gd = GaussianDiffusion(cfg["in_dims"], net, timesteps=cfg["timesteps"], time_scale=1000,
                               max_beta=cfg["max_beta"]).to(device).eval()
        fd = FastDiff()
        fd.load_state_dict({k: torch.from_numpy(v)
                            for k, v in synth.synth_params(synth.fastdiff_param_shapes(), seed + 1).items()})
        fd.remove_weight_norm()
        gd.set_compute_dtype(dtype)
        fd.set_compute_dtype(dtype)
        voc = FastDiffVocoder({"hop_size": HOP}, model=fd.to(device), reverse_step=4, device=device)
        return cls(gd, voc)

    @torch.no_grad()
    def __call__(self, cond, seed=None, utt_ids=None, lens=None):
        """Random draws are keyed by (seed, utterance id): row i of the batch is utterance
        ``utt_ids[i]`` (default i), and its output does not depend on the other rows.  ``lens``:
        a ragged batch (each row's frames, default all T): row i's first lens[i] frames (and
        lens[i] * hop samples) equal the utterance synthesized alone."""
        g = None if seed is None else 2 * seed
        mel = self.diffusion.sample(cond, seed=g, utt_ids=utt_ids, lens=lens)
        wav = self.vocoder.spec2wav_batch(mel, seed=None if seed is None else g + 1, utt_ids=utt_ids, lens=lens)
        return mel, wav


# SVS path (handler/base_config.yaml: 128 mels, 44.1 kHz, hop 512, teacher timesteps 4,
# NSF-HiFiGAN vocoder :216-219)
SVS_TEACHER = dict(audio_num_mel_bins=128, hidden_size=256, enc_layers=4, enc_ffn_kernel_size=9, dropout=0.1,
                   num_heads=2, num_spk=4, languages=["zh", "jp"], use_spk_id=True, use_lang_id=True,
                   use_dur_embed=True, use_voicing_embed=True, use_breath_embed=True, use_gender_id=False,
                   residual_layers=20, residual_channels=256, dilation_cycle_length=1, timesteps=4,
                   timescale=1000, schedule_type="vpsde", max_beta=40.0, spec_min=[-12], spec_max=[0])
SVS_HOP = 512
SVS_SAMPLE_RATE = 44100
SVS_VOCAB = 64

TOKEN_KEYS = ("txt_tokens", "lang_seq")
FRAME_KEYS = ("mel2ph", "f0", "voicing", "breath")


class SvsSynthesizer:
    """SVS segment inputs -> (mel [B,T,128], wav [B,T*512]): ProDiffTeacher.forward(infer=True)
    (handler/infer/handler.py:133-149 -> prodiff_teacher.py:148-168) then the NSF-HiFiGAN
    vocoder's spec2wav_torch (component/vocoder/nsf_hifigan.py:29-56), all on the GPU."""

    def __init__(self, teacher: ProDiffTeacher, generator: NsfGenerator, infer_step=4):
        self.teacher, self.generator, self.infer_step = teacher, generator, infer_step
        self.diffusion = teacher.diffusion
        self.mel_bins = self.diffusion.mel_bins

    def prepare(self):
        """Pack every handle now (see Synthesizer.prepare)."""
        self.teacher.cond_handle()
        self.diffusion.denoise_fn.handle()
        self.generator.handle()

    @classmethod
    def synthetic(cls, device, seed=0, dtype="fp32", **over):
        hp = dict(SVS_TEACHER, **over)
        t = ProDiffTeacher(SVS_VOCAB, hp)
        cp = synth.synth_cond_params(synth.cond_param_shapes(SVS_VOCAB, num_langs=len(hp["languages"]) + 1,
                                                             **{k: v for k, v in hp.items() if k != "num_langs"}),
                                     seed)
        wn = synth.synth_params(synth.wavenet_param_shapes(hp["audio_num_mel_bins"], hp["hidden_size"],
                                                           hp["residual_layers"], hp["residual_channels"]), seed + 1)
        sd = {k: torch.from_numpy(v) for k, v in cp.items()}
        sd.update({"diffusion.denoise_fn." + k: torch.from_numpy(v) for k, v in wn.items()})
        t.load_state_dict(sd, strict=False)
        h = dict(synth.NSF_DEFAULTS)
        g = NsfGenerator(h)
        g.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_params(synth.nsf_param_shapes(**h),
                                                                                  seed + 2).items()})
        t = t.to(device).eval().set_compute_dtype(dtype)
        g = g.to(device).eval().set_compute_dtype(dtype)
        return cls(t, g)

    @staticmethod
    def collate(items):
        """Per-utterance dicts -> one batch: token fields padded with 0 (PAD) to the longest, the
        frame fields (mel2ph, f0, voicing, breath) padded with 0 to the longest segment (mel2ph 0 =
        a padding frame, prodiff_teacher.py:118-146: a ragged batch, see ``lens``); ``ntok`` keeps
        each utterance's token count, ``nframes`` its frame count."""
        out = {"ntok": [int(it["txt_tokens"].shape[0]) for it in items],
               "nframes": [int(it["mel2ph"].shape[0]) for it in items]}
        for k in items[0]:
            vs = [it[k] for it in items]
            out[k] = _pad_stack(vs) if (k in TOKEN_KEYS or k in FRAME_KEYS) else torch.stack(vs)
        if "spk_mix_embed" in out:            # [B, 1, H]
            out["spk_mix_embed"] = out["spk_mix_embed"].reshape(len(items), -1, out["spk_mix_embed"].shape[-1])
        return out

    @torch.no_grad()
    def condition(self, batch):
        """cond [B,T,H] in one encoder pass over the token-padded batch.  Token padding is not
        neutral in the reference's batched FFT encoder (its FFN conv reads LayerNorm(0) = beta on
        padded rows, common_layers.py:668-669) and the reference encodes every segment alone
        (B=1), so each row's phoneme count goes to the encoder as ``txt_lens``: the FFN conv reads
        zero past it and every row equals its segment encoded alone (r05; rounds 2-4 ran one
        encoder pass per distinct phoneme count)."""
        b = {k: v for k, v in batch.items() if k not in ("ntok", "nframes")}
        B, Tt = int(b["txt_tokens"].shape[0]), int(b["txt_tokens"].shape[1])
        ntok = batch.get("ntok") or [Tt] * B
        n = max(ntok)
        tok = b.pop("txt_tokens")[:, :n]
        if "lang_seq" in b:
            b["lang_seq"] = b["lang_seq"][:, :n]
        return self.teacher.forward_condition(tok, b.pop("mel2ph"), b.pop("f0"),
                                              txt_lens=None if all(k == n for k in ntok) else ntok, **b)

    @torch.no_grad()
    def __call__(self, batch, seed=None, utt_ids=None, lens=None):
        """``lens`` (default: the batch's ``nframes``): each segment's frames in a ragged batch."""
        g = None if seed is None else 3 * seed
        if lens is None:
            lens = batch.get("nframes")
        cond = self.condition(batch)
        mel = self.diffusion.sample(cond, infer_step=self.infer_step, seed=g, utt_ids=utt_ids, lens=lens)
        wav = self.generator.synthesize(mel, batch["f0"], LOG10_TO_LN, seed=None if seed is None else g + 1,
                                        utt_ids=utt_ids, lens=lens)
        return mel, wav


def lpt_shards(lengths, world):
    """Longest-processing-time partition of utterances over ranks (sorted by length,
    each to the currently lightest rank).  Returns a list of index lists."""
    order = np.argsort(-np.asarray(lengths), kind="stable")
    load = np.zeros(world, np.int64)
    shards = [[] for _ in range(world)]
    for i in order:
        r = int(np.argmin(load))
        shards[r].append(int(i))
        load[r] += int(lengths[i])
    return [sorted(s) for s in shards]


def _numel(shape):
    return int(np.prod(shape)) if len(shape) else 1


def gather_to_root(t, root=0, shapes=None, force=False):
    """Point-to-point gather of per-rank tensors of DIFFERENT shapes to `root`
    (torch's NCCL backend -- RCCL on ROCm -- implements gather as sends to the
    root; gloo on CPU).  Every rank passes a tensor of the same ndim and dtype.

    The per-rank shapes are exchanged with one small all_gather unless the caller
    already knows them (``shapes``: one tuple per rank, e.g. from the shard plan,
    which saves that round trip).  Each rank's tensor is flattened and padded to
    the largest size, gathered, and trimmed on the root.  Returns the list of
    per-rank tensors (rank order) on the root, None elsewhere.  ``force`` runs the
    collective even at world size 1 (tests drive RCCL on a one-GPU box that way)."""
    if not dist.is_initialized() or (dist.get_world_size() == 1 and not force):
        return [t]
    world, rank = dist.get_world_size(), dist.get_rank()
    t = t.contiguous()
    if shapes is None:
        nd = t.dim()
        mine = torch.zeros(1 + nd, dtype=torch.int64, device=t.device)
        mine[0] = nd
        if nd:
            mine[1:] = torch.tensor(t.shape, dtype=torch.int64)
        allv = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        shapes = []
        for v in allv:
            v = v.cpu().tolist()
            if v[0] != nd:
                raise ValueError("gather_to_root: ranks passed tensors of different ndim")
            shapes.append(tuple(v[1:]))
    shapes = [tuple(int(d) for d in s) for s in shapes]
    if tuple(t.shape) != shapes[rank]:
        raise ValueError(f"gather_to_root: rank {rank} tensor {tuple(t.shape)} != planned {shapes[rank]}")
    n = max(_numel(s) for s in shapes)
    flat = t.reshape(-1)
    if flat.numel() < n:
        flat = torch.cat([flat, flat.new_zeros(n - flat.numel())])
    if rank == root:
        bufs = [torch.empty(n, dtype=t.dtype, device=t.device) for _ in range(world)]
        dist.gather(flat, gather_list=bufs, dst=root)
        return [b[:_numel(s)].reshape(s) for b, s in zip(bufs, shapes)]
    dist.gather(flat, dst=root)
    return None


def ragged_batches(lengths, idx, max_waste=0.15, max_frames=None):
    """Batches of utterances `idx` for one rank, as [(T_pad, [indices])] longest first.

    The samplers take ragged batches (``lens``: every conv reads zero past each row's own end, so
    a padded batch reproduces the reference's one-segment-at-a-time results,
    handler/infer/handler.py:373-388); padding only costs compute.  Utterances are sorted by
    length and a batch grows while its padded frames stay within (1 + max_waste) of its real
    frames (and, if given, its padded frames within max_frames).  Equal lengths give one batch."""
    order = sorted((int(i) for i in idx), key=lambda i: (-int(lengths[i]), i))
    out = []
    for i in order:
        L = int(lengths[i])
        if out:
            T, ids, tot = out[-1]
            n = len(ids) + 1
            if T * n <= (1.0 + max_waste) * (tot + L) and (max_frames is None or T * n <= max_frames):
                ids.append(i)
                out[-1] = (T, ids, tot + L)
                continue
        out.append((L, [i], L))
    return [(T, ids) for T, ids, _ in out]


def length_groups(lengths, idx):
    """Utterances `idx` grouped by exact length, longest first (the dense batches of rounds 1-4;
    kept for callers that want them -- distributed_synthesize uses ``ragged_batches``)."""
    groups = {}
    for i in idx:
        groups.setdefault(int(lengths[i]), []).append(int(i))
    return sorted(groups.items(), key=lambda kv: -kv[0])


def _pad_stack(items):
    """[T_i, ...] tensors -> one [B, max T_i, ...] tensor, zero past each row's T_i.  Equal lengths: one
    stack; otherwise one zero fill and a copy per row (F.pad per item cost a fill and a copy each, plus the
    stack: r06 trace, 8 copies per C3 job ahead of its first launch)."""
    T = max(int(c.shape[0]) for c in items)
    if all(int(c.shape[0]) == T for c in items):
        return torch.stack(list(items))
    out = items[0].new_zeros((len(items), T) + tuple(items[0].shape[1:]))
    for r, c in enumerate(items):
        out[r, :int(c.shape[0])] = c
    return out


def _default_collate(items):
    return _pad_stack(items)


class JobStreams:
    """Keeps up to ``depth`` synthesis jobs in flight on their own HIP streams (a serving loop's
    double buffering): ``with js.next(): distributed_synthesize(...)`` runs job i on stream
    i % depth, so one job's low-occupancy launches -- the ProDiff WaveNet stack puts one 64-frame
    window on a CU, 157 of 256 CUs at 8 x 861 frames; the NSF stages' small grids -- overlap the
    previous job's vocoder (bench.py --overlap: C3 -6% per job with 2 in flight, C5 -15% with 3, on
    one MI355X; profiles/r05_ab/job_overlap_ab.txt, job_overlap_depth_ab.txt).  The outputs of a job live on its stream: read them
    after ``torch.cuda.synchronize()`` or a wait on that stream.  depth 1 or a CPU device: the
    current stream, no-op."""

    def __init__(self, depth=2, device=None):
        self.depth = max(1, int(depth))
        dev = torch.device(device) if device is not None else None
        self.streams = None
        if self.depth > 1 and dev is not None and dev.type == "cuda":
            cur = torch.cuda.current_stream(dev)
            self.streams = [torch.cuda.Stream(dev) for _ in range(self.depth)]
            for s in self.streams:
                s.wait_stream(cur)      # inputs made on the current stream are ready
        self.i = 0

    def next(self):
        if self.streams is None:
            return contextlib.nullcontext()
        s = self.streams[self.i % self.depth]
        self.i += 1
        # inputs the caller made on its own stream since the last job are ready for this one (the
        # jobs themselves run on the side streams, so this does not order one job after another)
        s.wait_stream(torch.cuda.current_stream(s.device))
        return torch.cuda.stream(s)


_SIDE_STREAMS = {}


def _side_streams(dev, cur, n):
    """``n`` side streams for ragged batches issued from stream ``cur``, created once and reused
    by every later call (new streams per call came round-robin from torch's pool, and
    every module keeps one grow-only workspace per stream, so a serving loop accumulated up to ~32
    full-size workspaces).  Keyed by the issuing stream, so jobs in flight on different
    ``JobStreams`` streams keep separate side streams (and workspaces) and still overlap."""
    lst = _SIDE_STREAMS.setdefault((str(dev), cur.cuda_stream), [])
    while len(lst) < n:
        lst.append(torch.cuda.Stream(dev))
    return lst[:n]


def _set_marks(stats, m0, m1, m2):
    stats["marks"] = (m0, m1, m2)
    stats.pop("compute_ms", None)
    stats.pop("gather_ms", None)
    if not isinstance(m0, torch.cuda.Event):       # host clock readings: resolved already
        phase_ms(stats)


def phase_ms(stats):
    """``compute_ms`` / ``gather_ms`` of a ``distributed_synthesize`` job from the marks it left in
    ``stats`` (HIP events: the caller synchronises first -- this waits for the last mark anyway).
    Returns (compute_ms, gather_ms) and stores them in ``stats``."""
    if "compute_ms" not in stats:
        m0, m1, m2 = stats["marks"]
        if isinstance(m0, torch.cuda.Event):
            m2.synchronize()
            c, g = m0.elapsed_time(m1), m1.elapsed_time(m2)
        else:
            c, g = (m1 - m0) * 1e3, (m2 - m1) * 1e3
        stats["compute_ms"], stats["gather_ms"] = float(c), float(g)
    return stats["compute_ms"], stats["gather_ms"]


def distributed_synthesize(synth_fn, conds, root=0, seed=0, hop=HOP, device=None, stats=None,
                           collectives=False, max_waste=0.15, streams=4, max_frames=None):
    """Synthesize utterances sharded over the ranks of the default process group
    (SURVEY §8(e)); the reference runs them one by one, B=1 per segment
    (handler/infer/handler.py:373-388).

    synth_fn(cond [B,T,H], seed, utt_ids, lens) -> (mel [B,T,M], wav [B,T*hop]): one rank's
      batched synthesis (a ``Synthesizer``; an ``SvsSynthesizer`` takes per-utterance input
      dicts).  Its ``collate`` pads a batch's inputs to the longest (default: zero-pad [T_i,H]
      conditions), ``lens`` gives each row's frames (a ragged batch), ``mel_bins`` the mel
      channels.  Every batch gets the same ``seed`` and the global indices of its utterances as
      ``utt_ids``, and the samplers key their random draws by (seed, utterance id): an
      utterance's mel and waveform are the same at any world size, in any batch position, and
      padded or alone.
    conds: list over ALL utterances (same order on every rank) of [T_i,H] tensors
      on this rank's device, or (T_i, callable returning one) pairs, so that only
      this rank's shard is materialized.
    Utterances are LPT-partitioned by length (``lpt_shards``); each rank runs its shard in
    ragged batches of similar lengths (``ragged_batches``, padding <= max_waste), trims each
    utterance's outputs to its length, and one ragged gather per output kind brings them to the
    root, which un-permutes them.  The plan is deterministic and the mel channels known
    (``synth_fn.mel_bins``), so nothing but the outputs crosses ranks.  Returns on the root the
    lists [mel_i [T_i,M]], [wav_i [T_i*hop]] in input order; (None, None) elsewhere.
    ``stats`` (a dict, optional) receives where this rank's job went -- its shard's synthesis and
    the collectives after it -- as three marks (HIP events on the job's stream on a GPU, host clock
    readings on a CPU) with no synchronisation inside the job; ``phase_ms(stats)`` turns them into
    ``compute_ms`` / ``gather_ms`` once the caller has synchronised (r06: two
    ``torch.cuda.synchronize()`` per job had serialised every N > 1 bench step).
    ``collectives=True`` runs the ragged gathers even at world size 1 (otherwise
    short-circuited), so the N > 1 code path can be exercised on one GPU.
    ``streams``: a shard of several ragged batches runs them side by side on up to this many HIP
    streams (each with its own workspaces, ``_lib.Workspace``): a long utterance alone in its batch
    fills a fraction of the GPU (the WaveNet stack puts 32 frames on a CU), so it overlaps the
    others instead of running after them.  1 = one after the other on the current stream.
    ``max_frames``: cap on a batch's padded frames (``ragged_batches``); a shard split into several
    batches runs them on the streams side by side, so one batch's low-occupancy launches (the
    WaveNet stack puts 44 frames on a CU) overlap another's."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    lengths = [int(c.shape[0]) if torch.is_tensor(c) else int(c[0]) for c in conds]
    shards = lpt_shards(lengths, world)
    mel_parts, wav_parts = [], []
    M = getattr(synth_fn, "mel_bins", None)
    collate = getattr(synth_fn, "collate", _default_collate)
    plans = [ragged_batches(lengths, s, max_waste, max_frames) for s in shards]

    dev = device
    if dev is None:
        dev = next((c.device for c in conds if torch.is_tensor(c)), torch.device("cpu"))
    dev = torch.device(dev)

    def mark():
        if stats is None:
            return None
        if dev.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream(dev))
            return ev
        return time.perf_counter()
    plan = plans[rank]
    side = None
    if streams > 1 and len(plan) > 1 and dev.type == "cuda":
        if getattr(synth_fn, "prepare", None):
            synth_fn.prepare()
        cur = torch.cuda.current_stream(dev)
        side = _side_streams(dev, cur, min(streams, len(plan)))
        for s in side:
            s.wait_stream(cur)          # the inputs and the packed handles are ready

    m0 = mark()
    outs = []
    for k, (T, idx) in enumerate(plan):
        lens = [lengths[i] for i in idx]
        ctx = torch.cuda.stream(side[k % len(side)]) if side else contextlib.nullcontext()
        with ctx:
            cb = collate([conds[i] if torch.is_tensor(conds[i]) else conds[i][1]() for i in idx])
            if all(n == T for n in lens):
                mel, wav = synth_fn(cb, seed, utt_ids=idx)
            else:
                mel, wav = synth_fn(cb, seed, utt_ids=idx, lens=lens)
        outs.append((mel, wav, lens, T))
    if side:
        for s in side:
            cur.wait_stream(s)
        for mel, wav, _, _ in outs:     # made on a side stream, read (and freed) on the current one
            mel.record_stream(cur)
            wav.record_stream(cur)
    if world == 1 and not (collectives and dist.is_initialized()):
        # one rank, no gather: each utterance's outputs are views of its batch (no flatten / cat
        # copies of the whole job on the device)
        mels, wavs = [None] * len(lengths), [None] * len(lengths)
        for (mel, wav, lens, T), (_, idx) in zip(outs, plan):
            for r, (i, n) in enumerate(zip(idx, lens)):
                mels[i] = mel[r, :n]
                wavs[i] = wav[r, :n * hop]
        if stats is not None:
            m1 = mark()
            _set_marks(stats, m0, m1, m1)
        return mels, wavs
    for mel, wav, lens, T in outs:
        M = mel.shape[-1]
        if all(n == T for n in lens):
            mel_parts.append(mel.reshape(-1))
            wav_parts.append(wav.reshape(-1))
        else:
            for r, n in enumerate(lens):       # trim each row to its utterance
                mel_parts.append(mel[r, :n].reshape(-1))
                wav_parts.append(wav[r, :n * hop])
    if not mel_parts:     # an empty shard still takes part in the collectives
        mel_flat = torch.zeros(0, device=dev)
        wav_flat = torch.zeros(0, device=dev)
    else:
        mel_flat, wav_flat = torch.cat(mel_parts), torch.cat(wav_parts)
    m1 = mark()
    if world == 1 and not (collectives and dist.is_initialized()):
        mels_all, wavs_all = [mel_flat], [wav_flat]
    else:
        if getattr(synth_fn, "mel_bins", None) is None:   # (the same answer on every rank)
            # a synth_fn without `mel_bins`: every rank with a non-empty shard knows it (one small
            # all_reduce; the library's synthesizers declare it, so the bench never pays this)
            mt = torch.tensor([0 if not mel_parts else M], device=mel_flat.device)
            dist.all_reduce(mt, op=dist.ReduceOp.MAX)
            M = int(mt.item())
        mel_shapes = [(sum(lengths[i] for i in s) * M,) for s in shards]
        wav_shapes = [(sum(lengths[i] for i in s) * hop,) for s in shards]
        mels_all = gather_to_root(mel_flat, root, mel_shapes, force=collectives)
        wavs_all = gather_to_root(wav_flat, root, wav_shapes, force=collectives)
    if stats is not None:
        # (the gathers' completion: torch's process group makes the current stream wait for its
        # collective stream, so an event recorded here ends after them)
        _set_marks(stats, m0, m1, mark())
    if rank != root:
        return None, None
    mels, wavs = [None] * len(lengths), [None] * len(lengths)
    for r in range(world):
        mo, wo = 0, 0
        for T, idx in plans[r]:
            for i in idx:
                n = lengths[i]
                mels[i] = mels_all[r][mo:mo + n * M].reshape(n, M)
                wavs[i] = wavs_all[r][wo:wo + n * hop]
                mo += n * M
                wo += n * hop
    return mels, wavs
