"""N>1 path on CPU: utterance sharding (LPT), the ragged point-to-point gather to
the root and the un-permute back to input order, world sizes 2 and 3 over gloo
(the GPU run uses the same code over RCCL); and bench.py's own N-rank launcher
in its CPU dry-run mode."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from prodiff_amd.pipeline import distributed_synthesize, gather_to_root, length_groups, lpt_shards, ragged_batches

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOP = 4          # stub vocoder hop (keeps the test tensors small)
M = 3


def test_lpt_shards_balance_and_cover():
    lengths = [609, 286, 1917, 400, 512, 700, 1200, 333, 861, 861, 861, 90]
    for world in (1, 2, 3, 8):
        sh = lpt_shards(lengths, world)
        assert sorted(i for s in sh for i in s) == list(range(len(lengths)))
        loads = [sum(lengths[i] for i in s) for s in sh]
        # LPT bound: max load <= mean + max item
        assert max(loads) <= sum(lengths) / world + max(lengths)
    # equal lengths (C4): equal counts
    sh = lpt_shards([861] * 256, 8)
    assert all(len(s) == 32 for s in sh)
    # more ranks than utterances: empty shards are allowed
    sh = lpt_shards([5, 3], 4)
    assert sorted(len(s) for s in sh) == [0, 0, 1, 1]


def test_length_groups_exact():
    g = length_groups([5, 9, 3, 7, 7, 2], [0, 3, 4, 5])
    assert g == [(7, [3, 4]), (5, [0]), (2, [5])]


def test_ragged_batches_plan():
    """Longest first, padding within max_waste of the real frames, every utterance once."""
    lengths = [504, 522, 539, 720, 1197, 550, 550, 515, 1917, 286, 460, 579]
    plan = ragged_batches(lengths, range(len(lengths)), max_waste=0.15)
    assert sorted(i for _, ids in plan for i in ids) == list(range(len(lengths)))
    for T, ids in plan:
        assert T == max(lengths[i] for i in ids)
        assert T * len(ids) <= 1.15 * sum(lengths[i] for i in ids)
    assert plan[0] == (1917, [8]) and plan[1] == (1197, [4])
    assert [T for T, _ in plan] == sorted((T for T, _ in plan), reverse=True)
    # equal lengths: one dense batch; a frame cap splits it
    assert ragged_batches([861] * 8, range(8)) == [(861, list(range(8)))]
    assert [len(ids) for _, ids in ragged_batches([861] * 8, range(8), max_frames=861 * 3)] == [3, 3, 2]


def stub_synth(cond, seed, utt_ids=None, lens=None):
    """A deterministic stand-in for Synthesizer: per-utterance (independent of the batch
    it runs in), mel [B,T,M], wav [B,T*HOP].  Like the real samplers' draws it depends on
    (seed, utterance id), so the test sees that every batch gets the job's seed and the
    utterances' GLOBAL indices.  A ragged batch's zero padding is neutral (the real samplers
    read zero past each row's ``lens``)."""
    ids = torch.as_tensor(list(range(cond.shape[0])) if utt_ids is None else utt_ids, dtype=torch.float32)
    mel = cond[..., :M] * 2.0 + 1.0 + 1000.0 * ids[:, None, None] + seed
    wav = torch.repeat_interleave(cond[..., 0], HOP, dim=1) - cond[..., 1].sum(1, keepdim=True)
    return mel, wav


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _conds(lengths):
    g = torch.Generator().manual_seed(1234)
    return [torch.randn(T, 8, generator=g) for T in lengths]


def _worker(rank, world, port, q, lengths):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        conds = _conds(lengths)
        # only this rank's shard is materialized: the rest are (length, callable) stubs
        mine = set(lpt_shards(lengths, world)[rank])
        arg = [c if i in mine else (c.shape[0], None) for i, c in enumerate(conds)]
        mels, wavs = distributed_synthesize(stub_synth, arg, hop=HOP)
        # ragged gather with the shape exchange (no plan given)
        t = torch.full((rank + 1, 2 + rank), float(rank))
        g = gather_to_root(t)
        if rank == 0:
            q.put(([m.numpy() for m in mels], [w.numpy() for w in wavs], [x.numpy() for x in g]))
        else:
            assert mels is None and wavs is None and g is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,lengths", [(2, [5, 9, 3, 7, 7, 2]), (3, [4, 11, 6, 6]), (2, [6]),
                                          (2, [40, 41, 43, 44, 39, 12, 90])])
def test_distributed_synthesize_ragged(world, lengths):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, lengths)) for r in range(world)]
    for p in procs:
        p.start()
    mels, wavs, g = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # every utterance back in input order, equal to running it alone
    conds = _conds(lengths)
    assert len(mels) == len(lengths) == len(wavs)
    for i, c in enumerate(conds):
        em, ew = stub_synth(c[None], 0, utt_ids=[i])
        np.testing.assert_array_equal(mels[i], em[0].numpy())
        np.testing.assert_array_equal(wavs[i], ew[0].numpy())
        assert mels[i].shape == (lengths[i], M) and wavs[i].shape == (lengths[i] * HOP,)
    for r in range(world):
        np.testing.assert_array_equal(g[r], np.full((r + 1, 2 + r), float(r)))


@pytest.mark.parametrize("max_frames", [None, 20, 9])
def test_distributed_synthesize_max_frames_one_rank(max_frames):
    """One rank (no process group): a frame cap splits the shard into several batches (run side
    by side on streams on a GPU); every utterance still comes back in input order, equal to
    running it alone."""
    lengths = [5, 9, 3, 7, 7, 2, 9]
    conds = _conds(lengths)
    mels, wavs = distributed_synthesize(stub_synth, conds, hop=HOP, max_frames=max_frames)
    for i, c in enumerate(conds):
        em, ew = stub_synth(c[None], 0, utt_ids=[i])
        np.testing.assert_array_equal(mels[i].numpy(), em[0].numpy())
        np.testing.assert_array_equal(wavs[i].numpy(), ew[0].numpy())


def test_job_streams_cpu_is_a_no_op():
    """JobStreams on a CPU device (or depth 1) hands out null contexts: jobs run in order on the
    current stream, with the same outputs."""
    from prodiff_amd.pipeline import JobStreams
    lengths = [5, 9, 3]
    conds = _conds(lengths)
    for js in (JobStreams(2, "cpu"), JobStreams(1, None)):
        assert js.streams is None
        outs = []
        for j in range(3):
            with js.next():
                outs.append(distributed_synthesize(stub_synth, conds, seed=j, hop=HOP))
        for j, (mels, wavs) in enumerate(outs):
            for i, c in enumerate(conds):
                em, ew = stub_synth(c[None], j, utt_ids=[i])
                np.testing.assert_array_equal(mels[i].numpy(), em[0].numpy())


def test_bench_self_launches_n_ranks_dry_run():
    """`bench.py --gpus 2` without torchrun spawns 2 ranks itself (CPU dry run: gloo,
    stub synthesis, no GPU) and rank 0 reports n_gpus 2."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                          "--warmup", "1", "--dry-run"], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["dry_run"] is True
    assert d["config"]["global_batch"] == 2 * d["config"]["per_gpu_batch"]


def test_bench_jobs_in_flight_with_ranks_dry_run():
    """N > 1 ranks keep two jobs in flight by default (r06): each job's RCCL gather runs on the
    process group's collective stream beside the next job's compute.  The dry run (gloo, CPU)
    exercises the launcher, the schedule and the event-free phase marks; the line names the
    schedule and reports each rank's compute / gather split."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    for extra, depth in (([], 2), (["--overlap", "3"], 3), (["--overlap", "1"], 1)):
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                              "--warmup", "1", "--dry-run"] + extra, cwd=ROOT, env=env, capture_output=True,
                             text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-3000:]
        d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
        assert d["config"]["jobs_in_flight"] == depth
        if depth > 1:
            assert "RCCL gather" in d["config"]["schedule"] and "overlapping job i + 1" in d["config"]["schedule"]
        else:
            assert d["config"]["schedule"] is None
        ph = d["phases"]
        assert ph["compute_ms_per_step_slowest_rank"] >= ph["compute_ms_per_step_fastest_rank"] >= 0
        assert ph["gather_ms_per_step_max"] >= 0


def test_phase_marks_cpu():
    """distributed_synthesize's ``stats`` on a CPU device: host clock marks, resolved at once."""
    from prodiff_amd.pipeline import phase_ms
    lengths = [5, 9, 3]
    st = {}
    distributed_synthesize(stub_synth, _conds(lengths), hop=HOP, stats=st)
    c, g = phase_ms(st)
    assert c >= 0 and g == 0.0 and st["compute_ms"] == c and len(st["marks"]) == 3


class StubSvs:
    """Per-utterance dict inputs like SvsSynthesizer's (phoneme tokens + frame features),
    batched by the real SvsSynthesizer.collate; output independent of the batch."""
    from prodiff_amd.pipeline import SvsSynthesizer as _S
    collate = staticmethod(_S.collate)

    def __call__(self, batch, seed, utt_ids=None, lens=None):
        n = torch.tensor(batch["ntok"], dtype=torch.float32)[:, None]
        tok_sum = batch["txt_tokens"].float().sum(1, keepdim=True)        # pads are 0: neutral
        mel = batch["f0"][..., None].repeat(1, 1, M) + tok_sum[..., None] + n[..., None]
        wav = torch.repeat_interleave(batch["f0"], HOP, dim=1) - batch["voicing"].sum(1, keepdim=True)
        return mel, wav


def _svs_items(lengths, ntoks):
    g = torch.Generator().manual_seed(99)
    return [dict(txt_tokens=torch.randint(1, 50, (n,), generator=g), mel2ph=torch.zeros(T, dtype=torch.long),
                 f0=torch.rand(T, generator=g) * 500, voicing=torch.randn(T, generator=g),
                 spk_mix_embed=torch.randn(1, 8, generator=g))
            for T, n in zip(lengths, ntoks)]


def _svs_worker(rank, world, port, q, lengths, ntoks):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        items = _svs_items(lengths, ntoks)
        mels, wavs = distributed_synthesize(StubSvs(), [(T, (lambda it=it: it)) for T, it in zip(lengths, items)],
                                            hop=HOP)
        if rank == 0:
            q.put(([m.numpy() for m in mels], [w.numpy() for w in wavs]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_distributed_synthesize_svs_collate():
    """C5's path at world size 2: dict items with ragged phoneme counts (padded by
    SvsSynthesizer.collate) sharded and gathered back in input order."""
    lengths, ntoks = [6, 9, 6, 4, 9], [3, 5, 2, 4, 5]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_svs_worker, args=(r, 2, port, q, lengths, ntoks)) for r in range(2)]
    for p in procs:
        p.start()
    mels, wavs = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for i, it in enumerate(_svs_items(lengths, ntoks)):
        em, ew = StubSvs()(StubSvs.collate([it]), 0)
        np.testing.assert_allclose(mels[i], em[0].numpy(), rtol=0, atol=1e-4)
        np.testing.assert_allclose(wavs[i], ew[0].numpy(), rtol=0, atol=1e-4)
