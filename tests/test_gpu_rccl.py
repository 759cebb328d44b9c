"""RCCL (torch's ``nccl`` backend on ROCm) through the multi-GPU gather path, on one GPU.

The N > 1 bench runs exactly this code: ``distributed_synthesize`` -> the ``all_reduce`` of
the mel-bin count and two ragged ``gather_to_root`` calls (prodiff_amd/pipeline.py).  At world
size 1 those collectives are normally skipped, so the ``force`` / ``collectives`` flags run
them anyway on a one-rank ``nccl`` group: device tensors through RCCL's gather and
all_gather, ragged shapes, several dtypes, and the whole pipeline with and without the
collectives.  Two ranks cannot share one GPU under RCCL, so world size 2 and 3 are covered on
CPU (tests/test_multirank_gloo.py).  The per-segment semantics being parallelised are the
reference's handler loop (handler/infer/handler.py:373-388).
"""
import socket

import pytest
import torch
import torch.distributed as dist

from prodiff_amd import synth
from prodiff_amd.pipeline import JobStreams, Synthesizer, distributed_synthesize, gather_to_root, phase_ms

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_group():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=DEV)
    assert dist.get_backend() == "nccl"
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.int64])
def test_gather_to_root_rccl_roundtrip(nccl_group, dtype):
    g = torch.Generator(device=DEV).manual_seed(3)
    for shape in [(5, 7), (0,), (3, 1, 129), (220_416,)]:
        t = (torch.randn(shape, device=DEV, generator=g) * 100).to(dtype)
        # planned shapes (the bench's path) and exchanged shapes (one all_gather)
        for shapes in ([shape], None):
            out = gather_to_root(t, shapes=shapes, force=True)
            assert len(out) == 1 and out[0].device == t.device
            assert out[0].dtype == dtype and tuple(out[0].shape) == shape
            assert torch.equal(out[0], t)
    with pytest.raises(ValueError):
        gather_to_root(torch.zeros(4, device=DEV), shapes=[(5,)], force=True)


def test_all_reduce_rccl(nccl_group):
    mt = torch.tensor([80], device=DEV)
    dist.all_reduce(mt, op=dist.ReduceOp.MAX)
    assert int(mt.item()) == 80


def test_distributed_synthesize_collectives_bf16(nccl_group):
    """The bf16 pipeline the bench runs, ragged lengths, with the RCCL collectives forced on:
    equal to the short-circuited run element for element (the collectives only move bytes)."""
    syn = Synthesizer.synthetic(DEV, seed=3, dtype="bf16", residual_layers=4)
    lengths = [9, 7, 9, 5]
    conds = [torch.from_numpy(synth.synth_inputs(90 + i, (T, 256))).to(DEV) for i, T in enumerate(lengths)]
    stats = {}
    mels, wavs = distributed_synthesize(syn, conds, seed=5, stats=stats, collectives=True)
    mref, wref = distributed_synthesize(syn, conds, seed=5)
    torch.cuda.synchronize()
    c, g = phase_ms(stats)          # HIP event marks: no synchronisation inside the job (r06)
    assert c > 0 and g >= 0 and stats["gather_ms"] == g
    for i, T in enumerate(lengths):
        assert tuple(mels[i].shape) == (T, 80) and tuple(wavs[i].shape) == (T * 256,)
        assert torch.equal(mels[i], mref[i]) and torch.equal(wavs[i], wref[i])


def test_distributed_synthesize_jobs_in_flight_rccl(nccl_group):
    """The N > 1 bench schedule at world size 1 with the collectives forced on: jobs on two
    JobStreams streams, each job's gathers issued from its own stream (torch's collective stream
    waits for it), so job i's gather overlaps job i + 1's compute.  Every job equals the same job
    run alone, element for element."""
    syn = Synthesizer.synthetic(DEV, seed=3, dtype="bf16", residual_layers=4)
    lengths = [9, 7, 9, 5, 12]
    conds = [torch.from_numpy(synth.synth_inputs(70 + i, (T, 256))).to(DEV) for i, T in enumerate(lengths)]
    syn.prepare()
    torch.cuda.synchronize()
    js = JobStreams(2, DEV)
    outs, sts = [], []
    for j in range(4):
        st = {}
        with js.next():
            outs.append(distributed_synthesize(syn, conds, seed=j, stats=st, collectives=True, max_frames=20))
        sts.append(st)
    torch.cuda.synchronize()
    for j, (mels, wavs) in enumerate(outs):
        mref, wref = distributed_synthesize(syn, conds, seed=j)
        torch.cuda.synchronize()
        for i in range(len(lengths)):
            assert torch.equal(mels[i], mref[i]) and torch.equal(wavs[i], wref[i])
        c, g = phase_ms(sts[j])
        assert c > 0 and g >= 0
