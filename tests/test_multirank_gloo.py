"""N>1 path on CPU: utterance sharding (LPT) and the point-to-point gather to the
root, world_size 2 over gloo (the GPU run uses the same code over RCCL)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from prodiff_amd.pipeline import gather_to_root, lpt_shards


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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lengths = [5, 9, 3, 7, 7, 2]
    shards = lpt_shards(lengths, world)
    mine = shards[rank]
    # each rank "synthesises" its utterances: here a deterministic function of the index
    out = torch.zeros(len(shards[0]) + 2, 4)
    for j, i in enumerate(mine):
        out[j] = float(i) + torch.arange(4, dtype=torch.float32) / 10
    g = gather_to_root(out)
    if rank == 0:
        q.put((shards, g.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_to_root_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    shards, g = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert g.shape[0] == 2
    for r, s in enumerate(shards):
        for j, i in enumerate(s):
            np.testing.assert_allclose(g[r, j], i + np.arange(4) / 10, rtol=0, atol=1e-6)
