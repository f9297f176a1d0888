"""Multi-GPU path (config 4) on CPU: world_size-2 gloo ranks run bench.py's sharding and
aggregation helpers. Each rank owns distinct blocks (no data-path collective); the
only collectives are the timing barrier and the max-over-ranks reduction. The per-rank
CRC work is done by the oracle here (no GPU in this container) purely to exercise the
harness; the GPU numbers come from bench.py on the box."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out):
    import sys
    import time

    import torch
    import torch.distributed as dist

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "tests"))
    import bench
    from util import oracle_compute, oracle_verify, splitmix_bytes

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blocks, nbytes = 3, 1 << 20
    data = [splitmix_bytes(nbytes, bench.rank_seed(rank) + b) for b in range(blocks)]
    crcs = [oracle_compute(d, 512) for d in data]
    dist.barrier()
    t0 = time.perf_counter()
    bad = [oracle_verify(d, 512, c, False) for d, c in zip(data, crcs)]
    elapsed = time.perf_counter() - t0 + 0.01 * (rank + 1)  # make ranks differ
    dist.barrier()
    emax = bench.max_over_ranks(dist, elapsed, torch.device("cpu"))
    rate = bench.aggregate_rate(nbytes * blocks, world, emax)
    first = torch.tensor([int(data[0][:8].view(np.int64)[0])], dtype=torch.int64)
    firsts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(firsts, first)
    out[rank] = (elapsed, emax, rate, bad, [int(f.item()) for f in firsts])
    dist.destroy_process_group()


def test_two_rank_sharding_and_max_time():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rank_main, args=(world, port, out), nprocs=world, join=True)
    (e0, m0, r0, b0, f0), (e1, m1, r1, b1, f1) = out[0], out[1]
    assert m0 == m1 == pytest.approx(max(e0, e1))          # max over ranks, agreed by all
    assert r0 == pytest.approx(2 * 3 * (1 << 20) / m0 / 2**30)
    assert b0 == b1 == [-1, -1, -1]                          # every shard verifies clean
    assert f0 == f1 and f0[0] != f0[1]                       # ranks hold distinct blocks
