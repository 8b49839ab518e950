"""CPU, multi-process (gloo, world_size 2): image sharding and the padded-detection all-gather used by bench.py
for N > 1 (the path's single exchange step)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import yolosod_import  # noqa: F401  (spawned workers re-import this module before conftest runs)
from yolosod_amd.engine.predictor import gather_detections, shard_bounds


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 32, 33, 256):
        for w in (1, 2, 3, 8):
            seen = []
            for r in range(w):
                lo, hi = shard_bounds(n, r, w)
                seen.extend(range(lo, hi))
            assert seen == list(range(n))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B, D = 4, 300
        g = torch.Generator().manual_seed(rank)
        out = torch.randn(B, D, 6, generator=g)
        counts = torch.randint(0, D, (B,), generator=g, dtype=torch.int32)
        g_out, g_cnt = gather_detections(out, counts)
        ok = True
        for r in range(world):
            gr = torch.Generator().manual_seed(r)
            ro = torch.randn(B, D, 6, generator=gr)
            rc = torch.randint(0, D, (B,), generator=gr, dtype=torch.int32)
            ok &= torch.equal(g_out[r * B:(r + 1) * B], ro) and torch.equal(g_cnt[r * B:(r + 1) * B], rc)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_detections_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=90) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(r, True) for r in range(world)]
