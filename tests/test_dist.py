"""CPU, multi-process (gloo, world_size 2): image sharding and the padded-detection all-gather used by bench.py
for N > 1 (the path's single exchange step)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import yolosod_import  # noqa: F401  (spawned workers re-import this module before conftest runs)
import conftest  # noqa: F401,E402  (sys.path: repo root + tests/golden for the workers)
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
        index = torch.randint(-1, 34000, (B, D), generator=g, dtype=torch.int32)
        g_out, g_cnt, g_idx = gather_detections(out, counts, index)
        ok = True
        for r in range(world):
            gr = torch.Generator().manual_seed(r)
            ro = torch.randn(B, D, 6, generator=gr)
            rc = torch.randint(0, D, (B,), generator=gr, dtype=torch.int32)
            ri = torch.randint(-1, 34000, (B, D), generator=gr, dtype=torch.int32)
            sl = slice(r * B, (r + 1) * B)
            ok &= torch.equal(g_out[sl], ro) and torch.equal(g_cnt[sl], rc) and torch.equal(g_idx[sl], ri)
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


def _pad_rows(rows, idx, D=300):
    out = torch.zeros((len(rows), D, 6))
    index = torch.full((len(rows), D), -1, dtype=torch.int32)
    for i, (r, a) in enumerate(zip(rows, idx)):
        out[i, :len(r)] = torch.from_numpy(r)
        index[i, :len(r)] = torch.from_numpy(a.astype(np.int32))
    return out, torch.tensor([len(r) for r in rows], dtype=torch.int32), index


def _flow_worker(rank, world, port, n_images, q):
    """The bench's N > 1 flow on CPU: shard_bounds -> rank-local predict (the oracle NMS on precomputed
    predictions stands in for the GPU predictor) -> gather_detections, via engine.predictor.sharded_predict."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import recipes
        from oracle.nms import non_max_suppression_ref
        from yolosod_amd.engine.predictor import sharded_predict
        preds = recipes.synthetic_predictions(11, n_images, 3000, 10, n_clusters=6)  # one global batch [n, 14, A]

        def local_predict(p):
            rows, idx = non_max_suppression_ref(p.numpy().copy(), 0.25, 0.3, max_det=300)
            return _pad_rows(rows, idx)

        g_out, g_cnt, g_idx = sharded_predict(local_predict, n_images,
                                              lambda lo, hi: torch.from_numpy(preds[lo:hi].copy()))
        rows, idx = non_max_suppression_ref(preds.copy(), 0.25, 0.3, max_det=300)  # unsharded, one process
        ref_out, ref_cnt, ref_idx = _pad_rows(rows, idx)
        ok = (g_out.shape == ref_out.shape and torch.equal(g_cnt, ref_cnt) and torch.equal(g_out, ref_out)
              and torch.equal(g_idx, ref_idx)  # kept anchor indices survive the exchange, in global image order
              and int(ref_cnt.min()) > 0 and len(set(ref_cnt.tolist())) > 1)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_images", [8, 7])
def test_sharded_flow_matches_single_process_gloo(n_images):
    """World size 2: the gathered detections and kept anchor indices equal the single-process ones row for row, in
    global image order (distinct per-image counts make a shard-order error visible); 7 images = uneven shards."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flow_worker, args=(r, 2, port, n_images, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


def test_packed_detections_roundtrip():
    """The exchange buffer (one int32 row per image: fp32 row bits | kept indices | count) unpacks bit for bit,
    including NaN / -0.0 / inf rows and index -1 padding."""
    from yolosod_amd.engine.predictor import pack_detections, unpack_detections
    g = torch.Generator().manual_seed(5)
    out = torch.randn(3, 300, 6, generator=g)
    out[0, 0, 0], out[1, 2, 3], out[2, 4, 5] = float("nan"), -0.0, float("inf")
    counts = torch.tensor([0, 17, 300], dtype=torch.int32)
    index = torch.randint(-1, 34000, (3, 300), generator=g, dtype=torch.int32)
    p = pack_detections(out, counts, index)
    assert p.dtype == torch.int32 and tuple(p.shape) == (3, 7 * 300 + 1) and p.is_contiguous()
    o2, c2, i2 = unpack_detections(p, 300, True)
    assert torch.equal(o2.view(torch.int32), out.view(torch.int32)) and torch.equal(c2, counts)
    assert torch.equal(i2, index)
    o3, c3 = unpack_detections(pack_detections(out, counts), 300, False)
    assert torch.equal(o3.view(torch.int32), out.view(torch.int32)) and torch.equal(c3, counts)


def _count_collectives_worker(rank, world, port, q):
    """gather_detections issues exactly one collective (a single exchange latency per step)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []
        orig = dist.all_gather_into_tensor

        def counting(*a, **k):
            calls.append(1)
            return orig(*a, **k)

        dist.all_gather_into_tensor = counting
        try:
            out = torch.full((2, 300, 6), float(rank))
            g_out, g_cnt, g_idx = gather_detections(out, torch.tensor([rank, 1], dtype=torch.int32),
                                                    torch.full((2, 300), rank, dtype=torch.int32))
        finally:
            dist.all_gather_into_tensor = orig
        ok = (len(calls) == 1 and g_out.shape == (4, 300, 6) and g_cnt.tolist() == [0, 1, 1, 1]
              and torch.equal(g_idx[:2], torch.zeros(2, 300, dtype=torch.int32))
              and torch.equal(g_out[2:], torch.ones(2, 300, 6)))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_gather_detections_is_one_collective_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_count_collectives_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=90) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


def test_seeded_images_are_slices_of_one_global_batch():
    from yolosod_amd.engine.predictor import seeded_images
    full = seeded_images(0, 6, 32)
    for w in (1, 2, 3, 4):
        parts = [seeded_images(*shard_bounds(6, r, w), 32) for r in range(w)]
        assert torch.equal(torch.cat(parts), full)
