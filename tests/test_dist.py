"""Multi-process (world_size 2, gloo, CPU) tests of the scene-sharded path: dataset/GS.py:54-67 chunking,
train.py:170-176 metric reduce, and the bench's max-over-ranks timing."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from splatformer_amd import dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_scene_chunk_matches_reference_rule():
    # GS.py:57-67: chunk = n // world; the last rank takes the remainder
    assert dist.scene_chunk(9, 0, 2) == [0, 1, 2, 3]
    assert dist.scene_chunk(9, 1, 2) == [4, 5, 6, 7, 8]
    assert dist.scene_chunk(3, 0, 4) == [] and dist.scene_chunk(3, 3, 4) == [0, 1, 2]
    for n in range(0, 20):
        for w in (1, 2, 3, 8):
            got = sum((dist.scene_chunk(n, r, w) for r in range(w)), [])
            assert got == list(range(n))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        assert dist.init("gloo")
        r, w = dist.world()
        mine = dist.scene_chunk(7, r, w)
        # per-scene "psnr" = 10 + scene index, 3 images per scene
        psnr_sum = torch.tensor(float(sum(3 * (10 + i) for i in mine)), dtype=torch.float64)
        out = dist.reduce_metrics({"psnr": psnr_sum}, 3 * len(mine), len(mine))
        t = dist.max_over_ranks(1.5 + r)
        # DDP bucket average and SyncBN sums
        flat = torch.arange(6, dtype=torch.float32) * (r + 1)
        dist.allreduce_mean_(flat)
        sums = torch.tensor([1.0 + r, 10.0 * r, float(100 + r)], dtype=torch.float64)
        dist.allreduce_sum_(sums)
        dist.barrier()
        q.put((r, mine, out, t, flat.tolist(), sums.tolist()))
    finally:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()


def test_two_rank_reduce_and_timing():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, m0, o0, t0, f0, s0), (r1, m1, o1, t1, f1, s1) = res
    assert f0 == f1 == [1.5 * i for i in range(6)]
    assert s0 == s1 == [3.0, 10.0, 201.0]
    assert m0 + m1 == list(range(7))
    assert o1 == {}
    assert o0["num_images"] == 21 and o0["num_scenes"] == 7
    assert o0["psnr"] == pytest.approx(sum(10 + i for i in range(7)) / 7)
    assert t0 == t1 == 2.5
