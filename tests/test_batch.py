"""Mixed-length slide batches (config C5): LPT assignment and the data-parallel gather (CPU, gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gigapath import batch

SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]


def test_mixed_batch_sizes_are_c5():
    sizes = batch.mixed_batch_sizes()
    assert len(sizes) == 32 and min(sizes) >= 2000 and max(sizes) <= 100000
    assert sizes == batch.mixed_batch_sizes()          # seeded
    assert max(sizes) / min(sizes) > 10


def test_lpt_assignment_balances_and_covers():
    sizes = batch.mixed_batch_sizes()
    costs = [batch.slide_cost(n, SEGS, RATIOS) for n in sizes]
    for world in (1, 2, 4, 8):
        plan = batch.lpt_assign(costs, world)
        flat = sorted(i for r in plan for i in r)
        assert flat == list(range(len(sizes)))
        loads = [sum(costs[i] for i in r) for r in plan]
        # LPT bound: makespan <= 4/3 OPT; OPT >= max(mean load, largest job)
        assert max(loads) <= 4 / 3 * max(sum(costs) / world, max(costs)) + 1e-12
        for r in plan:                                      # each rank runs longest first
            assert [costs[i] for i in r] == sorted((costs[i] for i in r), reverse=True)


def test_pack_groups_respect_the_token_budget():
    sizes = batch.mixed_batch_sizes()
    order = list(range(len(sizes)))
    for budget in (50000, 200000, 1 << 21):
        groups = batch.pack_groups(sizes, order, budget)
        assert [i for g in groups for i in g] == order            # order kept, every slide once
        for g in groups:
            assert len(g) == 1 or sum(sizes[i] + 1 for i in g) <= budget
    assert len(batch.pack_groups(sizes, order, 1 << 21)) == 1       # the whole C5 batch fits one pack
    assert batch.pack_groups([10, 10], [0, 1], 5) == [[0], [1]]     # oversize slides stand alone


def test_cost_grows_superlinearly_with_tiles():
    c1, c2 = batch.slide_cost(10000, SEGS, RATIOS), batch.slide_cost(100000, SEGS, RATIOS)
    assert c2 > 10 * c1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, sizes, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gigapath import slide_encoder
        model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536)
        calls = []

        def fake_encode(x, c):          # stands in for the GPU forward: a deterministic per-slide value
            calls.append(int(x.shape[1]))
            v = torch.full((1, 768), float(x.shape[1])) + c.float().mean()
            return [v * (k + 1) for k in range(13)]

        slides = [(torch.zeros(n, 8), torch.ones(n, 2) * i) for i, n in enumerate(sizes)]
        out = batch.encode_slides(model, slides, all_layer_embed=True, encode_fn=fake_encode)
        dist.destroy_process_group()
        q.put((rank, (calls, [[o.numpy() for o in s] for s in out])))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_data_parallel_batch_gathers_every_slide_once():
    sizes = [3000, 50000, 2000, 12000, 7000, 90000, 4000]
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for v in res.values():
        assert not isinstance(v, str), v
    calls = sorted(n for r in range(world) for n in res[r][0])
    assert calls == sorted(sizes)                          # every slide encoded exactly once
    for r in range(world):
        outs = res[r][1]
        for i, n in enumerate(sizes):
            assert len(outs[i]) == 13
            for k in range(13):
                np.testing.assert_array_equal(outs[i][k], np.full((1, 768), (k + 1) * (n + i), dtype=np.float32))
