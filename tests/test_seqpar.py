"""Sequence-parallel bookkeeping and exchange (CPU: planner logic + gloo world_size 2..4).

The GPU half (the sharded forward against the single-device forward) is in test_gpu_seqpar.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as orc
from gigapath import seqpar

H, D = 16, 48
E, F = H * D, 4 * H * D
DEFAULT = ([1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16])
WSI250K = ([1024, 4870, 23170, 110217, 524288], [1, 2, 4, 8, 16])
SMALL_MISALIGNED = ([32, 60, 90, 123, 1000], [1, 2, 4, 8, 16])


def sparsify_ref(qkv, L, segs, ratios):
    """numpy restatement of gp_dilated_sparsify over all tokens: [L, 2C] per branch."""
    out = []
    p = np.arange(L)
    for sl, r in zip(segs, ratios):
        s = min(sl, L)
        C = (H // r) * D
        j = (p % s) % r
        cols = j[:, None] * C + np.arange(C)[None, :]
        k = np.take_along_axis(qkv[:, E:2 * E], cols, 1)
        v = np.take_along_axis(qkv[:, 2 * E:], cols, 1)
        out.append(np.concatenate([k, v], 1))
    return out


@pytest.mark.parametrize("L,world,sched", [
    (1025, 2, DEFAULT), (16385, 3, DEFAULT), (70001, 8, DEFAULT), (256001, 8, DEFAULT),
    (250001, 8, WSI250K), (1001, 5, SMALL_MISALIGNED), (3000, 7, SMALL_MISALIGNED), (37, 4, SMALL_MISALIGNED),
])
def test_plan_covers_every_row_the_merge_reads(L, world, sched):
    segs, ratios = sched
    plan = seqpar.ShardPlan(L, world, segs, ratios, H, D, F)
    # shards tile [0, L) contiguously
    assert [a for a, _ in plan.bounds[1:]] == [e for _, e in plan.bounds[:-1]]
    assert plan.bounds[0][0] == 0 and plan.bounds[-1][1] == L
    assert all(e > a for a, e in plan.bounds)
    for v in range(world):
        a, e = plan.bounds[v]
        for b, (sl, r) in enumerate(zip(segs, ratios)):
            geo = orc.branch_geometry(L, sl, r, H)
            s, m, nseg = geo["s"], geo["m"], geo["nseg"]
            g = m * r
            # every dense slot of the window maps to a sparse row (n, i, j) -- the merge reads it
            p = np.arange(a, e)
            n, t = p // g, p % g
            i, j = t // r, t % r
            assert (n < nseg).all()
            gather_tok = n * s + i * r + j
            valid = (i * r + j < s) & (gather_tok < L)
            # its query is local or in the q halo
            assert (gather_tok[valid] >= a - plan.q_halo[v]).all() and (gather_tok[valid] < e).all()
            # all keys of its segment are in the rank's K/V (receive) range
            lo, hi = plan.need[v][b]
            seg_lo, seg_hi = n * s, np.minimum((n + 1) * s, L)
            assert lo <= seg_lo.min() and hi >= seg_hi.max()
            # the all-to-all chunks from ranks 0..W-1, in rank order, tile [lo, hi) exactly
            chunks = [plan.chunk(w, v, b) for w in range(world)]
            got = [c for c in chunks if c[1] > c[0]]
            assert got[0][0] == lo and got[-1][1] == hi
            assert all(x[1] == y[0] for x, y in zip(got[:-1], got[1:]))
            assert sum(plan.recv_splits(v, b)) == hi - lo
        # every received range is owned by its sender
        for b, w, lo, hi in plan.recvs(v):
            wa, we = plan.bounds[w]
            assert wa <= lo < hi <= we
    # send and receive split tables agree pairwise
    for w in range(world):
        for v in range(world):
            for b in range(len(segs)):
                assert plan.send_splits(w, b)[v] == plan.recv_splits(v, b)[w]
            if v == w:
                continue
            hs = [(lo, hi) for dst, lo, hi in plan.halo_sends(w) if dst == v]
            hr = [(lo, hi) for src, lo, hi in plan.halo_recvs(v) if src == w]
            assert hs == hr


def test_balanced_bounds_equalise_modelled_cost():
    L = 256001
    cost = seqpar.token_cost(L, *DEFAULT, H, D, F)
    bounds = seqpar.balanced_bounds(cost, 8)
    per = np.array([cost[a:e].sum() for a, e in bounds])
    assert per.max() / per.mean() < 1.01
    # the last b=3 segment (70,638 real tokens) is cheaper per token than the first
    assert bounds[-1][1] - bounds[-1][0] > bounds[0][1] - bounds[0][0]


def test_shard_cuts_snap_to_segments_when_the_exchange_pays():
    """C4 on 8 ranks: the cuts land on multiples of 32,768, so the 32,768- and 1,024-token branches
    exchange nothing and the busiest rank pair carries ~27.5 MB per layer instead of ~49 MB.  The round-6
    planner (simulated launches, seqpar.LaunchModel) keeps round 5's plan unless its model scores another
    SP_PLAN_MARGIN better."""
    L = 256001
    plan = seqpar.ShardPlan(L, 8, *DEFAULT, H, D, F)
    assert all(a % 32768 == 0 for a, _ in plan.bounds)
    for b in (0, 2):                                       # s = 1024 and s = 32768
        assert not [x for x in plan.recvs(3) if x[0] == b]
    bal = seqpar.ShardPlan(L, 8, *DEFAULT, H, D, F,
                           bounds=seqpar.balanced_bounds(seqpar.token_cost(L, *DEFAULT, H, D, F), 8))
    assert plan.max_pair_bytes() < 0.6 * bal.max_pair_bytes()
    for n, w in [(70001, 8), (100001, 3), (16385, 4), (256001, 2), (256001, 4)]:
        p = seqpar.ShardPlan(n, w, *DEFAULT, H, D, F)
        assert not p.cheap_in_a
        os.environ["GIGAPATH_SP_PLANNER"] = "cost"
        try:
            r5 = seqpar.ShardPlan(n, w, *DEFAULT, H, D, F)
        finally:
            del os.environ["GIGAPATH_SP_PLANNER"]

        def sim(pl):
            return max(pl.model_rank(r)["total"] for r in range(w))
        # round 5's plan, or one the model scores at least SP_PLAN_MARGIN better
        assert p.bounds == r5.bounds or sim(p) < sim(r5) * (1 - seqpar.SP_PLAN_MARGIN), (n, w)


def test_round5_cost_planner_still_available(monkeypatch):
    """GIGAPATH_SP_PLANNER=cost: round 5's choice -- modelled token cost of the busiest rank + the busiest
    link's bytes, never worse than the cost-balanced cuts by that measure."""
    monkeypatch.setenv("GIGAPATH_SP_PLANNER", "cost")
    for n, w in [(70001, 2), (70001, 8), (100001, 3), (16385, 4), (256001, 2)]:
        p = seqpar.ShardPlan(n, w, *DEFAULT, H, D, F)
        assert not p.cheap_in_a
        cost = seqpar.token_cost(n, *DEFAULT, H, D, F)
        q = seqpar.ShardPlan(n, w, *DEFAULT, H, D, F, bounds=seqpar.balanced_bounds(cost, w))

        def model(pl):
            return (max(cost[a:e].sum() for a, e in pl.bounds) + pl.max_pair_bytes() / seqpar.LINK_BYTES_PER_S)
        assert model(p) <= model(q) * (1 + 1e-9), (n, w)


def test_branches_without_transfers():
    """Under 32,768-aligned cuts (C4, 8 ranks) the 1,024- and 32,768-token branches have no
    cross-rank rows: no sparsify rows, no all-to-all, no K/V buffer (the attention reads qkv)."""
    plan = seqpar.ShardPlan(256001, 8, *DEFAULT, H, D, F)
    assert plan.no_xfer == [True, False, True, False, False]
    ws = seqpar.ShardWorkspace(plan, 3, "cpu", F)
    for b in (0, 2):
        assert ws.send[b].shape[0] == 0 and ws.kvs[b].shape[0] == 0
        lo, hi = plan.need[3][b]
        assert plan.bounds[3][0] <= lo and hi <= plan.bounds[3][1]
    bal = seqpar.ShardPlan(256001, 8, *DEFAULT, H, D, F,
                           bounds=seqpar.balanced_bounds(seqpar.token_cost(256001, *DEFAULT, H, D, F), 8))
    assert not any(bal.no_xfer)


def test_key_parts_split_only_underfilled_launches(monkeypatch):
    """GIGAPATH_SP_KEY_PARTS=rule (round 5's item-count rule): at 256k / 8 ranks the long branches' launch
    (~384-480 8-wave items for 768 slots) splits both branches' keys in two; the filled launches (and every
    launch at W = 2) keep whole branches; the merge's entries never exceed GP_MAX_BRANCHES."""
    monkeypatch.setenv("GIGAPATH_SP_KEY_PARTS", "rule")
    segs, ratios = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]
    for W in (2, 4, 8):
        plan = seqpar.ShardPlan(256001, W, segs, ratios, 16, 48, 3072)
        for r in range(W):
            eng = seqpar.SeqParallelEngine(plan, r, None)
            kp = eng.parts()
            assert sum(kp) <= 8
            a, e = plan.bounds[r]
            for br in eng._launches():
                items = sum(seqpar.launch_items(plan.geo[b], 16, a, e) for b in br)
                under = items < 3 * 256 and max(plan.geo[b].m for b in br) >= seqpar.KEY_PARTS_MIN_KEYS
                assert all(kp[b] == 1 for b in br) == (not under), (W, r, br, items, kp)
            if W == 8 and not plan.cheap_in_a:
                assert kp == [1, 1, 1, 2, 2], (r, kp)
            if W == 2:
                assert kp == [1] * 5
    eng.key_parts = {4: 3}
    assert eng.parts() == [1, 1, 1, 1, 3]


def test_key_parts_chosen_by_simulated_launches():
    """Round 6: a launch's long branches (>= KEY_PARTS_MIN_KEYS keys per item) split into P parts only when
    the simulated launch (seqpar.LaunchModel) plus the merge's extra entries beats the whole launch by 2 %,
    and no other P in 2..4 within the merge's 8 entries would have been chosen instead; short branches stay
    whole.  At 256k / 8 ranks the 32,768-token ranks split the 185,363-token branch in two (round 5's
    measured best; (3, 2) was slower, profiles/r05_kp3_*)."""
    segs, ratios = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]
    m = seqpar.LAUNCH_MODEL
    for L, W in ((256001, 2), (256001, 4), (256001, 8), (70001, 8)):
        plan = seqpar.ShardPlan(L, W, segs, ratios, 16, 48, 3072)
        for r in range(W):
            eng = seqpar.SeqParallelEngine(plan, r, None)
            kp = eng.parts()
            assert sum(kp) <= 8
            a, e = plan.bounds[r]
            done = [1] * 5
            for br in eng._launches():
                long_ = [b for b in br if plan.geo[b].m >= seqpar.KEY_PARTS_MIN_KEYS]
                assert all(kp[b] == 1 for b in br if b not in long_)
                assert len({kp[b] for b in long_}) <= 1
                whole = plan.launch_time(r, br, done)
                P = kp[long_[0]] if long_ else 1
                if P > 1:
                    t = plan.launch_time(r, br, kp) + len(long_) * (P - 1) * (e - a) * m.merge_entry_s
                    assert t < 0.98 * whole, (L, W, r, br, kp)
                for b in long_:
                    done[b] = P
            if L == 256001 and W == 8 and e - a == 32768 and not plan.cheap_in_a:
                assert kp[3] == 2, (r, kp)


def test_key_parts_stay_off_for_short_launches():
    """A small sharded forward (5,000 tiles on 2 ranks, the GPU parity case) has under-filled launches of
    short items only: no key parts, so the merge keeps its 5-entry specialisation and the shards keep the
    single-device path's arithmetic (advice r05)."""
    segs, ratios = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]
    plan = seqpar.ShardPlan(5001, 2, segs, ratios, 16, 48, 3072)
    for r in range(2):
        assert seqpar.SeqParallelEngine(plan, r, None).parts() == [1] * 5


def test_attn_launch_params_match_the_kernel_build():
    """The planner reads the attention launch constants from the built library (gp_attn_launch_params),
    not from copies: 256-query 8-wave items, three resident workgroups per CU, the 4-wave switch below three
    items per CU, at most 64 key parts -- the values the key-part rule and its measurements assume."""
    from gigapath import _hip
    assert _hip.attn_launch_params() == {"qblk": 256, "wg_per_cu": 3, "small_per_cu": 3, "max_key_parts": 64}
    # the LDS-DMA layout condition key parts need (attn_fwd_impl's kv_desc_ok) on the engine's two layouts
    assert _hip.kv_layout_fast(0, 2 * 768, 3 * 768, 16)          # dense qkv rows
    assert _hip.kv_layout_fast(0, 2 * 48, 2 * 48, 16)            # exchanged rows, C = 48
    assert not _hip.kv_layout_fast(2 * 768, 0, 3 * 768, 16)      # v before k
    assert not _hip.kv_layout_fast(0, 2 * 768, 768, 16)          # stride shorter than v's offset + a head


def test_exchange_volume_is_sparse():
    """At 256k / 8 ranks each rank receives far less than the dense K/V (786 MB per layer)."""
    plan = seqpar.ShardPlan(256001, 8, *DEFAULT, H, D, F)
    dense = 256001 * 2 * E * 2
    vols = [plan.exchange_bytes(v) for v in range(8)]
    assert max(vols) < 0.45 * dense, [v / 1e6 for v in vols]
    assert plan.q_halo[0] == 0


def test_misaligned_schedule_has_q_halo():
    plan = seqpar.ShardPlan(256001, 8, *WSI250K, H, D, F)
    assert max(plan.q_halo) > 0            # 23170 % 4 != 0, 110217 % 8 != 0: dense slots shift right


# ------------------------------------------------------------------ gloo exchange
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _exchange_worker(rank, world, port, L, segs, ratios, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        rng = np.random.default_rng(7)
        qkv = rng.standard_normal((L, 3 * E)).astype(np.float32)      # same "global" projection on every rank
        ref = sparsify_ref(qkv, L, segs, ratios)
        plan = seqpar.ShardPlan(L, world, segs, ratios, H, D, F)
        ws = seqpar.ShardWorkspace(plan, rank, "cpu", F)
        a, e = plan.bounds[rank]
        for t in ws.kvs:
            t.fill_(float("nan"))
        ws.qkv_ext.fill_(float("nan"))
        ws.qkv.copy_(torch.from_numpy(qkv[a:e]).to(ws.qkv.dtype))
        for b in range(len(segs)):                       # this rank's sparsified rows, where sparsify writes
            if plan.no_xfer[b]:                          # them (its own rows of the receive buffer and, if
                continue                                 # the peers' chunks reach past those, a send buffer)
            for lo, hi, buf, off in ws.sparsify_dests(b):
                buf[off:off + hi - lo] = torch.from_numpy(ref[b][lo:hi]).to(buf.dtype)
        eng = seqpar.SeqParallelEngine(plan, rank, seqpar.Exchange())
        seqpar.Exchange.wait(eng.exchange(ws, list(range(len(segs))), halo=True))
        for b in range(len(segs)):
            if plan.no_xfer[b]:                 # read from qkv by the attention, never exchanged
                assert ws.kvs[b].shape[0] == 0
                continue
            lo, hi = plan.need[rank][b]
            base = ws.kv_base[b]
            got = ws.kvs[b][lo - base:hi - base].float().numpy()
            want = torch.from_numpy(ref[b][lo:hi]).to(ws.kvs[b].dtype).float().numpy()
            assert np.array_equal(got, want), ("branch", b)
        if ws.hq:
            got = ws.qkv_ext[:ws.hq].float().numpy()
            want = torch.from_numpy(qkv[a - ws.hq:a]).to(ws.qkv.dtype).float().numpy()
            assert np.array_equal(got, want)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as ex:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(ex)))


@pytest.mark.parametrize("world,L,sched", [(2, 3001, DEFAULT), (3, 5000, SMALL_MISALIGNED),
                                           (4, 2000, WSI250K)])
def test_gloo_exchange_delivers_every_needed_row(world, L, sched):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, L, sched[0], sched[1], q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


# ------------------------------------------------------------------ sharded forward, CPU stand-in kernels
SP_SCHED = ([64, 130, 250, 333, 1000], [1, 2, 4, 8, 16])      # multi-segment, misaligned (q halos)


def _sp_model(segs, ratios):
    from gigapath import slide_encoder
    cfg = orc.arch_config("gigapath_slide_enc12l768d")
    cfg["segment_length"], cfg["dilated_ratio"] = list(segs), list(ratios)
    m = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}, strict=True)
    m.encoder.args.segment_length, m.encoder.args.dilated_ratio = list(segs), list(ratios)
    return m.eval(), cfg


def _sp_forward_worker(rank, world, port, N, gp, q, local_first=False, monitor=False, key_parts=None):
    try:
        import sp_emulator
        sp_emulator.install()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(2)
        seqpar.SeqParallelEngine.local_first = local_first      # class defaults for the engine built below
        seqpar.SeqParallelEngine.key_parts = key_parts
        model, _ = _sp_model(*SP_SCHED)
        model.global_pool = gp
        model.enable_sequence_parallel()
        mon = seqpar.ExchangeMonitor(bound_s=300, rank=rank) if monitor else None
        model._sp.set_monitor(mon)
        x, coords = orc.synthetic_slide(N)
        with torch.no_grad():
            out = torch.stack(model._forward_sp(torch.from_numpy(x), torch.from_numpy(coords), True)).numpy()
            last = model._forward_sp(torch.from_numpy(x), torch.from_numpy(coords), False)[0].numpy()
        dist.destroy_process_group()
        q.put((rank, (out, last, mon.summary(len(model.encoder.layers)) if mon else None,
                      [(r["layer"], r["phase"]) for r in mon.records] if mon else None)))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world,N,gp,local_first,key_parts", [(2, 600, False, False, None), (3, 700, True, False, None),
                                                              (2, 600, False, True, None),
                                                              (2, 600, False, True, {1: 2, 4: 3})])
def test_sharded_forward_matches_oracle_with_cpu_kernels(world, N, gp, local_first, key_parts):
    """LongNetViT._forward_sp end to end over gloo with every HIP call replaced by an
    address-checking CPU stand-in (tests/sp_emulator.py): shard bounds, K/V and q-halo
    exchange, query windows, window merge, readouts, all-reduce/broadcast.  key_parts: branch 1's two key
    tiles in two parts, branch 4's one tile in three (two empty parts: o = 0, lse = -inf)."""
    monitor = world == 2 and not local_first and not key_parts
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sp_forward_worker, args=(r, world, port, N, gp, q, local_first, monitor, key_parts))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for v in res.values():
        assert not isinstance(v, str), v
    _, cfg = _sp_model(*SP_SCHED)
    W = {k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}
    x, coords = orc.synthetic_slide(N)
    ref = torch.stack(orc.slide_encoder_forward(W, x, coords, cfg, all_layer_embed=True, global_pool=gp)).numpy()
    ref_last = orc.slide_encoder_forward(W, x, coords, cfg, global_pool=gp)[0].numpy()
    for r in range(world):
        out, last, summ, recs = res[r]
        if monitor:      # every layer's three exchange phases timed, in both forwards
            nl = cfg["depth"]
            assert recs == [(li, ph) for _ in range(2) for li in range(nl) for ph in ("A", "B1", "B2")]
            assert summ["forwards"] == 2 and summ["kind"] == ["host_exchange"]
            assert set(summ["ms_per_layer_by_phase"]) == {"A", "B1", "B2"} and summ["ms_per_layer"] > 0
        for got, want in ((out, ref), (last, ref_last)):
            for idx in np.ndindex(*got.shape[:-1]):
                g_, w_ = got[idx].astype(np.float64), want[idx].astype(np.float64)
                rel = np.abs(g_ - w_).max() / np.abs(w_).max()
                cos = (g_ * w_).sum() / np.sqrt((g_ * g_).sum() * (w_ * w_).sum())
                assert rel <= 2e-2 and cos >= 0.9995, (r, idx, rel, cos)


_WATCHDOG_CHILD = """
import sys, time
sys.path.insert(0, %r)
from gigapath import seqpar
m = seqpar.ExchangeMonitor(bound_s=0.5, rank=5)
m.arm("layer 7 phase B1 branches [3, 4] peers [4, 6]")
time.sleep(30)
print("not reached")
"""


def test_exchange_watchdog_names_the_stuck_collective_and_exits():
    """A wait that outlives the bound ends the process (exit 3) and says which layer / phase /
    branches / peers it was stuck on -- instead of hanging until the launcher's timeout."""
    import subprocess
    import sys as _sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "prov-gigapath-replication_amd")
    p = subprocess.run([_sys.executable, "-c", _WATCHDOG_CHILD % pkg], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "rank 5" in p.stderr and "layer 7 phase B1 branches [3, 4] peers [4, 6]" in p.stderr
    assert "not reached" not in p.stdout
