"""Mixed-length batch (C5) on the GPU: every slide's output equals its own B = 1 forward, one
slide at a time and varlen-packed (one launch per op for all slides)."""
import numpy as np
import pytest
import torch

import oracle as orc
from gigapath import _hip, batch, runtime

SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]


def _model(**kw):
    from gigapath import slide_encoder
    cfg = orc.arch_config("gigapath_slide_enc12l768d")
    model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536, **kw)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}, strict=True)
    return model.cuda().eval()


def _slides(sizes, seed):
    out = []
    for i, n in enumerate(sizes):
        x, c = orc.synthetic_slide(n, seed_x=seed + i, seed_c=seed + 50 + i)
        out.append((torch.from_numpy(x[0]).cuda(), torch.from_numpy(c[0]).cuda()))
    return out


def _close(got, ref, tol=2e-2):
    g, r = got.float().flatten(), ref.float().flatten()
    rel = float((g - r).abs().max() / r.abs().max())
    cos = float((g @ r) / (g.norm() * r.norm()))
    assert rel <= tol and cos >= 0.9999, (rel, cos)

pytestmark = pytest.mark.gpu


def test_mixed_batch_equals_individual_forwards():
    from gigapath import slide_encoder
    cfg = orc.arch_config("gigapath_slide_enc12l768d")
    model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}, strict=True)
    model = model.cuda().eval()
    slides = []
    for i, n in enumerate([300, 2500, 1200, 5000]):
        x, c = orc.synthetic_slide(n, seed_x=10 + i, seed_c=20 + i)
        slides.append((torch.from_numpy(x[0]).cuda(), torch.from_numpy(c[0]).cuda()))
    out = batch.encode_slides(model, slides, all_layer_embed=True, packed=False)
    with torch.no_grad():
        for (x, c), got in zip(slides, out):
            ref = model(x[None], c[None], all_layer_embed=True)
            assert len(got) == len(ref) == 13
            for g, r in zip(got, ref):
                assert torch.equal(g, r)


def test_mixed_batch_graph_replays_bit_exact():
    """use_hip_graphs: slides replayed as captured graphs (two slides sharing a shape, so one graph
    is replayed twice per batch) -- every output equals the eager B = 1 forward."""
    from gigapath import slide_encoder
    cfg = orc.arch_config("gigapath_slide_enc12l768d")
    model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}, strict=True)
    model = model.cuda().eval()
    sizes = [400, 2600, 1300, 400, 5100, 900]
    slides = []
    for i, n in enumerate(sizes):
        x, c = orc.synthetic_slide(n, seed_x=30 + i, seed_c=40 + i)
        slides.append((torch.from_numpy(x[0]).cuda(), torch.from_numpy(c[0]).cuda()))
    with torch.no_grad():
        ref = [torch.stack(model(x[None], c[None], all_layer_embed=True)) for x, c in slides]
    model.use_hip_graphs = True
    model.graph_min_uses = 1
    for _ in range(2):                                    # capture pass, then pure replays
        out = batch.encode_slides(model, slides, all_layer_embed=True, packed=False)
        torch.cuda.synchronize()
        for got, want in zip(out, ref):
            assert torch.equal(torch.stack(got), want)
    assert len(model._graphs) == 5


@pytest.mark.parametrize("fmt", ["bf16", "bf16_overflow", "fp16_overflow"])
def test_varlen_attention_and_merge_bit_exact_per_slide(fmt):
    """One varlen launch over packed slides == the single-slide kernels on each slide's rows,
    bit for bit (same per-item math; each slide keeps its own segment schedule).  *_overflow: the
    first slide's head-0 scores spike 200 log2 units above the rest.  bf16: the no-max fast kernel's
    row sum overflows, the rows are flagged and the fixup pass recomputes them exactly; it rewrites only
    flagged rows, so the other slides' rows -- whose items may share a fixup block with the flagged
    ones -- keep the fast kernel's bits and still equal their own launches.  fp16: the exact running-
    max kernel (no fixup) on the same input."""
    H, D, E = 16, 48, 768
    Ls = [1025, 2897, 700, 6001, 12000]         # 6001 / 12000: several segments of branches 0-1
    T = sum(Ls)
    g = torch.Generator(device="cuda").manual_seed(5)
    qkv = torch.randn(T, 3 * E, device="cuda", generator=g)
    qkv[:, :E] *= 0.35
    if fmt.endswith("_overflow"):
        qkv[:1025, :D] = 0.0
        qkv[:1025, 0] = 8.0
        qkv[:1025, E:E + D] = 0.0
        qkv[150, E] = 25.0
    qkv = qkv.to(torch.float16 if fmt.startswith("fp16") else torch.bfloat16)
    vs = runtime.VarlenScratch(torch.device("cuda"), Ls, H, D, SEGS, RATIOS, qkv)
    for t in vs.outs + vs.lses:
        t.zero_()
    _hip.dilated_attn_fwd_varlen(vs.plan, True)
    ln_w = torch.rand(E, device="cuda") + 0.5
    ln_b = torch.randn(E, device="cuda") * 0.1
    merged = torch.empty(T, E, dtype=qkv.dtype, device="cuda")
    _hip.branch_merge_ln_varlen(vs.plan, ln_w, ln_b, 1e-5, merged)
    o_off = [0] * len(SEGS)
    l_off = [0] * len(SEGS)
    t0 = 0
    for L in Ls:
        rows = qkv[t0:t0 + L]
        sc = runtime.AttentionScratch(torch.device("cuda"), 1, L, H, D, SEGS, RATIOS, qkv.dtype)
        for t in sc.outs + sc.lses:
            t.zero_()
        _hip.dilated_attn_fwd(rows, rows[:, E:], rows[:, 2 * E:], 3 * E, 1, L, H, D, SEGS, RATIOS, sc.outs, sc.lses,
                              0.0, True)
        ref = torch.empty(L, E, dtype=qkv.dtype, device="cuda")
        _hip.branch_merge_ln(sc.outs, sc.lses, SEGS, RATIOS, 1, L, H, D, ln_w, ln_b, 1e-5, ref)
        torch.cuda.synchronize()
        for b in range(len(SEGS)):
            no, nl = sc.outs[b].numel(), sc.lses[b].numel()
            assert torch.equal(vs.outs[b][o_off[b]:o_off[b] + no], sc.outs[b]), (L, b)
            assert torch.equal(vs.lses[b][l_off[b]:l_off[b] + nl], sc.lses[b]), (L, b)
            o_off[b] += no
            l_off[b] += nl
        assert torch.equal(merged[t0:t0 + L], ref), L
        t0 += L
    assert o_off == vs.plan.o_elems and l_off == vs.plan.lse_elems


@pytest.mark.parametrize("global_pool", [False, True])
def test_forward_packed_matches_individual_forwards(global_pool):
    """Packed forward of 4 slides == each slide's own B = 1 forward (GEMM row-count rounding
    aside), 13 layer embeddings and the default single output."""
    model = _model(global_pool=global_pool)
    slides = _slides([300, 2500, 1200, 6100], seed=70)
    with torch.no_grad():
        for ale in (True, False):
            got = model.forward_packed(slides, all_layer_embed=ale)
            for (x, c), outs in zip(slides, got):
                ref = model(x[None], c[None], all_layer_embed=ale)
                assert len(outs) == len(ref) == (13 if ale else 1)
                for o, r in zip(outs, ref):
                    assert o.shape == r.shape == (1, 768)
                    _close(o, r)


def test_forward_packed_vs_oracle():
    cfg = orc.arch_config("gigapath_slide_enc12l768d")
    W = orc.make_weights(cfg, seed=0)
    model = _model()
    sizes = [300, 1100]
    slides = _slides(sizes, seed=90)
    with torch.no_grad():
        got = model.forward_packed(slides, all_layer_embed=True)
    Wt = {k: torch.from_numpy(v) for k, v in W.items()}
    for (x, c), outs in zip(slides, got):
        ref = torch.stack(orc.slide_encoder_forward(Wt, x[None].cpu().numpy(), c[None].cpu().numpy(), cfg,
                                                    all_layer_embed=True))
        _close(torch.stack(outs).cpu(), ref)


def test_packed_graph_replay_and_encode_slides():
    """use_hip_graphs: the packed forward as one graph replay equals the eager packed forward bit
    for bit; encode_slides (packed by default) returns every slide's outputs in input order."""
    model = _model()
    slides = _slides([400, 2600, 1300, 400, 5100], seed=110)
    with torch.no_grad():
        eager = model.forward_packed(slides, all_layer_embed=True)
        model.use_hip_graphs = True
        for _ in range(2):
            rep = model.forward_packed(slides, all_layer_embed=True)
            torch.cuda.synchronize()
            for a, b in zip(rep, eager):
                assert torch.equal(torch.stack(a), torch.stack(b))
        out = batch.encode_slides(model, slides, all_layer_embed=True)
        for (x, c), o in zip(slides, out):
            ref = model(x[None], c[None], all_layer_embed=True)
            _close(torch.stack(o), torch.stack(ref))


def test_forward_packed_edge_cases():
    """One-tile slides (L = 2: every branch a single short segment), a single slide, slides
    straddling the 1024-token segment edge, and the empty list."""
    model = _model()
    assert model.forward_packed([], all_layer_embed=True) == []
    slides = _slides([1, 1023, 1, 1024, 2047], seed=130)
    with torch.no_grad():
        got = model.forward_packed(slides, all_layer_embed=True)
        for (x, c), outs in zip(slides, got):
            ref = model(x[None], c[None], all_layer_embed=True)
            for o, r in zip(outs, ref):
                _close(o, r)
        one = model.forward_packed(slides[1:2], all_layer_embed=False)
        _close(one[0][0], model(slides[1][0][None], slides[1][1][None])[0])


@pytest.mark.timeout(600)
def test_c5_full_mixed_batch_packed_matches_individual_forwards():
    """Config C5 at its real size: the 32-slide batch of batch.mixed_batch_sizes() (2k-100k tiles,
    675,587 in all) encoded by encode_slides (varlen-packed, one forward) == every slide's own B = 1
    forward (GEMM row-count rounding aside), all 13 embeddings; the smallest slide also against the
    fp32 oracle."""
    sizes = batch.mixed_batch_sizes()
    assert len(sizes) == 32 and sum(sizes) == 675587
    model = _model()
    slides = _slides(sizes, seed=200)
    out = batch.encode_slides(model, slides, all_layer_embed=True)
    assert len(out) == 32
    with torch.no_grad():
        for (x, c), o in zip(slides, out):
            ref = model(x[None], c[None], all_layer_embed=True)
            assert len(o) == len(ref) == 13
            _close(torch.stack(o), torch.stack(ref))
    i = int(np.argmin(sizes))
    cfg = orc.arch_config("gigapath_slide_enc12l768d")
    Wt = {k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}
    x, c = slides[i]
    want = torch.stack(orc.slide_encoder_forward(Wt, x[None].cpu().numpy(), c[None].cpu().numpy(), cfg,
                                                 all_layer_embed=True))
    _close(torch.stack(out[i]).cpu(), want)
