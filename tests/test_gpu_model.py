"""Model-level parity of the MI355X slide encoder (run with -m gpu).

Tolerance: the build runs in bf16 and is compared with the reference in fp32;
the reference's OWN bf16-vs-fp32 deviation at N=1024 is 1.0-1.4e-2 (max|d|/max|ref|), so the
acceptance is max|d|/max|ref| <= max(2e-2, 1.5 x that) and cosine >= 0.9995 per output.
"""
import hashlib

import numpy as np
import pytest
import torch

import oracle as orc
from conftest import load_golden, record_parity

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = orc.arch_config("gigapath_slide_enc12l768d")


def close_enough(got, ref, ref_bf16_dev=0.0):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    rel = np.abs(got - ref).max() / np.abs(ref).max()
    cos = (got * ref).sum() / np.sqrt((got * got).sum() * (ref * ref).sum())
    return rel, cos, rel <= max(2e-2, 1.5 * ref_bf16_dev) and cos >= 0.9995


# the north star's stated bf16 tolerance on slide embeddings (BASELINE.json: "max-rel 1e-2"): the C3 / C4
# headline goldens must also stay inside it -- a regression guard below the survey's 2e-2 acceptance,
# since every moved rounding point (LN folds, residual epilogues) spends headroom
NORTH_STAR_REL = 1e-2


def check_vectors(test, name, got, ref, ref_bf16_dev=0.0, north_star=False):
    """Every output vector (last axis) within the model tolerance; the worst rel / cos is recorded
    (conftest.record_parity) so the headroom is on record, not only the pass.  north_star: the worst
    vector must also be within NORTH_STAR_REL (the C3 / C4 headline slides)."""
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    worst_rel, worst_cos = 0.0, 1.0
    for idx in np.ndindex(*got.shape[:-1]):
        rel, cos, ok = close_enough(got[idx], ref[idx], ref_bf16_dev)
        assert ok, (test, name, idx, rel, cos)
        worst_rel, worst_cos = max(worst_rel, rel), min(worst_cos, cos)
    tol = NORTH_STAR_REL if north_star else max(2e-2, 1.5 * ref_bf16_dev)
    record_parity(test, name, worst_rel, worst_cos, tol, 0.9995, int(np.prod(got.shape[:-1])))
    if north_star:
        assert worst_rel <= NORTH_STAR_REL, (test, name, "north-star max-rel", worst_rel)


@pytest.fixture(scope="module")
def model():
    from gigapath import slide_encoder
    m = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536)
    W = orc.make_weights(CFG, seed=0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    return m.to(DEV).eval()


def test_h5_slide_file_to_golden(model, golden_meta, tmp_path):
    """Slide-file input path (gigapath.slide_io, reference slide_datatset.py:170-193): the golden
    N = 1024 slide written as a CLAM-style h5 file (one tile per chunk, fp32 features, int64 coords),
    read back with get_images_from_path and fed to the encoder, matches the reference golden."""
    from gigapath import slide_io
    from h5_spec_writer import Writer
    g = load_golden("e2e_N1024_B1.npz")
    ent = [e for e in golden_meta["e2e"] if e["N"] == 1024 and e["B"] == 1][0]
    x, coords = orc.synthetic_slide(1024)
    w = Writer()
    w.dataset("features", x[0], layout="chunked", chunks=(1, x.shape[-1]))
    w.dataset("coords", coords[0].astype(np.int64), layout="chunked", chunks=(1, 2))
    p = str(tmp_path / "slide.h5")
    w.save(p)
    d = slide_io.get_images_from_path(p, max_tiles=100000)
    assert d["img_lens"] == 1024
    with torch.no_grad():
        got = torch.stack(model(d["imgs"][None].to(DEV), d["coords"][None].float().to(DEV),
                                all_layer_embed=True)).cpu().numpy()
    check_vectors("h5 slide file N=1024", "all_layer", got, g["all_layer"], ent.get("ref_bf16_rel_inf", 0.0))


@pytest.mark.parametrize("N,B", [(1024, 1), (4097, 1), (600, 2)])
def test_end_to_end_vs_reference_golden(model, golden_meta, N, B):
    g = load_golden("e2e_N%d_B%d.npz" % (N, B))
    ent = [e for e in golden_meta["e2e"] if e["N"] == N and e["B"] == B][0]
    x, coords = orc.synthetic_slide(N, B=B)
    xt, ct = torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV)
    with torch.no_grad():
        allv = torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy()
        last = model(xt, ct)[0].cpu().numpy()
        model.global_pool = True
        try:
            gp_all = torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy()
            gp_last = model(xt, ct)[0].cpu().numpy()
        finally:
            model.global_pool = False
    dev_bf16 = ent.get("ref_bf16_rel_inf", 0.0)
    for name, got in (("all_layer", allv), ("last", last), ("gp_all_layer", gp_all), ("gp_last", gp_last)):
        check_vectors("e2e N=%d B=%d" % (N, B), name, got, g[name], dev_bf16)


def test_c2_16k_end_to_end_vs_reference_golden(model, golden_meta):
    """Config C2 (16,384 tiles: 17 / 3 / 1 / 1 / 1 segments per branch) against the reference's own
    fp32 output (make_golden.py --e2e 16384), all 13 embeddings and the default output, eager and
    as a HIP-graph replay."""
    g = load_golden("e2e_N16384_B1.npz")
    x, coords = orc.synthetic_slide(16384)
    xt, ct = torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV)
    with torch.no_grad():
        allv = torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy()
        last = model(xt, ct)[0].cpu().numpy()
        model.use_hip_graphs = True
        model.graph_min_uses = 1
        try:
            rep = torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy()
            assert len(model._graphs) == 1
        finally:
            model.use_hip_graphs = False
            model.graph_min_uses = 2
            for k in list(model._graphs):
                model._drop_graph(k)
    assert np.array_equal(rep, allv)
    for name, got in (("all_layer", allv), ("last", last)):
        check_vectors("C2 e2e N=16384", name, got, g[name])


@pytest.mark.timeout(600)
def test_c3_70k_end_to_end_vs_reference_golden(model):
    """Config C3, the north star's headline slide (70,000 tiles: 69 / 13 / 3 / 1 / 1 segments, the
    8,751- and 4,376-row sparse branches), the FULL 12-layer forward against the reference's own
    fp32 output (make_golden.py --e2e 70000): all 13 embeddings, the default output and the two
    global-pool readouts, eager and as the HIP-graph replay bench.py times (bit-identical)."""
    g = load_golden("e2e_N70000_B1.npz")
    x, coords = orc.synthetic_slide(70000)
    xt, ct = torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV)
    with torch.no_grad():
        allv = torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy()
        last = model(xt, ct)[0].cpu().numpy()
        model.use_hip_graphs, model.graph_min_uses = True, 1
        try:
            rep = [torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy() for _ in range(2)]
        finally:
            model.use_hip_graphs, model.graph_min_uses = False, 2
            for k in list(model._graphs):
                model._drop_graph(k)
            model._graph_seen.clear()
        model.global_pool = True
        try:
            gp_all = torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy()
            gp_last = model(xt, ct)[0].cpu().numpy()
        finally:
            model.global_pool = False
    assert all(np.array_equal(r, allv) for r in rep)
    for name, got in (("all_layer", allv), ("last", last), ("gp_all_layer", gp_all), ("gp_last", gp_last)):
        check_vectors("C3 e2e N=70000", name, got, g[name], north_star=True)


@pytest.mark.timeout(300)
def test_resid_fused_path_vs_reference_golden(model, monkeypatch):
    """GIGAPATH_RESID_FUSED=1 (the residual epilogues and LN folds of DESIGN §3.4b; off by default since
    round 6, where the round-3 sequence measured faster) still matches the reference: config C2 (16,384
    tiles) against the reference's own fp32 output, every embedding within the model tolerance."""
    from gigapath import runtime
    g = load_golden("e2e_N16384_B1.npz")
    x, coords = orc.synthetic_slide(16384)
    xt, ct = torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV)
    eng = model.encoder.engine

    def repack():
        eng._packs.clear()
        eng._ws.clear()

    monkeypatch.setattr(runtime, "RESID_FUSED", True)
    repack()
    try:
        with torch.no_grad():
            allv = torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy()
        assert all(pl.resid_fused for pl in next(iter(eng._packs.values()))[1])
    finally:
        monkeypatch.setattr(runtime, "RESID_FUSED", False)
        repack()
    check_vectors("C2 e2e N=16384 resid-fused", "all_layer", allv, g["all_layer"])


def test_fp16_autocast_caller_vs_reference_golden(model, golden_meta):
    """The reference pipeline's call (pipeline.py:186-187): fp16 tile embeddings into
    model(x, coords, all_layer_embed=True) inside torch.cuda.amp.autocast(dtype=torch.float16).
    As the reference's Linear layers and flash-attn do under that autocast, the MI355X path then
    computes its 16-bit activations in fp16 (runtime.compute_format): fp16 GEMMs, the fp16 attention /
    merge / LN / GELU kernels; fp32 residual stream and readouts.  Outputs are fp32, within the model
    tolerance of the reference's fp32 golden, and closer to it than the bf16 path."""
    g = load_golden("e2e_N1024_B1.npz")
    ent = [e for e in golden_meta["e2e"] if e["N"] == 1024 and e["B"] == 1][0]
    x, coords = orc.synthetic_slide(1024)
    xt, ct = torch.from_numpy(x).to(DEV).half(), torch.from_numpy(coords).to(DEV)
    with torch.no_grad(), torch.cuda.amp.autocast(dtype=torch.float16):
        out = model(xt, ct, all_layer_embed=True)
        assert model.encoder.engine.ws.qkv.dtype == torch.float16          # computed in fp16
        assert model.encoder.engine.layers[0].w1.dtype == torch.float16
        last = model(xt, ct)[0]
    assert len(out) == 13 and all(o.dtype == torch.float32 for o in out) and last.dtype == torch.float32
    allv = torch.stack(out).cpu().numpy()
    for name, got in (("all_layer", allv), ("last", last.cpu().numpy())):
        check_vectors("fp16 autocast e2e N=1024", name, got, g[name], ent.get("ref_bf16_rel_inf", 0.0))
    with torch.no_grad():
        bf = torch.stack(model(xt.float(), ct, all_layer_embed=True)).cpu().numpy()
    assert model.encoder.engine.ws.qkv.dtype == torch.bfloat16                # outside autocast: bf16 again
    ref = g["all_layer"]
    e16 = np.abs(allv - ref).max() / np.abs(ref).max()
    ebf = np.abs(bf - ref).max() / np.abs(ref).max()
    assert e16 < 0.6 * ebf, (e16, ebf)


def test_fp16_graph_replay_and_packed_batch(model):
    """Under fp16 autocast the HIP-graph replay equals the eager fp16 forward bit for bit (graphs are
    keyed by the activation format), and the varlen-packed batch (fp16 exact attention kernel) matches
    each slide's own fp16 forward up to the GEMMs' row-count rounding."""
    sizes = [300, 1025, 77]
    slides = []
    for i, n in enumerate(sizes):
        x, c = orc.synthetic_slide(n, seed_x=40 + i, seed_c=60 + i)
        slides.append((torch.from_numpy(x[0]).to(DEV).half(), torch.from_numpy(c[0]).to(DEV)))
    x0, c0 = slides[1]
    with torch.no_grad(), torch.cuda.amp.autocast(dtype=torch.float16):
        eager = torch.stack(model(x0[None], c0[None], all_layer_embed=True))
        model.use_hip_graphs, model.graph_min_uses = True, 1
        try:
            g1 = torch.stack(model(x0[None], c0[None], all_layer_embed=True))
            g2 = torch.stack(model(x0[None], c0[None], all_layer_embed=True))
            packed = model.forward_packed(slides, all_layer_embed=True)
        finally:
            model.use_hip_graphs, model.graph_min_uses = False, 2
            for k in list(model._graphs):
                model._drop_graph(k)
            model._graph_seen.clear()
        single = [torch.stack(model(x[None], c[None], all_layer_embed=True)) for x, c in slides]
    assert torch.equal(eager, g1) and torch.equal(g1, g2)
    for i, (p, s1) in enumerate(zip(packed, single)):
        p = torch.stack(p)
        rel, cos, ok = close_enough(p.cpu().numpy().ravel(), s1.cpu().numpy().ravel())
        assert rel <= 5e-3 and cos >= 0.99999, (i, rel, cos)


def test_bf16_error_not_worse_than_reference_bf16(model, golden_meta):
    """At N=1024 the reference's own bf16 run deviates from its fp32 run by ~1.4e-2; ours must
    be at least as close to the fp32 reference."""
    g = load_golden("e2e_N1024_B1.npz")
    x, coords = orc.synthetic_slide(1024)
    with torch.no_grad():
        allv = torch.stack(model(torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV),
                                 all_layer_embed=True)).cpu().numpy()
    ours = np.abs(allv - g["all_layer"]).max() / np.abs(g["all_layer"]).max()
    theirs = np.abs(g["bf16_all_layer"] - g["all_layer"]).max() / np.abs(g["all_layer"]).max()
    assert ours <= theirs, (ours, theirs)


def test_dilated_attention_module_golden():
    """Reference DilatedAttention on a misaligned multi-segment schedule (s % r != 0, nseg > 1)."""
    from gigapath.torchscale.architecture.config import EncoderConfig
    from gigapath.torchscale.component.dilated_attention import DilatedAttention
    g = load_golden("dilated_attention_custom.npz")
    args = EncoderConfig(encoder_embed_dim=768, encoder_attention_heads=16, segment_length=list(g["segs"]),
                         dilated_ratio=list(g["ratios"]), flash_attention=True)
    mod = DilatedAttention(args, 768, 16, self_attention=True, subln=True)
    W = orc.make_weights(CFG, seed=0)
    pre = "encoder.layers.0.self_attn."
    mod.load_state_dict({k[len(pre):]: torch.from_numpy(v) for k, v in W.items() if k.startswith(pre)})
    mod = mod.to(DEV).eval()
    x = torch.from_numpy(g["x"]).to(DEV)
    with torch.no_grad():
        y = mod(x, x, x)[0].cpu().numpy()
    for b in range(y.shape[0]):
        rel, cos, ok = close_enough(y[b], g["y"][b])
        assert ok, (b, rel, cos)


@pytest.mark.parametrize("masked", [False, True])
def test_encoder_standalone_matches_oracle(masked):
    """Encoder.forward (reference signature) on random token embeddings, 2 layers.  masked: an
    encoder_padding_mask zeroes those embeddings before the first layer (encoder.py:358) and is not
    seen by the flash attention path (multihead_attention.py:103)."""
    from gigapath.torchscale.model.LongNet import make_longnet_from_name
    enc = make_longnet_from_name("LongNet_8_layers_768_dim", segment_length="[64, 128, 256, 512, 1024]",
                                 dropout=0.0, drop_path_rate=0.0)
    enc.layers = enc.layers[:2]
    enc.num_layers = 2
    cfg = dict(CFG, depth=2, segment_length=[64, 128, 256, 512, 1024])
    W = orc.make_weights(dict(cfg), seed=4)
    sd = {k[len("encoder."):]: torch.from_numpy(v) for k, v in W.items() if k.startswith("encoder.")}
    enc.load_state_dict(sd, strict=True)
    enc = enc.to(DEV).eval()
    rng = np.random.default_rng(2)
    x = torch.from_numpy(rng.standard_normal((1, 700, 768)).astype(np.float32))
    mask = torch.zeros(1, 700, dtype=torch.bool)
    if masked:
        mask[0, torch.from_numpy(rng.choice(700, 90, replace=False))] = True
    with torch.no_grad():
        out = enc(None, encoder_padding_mask=mask.to(DEV) if masked else None, token_embeddings=x.to(DEV),
                  return_all_hiddens=True)
    Wt = {k: torch.from_numpy(v) for k, v in W.items()}
    h = x * (1 - mask.unsqueeze(-1).float())
    states = [h]
    for li in range(2):
        h = orc.encoder_layer(h, Wt, "encoder.layers.%d" % li, cfg["segment_length"], cfg["dilated_ratio"], 16)
        states.append(h)
    ref_out = torch.nn.functional.layer_norm(h, (768,), Wt["encoder.layer_norm.weight"], Wt["encoder.layer_norm.bias"], 1e-5)
    rel, cos, ok = close_enough(out["encoder_out"].cpu().numpy(), ref_out.numpy())
    assert ok, (rel, cos)
    assert len(out["encoder_states"]) == 3
    for s_got, s_ref in zip(out["encoder_states"], states):
        rel, cos, ok = close_enough(s_got.cpu().numpy(), s_ref.numpy())
        assert ok, (rel, cos)
    assert torch.equal(out["encoder_embedding"].cpu(), x)
    if masked:
        assert not out["encoder_states"][0][0, mask[0]].any()


def test_out_of_range_coords_raise_index_error(model):
    x = torch.zeros(1, 3, 1536, device=DEV)
    c = torch.tensor([[[0.0, 0.0], [256.0 * 1000, 0.0], [5.0, 5.0]]], device=DEV)
    with pytest.raises(IndexError):
        with torch.no_grad():
            model(x, c)


def test_deterministic_and_batch_independent(model):
    x, coords = orc.synthetic_slide(3000)
    xt, ct = torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV)
    with torch.no_grad():
        a = torch.stack(model(xt, ct, all_layer_embed=True))
        b = torch.stack(model(xt, ct, all_layer_embed=True))
        c = torch.stack(model(torch.cat([xt, xt]), torch.cat([ct, ct]), all_layer_embed=True))
    assert torch.equal(a, b)
    assert torch.equal(c[:, 0], c[:, 1])
    assert (c[:, :1] - a).abs().max().item() <= 1e-5 * a.abs().max().item()


def test_full_size_70k_one_layer_vs_oracle(model):
    """C3 size (N = 70,000): embedding + layer 0 on the GPU vs the fp32 oracle (one layer keeps
    the CPU side to ~20 s)."""
    from gigapath.torchscale.architecture.encoder import EncoderLayer  # noqa: F401
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    N = 70000
    x, coords = orc.synthetic_slide(N)
    W = {k: torch.from_numpy(v) for k, v in orc.make_weights(CFG, seed=0).items()}
    h0 = torch.nn.functional.linear(torch.from_numpy(x), W["patch_embed.proj.weight"], W["patch_embed.proj.bias"])
    pos = orc.coords_to_pos(coords)
    h0 = h0 + torch.from_numpy(orc.pos_embed_rows(pos, orc.sincos_axis_table(768, 1000), 1000))
    h0 = torch.cat([W["cls_token"].view(1, 1, 768), h0], 1)
    with torch.no_grad():
        ref = orc.encoder_layer(h0, W, "encoder.layers.0", CFG["segment_length"], CFG["dilated_ratio"], 16)
        got, _ = model.encoder.layers[0](h0.to(DEV))
    got = got.cpu().numpy()[0]
    ref = ref.numpy()[0]
    rel, cos, ok = close_enough(got, ref)
    assert ok, (rel, cos)
    record_parity("C3 layer 0 vs oracle [70001,768]", "layer0", rel, cos, 2e-2, 0.9995)
    # per-token check on the CLS row and a sample of rows
    for t in [0, 1, 1023, 1024, 5791, 5792, 32767, 32768, 69999, 70000]:
        r2, c2, ok2 = close_enough(got[t], ref[t])
        assert c2 >= 0.999, (t, r2, c2)


def test_hip_graph_replay_matches_eager(model):
    """use_hip_graphs: one graph replay per input shape, bit-identical to the eager launches,
    across shape changes (each graph keeps its own workspace) and weight updates (re-capture,
    graphs of the old weights dropped); with the default graph_min_uses = 2 a shape seen once runs
    eagerly; the LRU byte budget evicts."""
    shapes = [1500, 700, 1500]
    x = {n: orc.synthetic_slide(n, seed_x=n) for n in set(shapes)}
    with torch.no_grad():
        eager = {n: torch.stack(model(torch.from_numpy(x[n][0]).to(DEV), torch.from_numpy(x[n][1]).to(DEV),
                                      all_layer_embed=True)) for n in set(shapes)}
        model.use_hip_graphs = True
        try:
            n0 = shapes[0]
            got = torch.stack(model(torch.from_numpy(x[n0][0]).to(DEV), torch.from_numpy(x[n0][1]).to(DEV),
                                    all_layer_embed=True))
            assert torch.equal(got, eager[n0]) and len(model._graphs) == 0     # first sighting: eager
            model._graph_seen.clear()
            model.graph_min_uses = 1
            for n in shapes:
                xt, ct = torch.from_numpy(x[n][0]).to(DEV), torch.from_numpy(x[n][1]).to(DEV)
                got = torch.stack(model(xt, ct, all_layer_embed=True))
                assert torch.equal(got, eager[n]), n
            assert len(model._graphs) == 2
            assert all(b > 0 for b in model._graph_bytes.values())
            # a weight update changes the packed-weight signature -> new capture, new result
            w = model.encoder.layers[3].ffn.fc2.weight
            saved = w.detach().clone()
            w.mul_(0.5)                  # in-place on the parameter: bumps its version
            n = shapes[0]
            got = torch.stack(model(torch.from_numpy(x[n][0]).to(DEV), torch.from_numpy(x[n][1]).to(DEV),
                                    all_layer_embed=True))
            assert not torch.equal(got, eager[n])
            assert len(model._graphs) == 1              # the old weights' graphs were dropped
            w.copy_(saved)
            got = torch.stack(model(torch.from_numpy(x[n][0]).to(DEV), torch.from_numpy(x[n][1]).to(DEV),
                                    all_layer_embed=True))
            assert torch.equal(got, eager[n])
            # byte budget: room for one graph only -> the least recently used one is evicted
            model.hip_graph_max_bytes = max(model._graph_bytes.values()) + 1
            for m in (700, 1500):
                got = torch.stack(model(torch.from_numpy(x[m][0]).to(DEV), torch.from_numpy(x[m][1]).to(DEV),
                                        all_layer_embed=True))
                assert torch.equal(got, eager[m]) and len(model._graphs) == 1
            with pytest.raises(IndexError):
                bad = torch.from_numpy(x[n][1]).to(DEV).clone()
                bad[0, 0, 0] = 256.0 * 1000
                model(torch.from_numpy(x[n][0]).to(DEV), bad)
        finally:
            model.use_hip_graphs = False
            model.graph_min_uses = 2
            model.hip_graph_max_bytes = 48 << 30
            for k in list(model._graphs):
                model._drop_graph(k)


@pytest.mark.parametrize("arch", ["gigapath_slide_enc24l1024d", "gigapath_slide_enc12l1536d"])
@pytest.mark.parametrize("half", [False, True])
def test_other_registered_archs_vs_oracle(arch, half):
    """24L1024d (D = 64) and 12L1536d (D = 96) end to end against the fp32 oracle, in bf16 and under
    the fp16 autocast caller (their register-staged fp16 attention kernels, F = 4096 / 6144 fp16 GELU)."""
    from gigapath import slide_encoder
    cfg = orc.arch_config(arch)
    m = slide_encoder.create_model("", arch, 1536)
    W = orc.make_weights(cfg, seed=0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    x, coords = orc.synthetic_slide(700)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16, enabled=half):
        got = torch.stack(m(torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV),
                            all_layer_embed=True)).cpu().numpy()
        assert m.encoder.engine.ws.qkv.dtype == (torch.float16 if half else torch.bfloat16)
    Wt = {k: torch.from_numpy(v) for k, v in W.items()}
    ref = torch.stack(orc.slide_encoder_forward(Wt, x, coords, cfg, all_layer_embed=True)).numpy()
    check_vectors("%s %s vs oracle N=700" % (arch, "fp16" if half else "bf16"), "all_layer", got, ref)


def test_classification_head_logits(model):
    from gigapath import classification_head
    head = classification_head.ClassificationHead(1536, 768, "0-6-12", n_classes=4, pretrained="")
    head.slide_encoder.load_state_dict(model.state_dict())
    head = head.to(DEV)
    x, coords = orc.synthetic_slide(900)
    xt, ct = torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV)
    logits = head(xt, ct)
    assert logits.shape == (1, 4) and logits.requires_grad
    with torch.no_grad():
        emb = model(xt, ct, all_layer_embed=True)
        want = head.classifier(torch.cat([emb[0], emb[6], emb[12]], -1))
    assert torch.allclose(logits.detach(), want, atol=1e-5)
    logits.sum().backward()                          # the classifier trains on frozen features
    assert head.classifier[0].weight.grad is not None


def _tiny_case(golden_meta, N, B):
    """(fp32 reference output, the reference's own worst per-vector bf16 deviation) of a tiny / ragged slide
    (tests/golden/make_golden.py --tiny: the reference itself, the model fixture's weights)."""
    ent = [e for e in golden_meta["tiny"]["cases"] if e["N"] == N and e["B"] == B][0]
    x, coords = orc.synthetic_slide(N, B=B)
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()   # noqa: E731
    assert sha(x) == ent["x_sha256"] and sha(coords) == ent["coords_sha256"]
    g = load_golden("tiny_slides.npz")
    return x, coords, g["N%d_B%d_fp32" % (N, B)], ent["ref_bf16_rel_vec_max"]


def check_tiny(test, got, ref, ref_dev):
    """Every [E] output vector within max(north-star 1e-2, 1.5 x the REFERENCE's own bf16-vs-fp32
    deviation at this size, worst vector) of the fp32 reference, cosine >= 0.9995 (verdict r04 item 5:
    the bound is pinned by the reference's own noise, not a flat 2e-2)."""
    tol = max(NORTH_STAR_REL, 1.5 * ref_dev)
    worst_rel, worst_cos = 0.0, 1.0
    for idx in np.ndindex(*got.shape[:-1]):
        g, r = np.asarray(got[idx], np.float64), np.asarray(ref[idx], np.float64)
        rel = np.abs(g - r).max() / np.abs(r).max()
        cos = (g * r).sum() / np.sqrt((g * g).sum() * (r * r).sum())
        assert rel <= tol and cos >= 0.9995, (test, idx, rel, cos, tol)
        worst_rel, worst_cos = max(worst_rel, rel), min(worst_cos, cos)
    record_parity(test + " (ref's own bf16 dev %.2e)" % ref_dev, "all_layer", worst_rel, worst_cos, tol, 0.9995,
                  int(np.prod(got.shape[:-1])))


@pytest.mark.parametrize("N,B", [(1, 1), (2, 1), (31, 1), (255, 1), (257, 1), (1023, 1), (5, 3)])
def test_tiny_and_ragged_slides_vs_reference(model, golden_meta, N, B):
    """Edge cases of the token count L = N + 1 (the CLS row included) against the reference's fp32 output
    (tests/golden/tiny_slides.npz): one-tile slides (every GEMM a single partial 256-row tile, attention
    segments of 2 tokens), lengths one short of / one past a 256-row tile, one short of the 1,024-token
    segment, and a batch of three 5-tile slides -- eager and through the HIP-graph replay (each shape
    captured on first reuse).  Bound: check_tiny (the reference's own bf16 deviation here is 1.4-2.0e-2)."""
    x, coords, ref, ref_dev = _tiny_case(golden_meta, N, B)
    xt, ct = torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV)
    with torch.no_grad():
        outs = [torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy() for _ in range(3)]
    for k, got in enumerate(outs):
        check_tiny("tiny/ragged N=%d B=%d run %d" % (N, B, k), got, ref, ref_dev)
    assert np.array_equal(outs[1], outs[2])     # graph replays agree with each other bit for bit


@pytest.mark.parametrize("N,B", [(1, 1), (257, 1), (5, 3)])
def test_tiny_and_ragged_slides_fp16_caller_vs_reference(model, golden_meta, N, B):
    """The same edge cases under the reference pipeline's fp16 autocast (fp16 GEMMs and GELU, the fp16
    attention) against the reference's fp32 output, same bound."""
    x, coords, ref, ref_dev = _tiny_case(golden_meta, N, B)
    xt, ct = torch.from_numpy(x).to(DEV).half(), torch.from_numpy(coords).to(DEV)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        outs = [torch.stack(model(xt, ct, all_layer_embed=True)).float().cpu().numpy() for _ in range(2)]
    for k, got in enumerate(outs):
        check_tiny("tiny/ragged fp16 N=%d B=%d run %d" % (N, B, k), got, ref, ref_dev)


@pytest.mark.parametrize("bad", [float("nan"), float("inf")])
def test_nonfinite_tile_propagates_like_reference(model, bad):
    """One non-finite feature in one tile: the reference's torch ops turn every layer output after the
    embedding into NaN (the tile's k / v row poisons every segment that holds it, then the CLS row), while
    the layer-0 readout (the CLS token before any layer) stays finite.  The kernels are built with
    -fno-honor-nans (csrc/Makefile: v_max without NaN canonicalisation); this pins that the NaN still
    propagates exactly as in the oracle instead of being absorbed by a max ("NaN inputs")."""
    Wt = {k: torch.from_numpy(v) for k, v in orc.make_weights(CFG, seed=0).items()}
    x, coords = orc.synthetic_slide(300)
    x[0, 7, 5] = bad
    ref = torch.stack(orc.slide_encoder_forward(Wt, x, coords, CFG, all_layer_embed=True)).numpy()
    xt, ct = torch.from_numpy(x).to(DEV), torch.from_numpy(coords).to(DEV)
    with torch.no_grad():
        for _ in range(2):                          # eager, then the captured graph
            got = torch.stack(model(xt, ct, all_layer_embed=True)).cpu().numpy()
            assert np.array_equal(np.isnan(got), np.isnan(ref)), [int(np.isnan(got[i]).sum()) for i in range(13)]
            assert np.isfinite(got[0]).all() and np.isnan(ref[1:]).all()
