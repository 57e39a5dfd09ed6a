"""Generate the golden vectors under tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference):  python tests/golden/make_golden.py
The outputs are data (inputs + expected outputs); the reference's source never leaves
/root/reference.  Weights and inputs are regenerated from seeds by oracle.make_weights /
oracle.synthetic_slide, and their sha256 is stored so a drifting generator is caught.
"""
import copy
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))   # repo root (for oracle)
sys.path.insert(0, HERE)

import ref_harness  # noqa: E402
import oracle as orc  # noqa: E402

torch.set_num_threads(os.cpu_count())


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def save(name, **arrs):
    np.savez_compressed(os.path.join(HERE, name), **arrs)
    print("wrote", name, {k: getattr(v, "shape", None) for k, v in arrs.items()})


def make_dilated_module(da, cfgmod, E, H, segs, ratios):
    args = cfgmod.EncoderConfig(encoder_embed_dim=E, encoder_attention_heads=H,
                                segment_length=str(list(segs)), dilated_ratio=str(list(ratios)),
                                flash_attention=True)
    mod = da.DilatedAttention(args, E, H, dropout=0.0, self_attention=True, subln=True)
    return mod.eval()


def index_maps(da, cfgmod, L, segs, ratios, H=16):
    """Decode gathering()/scattering() of the reference into integer maps (fp64 codes)."""
    mod = make_dilated_module(da, cfgmod, H, H, segs, ratios)
    out = {}
    x = (torch.arange(L, dtype=torch.float64) + 1).view(1, L, 1, 1).expand(1, L, H, 1).contiguous()
    for b, (sl, r) in enumerate(zip(segs, ratios)):
        g = mod.gathering(x, r, sl, is_causal=False, offset=0, is_kv=True, seq_parall=False)
        nseg = g.shape[0] // H
        tok = (g.view(nseg, H, -1).round().long() - 1).numpy()        # -1 == zero pad
        out["gather_%d" % b] = tok
    # scatter: branch b carries codes, every other branch has lse = -inf (weight 0)
    geos = [orc.branch_geometry(L, sl, r, H) for sl, r in zip(segs, ratios)]
    for b in range(len(segs)):
        outs, lses = [], []
        for bb, geo in enumerate(geos):
            nseg, m = geo["nseg"], geo["m"]
            if bb == b:
                code = (torch.arange(nseg * m, dtype=torch.float64) + 1).view(nseg, m, 1)
                o = code.expand(nseg, m, H).contiguous()
                l = torch.full((nseg, H, m), 0.5, dtype=torch.float64)
            else:
                o = torch.zeros(nseg, m, H, dtype=torch.float64)
                l = torch.full((nseg, H, m), -float("inf"), dtype=torch.float64)
            outs.append(o)
            lses.append(l)
        dense = mod.scattering(outs, lses, L, 1, offset=0)             # [1, L, H]
        c = dense[0].round().long().numpy() - 1                        # -1 == uncovered
        m = geos[b]["m"]
        out["scatter_n_%d" % b] = np.where(c >= 0, c // m, -1)
        out["scatter_i_%d" % b] = np.where(c >= 0, c % m, -1)
    return out


def main():
    t0 = time.time()
    se, da, cfgmod = ref_harness.load_reference()
    arch = "gigapath_slide_enc12l768d"
    cfg = orc.arch_config(arch)
    meta = {"arch": arch, "cfg": cfg}

    # ---------------- model, keys, param counts -------------------------------------------
    model = se.create_model("", arch, 1536).eval()
    sd = model.state_dict()
    meta["state_dict"] = [[k, list(v.shape)] for k, v in sd.items()]
    meta["n_params"] = int(sum(p.numel() for p in model.parameters()))
    meta["n_params_longnet"] = int(sum(p.numel() for p in model.encoder.parameters()))

    # ---------------- pos table factorisation -------------------------------------------
    tab = orc.sincos_axis_table(768, 1000)
    ref_pe = model.pos_embed[0].numpy()
    allp = np.arange(ref_pe.shape[0], dtype=np.int64)
    ours = orc.pos_embed_rows(allp, tab, 1000)
    meta["pos_table_bit_exact"] = bool(np.array_equal(ours.view(np.uint32), ref_pe.view(np.uint32)))
    assert meta["pos_table_bit_exact"]
    meta["pos_embed_sha256"] = sha(ref_pe)
    rs = np.random.Generator(np.random.PCG64(7))
    rows = np.concatenate([[0, 1, 2, 999, 1000, 1001, 999999, 1000000], rs.integers(0, 1000001, 56)])
    save("pos_embed_rows.npz", rows=rows, values=ref_pe[rows])

    # ---------------- coords_to_pos edge cases ------------------------------------------
    rc = np.random.Generator(np.random.PCG64(11))
    edge = np.array([[0, 0], [255.99, 255.99], [256, 256], [256.0001, 511.9999], [1e-7, 255.9999],
                     [255999.9, 255999.9], [256000, 5], [3, 256000], [255744, 255744],
                     [-0.5, 300], [12345.678, 98765.43], [999 * 256 + 255.5, 999 * 256 + 255.5]],
                    dtype=np.float32)
    rnd = (rc.random((2, 500, 2)) * 256000).astype(np.float32)
    c_all = np.concatenate([edge[None].repeat(2, 0), rnd], axis=1)
    pos_ref = model.coords_to_pos(torch.from_numpy(c_all), 256).numpy()
    assert np.array_equal(pos_ref, orc.coords_to_pos(c_all))
    save("coords_to_pos.npz", coords=c_all, pos=pos_ref)

    # ---------------- segment schedules -------------------------------------------------
    meta["schedules"] = {}
    for mw in (262144, 250000, 100000, 16384):
        s = eval(model.get_optimal_segment_length(mw, 256))
        assert s == orc.segment_schedule(mw, 256), (mw, s)
        meta["schedules"][str(mw)] = s

    # ---------------- dilated index maps --------------------------------------------------
    cases = []
    default = (cfg["segment_length"], cfg["dilated_ratio"])
    for L in (1, 7, 1025, 4098, 16385, 70001, 256001):
        cases.append(("default", L, default[0], default[1]))
    cases.append(("wsi250000", 30001, meta["schedules"]["250000"], [1, 2, 4, 8, 16]))
    cases.append(("custom", 200, [32, 60, 90, 120, 1000], [1, 2, 4, 8, 16]))
    cases.append(("custom_r3", 50, [16, 20, 45], [1, 3, 5]))   # head padding path (16 % 3 != 0)
    meta["index_maps"] = []
    samples = {}
    for tag, L, segs, ratios in cases:
        maps = index_maps(da, cfgmod, L, segs, ratios)
        ent = {"tag": tag, "L": L, "segs": list(segs), "ratios": list(ratios), "sha256": {}}
        for k, v in maps.items():
            v = v.astype(np.int64)
            ent["sha256"][k] = sha(v)
            if L <= 4098:
                samples["%s_%d_%s" % (tag, L, k)] = v
        meta["index_maps"].append(ent)
        print("maps", tag, L, "%.1fs" % (time.time() - t0))
    save("index_maps_small.npz", **samples)

    # ---------------- DilatedAttention module, custom misaligned multi-segment schedule ---
    segs, ratios = [32, 60, 90, 120, 1000], [1, 2, 4, 8, 16]
    mod = make_dilated_module(da, cfgmod, 768, 16, segs, ratios)
    W = orc.make_weights(cfg, seed=0, perturb=True)
    pre = "encoder.layers.0.self_attn."
    msd = {k[len(pre):]: torch.from_numpy(v) for k, v in W.items() if k.startswith(pre)}
    mod.load_state_dict(msd, strict=True)
    rx = np.random.Generator(np.random.PCG64(5))
    xa = rx.standard_normal((2, 200, 768)).astype(np.float32)
    with torch.no_grad():
        ya = mod(torch.from_numpy(xa), torch.from_numpy(xa), torch.from_numpy(xa))[0].numpy()
    save("dilated_attention_custom.npz", x=xa, y=ya, segs=np.array(segs), ratios=np.array(ratios))

    # ---------------- end-to-end slide encoder -----------------------------------------
    model.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    meta["weights_sha256"] = orc.weights_sha256(W)
    meta["e2e"] = []
    for N, B in ((1024, 1), (4097, 1), (600, 2)):
        x, coords = orc.synthetic_slide(N, B=B)
        res = {"x_sha256": sha(x), "coords_sha256": sha(coords)}
        with torch.no_grad():
            xt, ct = torch.from_numpy(x), torch.from_numpy(coords)
            t1 = time.time()
            allv = torch.stack(model(xt, ct, all_layer_embed=True), 0).numpy()
            res["sec_all_layer"] = time.time() - t1
            last = model(xt, ct)[0].numpy()
            model.global_pool = True
            gp = torch.stack(model(xt, ct, all_layer_embed=True), 0).numpy()
            gp_last = model(xt, ct)[0].numpy()
            model.global_pool = False
        arrs = dict(all_layer=allv, last=last, gp_all_layer=gp, gp_last=gp_last)
        if N == 1024:
            mb = copy.deepcopy(model).to(torch.bfloat16)   # .to() is in-place: keep fp32 model intact
            with torch.no_grad():
                bfv = torch.stack(mb(xt.bfloat16(), ct, all_layer_embed=True), 0).float().numpy()
            del mb
            arrs["bf16_all_layer"] = bfv
            res["ref_bf16_rel_inf"] = float(np.abs(bfv - allv).max() / np.abs(allv).max())
        save("e2e_N%d_B%d.npz" % (N, B), **arrs)
        res.update(N=N, B=B)
        meta["e2e"].append(res)
        print("e2e", N, B, "%.1fs" % (time.time() - t0))

    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("done %.1fs" % (time.time() - t0))


def add_e2e(N, B=1):
    """Append ONE end-to-end case to the existing golden set without regenerating the others:
    python tests/golden/make_golden.py --e2e 16384   (C2, ~1 min on 8 CPU threads;
    C3 = 70000 ~5 min, C4 = 256000 ~25 min).

    ONE fp32 reference forward with all_layer_embed=True; a forward hook on the reference's
    Encoder keeps its returned dict, so the default output (encoder_out, which the reference
    passes through encoder.layer_norm whatever return_all_hiddens is, encoder.py:387-388) and the
    global-pool readouts (slide_encoder.py:213-221) come from the same run through the
    reference's own `norm` module instead of three more forwards."""
    t0 = time.time()
    se, _, _ = ref_harness.load_reference()
    arch = "gigapath_slide_enc12l768d"
    cfg = orc.arch_config(arch)
    with open(os.path.join(HERE, "golden_meta.json")) as f:
        meta = json.load(f)
    W = orc.make_weights(cfg, seed=0, perturb=True)
    assert orc.weights_sha256(W) == meta["weights_sha256"]
    model = se.create_model("", arch, 1536).eval()
    model.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    x, coords = orc.synthetic_slide(N, B=B)
    res = {"x_sha256": sha(x), "coords_sha256": sha(coords)}
    kept = {}
    hook = model.encoder.register_forward_hook(lambda mod, inp, out: kept.update(out))
    with torch.no_grad():
        xt, ct = torch.from_numpy(x), torch.from_numpy(coords)
        t1 = time.time()
        allv = torch.stack(model(xt, ct, all_layer_embed=True), 0).numpy()
        res["sec_all_layer"] = time.time() - t1
        hook.remove()
        last = model.norm(kept["encoder_out"])[:, 0].numpy()
        gp = torch.stack([model.norm(h[:, 1:, :].mean(dim=1)) for h in kept["encoder_states"]],
                         0).numpy()
        gp_last = model.norm(kept["encoder_out"][:, 1:, :].mean(dim=1)).numpy()
        # the hooked states reproduce the returned list exactly (same tensors, same norm)
        chk = torch.stack([model.norm(h)[:, 0] for h in kept["encoder_states"]], 0).numpy()
        assert np.array_equal(chk, allv)
    del kept
    save("e2e_N%d_B%d.npz" % (N, B), all_layer=allv, last=last, gp_all_layer=gp, gp_last=gp_last)
    res.update(N=N, B=B)
    meta["e2e"] = [e for e in meta["e2e"] if not (e["N"] == N and e["B"] == B)] + [res]
    with open(os.path.join(HERE, "golden_meta.json")) as f2:
        meta2 = json.load(f2)          # another --e2e run may have appended meanwhile
    meta2["e2e"] = [e for e in meta2["e2e"] if not (e["N"] == N and e["B"] == B)] + [res]
    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta2, f, indent=1)
    print("e2e", N, B, "done %.1fs" % (time.time() - t0))


TINY_CASES = ((1, 1), (2, 1), (31, 1), (255, 1), (257, 1), (1023, 1), (5, 3))


def add_tiny():
    """The tiny / ragged slides of tests/test_gpu_model.py::test_tiny_and_ragged_slides_* as reference
    fixtures: python tests/golden/make_golden.py --tiny  (seconds).

    Weights = the tests' model fixture (oracle.make_weights(cfg, seed=0), no perturbation).  Per case the
    reference's fp32 all_layer_embed output AND the same reference model run in bf16 (weights and input
    cast, as for the N = 1024 case above), so the tests can bound the build's bf16 deviation by the
    reference's OWN bf16 deviation at that size instead of a flat tolerance.  The deviation is recorded
    per output vector, as tests/test_gpu_model.py::check_vectors measures it (max|d| / max|ref| of each
    [E] vector), worst over the vectors."""
    t0 = time.time()
    se, _, _ = ref_harness.load_reference()
    arch = "gigapath_slide_enc12l768d"
    cfg = orc.arch_config(arch)
    with open(os.path.join(HERE, "golden_meta.json")) as f:
        meta = json.load(f)
    W = orc.make_weights(cfg, seed=0)
    model = se.create_model("", arch, 1536).eval()
    model.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    mb = copy.deepcopy(model).to(torch.bfloat16)
    arrs, ents = {}, []
    for N, B in TINY_CASES:
        x, coords = orc.synthetic_slide(N, B=B)
        xt, ct = torch.from_numpy(x), torch.from_numpy(coords)
        with torch.no_grad():
            allv = torch.stack(model(xt, ct, all_layer_embed=True), 0).numpy()
            bfv = torch.stack(mb(xt.bfloat16(), ct, all_layer_embed=True), 0).float().numpy()
        vec = [float(np.abs(bfv[i] - allv[i]).max() / np.abs(allv[i]).max()) for i in np.ndindex(*allv.shape[:-1])]
        arrs["N%d_B%d_fp32" % (N, B)] = allv
        arrs["N%d_B%d_bf16" % (N, B)] = bfv
        ents.append({"N": N, "B": B, "x_sha256": sha(x), "coords_sha256": sha(coords),
                     "ref_bf16_rel_vec_max": max(vec),
                     "ref_bf16_rel_inf": float(np.abs(bfv - allv).max() / np.abs(allv).max())})
        print("tiny", N, B, "ref bf16 worst-vector rel %.3e" % max(vec))
    save("tiny_slides.npz", **arrs)
    meta["tiny"] = {"weights_sha256": orc.weights_sha256(W), "cases": ents}
    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("tiny done %.1fs" % (time.time() - t0))


if __name__ == "__main__":
    if len(sys.argv) == 2 and sys.argv[1] == "--tiny":
        add_tiny()
    elif len(sys.argv) == 3 and sys.argv[1] == "--e2e":
        add_e2e(int(sys.argv[2]))
    else:
        main()
