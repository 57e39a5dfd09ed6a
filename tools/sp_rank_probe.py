"""Per-rank compute of the sequence-parallel forward at W ranks, measured on ONE GPU (the pool's boxes
have one): for each rank r of the W-rank shard plan of the C4 slide, that rank's 12 encoder layers
(QKV GEMM + sparsify, windowed attention over all branches, merge, out-proj + residual, FFN + residual) run with
the K/V exchange replaced by nothing (the receive buffers hold random rows), as HIP-graph replays, timed
with HIP events.  max over ranks = the compute floor of the W-GPU forward's encoder; the plan's
received bytes per rank say what the RCCL exchange has to hide.  W = 1 is the same engine on the whole
slide (the reference point for the scaling ratio).

    python tools/sp_rank_probe.py [--tiles 256000] [--worlds 1,2,4,8] [--reps 3]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))

from gigapath import runtime, seqpar, slide_encoder   # noqa: E402


class NullExchange:
    device_comm = True

    def all_to_all(self, *a, **k):
        return None

    def p2p(self, *a, **k):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=256000)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ranks", default="", help="only these ranks of each W (default: all)")
    ap.add_argument("--local-first", default="0", help="comma list: 1 = transfer-free branches in a launch "
                    "of their own before the waits, 0 = in their size phase (the engine's default)")
    ap.add_argument("--lib", default="", help="another build of the library (tools/attn_lab A/B), in place of the product")
    ap.add_argument("--product-ref", action="store_true",
                    help="also time the product's one-GPU encoder on the whole slide (the scaling denominator)")
    ap.add_argument("--phases", default="2", help="comma list of attention launch splits to time: "
                    "2 = the plan's (short branches, long branches), 3 = the long branches split by "
                    "whole-sequence vs multi-segment, 1 = one launch")
    ap.add_argument("--key-parts", default="default",
                    help="comma list of key-part settings: default (the engine's rule), none, or b=P[/b=P...]")
    ap.add_argument("--bounds", default="plan", help="comma list: plan (ShardPlan's choice), balanced (the "
                    "cost-balanced cuts, never snapped to a segment multiple), cuts:c1/c2/... (explicit)")
    ap.add_argument("--planner", default="sim", help="comma list: sim (round 6: simulated launches, the default), "
                    "sim1 (the same with the cheap-exchange phase variant), "
                    "r5 (round 5's token-cost planner and item-count key-part rule)")
    ap.add_argument("--per-branch", action="store_true",
                    help="also time each branch's attention as a launch of its own (valid TFLOP/s per branch)")
    args = ap.parse_args()
    if args.lib:
        from gigapath import _hip
        _hip._lib = _hip.load_library(os.path.join(ROOT, args.lib))
    dev = torch.device("cuda", 0)
    model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536).to(dev).eval()
    enc = model.encoder
    layers = enc.engine.pack(enc, dev)
    pa = layers[0].attn
    F = enc.args.encoder_ffn_embed_dim
    L = args.tiles + 1
    g = torch.Generator(device=dev).manual_seed(0)
    out = {"tiles": args.tiles, "worlds": {}}
    def parse_kp(spec):
        if spec == "default":
            return None
        if spec == "none":
            return {}
        return {int(x.split("=")[0]): int(x.split("=")[1]) for x in spec.split("/")}
    for W, nph, lf, kps, bnd, pln in [(int(w), int(p), int(f), k, bd, pl) for w in args.worlds.split(",")
                                      for p in args.phases.split(",") for f in args.local_first.split(",")
                                      for k in args.key_parts.split(",") for bd in args.bounds.split(",")
                                      for pl in args.planner.split(",")]:
        os.environ["GIGAPATH_SP_PLANNER"] = "cost" if pln == "r5" else "sim"
        os.environ["GIGAPATH_SP_KEY_PARTS"] = "rule" if pln == "r5" else "sim"
        os.environ["GIGAPATH_SP_CHEAP_IN_A"] = "1" if pln == "sim1" else "0"
        cuts = None
        if bnd == "balanced":
            cuts = seqpar.balanced_bounds(seqpar.token_cost(L, pa.segs, pa.ratios, pa.H, pa.D, F), W)
        elif bnd.startswith("cuts:"):                  # explicit cuts, e.g. cuts:124928 at W = 2
            cs = [0] + [int(x) for x in bnd[5:].split("/")] + [L]
            assert len(cs) == W + 1, bnd
            cuts = [(cs[w], cs[w + 1]) for w in range(W)]
        plan = seqpar.ShardPlan(L, W, pa.segs, pa.ratios, pa.H, pa.D, F, bounds=cuts)
        if nph == 3:            # the round-2 plan: whole-sequence branches in a launch of their own
            long_ = plan.phase_b1
            plan.phase_b1 = [b for b in long_ if plan.geo[b].nseg > 1]
            plan.phase_b2 = [b for b in long_ if plan.geo[b].nseg == 1]
            if not plan.phase_b1:
                plan.phase_b1, plan.phase_b2 = plan.phase_b2, []
        elif nph == 1:
            plan.phase_a, plan.phase_b1, plan.phase_b2 = [], plan.phase_a + plan.phase_b1 + plan.phase_b2, []
        ranks = []
        sel = [int(r) for r in args.ranks.split(",") if r != "" and int(r) < W] or range(W)
        for r in sel:
            ws = seqpar.ShardWorkspace(plan, r, dev, F, torch.bfloat16)
            ws.x.normal_(generator=g)
            ws.a.copy_(ws.x)
            ws.shift[0].copy_(ws.x.mean(1))        # (gp_posembed_cls_ln's row means, for the residual epilogues)
            for kv in ws.kvs:
                kv.normal_(generator=g)
            if ws.hq:
                ws.qkv_ext[:ws.hq].normal_(generator=g)
            eng = seqpar.SeqParallelEngine(plan, r, NullExchange())
            eng.use_graphs = True
            eng.local_first = bool(lf)
            eng.key_parts = parse_kp(kps)
            x0 = ws.x.clone()
            with torch.no_grad():
                eng.run_layers(layers, ws, shift_ready=True)               # eager + capture
                best = 1e9
                for _ in range(args.reps):
                    ws.x.copy_(x0)
                    ws.a.copy_(x0)
                    ws.shift[0].copy_(x0.mean(1))
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    eng.run_layers(layers, ws, shift_ready=True)
                    e.record()
                    e.synchronize()
                    best = min(best, s.elapsed_time(e))
                # per-kernel-kind breakdown of one eager run (HIP events around each launch)
                ws.x.copy_(x0)
                ws.a.copy_(x0)
                ws.shift[0].copy_(x0.mean(1))
                runtime.TIMER.reset()
                runtime.TIMER.enabled = True
                eng.run_layers(layers, ws, shift_ready=True)
                spans = {k: round(v[1], 3) for k, v in sorted(runtime.TIMER.totals_ms().items())}
                runtime.TIMER.enabled = False
                per_branch = {}
                if args.per_branch:        # each branch alone, the engine's key parts, median of 5
                    a_, e_ = plan.bounds[r]
                    for b in range(len(plan.geo)):
                        ts = []
                        for _ in range(6):
                            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            s0.record()
                            eng.attention(pa, ws, [b], "br")
                            s1.record()
                            s1.synchronize()
                            ts.append(s0.elapsed_time(s1))
                        ms = sorted(ts[1:])[2]
                        fl = runtime.attention_valid_flops_window(L, [pa.segs[b]], [pa.ratios[b]], pa.H, pa.D, a_, e_)
                        per_branch[b] = {"ms": round(ms, 4), "valid_tflops": round(fl / ms / 1e9, 1),
                                         "parts": eng._kp[b]}
            a, b = plan.bounds[r]
            # modelled exposed transfer: per layer, both phases posted together after the head;
            # phase A's busiest incoming link must land before the short-branch attention (only the
            # local-first launch overlaps it), phase B's after A's and behind the short-branch attention.
            nl = len(layers)
            tA = plan.phase_pair_bytes(r, plan.phase_a, True) / seqpar.LINK_BYTES_PER_S * 1e3
            tB = plan.phase_pair_bytes(r, plan.phase_b, False) / seqpar.LINK_BYTES_PER_S * 1e3
            aL = spans.get("attn_local", 0.0) / nl
            aA = spans.get("attn_A", 0.0) / nl
            expA = max(0.0, tA - aL)
            expB = max(0.0, tA + tB - max(tA, aL) - aA)
            mod = plan.model_rank(r, eng.parts(), bool(lf))
            ranks.append({"rank": r, "tokens": b - a, "bounds": [a, b], "ms": round(best, 3), "key_parts": eng.parts(),
                          "model_ms": {k: round(v * nl * 1e3, 3) for k, v in mod.items()},
                          "phases": [plan.phase_a, plan.phase_b1, plan.phase_b2],
                          "recv_MB_per_layer": round(plan.exchange_bytes(r) / 1e6, 1), "spans_ms": spans,
                          "per_branch_attention": per_branch,
                          "link_ms_per_layer": {"A": round(tA, 3), "B": round(tB, 3)},
                          "modelled_exposed_ms": round(nl * (expA + expB), 3),
                          "ms_plus_exposed": round(best + nl * (expA + expB), 3)})
            del eng, ws
            torch.cuda.empty_cache()
        key = str(W) + ("" if nph == 2 else "/phases%d" % nph) + ("/local-first" if lf else "") + \
            ("" if kps == "default" else "/kp:" + kps) + ("" if bnd == "plan" else "/bounds:" + bnd) + \
            ("" if pln == "sim" else "/planner:" + pln)
        out["worlds"][key] = {"max_ms": max(x["ms"] for x in ranks), "ranks": ranks,
                              "max_ms_plus_exposed": max(x["ms_plus_exposed"] for x in ranks),
                              "link_bytes_per_s": seqpar.LINK_BYTES_PER_S}
        print(json.dumps({"W": key, "max_ms": out["worlds"][key]["max_ms"], "ms": [x["ms"] for x in ranks],
                          "attn_ms": [x["spans_ms"].get("attn") for x in ranks]}), flush=True)
    if "1" in out["worlds"]:
        t1 = out["worlds"]["1"]["max_ms"]
        out["compute_scaling"] = {W: round(t1 / v["max_ms"], 2) for W, v in out["worlds"].items()}
    if args.product_ref:
        # the denominator the verdict asks for: the PRODUCT's one-GPU encoder (runtime.EncoderEngine, no
        # sparsify, no windows) on the whole slide, same scope (12 layers from the embedding), graph replay
        E = pa.E
        wsp = enc.engine.workspace(dev, 1, L, E, F, pa.H, pa.segs, pa.ratios, torch.bfloat16)
        wsp.x.normal_(generator=g)
        x0 = wsp.x.clone()

        def run():
            wsp.x.copy_(x0)
            wsp.a.copy_(x0)
            torch.mean(wsp.x, 1, out=wsp.shift[0])
            enc.engine.run_layers(wsp, 1, L, shift_ready=True)
        with torch.no_grad():
            run()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                run()
            best = 1e9
            for _ in range(args.reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                gr.replay()
                e.record()
                e.synchronize()
                best = min(best, s.elapsed_time(e))
        out["product_1gpu_encoder_ms"] = round(best, 3)
        out["scaling_vs_product"] = {W: {"compute": round(best / v["max_ms"], 2),
                                         "compute_plus_modelled_exposed": round(best / v["max_ms_plus_exposed"], 2)}
                                     for W, v in out["worlds"].items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
