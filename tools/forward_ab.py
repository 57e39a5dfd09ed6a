"""Same-process, interleaved A/B of the whole 70k-tile forward (eager, all_layer_embed=True) across
library builds of the same ABI: per round every build runs one forward (after one warm-up each);
reports the median forward time and the median per-kernel spans (runtime.TIMER) of each build.

    python tools/forward_ab.py --libs prod,tools/attn_lab/liblab_x.so [--tiles 70000] [--rounds 5]

A library entry may carry host-path options after a colon: "prod:resid" / "prod:noresid" run the product
library with runtime.RESID_FUSED on (the residual epilogues) / off (the round-3 out-proj -> residual_layernorm
-> FFN -> residual_layernorm sequence, the default since round 6);
"prod:nomerge" with runtime.MERGE_IN_PRODUCER off (the next LN's statistics merged by the consumer's launch),
repacking the weights for it -- the in-process A/B of the residual epilogues.
"""
import argparse
import contextlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip, runtime, slide_encoder  # noqa: E402
from bench import make_slide  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="prod")
    ap.add_argument("--tiles", type=int, default=70000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    prod = _hip.load_library()
    libs = []
    for spec in args.libs.split(","):
        p = spec.split(":")[0]
        libs.append((spec, prod if p == "prod" else _hip.load_library(os.path.join(ROOT, p))))
    dev = torch.device("cuda")
    with contextlib.redirect_stdout(sys.stderr):
        model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536).to(dev).eval()
    model.use_hip_graphs = False
    x, coords = make_slide(args.tiles)
    xt, ct = torch.from_numpy(x).to(dev), torch.from_numpy(coords).to(dev)
    times = {p: [] for p, _ in libs}
    spans = {p: {} for p, _ in libs}
    outs = {}
    default_resid = runtime.RESID_FUSED      # the product default (GIGAPATH_RESID_FUSED; off since round 6)
    with torch.no_grad():
        for rnd in range(args.rounds + 1):
            for p, lib in libs:
                _hip._lib = lib
                runtime.MERGE_IN_PRODUCER = ":nomerge" not in p
                want = True if ":resid" in p else (False if ":noresid" in p else default_resid)
                if runtime.RESID_FUSED != want:        # (re)pack the weights for this host path
                    runtime.RESID_FUSED = want
                    model.encoder.engine._packs.clear()
                    model.encoder.engine._ws.clear()
                runtime.TIMER.reset()
                runtime.TIMER.enabled = rnd > 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                out = model(xt, ct, all_layer_embed=True)
                e1.record()
                torch.cuda.synchronize()
                runtime.TIMER.enabled = False
                _hip._lib = prod
                if rnd == 0:
                    outs[p] = out[-1].float().clone()
                    continue
                times[p].append(e0.elapsed_time(e1))
                for k, (n, ms) in runtime.TIMER.totals_ms().items():
                    spans[p].setdefault(k, []).append(ms)
    first = libs[0][0]
    res = []
    for p, ts in times.items():
        d = ((outs[p] - outs[first]).abs().max() / outs[first].abs().max()).item()
        row = {"lib": p, "forward_ms": round(statistics.median(ts), 3), "rel_diff_vs_first": d,
               "kernel_ms": {k: round(statistics.median(v), 3) for k, v in sorted(spans[p].items())}}
        print(json.dumps(row), flush=True)
        res.append(row)
    if args.out:
        json.dump({"tiles": args.tiles, "rounds": args.rounds, "results": res}, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
