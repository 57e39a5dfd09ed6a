"""Fit seqpar.LaunchModel to measured per-launch attention spans of tools/sp_rank_probe.py, and print the
model against every measured launch.  Host only (no GPU): reads the probe's JSON lines.

    python tools/sp_model_fit.py profiles/r06_fin_sp_rank_probe_w1_w8.log [more logs] [--fit]
"""
import argparse
import dataclasses
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))

from gigapath import seqpar  # noqa: E402

SEGS, RATIOS, H, D, F = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16], 16, 48, 3072


def samples(paths):
    """(plan, rank, kp, span, measured seconds per layer, rest seconds per layer, tokens) per measured launch."""
    out = []
    for path in paths:
        for line in open(path):
            if not line.startswith('{"tiles"'):
                continue
            d = json.loads(line)
            L = d["tiles"] + 1
            for key, v in d["worlds"].items():
                if "/phases" in key:
                    continue
                W = int(key.split("/")[0])
                cuts = None
                if "/bounds:cuts:" in key:
                    cs = [0] + [int(x) for x in key.split("/bounds:cuts:")[1].split("/")] + [L]
                    cuts = [(cs[i], cs[i + 1]) for i in range(W)]
                rk = v["ranks"]
                if "bounds" in rk[0]:       # round-6 probes record each rank's cuts and the plan's phases
                    cuts = [tuple(x["bounds"]) for x in sorted(rk, key=lambda x: x["rank"])]
                    if len(cuts) != W:
                        continue
                if cuts is None:            # older probes: the round-5 planner made their plans
                    os.environ["GIGAPATH_SP_PLANNER"] = "cost"
                plan = seqpar.ShardPlan(L, W, SEGS, RATIOS, H, D, F, bounds=cuts,
                                        cheap_in_a=("phases" in rk[0] and len(rk[0]["phases"][0]) > 2))
                os.environ.pop("GIGAPATH_SP_PLANNER", None)
                if "phases" in rk[0]:
                    plan.phase_a, plan.phase_b1, plan.phase_b2 = [list(x) for x in rk[0]["phases"]]
                    plan.phase_b = plan.phase_b1 + plan.phase_b2
                lf = "/local-first" in key
                for r in v["ranks"]:
                    a, e = plan.bounds[r["rank"]]
                    assert e - a == r["tokens"], (key, r["rank"], e - a, r["tokens"])
                    sp = r["spans_ms"]
                    rest = sum(x for k, x in sp.items() if not k.startswith("attn")) / 12e3
                    for name, br in plan.launches(lf):
                        if sp.get(name) is not None:
                            out.append((plan, r["rank"], r.get("key_parts", [1] * 5), br, name, sp[name] / 12e3, rest,
                                        r["tokens"], path, key))
    return out


def dedupe(smp):
    """One sample per distinct launch (same plan window, branches, key parts): the mean of its measurements."""
    groups = {}
    for x in smp:
        plan, rank, kp, br, name = x[:5]
        k = (plan.L, plan.world, plan.bounds[rank], tuple(kp), tuple(br), name)
        groups.setdefault(k, []).append(x)
    out = []
    for xs in groups.values():
        x = list(xs[0])
        x[5] = sum(y[5] for y in xs) / len(xs)
        out.append(tuple(x))
    return out


def evaluate(smp, model):
    lp = {"qblk": 256, "wg_per_cu": 3, "small_per_cu": 3, "max_key_parts": 64}
    err = []
    for plan, rank, kp, br, name, ms, rest, tok, path, key in smp:
        t = plan.launch_time(rank, br, kp, 256, lp, model)
        err.append((t, ms))
    return err


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("logs", nargs="+")
    ap.add_argument("--fit", action="store_true")
    ap.add_argument("--maxfev", type=int, default=300)
    ap.add_argument("--x0", type=float, nargs="*", default=None, help="start tile_s in us")
    args = ap.parse_args()
    smp = samples(args.logs)
    model = seqpar.LAUNCH_MODEL
    if args.fit:
        import numpy as np
        from scipy.optimize import minimize
        fs = dedupe(smp)
        print("fitting %d distinct launches" % len(fs))

        def mk(x):
            t, i, idle, lau, s1, s2, n4, a1 = [float(v) for v in x]
            cl = lambda v: min(max(v, 0.2), 1.0)
            s1, s2, a1 = cl(s1), cl(s2), cl(a1)
            s2 = max(s1, s2)
            return dataclasses.replace(model, tile_s=t * 1e-6, item_s=abs(i) * 1e-6, idle_frac=min(max(idle, 0), 1),
                                       launch_s=abs(lau) * 1e-6, share3=(s1, s2, 1.0), nw4_rate=n4,
                                       share4=(a1, a1 + 0.5 * (1 - a1), a1 + 0.8 * (1 - a1), 1.0))

        files = sorted({x[8] for x in fs})

        def loss(x):
            ev = evaluate(fs, mk(x))
            err = 0.0
            for f in files:      # one free time scale per log but the first (boxes differ by up to +-4 %)
                pr = [(t, ms) for (t, ms), smp_ in zip(ev, fs) if smp_[8] == f]
                sc = 1.0 if f == args.logs[0] else np.exp(np.mean([np.log(ms / t) for t, ms in pr]))
                err += sum((sc * t / ms - 1) ** 2 for t, ms in pr)
            return err / len(fs)
        x0 = [args.x0[0] if args.x0 else model.tile_s * 1e6, model.item_s * 1e6, model.idle_frac, model.launch_s * 1e6, model.share3[0],
              model.share3[1], model.nw4_rate, model.share4[0]]
        res = minimize(loss, x0, method="Nelder-Mead", options={"maxfev": args.maxfev, "xatol": 1e-3, "fatol": 1e-6})
        model = mk(res.x)
        print("fit:", model, "rms rel err %.4f" % res.fun ** 0.5)
    for (plan, rank, kp, br, name, ms, rest, tok, path, key), (t, _) in zip(smp, evaluate(smp, model)):
        print("%-40s W=%d r=%d %-10s %-14s kp=%s meas %.4f model %.4f ms (%+.1f%%)  rest/token %.2f ns"
              % (os.path.basename(path)[:40], plan.world, rank, name, br, kp, ms * 1e3, t * 1e3, 100 * (t / ms - 1),
                 rest / tok * 1e9))


if __name__ == "__main__":
    main()
