"""Tune the slide encoder's hipBLASLt GEMMs with PyTorch TunableOp on the GPU box and write the
winning solutions to prov-gigapath-replication_amd/gigapath/tuned/tunableop_results.csv, which
runtime.py loads (tuning disabled) on every later run.

    python tools/tune_gemms.py --tiles 70000 16384          # whole forwards of those slide sizes
    python tools/tune_gemms.py --sp-tiles 262144 --sp-worlds 1 2 4 8 [--packed-tiles 675587]
    python tools/tune_gemms.py --half --tiles 70000 16384   # the fp16 autocast caller's shapes

--sp-tiles tunes, for every rank of every listed world size, the five GEMM shapes that rank's
sequence-parallel forward issues (rows = its token window from seqpar.ShardPlan, patch rows =
its tiles), by calling the same torch.addmm / torch.mm forms the runtime uses (runtime.py:345-356,
seqpar.py:397-414, slide_encoder.py:509) on random data -- no 256k forward per shape.  --packed-tiles
adds the packed (C5) shapes of that many tiles over --packed-slides slides.  Existing entries of
--out are kept (loaded first, written back with the new ones).
"""
import argparse
import os
import sys
import time

# A tuning run under HIPBLASLT_WORKSPACE_SIZE=0 (meant to rule out the stream-K candidates) ended
# abnormally in round 2 with no fault text in its log: refused, before torch loads.
if os.environ.get("HIPBLASLT_WORKSPACE_SIZE", "").strip() in ("0", "0K", "0k"):
    sys.exit("tune_gemms.py: refusing to tune with HIPBLASLT_WORKSPACE_SIZE=0 (TunableOp still times the "
             "workspace-using candidates; see DESIGN.md §6.3)")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "prov-gigapath-replication_amd", "gigapath", "tuned", "tunableop_results.csv")

import torch  # noqa: E402

E, F, C_IN, H, D = 768, 3072, 1536, 16, 48
SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]


def sp_shapes(tiles, worlds):
    """{(rows, patch_rows)} over every rank of every world size (seqpar.ShardPlan's default bounds)."""
    from gigapath import seqpar
    L = tiles + 1
    out = set()
    for w in worlds:
        bounds = seqpar.ShardPlan(L, w, SEGS, RATIOS, H, D, F).bounds if w > 1 else [(0, L)]
        for a, e in bounds:
            out.add((e - a, (e - 1) - (max(a, 1) - 1)))
    return sorted(out)


def tune_rows(rows, patch_rows, log, bf=torch.bfloat16):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g).to(bf)  # noqa: E731
    a, f = r(rows, E), r(rows, F)
    qkv, y, fo = torch.empty(rows, 3 * E, device=dev, dtype=bf), torch.empty(rows, E, device=dev, dtype=bf), \
        torch.empty(rows, F, device=dev, dtype=bf)
    w_qkv, b_qkv, w_o, w1, b1, w2 = r(3 * E, E), r(3 * E), r(E, E), r(F, E), r(F), r(E, F)
    t0 = time.time()

    def step(name, fn):
        fn()
        torch.cuda.synchronize()
        log("rows %d %s: %.1f s" % (rows, name, time.time() - t0))
    step("qkv", lambda: torch.addmm(b_qkv, a, w_qkv.t(), out=qkv))       # QKV (+ bias)
    step("out", lambda: torch.mm(a, w_o.t(), out=y))                     # out-proj
    step("fc1", lambda: torch.addmm(b1, a, w1.t(), out=fo))              # fc1 (+ bias)
    step("fc2", lambda: torch.mm(f, w2.t(), out=y))                      # fc2
    if patch_rows > 0:
        xp, wp, bp = r(patch_rows, C_IN), r(E, C_IN), r(E)
        step("patch %d" % patch_rows, lambda: torch.addmm(bp, xp, wp.t(), out=y[:patch_rows]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, nargs="*", default=[])
    ap.add_argument("--sp-tiles", type=int, default=0)
    ap.add_argument("--sp-worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--packed-tiles", type=int, default=0)
    ap.add_argument("--packed-slides", type=int, default=32)
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--list", action="store_true", help="print the --sp-tiles shapes and exit (no GPU)")
    ap.add_argument("--rotating-mb", type=int, default=0,
                    help="TunableOp rotating buffer: time each candidate on operands cycled through this many MB "
                         "(cold caches, as inside the forward) instead of the same warm operands")
    ap.add_argument("--fresh", action="store_true", help="do not start from the entries already in --out")
    ap.add_argument("--half", action="store_true",
                    help="fp16 shapes: the reference pipeline's autocast(float16) caller (DESIGN.md §3.3)")
    args = ap.parse_args()
    log = lambda s: print(s, flush=True)  # noqa: E731
    shapes = sp_shapes(args.sp_tiles, args.sp_worlds) if args.sp_tiles else []
    if args.packed_tiles:
        shapes.append((args.packed_tiles + args.packed_slides, args.packed_tiles))
    if args.list:
        for s in shapes:
            log("rows %d patch %d" % s)
        return
    os.environ["GIGAPATH_NO_TUNED_GEMMS"] = "1"       # the file is loaded here, with tuning on
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_max_tuning_duration(60)
    torch.cuda.tunable.set_max_tuning_iterations(30)
    if args.rotating_mb:
        torch.cuda.tunable.set_rotating_buffer_size(args.rotating_mb)
    if os.path.exists(args.out) and not args.fresh:
        torch.cuda.tunable.read_file(args.out)
    torch.cuda.tunable.set_filename(args.out + ".exit.csv", False)   # TunableOp's own copy at exit
    n0 = len(torch.cuda.tunable.get_results())
    with torch.no_grad():
        for rows, patch_rows in shapes:
            tune_rows(rows, patch_rows, log, torch.float16 if args.half else torch.bfloat16)
        if args.tiles:
            import bench
            from gigapath import slide_encoder
            model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536).cuda().eval()
            for n in args.tiles:
                x, c = bench.make_slide(n)
                xt = torch.from_numpy(x).cuda()
                with torch.autocast("cuda", dtype=torch.float16, enabled=args.half):
                    model(xt.half() if args.half else xt, torch.from_numpy(c).cuda(), all_layer_embed=True)
                torch.cuda.synchronize()
                log("tuned shapes for %d tiles" % n)
    with open(args.out, "w") as fh:                # the loaded + new entries, TunableOp's CSV format
        for item in torch.cuda.tunable.get_validators():
            fh.write("Validator," + ",".join(str(v) for v in item) + "\n")
        for item in torch.cuda.tunable.get_results():
            fh.write(",".join(str(v) for v in item) + "\n")
    log("%d GEMM shapes (%d new) -> %s" % (len(torch.cuda.tunable.get_results()),
                                          len(torch.cuda.tunable.get_results()) - n0, args.out))


if __name__ == "__main__":
    main()
