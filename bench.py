"""Slide-encoder throughput benchmark (BASELINE.json metric) on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--tiles T]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Without a launcher (`WORLD_SIZE` unset), `--gpus N > 1` starts the N ranks itself: it runs
torch.distributed.run as a child process before anything touches the GPU.  Under a launcher,
WORLD_SIZE must equal --gpus (exit 2 otherwise).

A step = one gigapath_slide_enc12l768d forward (bf16, inference) over one synthetic slide of
--tiles tiles, inputs and weights resident in HBM.  Default: 70,000 tiles (BASELINE config C3,
the north star's 1-GPU target) at N = 1; 256,000 tiles (config C4, the north star's 8-GPU
scaling target) for the sequence-parallel runs at N > 1.
Multi-GPU (one process per GPU), --mode:
  sp       (default for N > 1) the SAME slide is sharded across the N ranks by sequence
           parallelism (seqpar.py: per-layer sparse K/V exchange over RCCL point-to-point);
           value = slide tiles / max-over-ranks wall time ("strong" scaling, C4's design);
  replica  every rank encodes its own slide, no collective: value = N x tiles / time ("weak");
  mixed    C5: a batch of 32 slides of 2k-100k tiles (log-uniform, seed 3), LPT-assigned to the
           ranks (batch.py, data parallel, one all-reduce of the outputs at the end), each rank's
           slides varlen-packed into one forward; value = batch tiles / time ("strong").
Rank 0 prints ONE JSON line including the attention kernel's roofline (HIP events around
every gp_dilated_attn_fwd launch in the timed region) and a CPU baseline (the fp32 oracle on
a bounded sample of the same workload, timed on this host).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "slide-encoder tiles/sec at 1/2/4/8 GPUs (12L768d LongNet); attn MFMA util %"
ARCH = "gigapath_slide_enc12l768d"
PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level table)
PEAK_HBM_GBS = 8000.0


def make_slide(n_tiles, seed=1, in_chans=1536, tile=256):
    """Synthetic slide of SURVEY §8(d): N(0,1) tile embeddings, distinct raster-sorted grid cells."""
    rx = np.random.Generator(np.random.PCG64(seed))
    x = rx.standard_normal((1, n_tiles, in_chans), dtype=np.float32)
    rc = np.random.Generator(np.random.PCG64(seed + 1))
    side = max(int(math.ceil(math.sqrt(n_tiles / 0.7))), int(math.ceil(math.sqrt(n_tiles))))
    cells = np.sort(rc.choice(side * side, size=n_tiles, replace=False))
    coords = np.stack([cells // side, cells % side], -1).astype(np.float32)[None] * tile
    return x, coords


def cgroup_cpu_quota():
    """CPUs granted by this job's cgroup CPU bandwidth limit (cgroup v2 cpu.max / v1 cfs quota), None if
    unlimited.  The GPU box's job shows 256 CPUs in its affinity mask under a 16-CPU quota
    ("1600000 100000", profiles/r04_f_cpu_facts.txt)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = float(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = float(f.read())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def host_cores():
    """(threads used for the CPU baseline, usable cores, os.cpu_count(), how usable was derived).
    Usable = the affinity mask, capped by the cgroup CPU quota: the GPU box's affinity mask lists the whole
    256-CPU machine while the job's cgroup grants 16 CPUs of bandwidth, and torch on 256 threads under that
    quota is throttled, not faster (r04_f: no output for 180 s, killed).  The CPU baseline runs on every
    usable core (the reference CPU path on the box's host cores)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    usable = max(1, min(aff, math.ceil(quota))) if quota else aff
    how = {"affinity": aff, "cgroup_cpu_quota": quota}
    return usable, usable, os.cpu_count() or usable, how


def cpu_baseline(n_tiles, threads, sample_tiles=70000, total_tflops=None):
    """fp32 CPU oracle on a bounded sample: patch embed + pos add + ONE of the 12 encoder layers of
    a slide of min(n_tiles, sample_tiles) tiles, extrapolated to the full 12-layer forward; for a
    larger workload (C4's 256k slide, the C5 batch) further scaled by the valid-FLOP ratio of the
    workload to the sampled forward (`total_tflops` = the workload's model TFLOP)."""
    import oracle
    torch.set_num_threads(threads)
    cfg = oracle.arch_config(ARCH)
    W = {k: torch.from_numpy(v) for k, v in oracle.make_weights(cfg, seed=0).items()
         if k.startswith(("patch_embed", "cls_token", "encoder.layers.0."))}
    ns = min(n_tiles, sample_tiles)
    x, coords = make_slide(ns)
    with torch.no_grad():
        t0 = time.perf_counter()
        h = torch.nn.functional.linear(torch.from_numpy(x), W["patch_embed.proj.weight"], W["patch_embed.proj.bias"])
        pos = oracle.coords_to_pos(coords)
        h = h + torch.from_numpy(oracle.pos_embed_rows(pos, oracle.sincos_axis_table(768, 1000), 1000))
        h = torch.cat([W["cls_token"].view(1, 1, 768), h], 1)
        t1 = time.perf_counter()
        oracle.encoder_layer(h, W, "encoder.layers.0", cfg["segment_length"], cfg["dilated_ratio"], 16)
        t2 = time.perf_counter()
    full = (t1 - t0) + cfg["depth"] * (t2 - t1)
    _, usable, ncpu, how = host_cores()
    res = {"value": round(ns / full, 2), "unit": "tiles/s", "cores": threads, "usable_cores": usable,
           "usable_from": how, "cpu_count": ncpu, "kind": "port",
           "sample": "EXTRAPOLATED: oracle fp32 torch-CPU, embed + 1 of 12 layers of the %d-tile slide (%.1f s), "
                     "x12 layers (%.1f s per forward)" % (ns, t2 - t0, full)}
    if total_tflops is not None and ns != n_tiles:
        from gigapath import runtime
        segs, ratios = cfg["segment_length"], cfg["dilated_ratio"]
        sample_tf = (runtime.gemm_flops(1, ns, 768, 3072, 1536, 12)
                     + 12 * runtime.attention_valid_flops(ns + 1, segs, ratios, 16, 48)) / 1e12
        secs = full * total_tflops / sample_tf
        res["value"] = round(n_tiles / secs, 2)
        res["sample"] += ("; scaled to the %d-tile workload by its valid FLOPs (%.2f / %.2f TFLOP): %.0f s"
                          % (n_tiles, total_tflops, sample_tf, secs))
    return res


def cpu_full_forwards(sizes, threads):
    """The fp32 CPU oracle's WHOLE 12-layer forward (all_layer_embed=True) of the C1 / C2 slides,
    timed in full (no extrapolation): BASELINE.md §4's CPU rows."""
    import oracle
    torch.set_num_threads(threads)
    cfg = oracle.arch_config(ARCH)
    W = {k: torch.from_numpy(v) for k, v in oracle.make_weights(cfg, seed=0).items()}
    res = {}
    for name, n in sizes:
        x, coords = make_slide(n)
        with torch.no_grad():
            t0 = time.perf_counter()
            out = oracle.slide_encoder_forward(W, x, coords, cfg, all_layer_embed=True)
            dt = time.perf_counter() - t0
        assert all(torch.isfinite(o).all() for o in out)
        res[name] = {"tiles": n, "value": round(n / dt, 2), "unit": "tiles/s", "seconds": round(dt, 2),
                     "cores": threads, "kind": "port", "sample": "full 12-layer fp32 forward, timed"}
    return res


def sp_rank_report(model, kt, rank, timing_steps, L, segs, ratios, monitor):
    """This rank's line of the N > 1 report: its shard, bytes over xGMI per layer, exposed exchange
    wait per layer (monitor), and its attention / sparsify kernels against their rooflines."""
    from gigapath import runtime
    plan = model._sp.plan
    a_w, b_w = plan.bounds[rank]
    nl = len(model.encoder.layers)
    recv = plan.exchange_bytes(rank)
    send = sum((hi - lo) * 2 * plan.C[b] * 2 for b, _, lo, hi in plan.sends(rank))
    send += sum((hi - lo) * 3 * plan.E * 2 for _, lo, hi in plan.halo_sends(rank))
    fl = runtime.attention_valid_flops_window(L, segs, ratios, 16, 48, a_w, b_w)
    # (the SP engine labels its attention launches by exchange phase: attn_local / attn_A / attn_B)
    ms_att = sum(v[1] for k, v in kt.items() if k.startswith("attn"))
    att_s = ms_att / max(timing_steps * nl, 1) / 1e3
    sp_bytes = sum((b_w - a_w) * 2 * plan.C[b] * 2 + sum(plan.send_splits(rank, b)) * 2 * plan.C[b] * 2
                   for b in range(len(plan.C)) if not plan.no_xfer[b])
    n_sp, ms_sp = kt.get("sparsify", (0, 0.0))
    rep = {"rank": rank, "tokens": [a_w, b_w], "recv_mb_per_layer": round(recv / 1e6, 2),
           "send_mb_per_layer": round(send / 1e6, 2),
           "attn_ms_per_layer": round(att_s * 1e3, 4),
           "attn_tflops": round(fl / att_s / 1e12, 1) if att_s > 0 else None,
           "attn_frac": round(fl / att_s / 1e12 / PEAK_BF16_TFLOPS, 4) if att_s > 0 else None,
           "sparsify_gbs": round(sp_bytes / (ms_sp / n_sp / 1e3) / 1e9, 1) if ms_sp > 0 else None,
           "kernel_ms_per_step": {k: round(v[1] / timing_steps, 3) for k, v in sorted(kt.items())}}
    if monitor is not None:
        rep["exchange_exposed"] = monitor.summary(nl)
    return rep


def config_label(n_tiles, world, sp):
    """BASELINE.json config this slide size is (C1..C4), or a plain description."""
    if sp:
        return "C4" if n_tiles == 256000 else "SP"
    return {1024: "C1", 16384: "C2", 70000: "C3", 256000: "C4's slide on one GPU"}.get(n_tiles,
                                                                                  "custom (%d tiles)" % n_tiles)


def spawn_ranks(ngpus):
    """`python bench.py --gpus N` without a launcher: start N ranks under torch.distributed.run as a
    CHILD process (nothing here has touched the GPU yet) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ngpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def pmc_traffic(n_tiles, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (tools/pmc_bench.sh ->
    profiles/pmc_traffic.json), or None when it was collected on a different workload."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    ks = [v for name, v in sorted(d.get("kernels", {}).items()) if name.startswith(kernel)]
    if d.get("tiles") != n_tiles or not ks:
        return None
    # the attention prefix also matches the small exact-fixup pass (another VAR of the same template):
    # the launch being priced is the heavy one
    return round(max(k["hbm_bytes_per_launch"] for k in ks))


def main():
    if os.environ.get("GP_BENCH_TRACE_AFTER"):           # debugging aid: dump every thread's stack
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["GP_BENCH_TRACE_AFTER"]), exit=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--tiles", type=int, default=None,
                    help="slide size (default 70000; 256000 for --mode sp at N > 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--mode", choices=["sp", "replica", "mixed"], default="sp")
    ap.add_argument("--timing-steps", type=int, default=2, help="eager steps with per-kernel HIP events")
    ap.add_argument("--mixed-slides", type=int, default=32, help="--mode mixed: slides in the batch")
    ap.add_argument("--no-graphs", action="store_true", help="eager launches instead of HIP graph replay")
    ap.add_argument("--no-cpu-full", action="store_true", help="skip the full C1/C2 CPU forwards")
    ap.add_argument("--no-c4-ref", action="store_true",
                    help="N = 1: skip the 256k-slide line (the workload the N > 1 runs shard)")
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr)
        sys.exit(2)
    if args.dry_run:        # launcher plumbing check only (tests/test_bench_cli.py): no GPU, no work
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": world}), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    sp = world > 1 and args.mode == "sp"
    mixed = args.mode == "mixed"
    if args.tiles is None:
        args.tiles = 256000 if sp else 70000
    # GP_BENCH_BACKEND=gloo: rehearsal of the multi-rank path with several ranks on one GPU
    backend = os.environ.get("GP_BENCH_BACKEND", "nccl")
    if backend != "nccl":                  # (RCCL refuses two ranks on one GPU: gloo only)
        local = local % torch.cuda.device_count()
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    import contextlib
    from gigapath import runtime, slide_encoder
    with contextlib.redirect_stdout(sys.stderr):       # keep stdout to the one JSON line
        model = slide_encoder.create_model("", ARCH, 1536).to(dev).eval()
    model.validate_positions = True
    if sp:
        model.enable_sequence_parallel()
    # graphs: the whole forward (1 GPU, C5) or, under SP, the per-layer compute segments between
    # the RCCL exchanges (collectives stay eager)
    model.use_hip_graphs = not args.no_graphs
    model.graph_min_uses = 1        # the bench repeats one shape: capture during the warm-up
    if mixed:
        from gigapath import batch
        sizes = batch.mixed_batch_sizes(n_slides=args.mixed_slides)
        slides = []
        for i, n in enumerate(sizes):
            x, coords = make_slide(n, seed=100 + 2 * i)
            slides.append((torch.from_numpy(x[0]).to(dev), torch.from_numpy(coords[0]).to(dev)))
        args.tiles = sum(sizes)

        def step():
            return batch.encode_slides(model, slides, all_layer_embed=True)[0]
    else:
        x, coords = make_slide(args.tiles, seed=1 if sp else 1 + rank)
        xt = torch.from_numpy(x).to(dev)
        ct = torch.from_numpy(coords).to(dev)

        def step():
            return model(xt, ct, all_layer_embed=True)

    monitor = None
    if sp:
        # exchange instrumentation + collective watchdog (seqpar.ExchangeMonitor) on the first warm-up
        # step and the per-kernel timing pass only: it syncs the host at every wait
        from gigapath import seqpar
        monitor = seqpar.ExchangeMonitor(bound_s=float(os.environ.get("GP_SP_WATCHDOG_S", "180")), rank=rank)
        model._sp.set_monitor(monitor)
    with torch.no_grad():
        for i in range(args.warmup):
            step()
            if monitor is not None and i == 0:
                torch.cuda.synchronize(dev)
                model._sp.set_monitor(None)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        # per-kernel timing pass (HIP events around every hot launch, on the launch stream): an
        # eager run of the same workload after the timed region, so the events do not add host
        # work to the timed steps; a kernel's duration does not depend on how it was launched
        runtime.TIMER.reset()
        runtime.TIMER.enabled = True
        if monitor is not None:              # drop the warm-up's records (it included graph capture)
            monitor._pending.clear()
            monitor.records.clear()
            model._sp.set_monitor(monitor)
        for _ in range(args.timing_steps):
            step()
        torch.cuda.synchronize(dev)
        runtime.TIMER.enabled = False
        if monitor is not None:
            model._sp.set_monitor(None)
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    assert all(torch.isfinite(o).all() for o in out)

    kt = runtime.TIMER.totals_ms()
    segs = model.encoder.layers[0].self_attn.args.segment_length
    ratios = model.encoder.layers[0].self_attn.args.dilated_ratio
    L = args.tiles + 1
    att_flops_launch = runtime.attention_valid_flops(L, segs, ratios, 16, 48)
    if mixed:
        # varlen packing: one attention launch per layer covers every slide of this rank
        from gigapath import batch as _b
        mine = _b.lpt_assign([_b.slide_cost(n, segs, ratios) for n in sizes], world)[rank]
        att_flops_launch = sum(runtime.attention_valid_flops(sizes[i] + 1, segs, ratios, 16, 48) for i in mine)
    n_att, ms_att = kt.get("attn", (0, 0.0))
    if sp:          # (the SP engine labels its launches by exchange phase: attn_local / attn_A / attn_B)
        ms_att = sum(v[1] for k, v in kt.items() if k.startswith("attn"))
        # this rank's attention launches cover its query window: price them with its share of the
        # valid FLOPs (two launches per layer: local branches, then exchanged ones)
        plan = model._sp.plan
        a_w, b_w = plan.bounds[rank]
        att_flops_launch = runtime.attention_valid_flops_window(L, segs, ratios, 16, 48, a_w, b_w)
        n_att = args.timing_steps * len(model.encoder.layers)   # per layer: both launches together
    avg_att_s = ms_att / max(n_att, 1) / 1e3
    achieved = att_flops_launch / avg_att_s / 1e12 if avg_att_s > 0 else 0.0
    if mixed:   # whole batch (all ranks)
        total_tf = sum(runtime.gemm_flops(1, n, 768, 3072, 1536, 12)
                       + 12 * runtime.attention_valid_flops(n + 1, segs, ratios, 16, 48) for n in sizes) / 1e12
    else:       # one slide (SP: shared by the ranks; replicas: one per rank)
        total_tf = (runtime.gemm_flops(1, args.tiles, 768, 3072, 1536, 12)
                    + 12 * runtime.attention_valid_flops(L, segs, ratios, 16, 48)) / 1e12
    plain = not (sp or mixed)          # the PMC summary was collected on the plain C3 run
    traffic = pmc_traffic(args.tiles, "dilated_attn32_kernel<48, true, 0,") if plain else None
    # HBM-bound merge kernel: algorithmic bytes per launch over its live launch time
    n_mg, ms_mg = kt.get("merge", (0, 0.0))
    if sp:
        merge_tok = b_w - a_w
    elif mixed:
        merge_tok = sum(sizes[i] + 1 for i in mine)
    else:
        merge_tok = L
    merge_bytes = runtime.merge_bytes(L, segs, ratios, 16, 48) * merge_tok / L
    merge_gbs = merge_bytes / (ms_mg / max(n_mg, 1) / 1e3) / 1e9 if ms_mg > 0 else 0.0
    value = (1 if (sp or mixed) else world) * args.tiles * args.steps / elapsed
    ms_step = elapsed / args.steps * 1e3
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "tiles/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "strong" if (sp or mixed) else "weak",
        "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (PCG64 N(0,1) 1536-d tile embeddings, distinct grid coords; random-init weights)",
        "config": {"workload": ("C5: %s forward of a 32-slide mixed batch (%d tiles, 2k-100k per slide), "
                                "LPT data parallel over %d GPUs, all_layer_embed=True" % (ARCH, args.tiles, world))
                               if mixed else
                               ("%s: %s forward, one %d-tile slide sharded over %d GPUs (sequence parallel), "
                                "all_layer_embed=True" % (config_label(args.tiles, world, sp), ARCH, args.tiles, world))
                               if sp else
                               ("%s: %s forward, one %d-tile slide per GPU, all_layer_embed=True"
                                % (config_label(args.tiles, world, sp), ARCH, args.tiles)),
                   "tiles_per_slide": args.tiles, "slides_per_gpu": (1.0 / world) if sp else 1,
                   "parallelism": ("dp%d-lpt" % world) if mixed else ("sp%d" % world) if sp else ("replica x%d" % world)},
        "roofline": {"bound": "mfma", "kernel": "gp_dilated_attn_fwd", "achieved": round(achieved, 2),
                     "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                     "traffic": traffic, "flops_per_launch": att_flops_launch, "avg_launch_ms": round(avg_att_s * 1e3, 4),
                     "launches": n_att},
        "attn_mfma_util_pct": round(100 * achieved / PEAK_BF16_TFLOPS, 2),
        "merge_roofline": {"bound": "hbm", "kernel": "gp_branch_merge_ln", "achieved": round(merge_gbs, 1),
                           "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(merge_gbs / PEAK_HBM_GBS, 4),
                           "traffic": pmc_traffic(args.tiles, "branch_merge_v3_kernel<5") if plain else None,
                           "bytes_per_launch": merge_bytes},
        "model_tflops": round(total_tf * args.steps * (1 if (sp or mixed) else world) / elapsed, 2),
        "kernel_ms_per_step": {k: round(v[1] / args.timing_steps, 3) for k, v in sorted(kt.items())},
        "launch": "hip-graph replay" if model.use_hip_graphs else "eager",
    }
    if sp:
        result["sp_exchange_mb_per_layer_rank0"] = round(model._sp.plan.exchange_bytes(0) / 1e6, 1)
        # the SP gather (gp_dilated_sparsify_dests): per branch that crosses a cut, read the K and V
        # head-group columns of this rank's tokens (2*C_b bf16 each) and write one row per destination
        # chunk (transfer-free branches are read in place by the attention: no sparsify bytes)
        plan = model._sp.plan
        a_w, b_w = plan.bounds[rank]
        sp_bytes = sum((b_w - a_w) * 2 * plan.C[b] * 2 + sum(plan.send_splits(rank, b)) * 2 * plan.C[b] * 2
                       for b in range(len(plan.C)) if not plan.no_xfer[b])
        n_sp, ms_sp = kt.get("sparsify", (0, 0.0))
        sp_gbs = sp_bytes / (ms_sp / max(n_sp, 1) / 1e3) / 1e9 if ms_sp > 0 else 0.0
        result["sparsify_roofline"] = {"bound": "hbm", "kernel": "gp_dilated_sparsify_dests",
                                       "achieved": round(sp_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                       "frac": round(sp_gbs / PEAK_HBM_GBS, 4), "traffic": None,
                                       "bytes_per_launch": sp_bytes}
        # every rank's view (shard, xGMI bytes, exposed exchange wait, kernel rooflines), gathered
        mine_rep = sp_rank_report(model, kt, rank, args.timing_steps, L, segs, ratios, monitor)
        reps = [None] * world
        dist.all_gather_object(reps, mine_rep)
        result["sp_ranks"] = reps
        result["sp_exchange_exposed_ms_per_layer_max"] = max(
            r["exchange_exposed"]["ms_per_layer"] for r in reps)
        result["sp_transport"] = "rccl" if backend == "nccl" else backend + " (host-staged rehearsal)"
    if world == 1 and plain and args.tiles == 70000 and not args.no_c4_ref:
        # the C4 256k slide on this one GPU, same process: the N > 1 lines shard THIS workload, so their
        # speedup over this line (not over the 70k `value`) is the sequence-parallel scaling
        x4, c4 = make_slide(256000, seed=1)
        x4t, c4t = torch.from_numpy(x4).to(dev), torch.from_numpy(c4).to(dev)
        del x4, c4
        print("bench: C4 256k reference line on this GPU ...", file=sys.stderr, flush=True)
        with torch.no_grad():
            for _ in range(2):
                model(x4t, c4t, all_layer_embed=True)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(3):
                model(x4t, c4t, all_layer_embed=True)
            torch.cuda.synchronize(dev)
            e4 = time.perf_counter() - t0
        result["c4_256k_same_gpu"] = {
            "workload": "C4 slide (256,000 tiles) forward on this one GPU, all_layer_embed=True, HIP-graph replay",
            "tiles_per_s": round(256000 * 3 / e4, 2), "ms_per_step": round(e4 / 3 * 1e3, 3), "steps": 3,
            "note": "the N > 1 lines shard this workload: their speedup over this line is the C4 scaling"}
        del x4t, c4t
    if rank == 0 and not args.no_cpu_baseline:
        threads, usable, ncpu, _ = host_cores()
        threads = args.cpu_threads or threads
        print("bench: CPU baseline on %d threads ..." % threads, file=sys.stderr, flush=True)
        result["cpu_baseline"] = cpu_baseline(args.tiles, threads, total_tflops=total_tf)
        if world == 1 and not mixed and not args.no_cpu_full:
            print("bench: CPU full forwards (C1, C2) ...", file=sys.stderr, flush=True)
            result["cpu_full_forwards"] = cpu_full_forwards([("C1", 1024), ("C2", 16384)], threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if monitor is not None:
        monitor.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
