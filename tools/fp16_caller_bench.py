"""The reference pipeline's caller (pipeline.py:186-187: fp16 tile embeddings under
torch.cuda.amp.autocast(dtype=torch.float16)) timed against the bf16 product path on one slide.

    python tools/fp16_caller_bench.py [--tiles 70000] [--steps 10]

HIP-graph replays of the whole forward (all_layer_embed=True) in both formats, same process, plus one
eager step per format with HIP events around the attention launches.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "prov-gigapath-replication_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gigapath import runtime, slide_encoder  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=70000)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import oracle as orc                       # synthetic slide generator only (bench inputs)
    dev = torch.device("cuda")
    model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536).to(dev).eval()
    model.use_hip_graphs = True
    model.graph_min_uses = 1
    x, coords = orc.synthetic_slide(args.tiles)
    xt, ct = torch.from_numpy(x).to(dev), torch.from_numpy(coords).to(dev)
    flops = runtime.attention_valid_flops(args.tiles + 1, [1024, 5792, 32768, 185363, 1048576],
                                          [1, 2, 4, 8, 16], 16, 48) * 12
    res = {}
    for name, inp, ac in (("bf16", xt, False), ("fp16_autocast", xt.half(), True)):
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16, enabled=ac):
            for _ in range(3):
                model(inp, ct, all_layer_embed=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                model(inp, ct, all_layer_embed=True)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.steps
            runtime.TIMER.reset()
            runtime.TIMER.enabled = True
            model(inp, ct, all_layer_embed=True)
            kt = runtime.TIMER.totals_ms()
            runtime.TIMER.enabled = False
        att = kt.get("attn", (0, 0.0))[1]
        res[name] = {"ms_per_forward": round(ms, 3), "tiles_per_s": round(args.tiles / ms * 1e3, 1),
                     "attn_ms": round(att, 3), "attn_tflops": round(flops / att / 1e9, 1) if att else None,
                     "kernel_ms": {k: round(v[1], 3) for k, v in sorted(kt.items())}}
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
