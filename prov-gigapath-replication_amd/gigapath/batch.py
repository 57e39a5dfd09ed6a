"""Mixed-length slide batches, data parallel over the GPUs of a node.

The reference encodes one slide per call; its fine-tuning collate pads a batch to the longest
slide (finetune/utils.py:63-98), which changes the result (padded tiles are attended to) and is
not the parity target.  Here every slide keeps its own B = 1 forward: with packed=False each
output is bit-identical to encoding the slide alone; the default varlen-packed path matches it up
to the GEMMs' row-count-dependent rounding (same attention and merge math per slide):

* slides are assigned to ranks by LPT (longest processing time first) on the modelled cost of
  a forward (valid attention FLOPs + GEMM FLOPs + row-kernel bytes, seqpar.token_cost), so the
  ranks finish together;
* each rank encodes its slides in descending cost order, inputs already on its device;
* one all-reduce of the [S, n_out, E] result table gives every rank every slide's outputs
  (slides not owned contribute zeros) -- the only collective, after all compute.
"""
from __future__ import annotations

import heapq
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import seqpar


def slide_cost(n_tiles: int, segs: Sequence[int], ratios: Sequence[int], H: int = 16, D: int = 48,
               F: int = 3072) -> float:
    """Modelled seconds of one forward over an n_tiles slide (relative scale is what matters)."""
    return float(seqpar.token_cost(n_tiles + 1, segs, ratios, H, D, F).sum())


def lpt_assign(costs: Sequence[float], world: int) -> List[List[int]]:
    """Longest-processing-time-first assignment: slide indices per rank, each rank's list in
    descending cost order.  Deterministic (ties broken by slide index, then rank)."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    heap = [(0.0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + costs[i], r))
    return out


def pack_groups(sizes: Sequence[int], order: Sequence[int], max_tokens: int) -> List[List[int]]:
    """Split `order` (slide indices) into consecutive groups of at most max_tokens packed tokens
    (N_i + 1 each); a slide larger than the budget forms its own group."""
    groups, cur, tok = [], [], 0
    for i in order:
        L = int(sizes[i]) + 1
        if cur and tok + L > max_tokens:
            groups.append(cur)
            cur, tok = [], 0
        cur.append(i)
        tok += L
    if cur:
        groups.append(cur)
    return groups


def encode_slides(model, slides: Sequence[Tuple[torch.Tensor, torch.Tensor]], all_layer_embed: bool = False,
                  group=None, encode_fn: Optional[Callable] = None, packed: Optional[bool] = None,
                  max_packed_tokens: int = 1 << 21) -> List[List[torch.Tensor]]:
    """Encode a list of (tile_embed [N_i, C] or [1, N_i, C], coords [N_i, 2] or [1, N_i, 2]) slides.

    Single process: every slide of this rank in one varlen-packed forward (model.forward_packed:
    per-token work over all slides' rows at once, one attention and one merge launch per layer
    with per-slide segment tables; groups of at most max_packed_tokens tokens), or, with
    packed=False or a custom encode_fn, sequential B = 1 forwards.  Under torch.distributed (one process per GPU,
    every rank passing the same list): LPT-sharded across the ranks of `group`, results
    all-reduced so every rank returns every slide's outputs.  Returns, per slide, the list the
    model's forward returns (1 or 1 + depth tensors of [1, E]).

    With ``model.use_hip_graphs`` each forward (packed group or slide) is a replay of its captured
    graph, one after another on one stream: replaying graphs of different slides concurrently on
    several streams hung the GPU on MI355X (32 slides over 4 streams; GEMM kernels that assume
    their workgroups are co-resident are the suspect) -- packing is the cross-slide batching."""
    import torch.distributed as dist
    if getattr(model, "_sp", None) is not None:
        raise ValueError("encode_slides is data parallel: call model.disable_sequence_parallel() first")
    if packed is None:
        packed = encode_fn is None and hasattr(model, "forward_packed")
    encode_fn = encode_fn or (lambda x, c: model(x, c, all_layer_embed=all_layer_embed))
    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if dist_on else 1
    rank = dist.get_rank(group) if dist_on else 0
    args = model.encoder.args
    segs, ratios = list(args.segment_length), list(args.dilated_ratio)
    sizes = [int(x.shape[-2]) for x, _ in slides]
    plan = lpt_assign([slide_cost(n, segs, ratios) for n in sizes], world)
    mine = plan[rank]
    n_out = (1 + len(model.encoder.layers)) if all_layer_embed else 1
    E = model.embed_dim
    dev = model.cls_token.device
    table = torch.zeros(len(slides), n_out, E, dtype=torch.float32, device=dev)

    def shaped(i):
        x, c = slides[i]
        x = x if x.dim() == 3 else x.unsqueeze(0)
        c = c if c.dim() == 3 else c.unsqueeze(0)
        return x, (c if c.dtype in (torch.float32, torch.float64) else c.float())

    with torch.no_grad():
        if packed:
            for grp in pack_groups(sizes, mine, max_packed_tokens):
                outs = model.forward_packed([slides[i] for i in grp], all_layer_embed)
                for i, o in zip(grp, outs):
                    table[i] = torch.stack([t.reshape(E).float() for t in o])
        else:
            for i in mine:
                x, c = shaped(i)
                outs = encode_fn(x, c)
                table[i] = torch.stack([o.reshape(E).float() for o in outs])
    if world > 1:
        if dist.get_backend(group) == "nccl" or not table.is_cuda:
            dist.all_reduce(table, group=group)
        else:
            h = table.cpu()
            dist.all_reduce(h, group=group)
            table.copy_(h)
    out_dtype = model.norm.weight.dtype
    return [[table[i, k:k + 1].to(out_dtype) for k in range(n_out)] for i in range(len(slides))]


def mixed_batch_sizes(n_slides: int = 32, lo: int = 2000, hi: int = 100000, seed: int = 3) -> List[int]:
    """C5's slide sizes: N_i = round(exp(U(ln lo, ln hi))) from PCG64(seed)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return [int(round(float(np.exp(u)))) for u in rng.uniform(np.log(lo), np.log(hi), n_slides)]

