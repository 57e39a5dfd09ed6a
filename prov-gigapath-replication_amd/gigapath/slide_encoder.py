"""Prov-GigaPath slide encoder — MI355X drop-in for ``gigapath.slide_encoder``.

Same public surface as the reference (gigapath/slide_encoder.py:32-270): ``PatchEmbed``,
``LongNetViT`` (constructor kwargs, ``forward(x, coords, all_layer_embed=False) -> list``,
``coords_to_pos``, ``get_optimal_segment_length``), ``create_model(pretrained, model_arch,
in_chans, local_dir, **kwargs)`` and the three registered architectures, with the same
247-key state dict.  The forward is inference-only and runs on a ROCm device:

    patch GEMM (hipBLASLt) -> gp_coords_to_pos -> gp_posembed_cls_ln (pos add + CLS + LN1)
    -> 12 x LongNet layer (runtime.EncoderEngine) -> LN readouts (gp_layernorm_f32 /
    gp_mean_tokens)

The 3.07 GB fp32 ``pos_embed`` buffer of the reference is replaced by its exact [G, E/2]
factor (see pos_embed.py); ``model.pos_embed`` is still available, built lazily on the CPU.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from functools import partial
from typing import Dict, List

import numpy as np
import torch
import torch.nn as nn

from . import _hip, runtime
from .pos_embed import axis_table, get_2d_sincos_pos_embed
from .torchscale.model.LongNet import make_longnet_from_name

_REGISTRY: Dict[str, callable] = {}


def register_model(fn):
    _REGISTRY[fn.__name__] = fn
    return fn


def list_models() -> List[str]:
    return sorted(_REGISTRY)


class PatchEmbed(nn.Module):
    """Slide patch embedding: Linear(in_chans -> embed_dim) (+ optional norm)."""

    def __init__(self, in_chans=1536, embed_dim=768, norm_layer=None, bias=True):
        super().__init__()
        self.proj = nn.Linear(in_chans, embed_dim, bias=bias)
        self.norm = norm_layer(embed_dim) if norm_layer else nn.Identity()

    def forward(self, x):
        if not isinstance(self.norm, nn.Identity):
            raise NotImplementedError("PatchEmbed norm is not used by the registered slide encoders")
        dev = x.device
        if dev.type != "cuda":
            raise RuntimeError("PatchEmbed (MI355X path) needs ROCm device tensors")
        B, L, C = x.shape
        act = runtime.call_act_dtype(self)
        with torch.autocast("cuda", enabled=False):
            y = torch.addmm(self.proj.bias.to(dev, act), x.reshape(B * L, C).to(act), self.proj.weight.to(dev, act).t())
        return y.view(B, L, -1).to(x.dtype)


class LongNetViT(nn.Module):
    """LongNet slide encoder backbone (reference gigapath/slide_encoder.py:54-223)."""

    def __init__(self, in_chans=1536, embed_dim=256, depth=12, slide_ngrids=1000, tile_size=256,
                 max_wsi_size=262144, norm_layer=nn.LayerNorm, global_pool=False, dropout=0.25,
                 drop_path_rate=0.1, **kwargs):
        super().__init__()
        self.patch_embed = PatchEmbed(in_chans, embed_dim)
        self.tile_size = tile_size
        self.slide_ngrids = slide_ngrids
        self.embed_dim = embed_dim
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.encoder_name = "LongNet_{}_layers_{}_dim".format(depth, embed_dim)
        if kwargs.get("mlp_ratio", 4.0) != 4.0:
            self.encoder_name += "_mlp{}".format(kwargs.get("mlp_ratio"))
        segment_length = self.get_optimal_segment_length(max_wsi_size, tile_size)
        self.encoder = make_longnet_from_name(self.encoder_name, drop_path_rate=drop_path_rate, dropout=dropout,
                                              segment_length=segment_length)
        self.norm = norm_layer(embed_dim)
        self.global_pool = global_pool
        self.validate_positions = True      # raise IndexError on out-of-range coords like the reference
        print("Global Pooling:", self.global_pool)
        self._top_sig = None
        self._top = None
        self._pos_full = None
        self._sp = None
        # HIP graphs: the whole single-device forward as one replay per input shape.  A graph keeps
        # its shape's workspace alive (~2 GB at 100k tiles, ~5 GB at 256k), so the cache is an LRU
        # bounded by entries AND bytes; a shape is captured only once it has been seen
        # graph_min_uses times (real slide sizes rarely repeat: a one-off slide runs eagerly instead of
        # paying an eager warm-up + capture it never replays); graphs of superseded weights are dropped
        self.use_hip_graphs = False
        self.max_hip_graphs = 16
        self.hip_graph_max_bytes = 48 << 30
        self.graph_min_uses = 2
        self._graphs = OrderedDict()
        self._graph_ws = {}
        self._graph_bytes = {}
        self._graph_seen = {}
        self._capture_streams = OrderedDict()
        self.max_capture_streams = 8
        self.initialize_vit_weights()

    # ---------------------------------------------------------------- sequence parallel
    def enable_sequence_parallel(self, group=None):
        """Shard every forward's tokens across the ranks of `group` (one process per GPU,
        torch.distributed initialised; RCCL for device transfers).  Every rank calls forward with
        the same full slide and gets the same outputs (seqpar.py)."""
        from . import seqpar
        self._sp = seqpar.SeqParallelContext(group)
        return self

    def disable_sequence_parallel(self):
        self._sp = None
        return self

    # ---------------------------------------------------------------- init / helpers
    def initialize_vit_weights(self):
        w = self.patch_embed.proj.weight.data
        torch.nn.init.xavier_uniform_(w.view([w.shape[0], -1]))
        torch.nn.init.normal_(self.cls_token, std=0.02)
        self.apply(self._init_weights)

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            torch.nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def get_optimal_segment_length(self, max_wsi_size: int = 262144, tile_size: int = 256) -> str:
        """Five segment lengths 2**linspace(10, log2((max_wsi/tile)^2), 5) (reference :137-154),
        rendered with plain ints (the reference's str(list(np.int64)) breaks under numpy>=2)."""
        max_seq_len = (max_wsi_size // tile_size) ** 2
        seg = np.power(2, np.linspace(np.log2(1024), int(np.log2(max_seq_len)), 5)).astype(int)
        return str([int(v) for v in seg])

    @property
    def pos_embed(self) -> torch.Tensor:
        """The reference's [1, G*G+1, E] fp32 table (3.07 GB at G=1000), built lazily on the CPU.
        The forward never uses it."""
        if self._pos_full is None:
            self._pos_full = torch.from_numpy(
                get_2d_sincos_pos_embed(self.embed_dim, self.slide_ngrids, cls_token=True)).float().unsqueeze(0)
        return self._pos_full

    def coords_to_pos(self, coords, tile_size: int = 256):
        """[B, N, 2] pixel coordinates -> [B, N] int64 flat pos-embed rows (reference :166-179)."""
        if coords.device.type != "cuda":
            raise RuntimeError("coords_to_pos (MI355X path) needs ROCm device tensors")
        c = coords if coords.dtype in (torch.float32, torch.float64) else coords.float()
        c = c.contiguous()
        pos = torch.empty(c.shape[:-1], dtype=torch.int64, device=c.device)
        _hip.coords_to_pos(c, self.slide_ngrids, tile_size, pos, None)
        return pos

    def _packed_top(self, dev):
        mods = (self.patch_embed, self.norm, self.encoder.layer_norm, self.encoder.layers[0].self_attn_layer_norm)
        sig = (str(dev), self.cls_token.data_ptr(), self.cls_token._version,
               tuple(runtime.param_signature(m) for m in mods))
        if sig != self._top_sig:
            f32 = runtime._f32
            ln1 = self.encoder.layers[0].self_attn_layer_norm
            self._top = dict(
                patch={},              # act -> (patch weight, patch bias) in that 16-bit format
                cls=f32(self.cls_token.reshape(-1), dev),
                tab=torch.from_numpy(axis_table(self.embed_dim, self.slide_ngrids)).to(dev),
                ln1_w=f32(ln1.weight, dev), ln1_b=f32(ln1.bias, dev), ln1_eps=float(ln1.eps),
                enc_w=f32(self.encoder.layer_norm.weight, dev), enc_b=f32(self.encoder.layer_norm.bias, dev),
                enc_eps=float(self.encoder.layer_norm.eps),
                norm_w=f32(self.norm.weight, dev), norm_b=f32(self.norm.bias, dev), norm_eps=float(self.norm.eps))
            self._top_sig = sig
        return self._top

    def _patch_gemm(self, top, x2d, out, gemm_ws=None):
        """out = x2d . Wp^T + bp in the call's activation format (runtime.linear: gp_linear or hipBLASLt,
        bias in the epilogue either way)."""
        act = out.dtype
        if act not in top["patch"]:
            dev = out.device
            bp = runtime._act(self.patch_embed.proj.bias, dev, act)
            top["patch"][act] = (runtime._act(self.patch_embed.proj.weight, dev, act), bp, bp.float().contiguous())
        wp, bp, bpf = top["patch"][act]
        with runtime.TIMER.span("gemm_patch"):
            runtime.linear(x2d.to(act), wp, bp, bpf, out, gemm_ws)

    # ---------------------------------------------------------------- forward
    @runtime.compute_format
    def forward(self, x, coords, all_layer_embed=False):
        """x [B, N, in_chans], coords [B, N, 2] (pixels) -> list of [B, E] slide embeddings:
        1 (final, after encoder.layer_norm) or, with all_layer_embed, 1 + depth (embedding and
        every layer output, before encoder.layer_norm), each through self.norm; CLS row, or the
        mean over tiles when global_pool (reference :181-223, encoder.py:360-388)."""
        self.encoder.check_eval()
        dev = self.cls_token.device
        if dev.type != "cuda" or x.device != dev or coords.device != dev:
            raise RuntimeError("LongNetViT (MI355X path): model, x and coords must be on the same ROCm device "
                               "(model %s, x %s, coords %s)" % (dev, x.device, coords.device))
        B, N, C = x.shape
        if coords.shape != (B, N, 2):
            raise ValueError("coords must be [B, N, 2], got %s" % (tuple(coords.shape),))
        if self._sp is not None and self._sp.world > 1:
            return self._forward_sp(x, coords, all_layer_embed)
        if self.use_hip_graphs and not runtime.TIMER.enabled:
            return self._forward_graphed(x, coords, all_layer_embed)
        return self._forward_device(x, coords, all_layer_embed, self.validate_positions)

    def _forward_graphed(self, x, coords, all_layer_embed):
        """Replay of a HIP graph holding the whole forward (~170 launches) for this input shape:
        captured on first use per (shape, dtypes, options, weights version), inputs copied into the
        graph's static buffers, outputs cloned out.  Coordinates are validated eagerly first (one
        small kernel + one sync, as in the eager path)."""
        c = coords if coords.dtype in (torch.float32, torch.float64) else coords.float()
        if self.validate_positions:
            self.check_positions([c])
        ent = self.graph_entry(x, c, all_layer_embed)
        if ent is None:                          # shape not (yet) worth a capture
            return self._forward_device(x, coords, all_layer_embed, False)
        graph, sx, sc, outs = ent
        sx.copy_(x)
        sc.copy_(c)
        runtime.replay_graph(graph)
        return self._clone_outputs(outs)

    @staticmethod
    def _clone_outputs(outs):
        """Copies of the graph's static outputs.  The readouts are views of one [n_out, B, E] table: one
        copy of the table (one copy launch instead of 13 for all_layer_embed) and the same views into it."""
        base = outs[0]._base if outs else None
        if base is not None and base.is_contiguous() and all(o._base is base for o in outs):
            nb = base.clone()
            off = base.storage_offset()
            return [nb.as_strided(o.size(), o.stride(), o.storage_offset() - off) for o in outs]
        return [o.clone() for o in outs]

    def check_positions(self, coords_list):
        """Raise IndexError if any tile of any slide maps outside pos_embed (reference :200 indexing);
        one small kernel per slide, one host sync for all of them."""
        dev = self.cls_token.device
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        for c in coords_list:
            pos = torch.empty(c.numel() // 2, dtype=torch.int64, device=dev)
            _hip.coords_to_pos(c.contiguous(), self.slide_ngrids, self.tile_size, pos, err)
        if int(err.item()) > 0:
            raise IndexError("coords map outside pos_embed (%d rows): %d tiles" %
                             (self.slide_ngrids ** 2 + 1, int(err.item())))

    def graph_stream(self):
        """The side stream graphs are captured on: one per (device, CALLER stream).  A captured GEMM
        bakes the hipBLASLt workspace of the stream it was captured on (PyTorch keeps one per
        (handle, stream): ATen/cuda/CUDAContextLight.h cublaslt_handle_stream_to_workspace) and the
        engine's activation workspace of that stream, so graphs of different caller streams never
        share either and may replay concurrently; graphs of one caller stream replay in its order."""
        dev = self.cls_token.device
        key = (str(dev), int(torch.cuda.current_stream(dev).cuda_stream))
        if key not in self._capture_streams:
            # LRU-bounded: a captured graph replays on whatever stream calls it, so an evicted capture
            # stream costs only a new stream object at the next capture from that caller stream
            while len(self._capture_streams) >= self.max_capture_streams:
                self._capture_streams.pop(next(iter(self._capture_streams)))
            self._capture_streams[key] = torch.cuda.Stream(device=dev)
        self._capture_streams.move_to_end(key)
        return self._capture_streams[key]

    def graph_entry(self, x, c, all_layer_embed):
        """(graph, static x, static coords, static outputs) for this input shape, captured if not
        cached and seen graph_min_uses times; None while the shape should run eagerly.  No
        validation, no replay."""
        dev = self.cls_token.device
        self._packed_top(dev)
        self.encoder.engine.pack(self.encoder, dev)
        key = (str(dev), int(torch.cuda.current_stream(dev).cuda_stream), tuple(x.shape), x.dtype, c.dtype,
               runtime.act_dtype(), bool(all_layer_embed), bool(self.global_pool), self._top_sig,
               self.encoder.engine._sig)
        ent = self._graph_lookup(key)
        if ent is None and self._graph_wanted(key):
            ent = self._capture(key, x, c, lambda sx, sc: self._forward_device(sx, sc, all_layer_embed, False),
                                lambda st: self.encoder.engine.stream_workspace(st, packed=False))
        return ent

    def _graph_lookup(self, key):
        ent = self._graphs.get(key)
        if ent is not None:
            self._graphs.move_to_end(key)       # LRU
        return ent

    def _graph_wanted(self, key) -> bool:
        """Count a miss; True once the shape has been seen graph_min_uses times."""
        if len(self._graph_seen) > 4096:
            self._graph_seen.clear()
        n = self._graph_seen.get(key, 0) + 1
        self._graph_seen[key] = n
        return n >= self.graph_min_uses

    def _drop_graph(self, key):
        self._graphs.pop(key, None)
        self._graph_ws.pop(key, None)
        self._graph_bytes.pop(key, None)

    @staticmethod
    def _tensor_bytes(obj, seen=None) -> int:
        """Device bytes held by the tensors of a workspace object (recursing into lists / scratch)."""
        seen = set() if seen is None else seen
        tot = 0
        items = obj.__dict__.values() if hasattr(obj, "__dict__") else obj
        for v in items:
            if isinstance(v, torch.Tensor):
                if v.is_cuda and v.data_ptr() not in seen:
                    seen.add(v.data_ptr())
                    tot += v.untyped_storage().nbytes()
            elif isinstance(v, (list, tuple)) or hasattr(v, "outs"):
                tot += LongNetViT._tensor_bytes(v, seen)
        return tot

    @staticmethod
    def _tensors_of(obj, seen=None):
        """Every CUDA tensor reachable from a workspace object / list / tuple (once each)."""
        seen = set() if seen is None else seen
        if isinstance(obj, torch.Tensor):
            if obj.is_cuda and id(obj) not in seen:
                seen.add(id(obj))
                yield obj
            return
        if obj is None or isinstance(obj, (int, float, str, bool)) or id(obj) in seen:
            return
        seen.add(id(obj))
        items = obj if isinstance(obj, (list, tuple)) else (obj.__dict__.values() if hasattr(obj, "__dict__") else ())
        for v in items:
            yield from LongNetViT._tensors_of(v, seen)

    @staticmethod
    def _weights_sig(key):
        """(top weights signature, encoder (device, param_signature)) of a graph key, whose last two
        entries are self._top_sig and EncoderEngine._sig = (device, param_signature, act)."""
        eng = key[-1]
        return key[-2], (tuple(eng[:2]) if isinstance(eng, tuple) else eng)

    def _capture(self, key, x, c, run, workspace):
        """Capture run(static_x, static_coords) -> outputs on the side stream (after one eager
        warm-up run there: allocations, TunableOp lookups) and cache it under `key`, keeping the
        workspace the graph bakes in (workspace(capture stream): the one the captured run itself used,
        not whichever the engine used last) alive with it."""
        # superseded weights never replay: drop graphs whose (top, encoder) WEIGHT signatures differ.
        # The encoder signature's activation format is left out of that comparison (it stays in the
        # lookup key): a bf16 and an fp16 caller each keep their graphs, as pack() keeps one packing
        # per format
        sig = self._weights_sig(key)
        for old in [k for k in self._graphs if self._weights_sig(k) != sig]:
            self._drop_graph(old)
        stream = self.graph_stream()
        # the static input is kept in the activation format (the forward's first use converts to it
        # anyway): the per-replay sx.copy_(x) then converts while copying, instead of a full-precision
        # copy plus a conversion pass inside the graph (one 0.86 GB HBM round trip fewer at 70k tiles)
        sx, sc = x.detach().to(runtime.act_dtype(), copy=True).contiguous(), c.detach().clone().contiguous()
        cur = torch.cuda.current_stream()
        stream.wait_stream(cur)
        with torch.cuda.stream(stream):
            run(sx, sc)
        graph = torch.cuda.CUDAGraph()
        n_blaslt = runtime.BLASLT_ISSUED[0]
        with torch.cuda.graph(graph, stream=stream, capture_error_mode="thread_local"):
            outs = run(sx, sc)
        # a graph with hipBLASLt GEMMs in it replays in the device's hipBLASLt event chain (runtime.replay_graph)
        graph.gp_blaslt = runtime.capture_uses_blaslt(n_blaslt)
        cur.wait_stream(stream)
        # the graph bakes this shape's workspace: keep it alive with the graph (and ONLY with it: the
        # engine forgets it, so evicting the graph frees it); evict least recently used graphs beyond
        # the entry and byte budgets
        ws = workspace(stream)
        if ws is None:
            raise RuntimeError("HIP graph capture: no engine workspace recorded for the capture stream")
        self.encoder.engine.detach_workspace(ws)
        # The workspace was allocated on the capture stream, but the graph replays on the caller stream
        # `cur` (part of the key).  The caching allocator orders a freed block's reuse only against its
        # allocation stream, so without this, dropping the graph (LRU eviction, new weights) while a replay
        # is still queued on `cur` could hand its memory to another allocation.  record_stream
        # makes each block's free wait for the work queued on `cur` at that moment.
        for t in self._tensors_of((ws, sx, sc, outs)):
            t.record_stream(cur)
        nbytes = self._tensor_bytes(ws) + sx.untyped_storage().nbytes() + sc.untyped_storage().nbytes()
        while self._graphs and (len(self._graphs) >= self.max_hip_graphs or
                                sum(self._graph_bytes.values()) + nbytes > self.hip_graph_max_bytes):
            self._drop_graph(next(iter(self._graphs)))
        ent = (graph, sx, sc, outs)
        self._graphs[key] = ent
        self._graph_ws[key] = ws
        self._graph_bytes[key] = nbytes
        return ent

    # ---------------------------------------------------------------- varlen packing (C5)
    @runtime.compute_format
    def forward_packed(self, slides, all_layer_embed=False):
        """Several slides in ONE forward (config C5 "varlen segment packing").

        slides: [(x_i [N_i, C] or [1, N_i, C], coords_i [N_i, 2] or [1, N_i, 2]), ...].  The tokens
        of all slides are packed into T = sum(N_i + 1) rows (each slide's CLS first); every
        per-token op (GEMMs, LNs, GELU, residuals) runs once over the T rows, and the dilated
        attention and branch merge run as one varlen launch each in which every slide keeps its
        own segment schedule (s = min(sl, L_i), no cross-slide attention).  Each slide's outputs
        are therefore those of its own B = 1 forward (up to the GEMMs' row-count-dependent
        rounding).  Returns one output list per slide, as forward(x_i[None], c_i[None])."""
        self.encoder.check_eval()
        dev = self.cls_token.device
        xs, cs = [], []
        for x, c in slides:
            x = x[0] if x.dim() == 3 else x
            c = c[0] if c.dim() == 3 else c
            if x.device != dev or c.device != dev:
                raise RuntimeError("forward_packed: slides must be on the model's device %s" % dev)
            if c.shape != (x.shape[0], 2):
                raise ValueError("forward_packed: coords must be [N, 2] per slide")
            xs.append(x)
            cs.append(c if c.dtype in (torch.float32, torch.float64) else c.float())
        if not xs:
            return []
        if self._sp is not None and self._sp.world > 1:
            raise ValueError("forward_packed is single-device: disable sequence parallelism first")
        if self.encoder.layers[0].self_attn.head_dim != 48 or len({c.dtype for c in cs}) != 1 or \
                len({x.dtype for x in xs}) != 1:
            # the varlen kernels cover D = 48 (the 12L768d arch): other archs run slide by slide
            return [self.forward(x[None], c[None], all_layer_embed) for x, c in zip(xs, cs)]
        Ns = tuple(int(x.shape[0]) for x in xs)
        x_cat = torch.cat(xs, 0)
        c_cat = torch.cat(cs, 0)
        if self.validate_positions:
            self.check_positions([c_cat])
        if self.use_hip_graphs and not runtime.TIMER.enabled:
            self._packed_top(dev)
            self.encoder.engine.pack(self.encoder, dev)
            key = ("packed", str(dev), int(torch.cuda.current_stream(dev).cuda_stream), Ns, x_cat.dtype,
                   c_cat.dtype, runtime.act_dtype(), bool(all_layer_embed), bool(self.global_pool),
                   self._top_sig, self.encoder.engine._sig)
            ent = self._graph_lookup(key)
            if ent is None and self._graph_wanted(key):
                ent = self._capture(key, x_cat, c_cat,
                                    lambda sx, sc: self._forward_packed_device(sx, sc, Ns, all_layer_embed),
                                    lambda st: self.encoder.engine.stream_workspace(st, packed=True))
            if ent is None:
                res = self._forward_packed_device(x_cat, c_cat, Ns, all_layer_embed)
            else:
                graph, sx, sc, res = ent
                sx.copy_(x_cat)
                sc.copy_(c_cat)
                runtime.replay_graph(graph)
                res = res.clone()
        else:
            res = self._forward_packed_device(x_cat, c_cat, Ns, all_layer_embed)
        out_dtype = self.norm.weight.dtype
        return [[res[k, i:i + 1].to(out_dtype) for k in range(res.shape[0])] for i in range(len(Ns))]

    def _forward_packed_device(self, x_cat, c_cat, Ns, all_layer_embed):
        """Eager packed forward (captured as is by forward_packed): x_cat [sum N_i, C], c_cat
        [sum N_i, 2] -> [n_out, S, E] fp32."""
        dev = self.cls_token.device
        E, S = self.embed_dim, len(Ns)
        Ls = [n + 1 for n in Ns]
        top = self._packed_top(dev)
        eng = self.encoder.engine
        layers = eng.pack(self.encoder, dev)
        pa = layers[0].attn
        ws = eng.workspace_packed(dev, Ls, E, self.encoder.args.encoder_ffn_embed_dim, pa.H, pa.segs, pa.ratios)
        Nt, T = int(sum(Ns)), int(sum(Ls))
        if not hasattr(ws, "pos"):
            ws.pos = torch.empty(Nt, dtype=torch.int64, device=dev)
        xp = ws.y[:Nt]
        self._patch_gemm(top, x_cat, xp, ws.gemm_ws)
        _hip.coords_to_pos(c_cat.contiguous(), self.slide_ngrids, self.tile_size, ws.pos, None)
        with runtime.TIMER.span("posembed"):
            n0 = 0
            for i, n in enumerate(Ns):            # slide i's CLS + tiles -> packed rows tok_off[i] ..
                t0 = ws.tok_off[i]
                _hip.posembed_cls_ln(xp[n0:n0 + n], ws.pos[n0:n0 + n], top["tab"], top["cls"], 1, n, E,
                                     self.slide_ngrids, top["ln1_w"], top["ln1_b"], top["ln1_eps"],
                                     ws.x[t0:t0 + n + 1], ws.a[t0:t0 + n + 1], ws.shift[0, t0:t0 + n + 1])
                n0 += n
        n_out = (1 + len(layers)) if all_layer_embed else 1
        res = torch.empty(n_out, S, E, dtype=torch.float32, device=dev)
        pool = torch.empty(S, E, dtype=torch.float32, device=dev)

        def readout(slot: int):
            if self.global_pool:
                for i, L in enumerate(Ls):
                    t0 = ws.tok_off[i]
                    _hip.mean_tokens(ws.x[t0:t0 + L], 1, L, E, 1, pool[i:i + 1])
            else:
                torch.index_select(ws.x, 0, ws.cls_idx, out=pool)
            _hip.layernorm_f32(pool, E, top["norm_w"], top["norm_b"], top["norm_eps"], res[slot], S, E)

        if all_layer_embed:
            readout(0)
        eng.run_layers(ws, 1, T, readout if all_layer_embed else None, shift_ready=True)
        if not all_layer_embed:
            if self.global_pool:
                _hip.layernorm_f32(ws.x, E, top["enc_w"], top["enc_b"], top["enc_eps"], ws.x, T, E)
                readout(0)
            else:
                cls_rows = torch.index_select(ws.x, 0, ws.cls_idx)
                _hip.layernorm_f32(cls_rows, E, top["enc_w"], top["enc_b"], top["enc_eps"], cls_rows, S, E)
                _hip.layernorm_f32(cls_rows, E, top["norm_w"], top["norm_b"], top["norm_eps"], res[0], S, E)
        return res

    def _forward_device(self, x, coords, all_layer_embed, validate):
        """The eager forward: every launch on the current stream (captured as is by _capture)."""
        dev = self.cls_token.device
        B, N, C = x.shape
        E, L, M = self.embed_dim, N + 1, B * (N + 1)
        top = self._packed_top(dev)
        eng = self.encoder.engine
        layers = eng.pack(self.encoder, dev)
        pa = layers[0].attn
        ws = eng.workspace(dev, B, L, E, self.encoder.args.encoder_ffn_embed_dim, pa.H, pa.segs, pa.ratios)
        if not hasattr(ws, "pos") or ws.pos.numel() != B * N:
            ws.pos = torch.empty(B * N, dtype=torch.int64, device=dev)
            ws.err = torch.zeros(1, dtype=torch.int32, device=dev)

        # patch embedding (bias epilogue) into the spare 16-bit buffer
        xp = ws.y[:B * N]
        self._patch_gemm(top, x.reshape(B * N, C), xp, ws.gemm_ws)
        c = coords if coords.dtype in (torch.float32, torch.float64) else coords.float()
        ws.err.zero_()
        _hip.coords_to_pos(c.contiguous(), self.slide_ngrids, self.tile_size, ws.pos, ws.err)
        if validate and int(ws.err.item()) > 0:
            raise IndexError("coords map outside pos_embed (%d rows): %d tiles" %
                             (self.slide_ngrids ** 2 + 1, int(ws.err.item())))
        with runtime.TIMER.span("posembed"):
            _hip.posembed_cls_ln(xp, ws.pos, top["tab"], top["cls"], B, N, E, self.slide_ngrids, top["ln1_w"],
                                 top["ln1_b"], top["ln1_eps"], ws.x, ws.a, ws.shift[0])

        n_out = (1 + len(layers)) if all_layer_embed else 1
        res = torch.empty(n_out, B, E, dtype=torch.float32, device=dev)
        pool = torch.empty(B, E, dtype=torch.float32, device=dev) if self.global_pool else None

        def readout(slot: int):
            if self.global_pool:
                _hip.mean_tokens(ws.x, B, L, E, 1, pool)
                _hip.layernorm_f32(pool, E, top["norm_w"], top["norm_b"], top["norm_eps"], res[slot], B, E)
            else:
                _hip.layernorm_f32(ws.x, L * E, top["norm_w"], top["norm_b"], top["norm_eps"], res[slot], B, E)

        if all_layer_embed:
            readout(0)
        eng.run_layers(ws, B, L, readout if all_layer_embed else None, shift_ready=True)
        if not all_layer_embed:
            if self.global_pool:
                _hip.layernorm_f32(ws.x, E, top["enc_w"], top["enc_b"], top["enc_eps"], ws.x, M, E)
                readout(0)
            else:
                cls_rows = torch.empty(B, E, dtype=torch.float32, device=dev)
                _hip.layernorm_f32(ws.x, L * E, top["enc_w"], top["enc_b"], top["enc_eps"], cls_rows, B, E)
                _hip.layernorm_f32(cls_rows, E, top["norm_w"], top["norm_b"], top["norm_eps"], res[0], B, E)
        out_dtype = self.norm.weight.dtype
        return [res[i].to(out_dtype) for i in range(n_out)]


    def _forward_sp(self, x, coords, all_layer_embed):
        """Sequence-parallel forward of one slide (B = 1): this rank embeds and encodes tokens
        [a, b) and exchanges sparsified K/V per layer; rank 0 reads out the CLS row (global pool:
        all-reduced token sums) and broadcasts the result."""
        sp = self._sp
        B, N, C = x.shape
        if B != 1:
            raise ValueError("sequence parallel forward takes one slide (B = 1), got B = %d" % B)
        dev = self.cls_token.device
        E, L = self.embed_dim, N + 1
        top = self._packed_top(dev)
        eng = self.encoder.engine
        layers = eng.pack(self.encoder, dev)
        pa = layers[0].attn
        F = self.encoder.args.encoder_ffn_embed_dim
        plan, ws, spe = sp.prepare(dev, L, pa.segs, pa.ratios, pa.H, pa.D, F, runtime.act_dtype())
        spe.use_graphs = self.use_hip_graphs
        a, e = plan.bounds[sp.rank]
        t0, t1 = max(a, 1) - 1, e - 1                      # tiles of this shard (token = tile + 1)
        nt = t1 - t0
        if not hasattr(ws, "pos") or ws.pos.numel() != nt:
            ws.pos = torch.empty(max(nt, 1), dtype=torch.int64, device=dev)
            ws.err = torch.zeros(1, dtype=torch.int32, device=dev)
        xp = ws.y[:nt]
        if nt > 0:
            self._patch_gemm(top, x[0, t0:t1], xp, ws.gemm_ws)
        c = coords if coords.dtype in (torch.float32, torch.float64) else coords.float()
        ws.err.zero_()
        if nt > 0:
            _hip.coords_to_pos(c[0, t0:t1].contiguous(), self.slide_ngrids, self.tile_size, ws.pos[:nt], ws.err)
        if self.validate_positions:
            err = sp.exchange.all_reduce_(ws.err.clone())
            if int(err.item()) > 0:
                raise IndexError("coords map outside pos_embed (%d rows): %d tiles" %
                                 (self.slide_ngrids ** 2 + 1, int(err.item())))
        with runtime.TIMER.span("posembed"):
            _hip.posembed_cls_ln(xp, ws.pos, top["tab"], top["cls"] if a == 0 else None, 1, nt, E, self.slide_ngrids,
                                 top["ln1_w"], top["ln1_b"], top["ln1_eps"], ws.x, ws.a, ws.shift[0])
        n_out = (1 + len(layers)) if all_layer_embed else 1
        res = torch.zeros(n_out, 1, E, dtype=torch.float32, device=dev)
        pool = torch.empty(1, E, dtype=torch.float32, device=dev)

        def pooled(src):
            """mean over tiles 1..L-1 of src (this shard's [n, E] rows), all-reduced."""
            start = 1 if a == 0 else 0
            if ws.n > start:
                _hip.mean_tokens(src, 1, ws.n, E, start, pool)
                pool.mul_(float(ws.n - start))
            else:
                pool.zero_()
            sp.exchange.all_reduce_(pool)
            pool.div_(float(L - 1))
            return pool

        def readout(slot: int):
            if self.global_pool:
                _hip.layernorm_f32(pooled(ws.x), E, top["norm_w"], top["norm_b"], top["norm_eps"], res[slot], 1, E)
            elif a == 0:
                _hip.layernorm_f32(ws.x, E, top["norm_w"], top["norm_b"], top["norm_eps"], res[slot], 1, E)

        if all_layer_embed:
            readout(0)
        spe.run_layers(layers, ws, readout if all_layer_embed else None, weights_sig=eng._sig, shift_ready=True)
        if not all_layer_embed:
            if self.global_pool:
                _hip.layernorm_f32(ws.x, E, top["enc_w"], top["enc_b"], top["enc_eps"], ws.x, ws.n, E)
                readout(0)
            elif a == 0:
                cls_rows = torch.empty(1, E, dtype=torch.float32, device=dev)
                _hip.layernorm_f32(ws.x, E, top["enc_w"], top["enc_b"], top["enc_eps"], cls_rows, 1, E)
                _hip.layernorm_f32(cls_rows, E, top["norm_w"], top["norm_b"], top["norm_eps"], res[0], 1, E)
        if not self.global_pool:
            sp.exchange.broadcast_(res, 0)
        out_dtype = self.norm.weight.dtype
        return [res[i].to(out_dtype) for i in range(n_out)]


def create_model(pretrained: str, model_arch: str, in_chans: int,
                 local_dir: str = os.path.join(os.path.expanduser("~"), ".cache/"), **kwargs):
    """Build a registered slide encoder and (optionally) load ``{"model": state_dict}`` weights
    with strict=False semantics (reference :226-252)."""
    if model_arch not in _REGISTRY:
        raise RuntimeError("Unknown model (%s)" % model_arch)
    model = _REGISTRY[model_arch](in_chans=in_chans, **kwargs)
    if pretrained.startswith("hf_hub:"):
        import huggingface_hub
        hub_name = pretrained.split(":")[1]
        huggingface_hub.hf_hub_download(hub_name, filename="slide_encoder.pth", local_dir=local_dir,
                                        force_download=True)
        local_path = os.path.join(local_dir, "slide_encoder.pth")
    else:
        local_path = pretrained
    if os.path.exists(local_path):
        state_dict = torch.load(local_path, map_location="cpu", weights_only=True)["model"]
        missing_keys, unexpected_keys = model.load_state_dict(state_dict, strict=False)
        for k in missing_keys:
            print("Missing ", k)
        for k in unexpected_keys:
            print("Unexpected ", k)
        print("\033[92m Successfully Loaded Pretrained GigaPath model from {} \033[00m".format(pretrained))
    else:
        print("\033[93m Pretrained weights not found at {}. Randomly initialized the model! \033[00m".format(local_path))
    return model


@register_model
def gigapath_slide_enc12l768d(**kwargs):
    return LongNetViT(embed_dim=768, depth=12, mlp_ratio=4, norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)


@register_model
def gigapath_slide_enc24l1024d(**kwargs):
    return LongNetViT(embed_dim=1024, depth=24, mlp_ratio=4, norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)


@register_model
def gigapath_slide_enc12l1536d(**kwargs):
    return LongNetViT(embed_dim=1536, depth=12, mlp_ratio=4, norm_layer=partial(nn.LayerNorm, eps=1e-6), **kwargs)
