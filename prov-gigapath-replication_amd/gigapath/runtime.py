"""MI355X execution engine of the LongNet slide-encoder forward.

Per layer the engine issues 8 kernels on torch's current HIP stream (M = B*L tokens):

    qkv  = LN1(x) . Wqkv^T + bqkv         gp_linear_ln (MFMA GEMM, LN1 folded; layer 0: gp_linear of
                                           the pos-embed kernel's LN1)              [M, 3E] bf16
    attn = gp_dilated_attn_fwd(qkv)        ONE launch, all dilation branches  sparse o / lse
    a    = LN_inner(merge(attn))           gp_branch_merge_ln                 [M, E] bf16
    x   += a . Wo^T + bo                   gp_linear_resid (fp32 residual stream updated in the epilogue,
                                           which also writes xb = gamma2 (x - s) and LN statistics)
    f    = gelu(LN2(x) . W1^T + b1), stats gp_ffn_fc1_gelu_ln (LN2 folded; GELU + LN statistics epilogue)
    x   += LN_ffn(f) . W2^T + b2           gp_ffn_fc2_ln_resid (LN folded; residual + the next layer's
                                           xb = gamma1' (x - s) and statistics in the epilogue)

(plus a split-K reduce after a GEMM whose last round of tiles is split).  That fused form (each LayerNorm
folded into the GEMM that consumes it, from the 16-bit xb = act(gamma (x - s)) and per-256-column
statistics its producer wrote; s = the row mean before the add; gp_gemm_impl.h) runs under
GIGAPATH_RESID_FUSED=1.  The default (round 6, faster: see RESID_FUSED below), and shapes outside the GEMM
kernels' instantiations, GIGAPATH_OWN_GEMMS=0 or GIGAPATH_FFN_FUSED=0, run the round-3 sequence:
gp_linear out-proj -> gp_residual_layernorm -> gp_ffn_fc1_gelu -> gp_ffn_fc2_ln -> gp_residual_layernorm
(hipBLASLt for uncovered GEMMs; for an uncovered FFN hipBLASLt fc1 + gp_gelu_layernorm + hipBLASLt fc2).

which is EncoderLayer.forward (torchscale/architecture/encoder.py:116-162) with
DilatedAttention.forward (component/dilated_attention.py:133-217) and the FFN
(component/feedforward_network.py:131-142) in eval mode.  The residual stream stays fp32;
GEMM operands are 16-bit (bf16, or fp16 under the caller's fp16 autocast) with fp32 accumulation.  Weights are packed once per parameter
version (fused QKV weight, bf16 GEMM operands, fp32 norms/biases) and workspaces are reused
across calls of the same shape.  No CPU fallback exists: every non-GEMM op is a HIP kernel.
"""
from __future__ import annotations

import functools
import math
import os
import threading
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _hip

_TUNED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "tunableop_results.csv")
_tuned_loaded = False


def use_tuned_gemms(dev=None):
    """Load the hipBLASLt solutions tools/tune_gemms.py selected for the slide encoder's GEMM
    shapes (PyTorch TunableOp, tuning itself off).  Shapes not in the file keep hipBLASLt's
    default heuristic.  GIGAPATH_NO_TUNED_GEMMS=1 disables it."""
    global _tuned_loaded
    path = os.environ.get("GIGAPATH_TUNED_GEMMS_FILE", _TUNED)     # an alternative tuning (A/B runs)
    if _tuned_loaded or os.environ.get("GIGAPATH_NO_TUNED_GEMMS") == "1" or not os.path.exists(path):
        return
    if dev is None or torch.device(dev).type != "cuda":
        return
    _tuned_loaded = True
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(False)
    torch.cuda.tunable.record_untuned_enable(False)
    torch.cuda.tunable.read_file(path)


_ACT = threading.local()


def call_act_dtype(module: Optional[torch.nn.Module] = None) -> torch.dtype:
    """The 16-bit activation format of a call: fp16 inside torch.autocast("cuda", float16) -- the
    reference pipeline runs the slide encoder that way (pipeline.py:186-187), so its Linear layers
    and flash-attn compute in fp16 -- or for a module whose parameters are fp16 (model.half());
    bf16 (BASELINE's dtype) otherwise, including under bf16 autocast."""
    if torch.is_autocast_enabled("cuda"):
        return torch.float16 if torch.get_autocast_dtype("cuda") == torch.float16 else torch.bfloat16
    if module is not None:
        p = next(module.parameters(), None)
        if p is not None and p.dtype == torch.float16:
            return torch.float16
    return torch.bfloat16


def act_dtype() -> torch.dtype:
    """The activation format of the compute_format call in progress on this thread (bf16 outside)."""
    return getattr(_ACT, "dtype", None) or torch.bfloat16


def compute_format(fn):
    """Decorator of the module forwards: fixes the call's activation format (call_act_dtype) for the
    whole call, nested forwards included, then runs with autocast off (autocast must not retarget
    the GEMMs that write into the 16-bit workspaces with out=).  Every 16-bit activation, GEMM operand
    and kernel format of the call follows it; the residual stream, LN parameters, LSEs and readouts
    stay fp32; outputs keep the model's parameter dtype, as the reference's autocast LayerNorm
    readout does."""
    @functools.wraps(fn)
    def wrapped(self, *args, **kw):
        outer = getattr(_ACT, "dtype", None)
        _ACT.dtype = outer if outer is not None else call_act_dtype(self)
        try:
            with torch.autocast("cuda", enabled=False):
                return fn(self, *args, **kw)
        finally:
            _ACT.dtype = outer
    return wrapped


# ------------------------------------------------------------------------------------------
# optional live timing of the hot kernels (bench.py: roofline "achieved" numbers)
# ------------------------------------------------------------------------------------------
class KernelTimer:
    """Records HIP events (on the launch stream) around selected kernels when enabled."""

    def __init__(self):
        self.enabled = False
        self.events: Dict[str, List[Tuple[torch.cuda.Event, torch.cuda.Event]]] = {}

    def reset(self):
        self.events = {}

    def span(self, name: str):
        timer = self

        class _Span:
            def __enter__(self_inner):
                if timer.enabled:
                    self_inner.e0 = torch.cuda.Event(enable_timing=True)
                    self_inner.e1 = torch.cuda.Event(enable_timing=True)
                    self_inner.e0.record()
                return self_inner

            def __exit__(self_inner, *exc):
                if timer.enabled:
                    self_inner.e1.record()
                    timer.events.setdefault(name, []).append((self_inner.e0, self_inner.e1))
                return False

        return _Span()

    def totals_ms(self) -> Dict[str, Tuple[int, float]]:
        """name -> (launch count, summed milliseconds).  Synchronises."""
        torch.cuda.synchronize()
        return {k: (len(v), sum(a.elapsed_time(b) for a, b in v)) for k, v in self.events.items()}


TIMER = KernelTimer()


# ------------------------------------------------------------------------------------------
# geometry (dilated_attention.py:16-31, 76-98)
# ------------------------------------------------------------------------------------------
def branch_geometry(L: int, sl: int, r: int) -> Tuple[int, int, int]:
    """(s, nseg, m) of one branch at sequence length L."""
    s = min(sl, L)
    return s, -(-L // s), -(-s // r)


def attention_valid_flops(L: int, segs: Sequence[int], ratios: Sequence[int], H: int, D: int, B: int = 1) -> float:
    """Algorithmic FLOPs of one layer's dilated attention: 4*D*c^2 per (segment, head), c = real
    (non-pad) tokens the head sees in that segment.  Zero pads count 0."""
    tot = 0
    for sl, r in zip(segs, ratios):
        s, nseg, m = branch_geometry(L, sl, r)
        hp = H + ((r - H % r) % r)
        hpg = hp // r
        for n in range(nseg):
            rem = min(L - n * s, s)
            for h in range(H):
                j = h // hpg
                lim = rem - j
                c = -(-lim // r) if lim > 0 else 0
                tot += 4 * D * c * c
    return float(tot * B)


# ------------------------------------------------------------------------------------------
# packed weights
# ------------------------------------------------------------------------------------------
def _act(t: torch.Tensor, dev, act: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """A 16-bit GEMM operand copy (bf16 or fp16)."""
    return t.detach().to(device=dev, dtype=act).contiguous()


def _bf16(t: torch.Tensor, dev) -> torch.Tensor:
    return _act(t, dev, torch.bfloat16)


def _f32(t: torch.Tensor, dev) -> torch.Tensor:
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


LOG2E = 1.4426950408889634


@dataclass
class PackedAttention:
    """Packed DilatedAttention weights.  The softmax scale D^-0.5 and log2(e) are folded into the
    Q rows of the fused projection (in fp32, before the single 16-bit rounding of the GEMM output),
    so the attention kernel consumes log2-domain logits (gp_dilated_attn_fwd q_log2_prescaled).
    16-bit operands are in `act` (bf16, or fp16 for the caller's fp16 autocast)."""
    E: int
    H: int
    D: int
    segs: List[int]
    ratios: List[int]
    w_qkv: torch.Tensor      # [3E, E] act (q * scale*log2e | k | v rows)
    b_qkv: torch.Tensor      # [3E] act
    w_o: torch.Tensor        # [E, E] act
    b_o: torch.Tensor        # [E] fp32 (added in the residual kernel)
    b_o_act: torch.Tensor    # [E] act (standalone module forward)
    ln_w: torch.Tensor
    ln_b: torch.Tensor
    ln_eps: float

    prescaled: bool = True
    b_qkv_f32: Optional[torch.Tensor] = None   # [3E] fp32 (gp_linear's bias)
    # fp16 packing only: the engine's QKV GEMMs write the V third of qkv in bf16 and the attention reads it so
    # (GP_FMT_F16_VBF16): bf16 P.V at the bf16 kernel's speed instead of the exact fp16 running-max kernel
    # (DESIGN §3.3).  Every engine producer and consumer of qkv passes it; the standalone module does not.
    v_bf16: bool = False

    def qkv_parts(self, qkv: torch.Tensor):
        """(q, k, v) column views of a fused [M, 3E] qkv buffer this layer's engine wrote, each with the dtype
        its bytes hold: with v_bf16 the V third of an fp16 qkv is bf16, so v is viewed as bfloat16 (reading
        qkv[:, 2E:] as fp16 would silently misread it).  Readers of ws.qkv outside the engine's own entry
        points go through here (advice r05)."""
        E = self.E
        q, k, v = qkv[:, :E], qkv[:, E:2 * E], qkv[:, 2 * E:3 * E]
        if self.v_bf16 and qkv.dtype == torch.float16:
            v = v.view(torch.bfloat16)
        return q, k, v

    @staticmethod
    def from_module(m, dev, act: torch.dtype = torch.bfloat16) -> "PackedAttention":
        E, H = m.embed_dim, m.num_heads
        D = E // H
        qs = (D ** -0.5) * LOG2E if D in (48, 64) else 1.0   # D=96 uses the generic kernel
        wq = m.q_proj.weight.detach().to(device=dev, dtype=torch.float32) * qs
        bq = m.q_proj.bias.detach().to(device=dev, dtype=torch.float32) * qs
        b_qkv = torch.cat([bq, _f32(m.k_proj.bias, dev), _f32(m.v_proj.bias, dev)], 0)
        return PackedAttention(
            E=E, H=H, D=D, segs=list(m.args.segment_length), ratios=list(m.args.dilated_ratio),
            w_qkv=_act(torch.cat([wq, _f32(m.k_proj.weight, dev), _f32(m.v_proj.weight, dev)], 0), dev, act),
            b_qkv=_act(b_qkv, dev, act), b_qkv_f32=_act(b_qkv, dev, act).float().contiguous(),
            w_o=_act(m.out_proj.weight, dev, act), b_o=_f32(m.out_proj.bias, dev),
            b_o_act=_act(m.out_proj.bias, dev, act),
            ln_w=_f32(m.inner_attn_ln.weight, dev), ln_b=_f32(m.inner_attn_ln.bias, dev),
            ln_eps=float(m.inner_attn_ln.eps), prescaled=D in (48, 64),
            v_bf16=(act == torch.float16 and D == 48 and OWN_GEMMS and _hip.gemm_supported(3 * E, E)))


@dataclass
class PackedLayer:
    attn: PackedAttention
    ln1_w: torch.Tensor
    ln1_b: torch.Tensor
    ln1_eps: float
    ln2_w: torch.Tensor
    ln2_b: torch.Tensor
    ln2_eps: float
    w1: torch.Tensor         # [F, E] act
    b1: torch.Tensor         # [F] act
    fln_w: torch.Tensor      # [F] fp32
    fln_b: torch.Tensor
    fln_eps: float
    w2: torch.Tensor         # [E, F] act
    b2: torch.Tensor         # [E] fp32
    # the fused FFN (gp_ffn_fc1_gelu / gp_ffn_fc2_ln), None when its kernels do not cover the shape:
    b1_f32: Optional[torch.Tensor] = None   # [F] fp32
    w2g: Optional[torch.Tensor] = None      # [E, F] act: W2 * gamma_ffn (LN weight folded into fc2)
    c2: Optional[torch.Tensor] = None       # [E] fp32: row sums of w2g as rounded
    d2: Optional[torch.Tensor] = None       # [E] fp32: W2 . beta_ffn + b2
    # the residual stream inside the GEMMs (gp_linear_ln / gp_ffn_fc1_gelu_ln fold the pre-LNs):
    c_qkv: Optional[torch.Tensor] = None    # [3E] fp32: w_qkv . gamma1 (w_qkv as rounded)
    d_qkv: Optional[torch.Tensor] = None    # [3E] fp32: w_qkv . beta1 + b_qkv
    c1: Optional[torch.Tensor] = None       # [F] fp32: w1 . gamma2
    d1: Optional[torch.Tensor] = None       # [F] fp32: w1 . beta2 + b1

    @property
    def ffn_fused(self) -> bool:
        return self.w2g is not None

    @property
    def resid_fused(self) -> bool:
        return self.c1 is not None

    @staticmethod
    def from_module(layer, dev, act: torch.dtype = torch.bfloat16) -> "PackedLayer":
        ffn = layer.ffn
        pl = PackedLayer(
            attn=PackedAttention.from_module(layer.self_attn, dev, act),
            ln1_w=_f32(layer.self_attn_layer_norm.weight, dev), ln1_b=_f32(layer.self_attn_layer_norm.bias, dev),
            ln1_eps=float(layer.self_attn_layer_norm.eps),
            ln2_w=_f32(layer.final_layer_norm.weight, dev), ln2_b=_f32(layer.final_layer_norm.bias, dev),
            ln2_eps=float(layer.final_layer_norm.eps),
            w1=_act(ffn.fc1.weight, dev, act), b1=_act(ffn.fc1.bias, dev, act),
            fln_w=_f32(ffn.ffn_layernorm.weight, dev), fln_b=_f32(ffn.ffn_layernorm.bias, dev),
            fln_eps=float(ffn.ffn_layernorm.eps),
            w2=_act(ffn.fc2.weight, dev, act), b2=_f32(ffn.fc2.bias, dev))
        F, E = pl.w1.shape
        if ffn_fusable(E, F) or resid_fusable(E, F):
            # LN(h) . W2^T + b2 = rstd (h . (W2 gamma)^T - mean c) + d  (csrc/gp_gemm_impl.h, "LN fold")
            w2 = ffn.fc2.weight.detach().to(device=dev, dtype=torch.float64)
            g = ffn.ffn_layernorm.weight.detach().to(device=dev, dtype=torch.float64)
            be = ffn.ffn_layernorm.bias.detach().to(device=dev, dtype=torch.float64)
            pl.w2g = (w2 * g[None, :]).to(act).contiguous()
            pl.c2 = pl.w2g.double().sum(1).float().contiguous()
            pl.d2 = (w2 @ be + ffn.fc2.bias.detach().to(device=dev, dtype=torch.float64)).float().contiguous()
            pl.b1_f32 = _f32(ffn.fc1.bias, dev)
        if resid_fusable(E, F):
            # LN(x) . W^T + b = rstd (xb . W^T - mean' c) + d with xb = act(gamma (x - s)): c = W . gamma
            # (W as the GEMM rounds it), d = W . beta + b (csrc/gp_gemm_impl.h, "the residual epilogues")
            def fold(w_act, ln, b):
                wd = w_act.double()
                return ((wd @ ln.weight.detach().to(device=dev, dtype=torch.float64)).float().contiguous(),
                        (wd @ ln.bias.detach().to(device=dev, dtype=torch.float64) + b.double()).float().contiguous())
            pl.c_qkv, pl.d_qkv = fold(pl.attn.w_qkv, layer.self_attn_layer_norm, pl.attn.b_qkv_f32)
            pl.c1, pl.d1 = fold(pl.w1, layer.final_layer_norm, _f32(ffn.fc1.bias, dev))
        return pl


FFN_FUSED = os.environ.get("GIGAPATH_FFN_FUSED", "1") != "0"
# the residual adds + pre-LNs inside the out-proj / fc2 epilogues and the QKV / fc1 folds (round 4), OFF by
# default since round 6: the round-3 sequence (plain out-proj / fc2 -> gp_residual_layernorm -> plain QKV / fc1)
# is faster in the HIP-graph forward on every measurement (r05: 30.96 / 31.08 / 30.92 vs 30.73 / 30.74 /
# 30.69 ms; r06_base: 29.51 / 29.39 / 29.48 vs 29.38 / 29.27 / 29.06 ms, profiles/r06_base_*) and stays
# inside the north star's 1e-2 at the headline slides (C3 max-rel 8.57e-3, C4 8.14e-3 vs 7.73e-3 / 6.45e-3
# fused, profiles/r06_base_golden_rel_resid_fused_on_off.jsonl).  =1 picks the fused epilogues (more
# parity headroom: the residual stream is rounded once per layer fewer).
RESID_FUSED = os.environ.get("GIGAPATH_RESID_FUSED", "0") == "1"
# the QKV / out-proj / patch projections on gp_linear (own MFMA GEMM, the default) instead of hipBLASLt.
# With every GEMM of the forward on gp_gemm.hip kernels (persistent, data-parallel tiles, no workgroup ever
# waits on another) concurrent HIP-graph replays on several streams run (tests/test_gpu_concurrent.py,
# r03_p: 6.3 s); with hipBLASLt's stream-K QKV / patch GEMMs the same test hung (r03_o, > 180 s).
OWN_GEMMS = os.environ.get("GIGAPATH_OWN_GEMMS", "1") == "1"


def linear(a: torch.Tensor, w: torch.Tensor, b_act: Optional[torch.Tensor], b_f32: Optional[torch.Tensor],
           out: torch.Tensor, gemm_ws: Optional[torch.Tensor] = None, v_bf16: bool = False):
    """out = a . w^T (+ b): nn.Linear on gp_linear when OWN_GEMMS and its instantiations cover the
    shape, else hipBLASLt (torch.addmm / mm).  b_act / b_f32: the bias in the act format / fp32.
    v_bf16: a fused fp16 QKV whose V third is written in bf16 (PackedAttention.v_bf16; own GEMM only)."""
    N, K = w.shape
    if OWN_GEMMS and a.is_cuda and _hip.gemm_supported(N, K) and (b_act is None or b_f32 is not None):
        if gemm_ws is not None and gemm_ws.numel() < _hip.gemm_workspace_bytes(a.shape[0], N, K):
            gemm_ws = None                   # (no split of the last round of tiles)
        # gp_linear's operand contract (row-major, 16-byte aligned rows): a strided or offset caller tensor
        # is copied once instead of being refused
        if not _gemm_rows_ok(a):
            a = a.clone(memory_format=torch.contiguous_format)
        if _gemm_rows_ok(out):
            _hip.linear(a, w, b_f32, out, gemm_ws, v_bf16=v_bf16)
        else:
            tmp = torch.empty(out.shape, dtype=out.dtype, device=out.device)
            _hip.linear(a, w, b_f32, tmp, gemm_ws, v_bf16=v_bf16)
            out.copy_(tmp)
    else:
        if v_bf16:
            raise RuntimeError("runtime.linear: a bf16 V third needs the own GEMM (OWN_GEMMS and a covered shape)")
        with blaslt_serialized():
            if b_act is not None:
                torch.addmm(b_act, a, w.t(), out=out)
            else:
                torch.mm(a, w.t(), out=out)


def _gemm_rows_ok(t: torch.Tensor) -> bool:
    """gp_linear's layout: row-major rows (unit column stride), rows a multiple of 8 elements apart,
    a 16-byte aligned base."""
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0


# hipBLASLt GEMMs (shapes outside the own kernels, GIGAPATH_OWN_GEMMS=0 / GIGAPATH_FFN_FUSED=0): its tuned
# stream-K kernels spin on flags of peer workgroups, and concurrent forwards / graph replays on several
# streams hung with them (r03_o).  Every such GEMM issued outside a capture is ordered after
# the previous one on ANY stream of the device (an event chain, no host sync), and a captured graph that
# contains one (BLASLT_ISSUED moved during its capture) replays under the same chain
# (LongNetViT._replay): hipBLASLt never runs on two streams at once.
BLASLT_ISSUED = [0]
_BLASLT_LOCK = threading.RLock()
_BLASLT_LAST: Dict[int, torch.cuda.Event] = {}


def capture_uses_blaslt(before: int) -> bool:
    """True when a hipBLASLt GEMM was issued since BLASLT_ISSUED[0] was `before` (a capture's contents)."""
    return BLASLT_ISSUED[0] != before


def replay_graph(graph) -> None:
    """graph.replay() on the current stream; a graph holding hipBLASLt GEMMs (graph.gp_blaslt, set at
    capture) replays in the device's hipBLASLt event chain (blaslt_serialized)."""
    if getattr(graph, "gp_blaslt", False):
        with blaslt_serialized():
            graph.replay()
    else:
        graph.replay()


class blaslt_serialized:
    """Context of one hipBLASLt launch (or one graph replay containing some) on the current stream."""

    def __enter__(self):
        BLASLT_ISSUED[0] += 1
        self._chain = torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing()
        if self._chain:
            _BLASLT_LOCK.acquire()
            self._stream = torch.cuda.current_stream()
            ev = _BLASLT_LAST.get(self._stream.device.index)
            if ev is not None:
                self._stream.wait_event(ev)
        return self

    def __exit__(self, *exc):
        if self._chain:
            try:
                ev = torch.cuda.Event()
                ev.record(self._stream)
                _BLASLT_LAST[self._stream.device.index] = ev
            finally:
                _BLASLT_LOCK.release()
        return False


def ffn_fusable(E: int, F: int) -> bool:
    """The fused FFN kernels cover fc1 [F, E] (K = E) and fc2 [E, F] (K = F)."""
    return (FFN_FUSED and E in _hip.GEMM_K_E and F in _hip.GEMM_K_F and _hip.gemm_supported(F, E)
            and _hip.gemm_supported(E, F))


def resid_fusable(E: int, F: int) -> bool:
    """Every GEMM of the layer on the residual-epilogue / LN-fold kernels: QKV [3E, E], out-proj [E, E],
    fc1 [F, E] with K = E and fc2 [E, F] with K = F (the three registered archs)."""
    return (RESID_FUSED and FFN_FUSED and OWN_GEMMS and E in _hip.GEMM_K_E and F in _hip.GEMM_K_F
            and all(_hip.gemm_supported(n, k) for n, k in ((3 * E, E), (E, E), (F, E), (E, F))))


def resid_buffers(dev, M: int, E: int):
    """(xstats [E/256 + 1, M, 2], shift [2, M]) of the residual epilogues (fp32).  The two shift rows are
    each padded to a multiple of 4 floats, so both start 16-byte aligned (the GEMMs LDS-DMA them)."""
    mp = (M + 3) // 4 * 4
    return (torch.empty((E // 256 + 1) * M * 2, dtype=torch.float32, device=dev),
            torch.empty(2, mp, dtype=torch.float32, device=dev)[:, :M])


# the residual producers (out-proj, fc2) merge the next LayerNorm's statistics themselves (round 5: in their
# split-tail reduce launch, so the 24 row_stats launches of the consumers go away; the result is the same bits)
MERGE_IN_PRODUCER = os.environ.get("GIGAPATH_MERGE_IN_PRODUCER", "1") != "0"


def fused_qkv(pl: "PackedLayer", ws, qkv: torch.Tensor):
    """QKV of a layer after the first: LN1 folded, A = ws.y (the previous fc2's xb); the statistics merge
    (shift[1] -> shift[0]) is the previous fc2's (MERGE_IN_PRODUCER) or done here."""
    pa = pl.attn
    E = pa.E
    _hip.linear_ln(ws.y, pa.w_qkv, ws.xstats, E // 256, pl.c_qkv, pl.d_qkv, pl.ln1_eps, ws.shift[1], ws.shift[0],
                   qkv, ws.gemm_ws, v_bf16=pa.v_bf16, merged=MERGE_IN_PRODUCER)


def fused_post_attention(pl: "PackedLayer", nxt: Optional["PackedLayer"], ws):
    """out-proj + residual, fc1 (+ folded LN2, GELU), fc2 (+ folded ffn LN, residual, the next layer's
    xb) on ws.a (the merge output).  Shift schedule: out-proj reads shift[0] (the row mean of x before it),
    fc1's merge writes shift[1], fc2 reads it; the next QKV maps shift[1] -> shift[0]."""
    pa = pl.attn
    E = pa.E
    mp = MERGE_IN_PRODUCER
    with TIMER.span("gemm_out"):
        _hip.linear_resid(ws.a, pa.w_o, pa.b_o, ws.x, ws.shift[0], pl.ln2_w, ws.y, ws.xstats, ws.gemm_ws,
                          eps_next=pl.ln2_eps if mp else None, s_out=ws.shift[1] if mp else None)
    with TIMER.span("gemm_fc1"):
        _hip.ffn_fc1_gelu_ln(ws.y, pl.w1, ws.xstats, E // 256, pl.c1, pl.d1, pl.ln2_eps, ws.shift[0], ws.shift[1],
                             ws.f, ws.fstats, merged=mp)
    with TIMER.span("gemm_fc2"):
        last = nxt is None
        _hip.ffn_fc2_ln_resid(ws.f, pl.w2g, ws.fstats, pl.c2, pl.d2, pl.fln_eps, ws.x, ws.shift[1],
                              None if last else nxt.ln1_w, ws.y, ws.xstats, ws.gemm_ws,
                              eps_next=None if (last or not mp) else nxt.ln1_eps,
                              s_out=None if (last or not mp) else ws.shift[0])


def ffn_forward(pl: "PackedLayer", a: torch.Tensor, f: torch.Tensor, y: torch.Tensor, fstats, gemm_ws,
                M: int, F: int) -> Optional[torch.Tensor]:
    """FeedForwardNetwork.forward (feedforward_network.py:131-142) without its residual: y = FFN(a).
    Returns the bias the residual add still owes (b2 on the unfused path, None when fused)."""
    if pl.ffn_fused and fstats is not None:
        with TIMER.span("gemm_fc1"):
            _hip.ffn_fc1_gelu(a, pl.w1, pl.b1_f32, f, fstats)
        with TIMER.span("gemm_fc2"):
            _hip.ffn_fc2_ln(f, pl.w2g, fstats, pl.c2, pl.d2, pl.fln_eps, y, gemm_ws)
        return None
    with TIMER.span("gemm_fc1"), blaslt_serialized():
        torch.addmm(pl.b1, a, pl.w1.t(), out=f)
    with TIMER.span("gelu_ln"):
        _hip.gelu_layernorm(f, pl.fln_w, pl.fln_b, pl.fln_eps, f, M, F)
    with TIMER.span("gemm_fc2"), blaslt_serialized():
        torch.mm(f, pl.w2.t(), out=y)
    return pl.b2


def ffn_buffers(dev, M: int, E: int, F: int):
    """(stats, GEMM workspace) of the fused FFN for M rows, or (None, workspace) when it does not apply."""
    if not (ffn_fusable(E, F) or resid_fusable(E, F)):
        return None, gemm_workspace(dev, M, E, F)
    stats = torch.empty((F // 256 + 1) * M * 2, dtype=torch.float32, device=dev)
    return stats, gemm_workspace(dev, M, E, F)


def gemm_workspace(dev, M: int, E: int, F: int) -> torch.Tensor:
    """Split-K workspace of the own GEMMs of M rows: fc2 (E x F) and, with OWN_GEMMS, QKV / out-proj."""
    nb = 0
    if torch.device(dev).type == "cuda":
        shapes = [(E, F)] + ([(3 * E, E), (E, E)] if OWN_GEMMS else [])
        nb = max([_hip.gemm_workspace_bytes(M, n, k) for n, k in shapes if _hip.gemm_supported(n, k)], default=0)
    return torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)


def param_signature(module: torch.nn.Module) -> tuple:
    return tuple((p.data_ptr(), p._version, p.dtype) for p in module.parameters())


# ------------------------------------------------------------------------------------------
# the dilated attention core (gather + attention + merge + inner LN), shared by the engine
# and by the standalone DilatedAttention module
# ------------------------------------------------------------------------------------------
class AttentionScratch:
    def __init__(self, dev, B: int, L: int, H: int, D: int, segs, ratios, act: torch.dtype = torch.bfloat16):
        self.key = (B, L, H, D, tuple(segs), tuple(ratios), act)
        self.outs, self.lses = [], []
        for sl, r in zip(segs, ratios):
            s, nseg, m = branch_geometry(L, sl, r)
            self.outs.append(torch.empty(B * nseg * m * H * D, dtype=act, device=dev))
            self.lses.append(torch.empty(B * nseg * H * m, dtype=torch.float32, device=dev))


class VarlenScratch:
    """Packed per-branch outputs of several slides (slide-major regions) and the varlen work table
    bound to one qkv buffer (config C5 packing, _hip.VarlenPlan)."""

    def __init__(self, dev, Ls: Sequence[int], H: int, D: int, segs, ratios, qkv: torch.Tensor):
        self.plan = _hip.VarlenPlan(Ls, H, D, segs, ratios)
        self.outs = [torch.empty(n, dtype=qkv.dtype, device=dev) for n in self.plan.o_elems]
        self.lses = [torch.empty(n, dtype=torch.float32, device=dev) for n in self.plan.lse_elems]
        self.plan.bind(qkv, self.outs, self.lses)


def dilated_attention_core(pa: PackedAttention, qkv: torch.Tensor, B: int, L: int, scratch: AttentionScratch,
                           out: torch.Tensor, inner_ln: bool = True, v_bf16: bool = False):
    """qkv: [B*L, 3E] 16-bit (q | k | v; v_bf16: an fp16 qkv whose V third is bf16, see PackedAttention);
    out: [B*L, E] same format = inner_attn_ln(merge(branches)).  With a VarlenScratch (bound to this qkv),
    every packed slide in one launch each."""
    E, H, D = pa.E, pa.H, pa.D
    if isinstance(scratch, VarlenScratch):
        if not pa.prescaled:
            raise RuntimeError("varlen packing needs the pre-scaled q of D = 48")
        with TIMER.span("attn"):
            _hip.dilated_attn_fwd_varlen(scratch.plan, True, v_bf16=v_bf16)
        with TIMER.span("merge"):
            _hip.branch_merge_ln_varlen(scratch.plan, pa.ln_w if inner_ln else None, pa.ln_b if inner_ln else None,
                                        pa.ln_eps, out)
        return
    with TIMER.span("attn"):
        _hip.dilated_attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], 3 * E, B, L, H, D, pa.segs, pa.ratios,
                              scratch.outs, scratch.lses, 0.0, pa.prescaled, v_bf16=v_bf16)
    with TIMER.span("merge"):
        _hip.branch_merge_ln(scratch.outs, scratch.lses, pa.segs, pa.ratios, B, L, H, D,
                             pa.ln_w if inner_ln else None, pa.ln_b if inner_ln else None, pa.ln_eps, out)


# ------------------------------------------------------------------------------------------
# encoder engine
# ------------------------------------------------------------------------------------------
class Workspace:
    def __init__(self, dev, B: int, L: int, E: int, F: int, H: int, segs, ratios, act: torch.dtype = torch.bfloat16):
        M = B * L
        self.key = (str(dev), B, L, E, F, H, tuple(segs), tuple(ratios), act)
        self.x = torch.empty(M, E, dtype=torch.float32, device=dev)
        self.a = torch.empty(M, E, dtype=act, device=dev)
        # fused q | k | v; NOTE under the fp16 caller (PackedAttention.v_bf16) the V third holds bf16 bits
        # although the tensor is fp16: read it through PackedAttention.qkv_parts
        self.qkv = torch.empty(M, 3 * E, dtype=act, device=dev)
        self.y = torch.empty(M, E, dtype=act, device=dev)
        self.y2 = torch.empty(M, E, dtype=act, device=dev)     # fc2 output (y keeps the out-proj's: RESID2)
        self.f = torch.empty(M, F, dtype=act, device=dev)
        self.fstats, self.gemm_ws = ffn_buffers(dev, M, E, F)
        self.xstats, self.shift = resid_buffers(dev, M, E)
        self.attn = AttentionScratch(dev, B, L, H, E // H, segs, ratios, act)


class PackedWorkspace(Workspace):
    """Workspace of several slides packed token-major: T = sum(L_i) rows, slide i at rows
    [tok_off[i], tok_off[i] + L_i) with its CLS first; attention through a VarlenScratch."""

    def __init__(self, dev, Ls: Sequence[int], E: int, F: int, H: int, segs, ratios,
                 act: torch.dtype = torch.bfloat16):
        self.Ls = [int(x) for x in Ls]
        T = sum(self.Ls)
        M = T
        self.key = (str(dev), tuple(self.Ls), E, F, H, tuple(segs), tuple(ratios), act)
        self.x = torch.empty(M, E, dtype=torch.float32, device=dev)
        self.a = torch.empty(M, E, dtype=act, device=dev)
        self.qkv = torch.empty(M, 3 * E, dtype=act, device=dev)   # (V third: see Workspace, qkv_parts)
        self.y = torch.empty(M, E, dtype=act, device=dev)
        self.y2 = torch.empty(M, E, dtype=act, device=dev)
        self.f = torch.empty(M, F, dtype=act, device=dev)
        self.fstats, self.gemm_ws = ffn_buffers(dev, M, E, F)
        self.xstats, self.shift = resid_buffers(dev, M, E)
        self.attn = VarlenScratch(dev, self.Ls, H, E // H, segs, ratios, self.qkv)
        self.tok_off = self.attn.plan.tok_off
        self.cls_idx = torch.tensor(self.tok_off[:-1], dtype=torch.int64, device=dev)


class EncoderEngine:
    """Runs the 12-layer (or 24-) LongNet stack on one device for inputs already embedded."""

    def __init__(self):
        self._sig = None
        self.layers: List[PackedLayer] = []
        self._packs: Dict[torch.dtype, tuple] = {}     # act -> (signature, packed layers)
        # activation workspaces per CALLER STREAM: two streams never share activation buffers, so
        # forwards issued on different streams can run concurrently; ws / pws = the last one used.
        # LRU-bounded (max_stream_workspaces): a caller using a fresh stream per request does not grow
        # them without limit.  A HIP graph's workspace is detached from these maps after its capture
        # (detach_workspace) and lives exactly as long as the graph (LongNetViT._graph_ws).
        self._ws: "OrderedDict[int, Workspace]" = OrderedDict()
        self._pws: "OrderedDict[int, PackedWorkspace]" = OrderedDict()
        self.ws: Optional[Workspace] = None
        self.pws: Optional[PackedWorkspace] = None

    def pack(self, encoder, dev, act: Optional[torch.dtype] = None):
        """Packed layers for the activation format `act` (default: the current call's, act_dtype());
        one packing per format is kept, so alternating bf16 / fp16 callers do not repack."""
        use_tuned_gemms(dev)
        act = act or act_dtype()
        sig = (str(dev), param_signature(encoder), act)
        ent = self._packs.get(act)
        if ent is None or ent[0] != sig:
            ent = (sig, [PackedLayer.from_module(l, dev, act) for l in encoder.layers])
            self._packs[act] = ent
        self._sig, self.layers = ent
        return self.layers

    @staticmethod
    def _stream_key(dev) -> int:
        return int(torch.cuda.current_stream(dev).cuda_stream) if torch.device(dev).type == "cuda" else 0

    # (8 = LongNetViT.max_capture_streams: the documented 4-stream concurrent pattern plus the default stream
    # and the capture side streams stay cached; beyond it an eager call on yet another stream evicts the least
    # recently used workspace and reallocates its own -- correct, but hundreds of MB per call at 20-70k tiles)
    max_stream_workspaces = 8

    def _cached(self, table, key, make):
        sk = self._stream_key(self._dev_of(key))
        ws = table.get(sk)
        if ws is None or ws.key != key:
            table.pop(sk, None)                # (a HIP graph that baked the old one keeps it alive)
            while len(table) >= self.max_stream_workspaces:
                old = next(iter(table))        # least recently used caller stream
                table.pop(old)
            ws = table[sk] = make()
        table.move_to_end(sk)
        return ws

    @staticmethod
    def _dev_of(key):
        return torch.device(key[0])

    def workspace(self, dev, B, L, E, F, H, segs, ratios, act: Optional[torch.dtype] = None) -> Workspace:
        act = act or act_dtype()
        key = (str(dev), B, L, E, F, H, tuple(segs), tuple(ratios), act)
        self.ws = self._cached(self._ws, key, lambda: Workspace(dev, B, L, E, F, H, segs, ratios, act))
        return self.ws

    def workspace_packed(self, dev, Ls, E, F, H, segs, ratios, act: Optional[torch.dtype] = None) -> PackedWorkspace:
        act = act or act_dtype()
        key = (str(dev), tuple(int(x) for x in Ls), E, F, H, tuple(segs), tuple(ratios), act)
        self.pws = self._cached(self._pws, key, lambda: PackedWorkspace(dev, Ls, E, F, H, segs, ratios, act))
        return self.pws

    def stream_workspace(self, stream, packed: bool = False):
        """The workspace the engine keeps for `stream` (the one a forward issued on that stream used),
        or None."""
        table = self._pws if packed else self._ws
        return table.get(int(stream.cuda_stream)) if stream is not None else None

    def detach_workspace(self, ws) -> None:
        """Forget `ws` (a HIP graph's baked workspace): the next eager call on its stream allocates a new
        one, and the graph cache alone decides how long `ws` lives."""
        for table in (self._ws, self._pws):
            for k in [k for k, v in table.items() if v is ws]:
                table.pop(k)
        if self.ws is ws:
            self.ws = None
        if self.pws is ws:
            self.pws = None

    def run_layers(self, ws: Workspace, B: int, L: int, layer_hook=None, shift_ready: bool = False):
        """ws.x holds the fp32 embedding and ws.a = LN1_0(ws.x) (16-bit).  Runs every layer in
        place; layer_hook(i) is called after layer i-1 finishes (i = 1..depth).  shift_ready: ws.shift[0]
        already holds the row means of ws.x (gp_posembed_cls_ln's row_mean); otherwise they are computed."""
        M = B * L
        E = ws.x.shape[1]
        F = ws.f.shape[1]
        nl = len(self.layers)
        if self.layers and all(pl.resid_fused for pl in self.layers) and ws.fstats is not None:
            if not shift_ready:
                torch.mean(ws.x, 1, out=ws.shift[0])
            for li, pl in enumerate(self.layers):
                pa = pl.attn
                with TIMER.span("gemm_qkv"):
                    if li == 0:
                        linear(ws.a, pa.w_qkv, pa.b_qkv, pa.b_qkv_f32, ws.qkv, ws.gemm_ws, v_bf16=pa.v_bf16)
                    else:
                        fused_qkv(pl, ws, ws.qkv)
                dilated_attention_core(pa, ws.qkv, B, L, ws.attn, ws.a, v_bf16=pa.v_bf16)
                fused_post_attention(pl, self.layers[li + 1] if li + 1 < nl else None, ws)
                if layer_hook is not None:
                    layer_hook(li + 1)
            return
        for li, pl in enumerate(self.layers):
            pa = pl.attn
            with TIMER.span("gemm_qkv"):
                linear(ws.a, pa.w_qkv, pa.b_qkv, pa.b_qkv_f32, ws.qkv, ws.gemm_ws, v_bf16=pa.v_bf16)
            dilated_attention_core(pa, ws.qkv, B, L, ws.attn, ws.a, v_bf16=pa.v_bf16)
            with TIMER.span("gemm_out"):
                linear(ws.a, pa.w_o, None, None, ws.y, ws.gemm_ws)
            nxt = self.layers[li + 1] if li + 1 < nl else None
            residual_pair(pl, nxt, ws, M, E, F)
            if layer_hook is not None:
                layer_hook(li + 1)


# the layer's two residual adds as gp_residual2_layernorm (round 6): the first leaves x unwritten, the second
# recomputes x1 from x and the out-proj output y and adds the fc2 output -- 22 instead of 24 bytes per element,
# bit-identical to the two gp_residual_layernorm passes (=0 restores those)
RESID2 = os.environ.get("GIGAPATH_RESID2", "1") != "0"


def residual_pair(pl: "PackedLayer", nxt: Optional["PackedLayer"], ws, M: int, E: int, F: int):
    """The unfused layer tail after the out-proj GEMM wrote ws.y: residual + LN2, FFN, residual + the next
    layer's LN1 (encoder.py:141-162)."""
    pa = pl.attn
    ln1 = (nxt.ln1_w, nxt.ln1_b, nxt.ln1_eps) if nxt else (None, None, 1e-5)
    if RESID2:
        with TIMER.span("resid_ln"):
            _hip.residual2_layernorm(ws.x, ws.y, pa.b_o, None, None, pl.ln2_w, pl.ln2_b, pl.ln2_eps, ws.a, M, E)
        b2 = ffn_forward(pl, ws.a, ws.f, ws.y2, ws.fstats, ws.gemm_ws, M, F)
        with TIMER.span("resid_ln"):
            _hip.residual2_layernorm(ws.x, ws.y, pa.b_o, ws.y2, b2, ln1[0], ln1[1], ln1[2], ws.a, M, E)
        return
    with TIMER.span("resid_ln"):
        _hip.residual_layernorm(ws.x, ws.y, pa.b_o, pl.ln2_w, pl.ln2_b, pl.ln2_eps, ws.a, M, E)
    b2 = ffn_forward(pl, ws.a, ws.f, ws.y, ws.fstats, ws.gemm_ws, M, F)
    with TIMER.span("resid_ln"):
        _hip.residual_layernorm(ws.x, ws.y, b2, ln1[0], ln1[1], ln1[2], ws.a, M, E)


def gemm_flops(B: int, N: int, E: int, F: int, C: int, depth: int) -> float:
    L = N + 1
    return float(2 * B * L * (4 * E * E + 2 * E * F) * depth + 2 * B * N * C * E)


def merge_bytes(L: int, segs: Sequence[int], ratios: Sequence[int], H: int, D: int, B: int = 1) -> float:
    """Algorithmic HBM bytes of one gp_branch_merge_ln launch (16-bit o, fp32 lse, 16-bit out): per token,
    branch b contributes the E/r_b covered output columns and H/r_b LSE values."""
    E = H * D
    per_tok = sum(E / r * 2 + H / r * 4 for r in ratios) + E * 2
    return float(B * L * per_tok)


def attention_valid_flops_window(L: int, segs: Sequence[int], ratios: Sequence[int], H: int, D: int, lo: int,
                                 hi: int) -> float:
    """Valid attention FLOPs of the query rows whose sparse_to_dense slot lies in [lo, hi) (one
    sequence-parallel shard): each such (row, head) costs 4*D*c, c = real keys of its segment."""
    tot = 0.0
    p = np.arange(lo, hi, dtype=np.int64)
    for sl, r in zip(segs, ratios):
        s, nseg, m = branch_geometry(L, sl, r)
        hp = H + ((r - H % r) % r)
        hpg = hp // r
        g = m * r
        n = p // g
        j = (p % g) % r
        seg_len = np.minimum(L - n * s, s)                 # real tokens of the row's segment
        rem = seg_len - j
        c = np.where(rem > 0, -(-rem // r), 0)
        heads = np.clip(H - j * hpg, 0, hpg)
        real_q = (p % g) < seg_len                         # a zero-padded query row is not valid work
        tot += float((4.0 * D * c * heads * real_q).sum())
    return tot
