"""ctypes binding of libgigapath_hip.so (the C ABI declared in include/gigapath_hip.h).

Tensors are passed as raw device pointers; every call is enqueued on torch's *current*
HIP stream.  There is no fallback: if the library is missing or a call fails, this module
raises.  torch is imported first so that its bundled HIP runtime (same soname,
libamdhip64.so.7) is the one the library binds to.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libgigapath_hip.so")
ABI_VERSION = 10
MAX_BRANCHES = 8
MAX_DESTS = 8

c_i32, c_i64, c_f32, c_f64, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_void_p


class GpRowDest(ctypes.Structure):
    """struct GpRowDest (include/gigapath_hip.h)."""
    _fields_ = [("tok_lo", c_i64), ("tok_hi", c_i64), ("dst", c_vp)]


class GpAttnBranch(ctypes.Structure):
    """struct GpAttnBranch (include/gigapath_hip.h)."""
    _fields_ = [("seg_len", c_i32), ("ratio", c_i32), ("k", c_vp), ("v", c_vp), ("kv_row_stride", c_i64),
                ("kv_tok_base", c_i64), ("kv_sparse_cols", c_i32), ("o", c_vp), ("lse", c_vp),
                ("key_part", c_i32), ("key_parts", c_i32)]

# name -> argtypes (mirrors include/gigapath_hip.h)
SIGNATURES = {
    "gp_abi_version": [],
    "gp_last_error_string": [],
    "gp_coords_to_pos": [c_vp, c_i32, c_i64, c_i32, c_f64, c_vp, c_vp, c_vp],
    "gp_posembed_cls_ln": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp,
                           c_i32, c_vp],
    "gp_dilated_gather": [c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp],
    "gp_dilated_attn_fwd": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp,
                            c_f32, c_i32, c_i32, c_vp],
    "gp_dilated_attn_fwd_ex": [c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i64, c_i64, c_vp, c_i32, c_f32,
                               c_i32, c_i32, c_vp],
    "gp_attn_launch_params": [c_vp, c_i32],
    "gp_dilated_sparsify": [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp,
                            c_vp, c_vp],
    "gp_dilated_sparsify_dests": [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_i32,
                                  c_vp, c_vp, c_vp],
    "gp_branch_merge_ln_window": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp,
                                  c_f32, c_vp, c_i32, c_vp],
    "gp_seg_attn_fwd": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_f32, c_vp, c_vp, c_vp],
    "gp_seg_attn_fwd_f16": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_f32, c_vp, c_vp, c_vp],
    "gp_branch_merge_ln": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_f32, c_vp, c_i32,
                           c_vp],
    "gp_residual_layernorm": [c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_i64, c_i32, c_i32, c_vp],
    "gp_residual2_layernorm": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_i64, c_i32, c_i32, c_vp],
    "gp_gelu_layernorm": [c_vp, c_vp, c_vp, c_f32, c_vp, c_i64, c_i32, c_i32, c_vp],
    "gp_layernorm_f32": [c_vp, c_i64, c_vp, c_vp, c_f32, c_vp, c_i64, c_i32, c_vp],
    "gp_mean_tokens": [c_vp, c_i64, c_i64, c_i32, c_i64, c_vp, c_vp],
    "gp_varlen_plan_bytes": [c_i32, c_i32],
    "gp_varlen_plan": [c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp],
    "gp_dilated_attn_fwd_varlen": [c_vp, c_vp, c_i32, c_i32, c_vp],
    "gp_branch_merge_ln_varlen": [c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_i32, c_vp],
    "gp_gemm_workspace_bytes": [c_i64, c_i64, c_i64],
    "gp_linear": [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i32, c_vp],
    "gp_ffn_fc1_gelu": [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_i32, c_vp],
    "gp_ffn_fc2_ln": [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_f32, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64,
                      c_i32, c_vp],
    "gp_linear_resid": [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_f32, c_vp, c_i64,
                        c_i64, c_i64, c_vp, c_i64, c_i32, c_vp],
    "gp_linear_ln": [c_vp, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64,
                     c_i64, c_vp, c_i64, c_i32, c_vp],
    "gp_ffn_fc1_gelu_ln": [c_vp, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_i64, c_vp,
                           c_i64, c_i64, c_i64, c_i32, c_vp],
    "gp_ffn_fc2_ln_resid": [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_f32, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                            c_vp, c_f32, c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i32, c_vp],
}
_RESTYPES = {"gp_last_error_string": ctypes.c_char_p, "gp_varlen_plan_bytes": c_i64, "gp_gemm_workspace_bytes": c_i64}

_lib = None


class HipLibraryError(RuntimeError):
    pass


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load (once) and type the C ABI.  Raises HipLibraryError if it is absent.  `path` loads another
    build of the same ABI without installing it (tools/attn_lab's A/B library); the typed wrappers
    below always call the in-tree product library."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise HipLibraryError(
            "libgigapath_hip.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C prov-gigapath-replication_amd/csrc`" % p)
    lib = ctypes.CDLL(p)
    for name, args in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if path is None:
                raise
            continue                        # a lab build exporting a subset of the ABI
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    if lib.gp_abi_version() != ABI_VERSION:
        raise HipLibraryError("ABI mismatch: library %d, binding %d" % (lib.gp_abi_version(), ABI_VERSION))
    if path is None:
        _lib = lib
    return lib


def _check(rc: int, name: str):
    if rc != 0:
        msg = _lib.gp_last_error_string().decode(errors="replace")
        raise RuntimeError("%s failed (rc=%d): %s" % (name, rc, msg))


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def _dev(t: torch.Tensor, dtype=None, name="tensor"):
    if not t.is_cuda:
        raise RuntimeError("gigapath HIP path: %s must be a ROCm device tensor (got %s)" % (name, t.device))
    if dtype is not None and t.dtype != dtype:
        raise TypeError("gigapath HIP path: %s must be %s (got %s)" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError("gigapath HIP path: %s must be contiguous" % name)
    return t


FMT_BF16, FMT_F16, FMT_F16_VBF16 = 0, 1, 2   # GP_FMT_* (include/gigapath_hip.h)
ACT_DTYPES = (torch.bfloat16, torch.float16)


def fmt_of(dtype: torch.dtype) -> int:
    """The C ABI's 16-bit activation format of a torch dtype (bf16 or fp16; anything else raises)."""
    if dtype == torch.bfloat16:
        return FMT_BF16
    if dtype == torch.float16:
        return FMT_F16
    raise TypeError("gigapath HIP path: 16-bit activations must be bf16 or fp16 (got %s)" % dtype)


def qkv_fmt_of(dtype: torch.dtype, v_bf16: bool) -> int:
    """The format of a fused q | k | v buffer: fmt_of(dtype), or FMT_F16_VBF16 for an fp16 buffer whose V
    third holds bf16 (written by linear / linear_ln with v_bf16, read by the attention entry points)."""
    f = fmt_of(dtype)
    return FMT_F16_VBF16 if (v_bf16 and f == FMT_F16) else f


def _i32_array(vals: Sequence[int]):
    return (ctypes.c_int32 * len(vals))(*[int(v) for v in vals])


def _ptr_array(ts: Sequence[torch.Tensor]):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


# ------------------------------------------------------------------------------------------
# typed wrappers
# ------------------------------------------------------------------------------------------
def coords_to_pos(coords: torch.Tensor, grid: int, tile_size: float, pos_out: torch.Tensor,
                  err_count: Optional[torch.Tensor]):
    lib = load_library()
    _dev(coords, name="coords")
    if coords.dtype not in (torch.float32, torch.float64):
        raise TypeError("coords must be float32 or float64")
    _dev(pos_out, torch.int64, "pos")
    n = coords.numel() // 2
    _check(lib.gp_coords_to_pos(_ptr(coords), int(coords.dtype == torch.float64), n, grid, float(tile_size),
                                _ptr(pos_out), _ptr(err_count), _stream()), "gp_coords_to_pos")


def posembed_cls_ln(xp, pos, tab, cls, B, N, E, G, ln_w, ln_b, eps, x_out, ln_out, row_mean=None):
    """row_mean ([rows] fp32 or None): each x_out row's mean (the first residual epilogue's shift)."""
    lib = load_library()
    fmt = fmt_of(xp.dtype)
    _dev(xp, name="xp"); _dev(pos, torch.int64, "pos"); _dev(tab, torch.float32, "tab")
    if cls is not None:
        _dev(cls, torch.float32, "cls")
    _dev(x_out, torch.float32, "x_out")
    if ln_out is not None:
        _dev(ln_out, xp.dtype, "ln_out")
    if row_mean is not None:
        _dev(row_mean, torch.float32, "row_mean")
        if row_mean.numel() < B * (N + (cls is not None)):
            raise ValueError("posembed_cls_ln: row_mean holds fewer than the output rows")
    _check(lib.gp_posembed_cls_ln(_ptr(xp), _ptr(pos), _ptr(tab), _ptr(cls), B, N, E, G, _ptr(ln_w), _ptr(ln_b),
                                  eps, _ptr(x_out), _ptr(ln_out), _ptr(row_mean), fmt, _stream()),
           "gp_posembed_cls_ln")


def dilated_gather(src, row_stride, col_off, B, L, H, D, sl, r, dst):
    lib = load_library()
    fmt_of(src.dtype)
    _dev(src, name="src"); _dev(dst, src.dtype, "dst")
    _check(lib.gp_dilated_gather(_ptr(src), row_stride, col_off, B, L, H, D, sl, r, _ptr(dst), _stream()),
           "gp_dilated_gather")


def dilated_attn_fwd(q, k, v, row_stride, B, L, H, D, segs, ratios, outs, lses, softmax_scale=0.0,
                     q_log2_prescaled=False, v_bf16=False):
    """v_bf16 (fp16 q only): v holds bf16 values (the fused QKV of linear(..., v_bf16=True)); o stays fp16."""
    lib = load_library()
    fmt = qkv_fmt_of(q.dtype, v_bf16)
    for t in (q, k, v):
        if not t.is_cuda or t.dtype != q.dtype:
            raise TypeError("q/k/v must be device tensors of one 16-bit dtype")
    for o in outs:
        _dev(o, q.dtype, "o")
    oa, la = _ptr_array(outs), _ptr_array(lses)
    _check(lib.gp_dilated_attn_fwd(_ptr(q), _ptr(k), _ptr(v), row_stride, B, L, H, D, _i32_array(segs),
                                   _i32_array(ratios), len(segs), oa, la, float(softmax_scale),
                                   int(bool(q_log2_prescaled)), fmt, _stream()),
           "gp_dilated_attn_fwd")


def attn_branch(sl, r, k, v, kv_row_stride, kv_tok_base, kv_sparse_cols, o, lse, key_part=0,
                key_parts=1) -> GpAttnBranch:
    """One GpAttnBranch descriptor; k / v are device tensors (views allowed) or raw pointers.  key_part /
    key_parts (ABI 10): attend to one part of the keys only (GpAttnBranch.key_parts)."""
    kp = k if isinstance(k, int) else k.data_ptr()
    vp = v if isinstance(v, int) else v.data_ptr()
    return GpAttnBranch(int(sl), int(r), kp, vp, int(kv_row_stride), int(kv_tok_base), int(bool(kv_sparse_cols)),
                        o.data_ptr(), lse.data_ptr(), int(key_part), int(key_parts))


def dilated_attn_fwd_ex(q, q_row_stride, q_tok_base, B, L, H, D, win_lo, win_hi, branches, softmax_scale=0.0,
                        q_log2_prescaled=False, v_bf16=False):
    """branches: sequence of GpAttnBranch (attn_branch).  v_bf16: as dilated_attn_fwd."""
    lib = load_library()
    if not q.is_cuda:
        raise TypeError("q must be a device tensor")
    fmt = qkv_fmt_of(q.dtype, v_bf16)     # k / o of the descriptors are in q's format, v too unless v_bf16
    arr = (GpAttnBranch * len(branches))(*branches)
    _check(lib.gp_dilated_attn_fwd_ex(_ptr(q), q_row_stride, q_tok_base, B, L, H, D, win_lo, win_hi,
                                      ctypes.cast(arr, c_vp), len(branches), float(softmax_scale),
                                      int(bool(q_log2_prescaled)), fmt, _stream()), "gp_dilated_attn_fwd_ex")


def attn_launch_params() -> dict:
    """The built library's attention launch constants (gp_attn_launch_params): query rows per 8-wave work
    item, resident 8-wave workgroups per CU, the under-filled threshold (items per CU; 0 = the 4-wave switch
    is off) and the largest key_parts.  Host only: works without a GPU."""
    lib = load_library()
    buf = (c_i32 * 4)()
    _check(lib.gp_attn_launch_params(ctypes.cast(buf, c_vp), 4), "gp_attn_launch_params")
    return {"qblk": buf[0], "wg_per_cu": buf[1], "small_per_cu": buf[2], "max_key_parts": buf[3]}


def kv_layout_fast(k_ptr: int, v_ptr: int, kv_row_stride: int, ratio: int, D: int = 48) -> bool:
    """gp_attn.hip's LDS-DMA layout condition for one branch (attn_fwd_impl's kv_desc_ok): v at or after k,
    a row stride covering v's offset plus one head, 32-bit tile offsets.  Key parts need it."""
    dv = int(v_ptr) - int(k_ptr)
    rs2 = 2 * int(kv_row_stride)
    return dv >= 0 and rs2 >= dv + 2 * D and dv + 64 * int(ratio) * rs2 < 0x7fffffff


def dilated_sparsify(src, src_row_stride, k_col, v_col, tok_lo, n_tok, L, H, D, segs, ratios, dsts, dst_bases=None):
    lib = load_library()
    fmt_of(src.dtype)
    _dev(src, name="src")
    for t in dsts:
        _dev(t, src.dtype, "dst")
    bases = None if dst_bases is None else (ctypes.c_int64 * len(dst_bases))(*[int(b) for b in dst_bases])
    _check(lib.gp_dilated_sparsify(_ptr(src), src_row_stride, k_col, v_col, tok_lo, n_tok, L, H, D, _i32_array(segs),
                                   _i32_array(ratios), len(segs), _ptr_array(dsts), bases, _stream()),
           "gp_dilated_sparsify")


def dilated_sparsify_dests(src, src_row_stride, k_col, v_col, tok_lo, n_tok, L, H, D, segs, ratios, dests):
    """dests[b] = list of (tok_lo, tok_hi, tensor, row_offset): token p of branch b is written to
    row row_offset + (p - tok_lo) of that [rows, 2C] bf16 tensor."""
    lib = load_library()
    fmt_of(src.dtype)
    _dev(src, name="src")
    arr = (GpRowDest * (MAX_DESTS * len(segs)))()
    nd = (ctypes.c_int32 * len(segs))()
    for b, lst in enumerate(dests):
        if len(lst) > MAX_DESTS:
            raise ValueError("at most %d destinations per branch" % MAX_DESTS)
        nd[b] = len(lst)
        for d, (lo, hi, t, off) in enumerate(lst):
            _dev(t, src.dtype, "dst")
            if off < 0 or off + (hi - lo) > t.shape[0]:
                raise ValueError("sparsify destination rows [%d, %d) outside a %d-row buffer" % (off, off + hi - lo,
                                                                                               t.shape[0]))
            arr[b * MAX_DESTS + d] = GpRowDest(int(lo), int(hi), t.data_ptr() + int(off) * t.stride(0) * 2)
    _check(lib.gp_dilated_sparsify_dests(_ptr(src), src_row_stride, k_col, v_col, tok_lo, n_tok, L, H, D,
                                         _i32_array(segs), _i32_array(ratios), len(segs), ctypes.cast(arr, c_vp),
                                         nd, _stream()), "gp_dilated_sparsify_dests")


def branch_merge_ln_window(outs, lses, segs, ratios, B, L, tok_lo, n_tok, H, D, ln_w, ln_b, eps, out):
    lib = load_library()
    fmt = fmt_of(out.dtype)
    _dev(out, name="out")
    for o in outs:
        _dev(o, out.dtype, "o")
    _check(lib.gp_branch_merge_ln_window(_ptr_array(outs), _ptr_array(lses), _i32_array(segs), _i32_array(ratios),
                                         len(segs), B, L, tok_lo, n_tok, H, D, _ptr(ln_w), _ptr(ln_b), eps, _ptr(out),
                                         fmt, _stream()), "gp_branch_merge_ln_window")


def seg_attn_fwd(q, k, v, o, lse, softmax_scale=0.0):
    """flash_attn_func seam: bf16 q/k/v/o -> gp_seg_attn_fwd, fp16 -> gp_seg_attn_fwd_f16."""
    lib = load_library()
    nb, sl, H, D = q.shape
    dt = q.dtype if q.dtype in (torch.bfloat16, torch.float16) else torch.bfloat16
    for nm, t in (("q", q), ("k", k), ("v", v), ("o", o)):
        _dev(t, dt, nm)
    _dev(lse, torch.float32, "lse")
    fn, name = (lib.gp_seg_attn_fwd_f16, "gp_seg_attn_fwd_f16") if dt == torch.float16 else \
        (lib.gp_seg_attn_fwd, "gp_seg_attn_fwd")
    _check(fn(_ptr(q), _ptr(k), _ptr(v), nb, sl, H, D, float(softmax_scale), _ptr(o), _ptr(lse), _stream()), name)


def branch_merge_ln(outs, lses, segs, ratios, B, L, H, D, ln_w, ln_b, eps, out):
    lib = load_library()
    fmt = fmt_of(out.dtype)
    _dev(out, name="out")
    for o in outs:
        _dev(o, out.dtype, "o")
    _check(lib.gp_branch_merge_ln(_ptr_array(outs), _ptr_array(lses), _i32_array(segs), _i32_array(ratios),
                                  len(segs), B, L, H, D, _ptr(ln_w), _ptr(ln_b), eps, _ptr(out), fmt, _stream()),
           "gp_branch_merge_ln")


def residual_layernorm(x, y, bias, ln_w, ln_b, eps, ln_out, rows, cols):
    lib = load_library()
    fmt = fmt_of(y.dtype)
    _dev(x, torch.float32, "x"); _dev(y, name="y")
    if ln_out is not None:
        _dev(ln_out, y.dtype, "ln_out")
    _check(lib.gp_residual_layernorm(_ptr(x), _ptr(y), _ptr(bias), _ptr(ln_w), _ptr(ln_b), eps, _ptr(ln_out),
                                     rows, cols, fmt, _stream()), "gp_residual_layernorm")


def residual2_layernorm(x, y1, b1, y2, b2, ln_w, ln_b, eps, ln_out, rows, cols):
    """gp_residual2_layernorm: y2 None -> ln_out = LN(x + (y1 + b1)), x unchanged; else x = x + (y1 + b1) +
    (y2 + b2) (two roundings, as two residual_layernorm calls) and ln_out = LN(x)."""
    lib = load_library()
    fmt = fmt_of(y1.dtype)
    _dev(x, torch.float32, "x"); _dev(y1, name="y1")
    if y2 is not None:
        _dev(y2, y1.dtype, "y2")
    if ln_out is not None:
        _dev(ln_out, y1.dtype, "ln_out")
    _check(lib.gp_residual2_layernorm(_ptr(x), _ptr(y1), _ptr(b1), _ptr(y2), _ptr(b2), _ptr(ln_w), _ptr(ln_b), eps,
                                      _ptr(ln_out), rows, cols, fmt, _stream()), "gp_residual2_layernorm")


def gelu_layernorm(h, ln_w, ln_b, eps, out, rows, cols):
    lib = load_library()
    fmt = fmt_of(h.dtype)
    _dev(h, name="h"); _dev(out, h.dtype, "out")
    _check(lib.gp_gelu_layernorm(_ptr(h), _ptr(ln_w), _ptr(ln_b), eps, _ptr(out), rows, cols, fmt, _stream()),
           "gp_gelu_layernorm")


def layernorm_f32(x, row_stride, ln_w, ln_b, eps, out, rows, cols):
    lib = load_library()
    if not x.is_cuda or x.dtype != torch.float32:
        raise TypeError("x must be an fp32 device tensor")
    _dev(out, torch.float32, "out")
    _check(lib.gp_layernorm_f32(_ptr(x), row_stride, _ptr(ln_w), _ptr(ln_b), eps, _ptr(out), rows, cols,
                                _stream()), "gp_layernorm_f32")


def mean_tokens(x, B, L, E, start, out):
    lib = load_library()
    _dev(x, torch.float32, "x"); _dev(out, torch.float32, "out")
    _check(lib.gp_mean_tokens(_ptr(x), B, L, E, start, _ptr(out), _stream()), "gp_mean_tokens")


# ------------------------------------------------------------------------------------------
# varlen packing (several slides in one launch per op; include/gigapath_hip.h "Varlen packing")
# ------------------------------------------------------------------------------------------
class VarlenPlan:
    """Work table of `Ls` slides packed token-major in one [T, 3E] qkv buffer.

    ``VarlenPlan(Ls, H, D, segs, ratios)`` sizes the packed per-branch outputs (``o_elems``,
    ``lse_elems``); ``bind(qkv, outs, lses)`` writes the table (device pointers into those
    tensors) and copies it to the device.  The tensors must outlive every launch using the plan."""

    def __init__(self, Ls: Sequence[int], H: int, D: int, segs: Sequence[int], ratios: Sequence[int]):
        lib = load_library()
        self.Ls = [int(x) for x in Ls]
        self.H, self.D, self.segs, self.ratios = H, D, list(segs), list(ratios)
        nb = len(self.segs)
        self._L = (c_i64 * len(self.Ls))(*self.Ls)
        o_el, l_el = (c_i64 * nb)(), (c_i64 * nb)()
        _check(lib.gp_varlen_plan(self._L, len(self.Ls), H, D, _i32_array(self.segs), _i32_array(self.ratios), nb,
                                  None, 3 * H * D, None, None, None, 0, o_el, l_el), "gp_varlen_plan")
        self.o_elems, self.lse_elems = list(o_el), list(l_el)
        self.nbytes = int(lib.gp_varlen_plan_bytes(len(self.Ls), nb))
        self.tok_off = [0]
        for L in self.Ls:
            self.tok_off.append(self.tok_off[-1] + L)
        self.host = None
        self.dev = None

    def bind(self, qkv: torch.Tensor, outs: Sequence[torch.Tensor], lses: Sequence[torch.Tensor]):
        lib = load_library()
        self.fmt = fmt_of(qkv.dtype)
        _dev(qkv, name="qkv")
        if qkv.shape[0] < self.tok_off[-1] or qkv.shape[1] != 3 * self.H * self.D:
            raise ValueError("VarlenPlan.bind: qkv must be [>= %d, %d]" % (self.tok_off[-1], 3 * self.H * self.D))
        for b, (o, l) in enumerate(zip(outs, lses)):
            _dev(o, qkv.dtype, "o[%d]" % b); _dev(l, torch.float32, "lse[%d]" % b)
            if o.numel() < self.o_elems[b] or l.numel() < self.lse_elems[b]:
                raise ValueError("VarlenPlan.bind: branch %d outputs too small" % b)
        host = (ctypes.c_uint8 * self.nbytes)()
        o_el, l_el = (c_i64 * len(self.segs))(), (c_i64 * len(self.segs))()
        _check(lib.gp_varlen_plan(self._L, len(self.Ls), self.H, self.D, _i32_array(self.segs),
                                  _i32_array(self.ratios), len(self.segs), _ptr(qkv), 3 * self.H * self.D,
                                  _ptr_array(outs), _ptr_array(lses), host, self.nbytes, o_el, l_el),
               "gp_varlen_plan")
        self.host = host
        self.dev = torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8).to(qkv.device)
        self._keep = (qkv, list(outs), list(lses))
        return self


def dilated_attn_fwd_varlen(plan: VarlenPlan, q_log2_prescaled: bool = True, v_bf16: bool = False):
    lib = load_library()
    fmt = FMT_F16_VBF16 if (v_bf16 and plan.fmt == FMT_F16) else plan.fmt
    _check(lib.gp_dilated_attn_fwd_varlen(plan.host, _ptr(plan.dev), int(bool(q_log2_prescaled)), fmt,
                                          _stream()), "gp_dilated_attn_fwd_varlen")


def branch_merge_ln_varlen(plan: VarlenPlan, ln_w, ln_b, eps, out):
    lib = load_library()
    _dev(out, name="out")
    if fmt_of(out.dtype) != plan.fmt:
        raise TypeError("branch_merge_ln_varlen: out must be in the plan's 16-bit format")
    _check(lib.gp_branch_merge_ln_varlen(plan.host, _ptr(plan.dev), _ptr(ln_w), _ptr(ln_b), eps, _ptr(out),
                                         plan.fmt, _stream()), "gp_branch_merge_ln_varlen")


# ------------------------------------------------------------------------------------------
# projection GEMMs (include/gigapath_hip.h "Projection GEMMs on MFMAs")
# ------------------------------------------------------------------------------------------
GEMM_K_E = (768, 1024, 1536)        # K = E of the three registered archs (QKV, out-proj, fc1; patch 1536)
GEMM_K_F = (3072, 4096, 6144)       # K = F = 4E (fc2)
GEMM_K = GEMM_K_E + GEMM_K_F


def gemm_supported(N: int, K: int) -> bool:
    """Shapes the MFMA GEMM kernels are instantiated for (N a multiple of 256, K = E or 4E of a registered arch;
    gp_linear / gp_linear_ln cover both, the residual / fc1 epilogues K = E, the fc2 epilogues K = 4E)."""
    return N % 256 == 0 and N > 0 and K in GEMM_K


def gemm_workspace_bytes(M: int, N: int, K: int) -> int:
    return int(load_library().gp_gemm_workspace_bytes(M, N, K))


def _rows(t, name):
    if not t.is_cuda or t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("gigapath HIP path: %s must be a row-major 2-D device tensor" % name)
    return t


def _ws(ws):
    return (None, 0) if ws is None else (ws.data_ptr(), ws.numel() * ws.element_size())


def linear(a, w, bias, out, ws=None, v_bf16=False):
    """out = a . w^T (+ bias): a [M, K], w [N, K], out [M, N] act; bias [N] fp32 or None.  v_bf16 (fp16 a, a
    fused q | k | v output): the last third of out's columns is written in bf16 (FMT_F16_VBF16)."""
    lib = load_library()
    fmt = qkv_fmt_of(a.dtype, v_bf16)
    _rows(a, "a"); _rows(w, "w"); _rows(out, "out")
    if w.dtype != a.dtype or out.dtype != a.dtype:
        raise TypeError("linear: a, w and out must share one 16-bit dtype")
    if bias is not None:
        _dev(bias, torch.float32, "bias")
    wp, wb = _ws(ws)
    _check(lib.gp_linear(_ptr(a), a.stride(0), _ptr(w), w.stride(0), _ptr(bias), _ptr(out), out.stride(0), a.shape[0],
                         w.shape[0], a.shape[1], wp, wb, fmt, _stream()), "gp_linear")


def ffn_fc1_gelu(a, w1, b1, h, stats):
    """h = act(gelu(a . w1^T + b1)), stats [F/256 + 1, M, 2] fp32 (per 256-column (mean, M2) of h; the
    last plane is gp_ffn_fc2_ln's row (mean, rstd))."""
    lib = load_library()
    fmt = fmt_of(a.dtype)
    _rows(a, "a"); _rows(w1, "w1"); _rows(h, "h")
    if w1.dtype != a.dtype or h.dtype != a.dtype:
        raise TypeError("ffn_fc1_gelu: a, w1 and h must share one 16-bit dtype")
    _dev(stats, torch.float32, "stats")
    M, F = a.shape[0], w1.shape[0]
    if stats.numel() < (F // 256 + 1) * M * 2:
        raise ValueError("ffn_fc1_gelu: stats must hold [F/256 + 1, M, 2] floats")
    if b1 is not None:
        _dev(b1, torch.float32, "b1")
    _check(lib.gp_ffn_fc1_gelu(_ptr(a), a.stride(0), _ptr(w1), w1.stride(0), _ptr(b1), _ptr(h), h.stride(0),
                               _ptr(stats), M, F, a.shape[1], fmt, _stream()), "gp_ffn_fc1_gelu")


def ffn_fc2_ln(h, w2g, stats, c, d, eps, y, ws=None):
    """y = act(LN(h) . w2^T + b2) through the fold: w2g = w2 * gamma, c = rowsum(w2g), d = w2 . beta + b2."""
    lib = load_library()
    fmt = fmt_of(h.dtype)
    _rows(h, "h"); _rows(w2g, "w2g"); _rows(y, "y")
    if w2g.dtype != h.dtype or y.dtype != h.dtype:
        raise TypeError("ffn_fc2_ln: h, w2g and y must share one 16-bit dtype")
    for nm, t in (("stats", stats), ("c", c), ("d", d)):
        _dev(t, torch.float32, nm)
    M, F, N = h.shape[0], h.shape[1], w2g.shape[0]
    if stats.numel() < (F // 256 + 1) * M * 2:
        raise ValueError("ffn_fc2_ln: stats must hold [F/256 + 1, M, 2] floats")
    wp, wb = _ws(ws)
    _check(lib.gp_ffn_fc2_ln(_ptr(h), h.stride(0), _ptr(w2g), w2g.stride(0), _ptr(stats), _ptr(c), _ptr(d), float(eps),
                             _ptr(y), y.stride(0), M, N, F, wp, wb, fmt, _stream()), "gp_ffn_fc2_ln")


# ------------------------------------------------------------------------------------------
# the residual stream inside the GEMMs (include/gigapath_hip.h, ABI 7)
# ------------------------------------------------------------------------------------------
def _f32_vec(t, n, name):
    _dev(t, torch.float32, name)
    if t.numel() < n:
        raise ValueError("%s must hold %d floats" % (name, n))
    return t


def _merge_args(gamma, xstats, N, M, eps_next, s_out, who):
    """The producer-side statistics merge (round 5): s_out [M] fp32 and eps_next, xstats with plane N/256."""
    if s_out is None:
        return 0.0, None
    if gamma is None or eps_next is None or eps_next <= 0:
        raise ValueError("%s: s_out (the statistics merge) needs gamma and eps_next > 0" % who)
    _f32_vec(s_out, M, "s_out"); _f32_vec(xstats, (N // 256 + 1) * M * 2, "xstats")
    return float(eps_next), s_out


def linear_resid(a, w, bias, x, shift, gamma, xb, xstats, ws=None, eps_next=None, s_out=None):
    """x += a . w^T + bias (fp32 x [M, N], in place); with gamma: xb = act(gamma * (x - shift)) [M, N] and
    xstats [N/256 (+1), M, 2] (mean, M2) of x - shift per 256-column group.  gamma None: x only.
    s_out (round 5): also merge the groups into plane N/256 (mean, rstd with eps_next) and write s_out = shift
    + the row mean -- the next LN-folding GEMM is then called with merged=True (no merge launch there)."""
    lib = load_library()
    fmt = fmt_of(a.dtype)
    _rows(a, "a"); _rows(w, "w"); _rows(x, "x")
    M, K, N = a.shape[0], a.shape[1], w.shape[0]
    if w.dtype != a.dtype or x.dtype != torch.float32 or x.shape[0] < M or x.shape[1] < N:
        raise TypeError("linear_resid: a / w share one 16-bit dtype; x is fp32 [M, N]")
    if bias is not None:
        _f32_vec(bias, N, "bias")
    if gamma is not None:
        _f32_vec(gamma, N, "gamma"); _f32_vec(shift, M, "shift"); _f32_vec(xstats, N // 256 * M * 2, "xstats")
        _rows(xb, "xb")
        if xb.dtype != a.dtype:
            raise TypeError("linear_resid: xb must be in a's 16-bit dtype")
    eps_next, s_out = _merge_args(gamma, xstats, N, M, eps_next, s_out, "linear_resid")
    wp, wb = _ws(ws)
    _check(lib.gp_linear_resid(_ptr(a), a.stride(0), _ptr(w), w.stride(0), _ptr(bias), _ptr(x), x.stride(0),
                               _ptr(shift if gamma is not None else None), _ptr(gamma),
                               _ptr(xb if gamma is not None else None), xb.stride(0) if gamma is not None else 0,
                               _ptr(xstats if gamma is not None else None), eps_next, _ptr(s_out), M, N, K, wp, wb,
                               fmt, _stream()), "gp_linear_resid")


def linear_ln(a, w, stats, nst, c, d, eps, s_in, s_out, out, ws=None, v_bf16=False, merged=False):
    """out = act(LN(x) . w^T + b) through the fold: a = xb = act(gamma * (x - s_in)), stats planes 0 .. nst-1
    merged into plane nst (s_out = s_in + mean' when given), c = w . gamma, d = w . beta + b.  v_bf16: as
    linear.  merged: the producer already merged plane nst and wrote s_out (linear_resid(..., s_out=))."""
    lib = load_library()
    fmt = qkv_fmt_of(a.dtype, v_bf16)
    _rows(a, "a"); _rows(w, "w"); _rows(out, "out")
    if w.dtype != a.dtype or out.dtype != a.dtype:
        raise TypeError("linear_ln: a, w and out must share one 16-bit dtype")
    M, K, N = a.shape[0], a.shape[1], w.shape[0]
    _f32_vec(stats, (nst + 1) * M * 2, "stats"); _f32_vec(c, N, "c"); _f32_vec(d, N, "d")
    for nm, t in (("s_in", s_in), ("s_out", s_out)):
        if t is not None:
            _f32_vec(t, M, nm)
    wp, wb = _ws(ws)
    _check(lib.gp_linear_ln(_ptr(a), a.stride(0), _ptr(w), w.stride(0), _ptr(stats), -int(nst) if merged else int(nst),
                            _ptr(c), _ptr(d),
                            float(eps), _ptr(s_in), _ptr(s_out), _ptr(out), out.stride(0), M, N, K, wp, wb, fmt,
                            _stream()), "gp_linear_ln")


def ffn_fc1_gelu_ln(a, w1, xstats, nst, c1, d1, eps, s_in, s_out, h, hstats, merged=False):
    """gp_ffn_fc1_gelu with final_layer_norm folded as in linear_ln (a = xb; merged as there)."""
    lib = load_library()
    fmt = fmt_of(a.dtype)
    _rows(a, "a"); _rows(w1, "w1"); _rows(h, "h")
    if w1.dtype != a.dtype or h.dtype != a.dtype:
        raise TypeError("ffn_fc1_gelu_ln: a, w1 and h must share one 16-bit dtype")
    M, K, F = a.shape[0], a.shape[1], w1.shape[0]
    _f32_vec(xstats, (nst + 1) * M * 2, "xstats"); _f32_vec(c1, F, "c1"); _f32_vec(d1, F, "d1")
    _f32_vec(hstats, (F // 256 + 1) * M * 2, "hstats")
    for nm, t in (("s_in", s_in), ("s_out", s_out)):
        if t is not None:
            _f32_vec(t, M, nm)
    _check(lib.gp_ffn_fc1_gelu_ln(_ptr(a), a.stride(0), _ptr(w1), w1.stride(0), _ptr(xstats),
                                  -int(nst) if merged else int(nst), _ptr(c1),
                                  _ptr(d1), float(eps), _ptr(s_in), _ptr(s_out), _ptr(h), h.stride(0), _ptr(hstats),
                                  M, F, K, fmt, _stream()), "gp_ffn_fc1_gelu_ln")


def ffn_fc2_ln_resid(h, w2g, hstats, c, d, eps, x, shift, gamma, xb, xstats, ws=None, eps_next=None, s_out=None):
    """x += fc2(ffn_layernorm(h)) through the fold; with gamma: xb / xstats (and the merge: s_out, eps_next) as
    linear_resid."""
    lib = load_library()
    fmt = fmt_of(h.dtype)
    _rows(h, "h"); _rows(w2g, "w2g"); _rows(x, "x")
    M, F, N = h.shape[0], h.shape[1], w2g.shape[0]
    if w2g.dtype != h.dtype or x.dtype != torch.float32 or x.shape[0] < M or x.shape[1] < N:
        raise TypeError("ffn_fc2_ln_resid: h / w2g share one 16-bit dtype; x is fp32 [M, N]")
    _f32_vec(hstats, (F // 256 + 1) * M * 2, "hstats"); _f32_vec(c, N, "c"); _f32_vec(d, N, "d")
    if gamma is not None:
        _f32_vec(gamma, N, "gamma"); _f32_vec(shift, M, "shift"); _f32_vec(xstats, N // 256 * M * 2, "xstats")
        _rows(xb, "xb")
        if xb.dtype != h.dtype:
            raise TypeError("ffn_fc2_ln_resid: xb must be in h's 16-bit dtype")
    eps_next, s_out = _merge_args(gamma, xstats, N, M, eps_next, s_out, "ffn_fc2_ln_resid")
    wp, wb = _ws(ws)
    _check(lib.gp_ffn_fc2_ln_resid(_ptr(h), h.stride(0), _ptr(w2g), w2g.stride(0), _ptr(hstats), _ptr(c), _ptr(d),
                                   float(eps), _ptr(x), x.stride(0), _ptr(shift if gamma is not None else None),
                                   _ptr(gamma), _ptr(xb if gamma is not None else None),
                                   xb.stride(0) if gamma is not None else 0,
                                   _ptr(xstats if gamma is not None else None), eps_next, _ptr(s_out), M, N, F, wp,
                                   wb, fmt, _stream()), "gp_ffn_fc2_ln_resid")
