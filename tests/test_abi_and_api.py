"""CPU-side checks of the product: the C-ABI library loads and exports every symbol the header
declares, and the Python drop-in mirrors the reference API (no GPU needed, no compute calls)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest
import torch

from conftest import GOLDEN, PKG_ROOT, ROOT, load_golden

HEADER = os.path.join(ROOT, "include", "gigapath_hip.h")


def _lib_path():
    from gigapath import _hip
    if not os.path.exists(_hip.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(PKG_ROOT, "csrc"), "-j8"], check=True,
                       stdout=subprocess.DEVNULL)
    return _hip.LIB_PATH


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gp_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for f in ("gp_coords_to_pos", "gp_posembed_cls_ln", "gp_dilated_gather", "gp_dilated_attn_fwd",
              "gp_seg_attn_fwd", "gp_branch_merge_ln", "gp_residual_layernorm", "gp_gelu_layernorm",
              "gp_layernorm_f32", "gp_mean_tokens", "gp_abi_version", "gp_last_error_string"):
        assert f in fns


def test_library_exports_every_header_symbol():
    path = _lib_path()
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gp_[a-z0-9_]+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


def test_library_loads_and_binding_covers_header():
    _lib_path()
    from gigapath import _hip
    lib = _hip.load_library()
    assert lib.gp_abi_version() == _hip.ABI_VERSION
    assert set(_hip.SIGNATURES) == set(header_functions())
    assert lib.gp_last_error_string() == b""


def test_library_is_gfx950_code():
    blob = open(_lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob          # embedded code-object target id


def test_argument_errors_are_reported_without_gpu():
    """Bad arguments are rejected on the host before any launch (GP_EARG + message)."""
    _lib_path()
    from gigapath import _hip
    lib = _hip.load_library()
    rc = lib.gp_dilated_attn_fwd(None, None, None, 0, 1, 10, 16, 40, None, None, 1, None, None, 0.0, 0, 0, None)
    assert rc == -1
    assert b"head dim 40" in lib.gp_last_error_string()
    rc = lib.gp_residual_layernorm(None, None, None, None, None, 1e-5, None, 4, 100, 0, None)
    assert rc == -1 and b"cols=100" in lib.gp_last_error_string()
    rc = lib.gp_gelu_layernorm(None, None, None, 1e-5, None, 4, 3072, 7, None)     # fmt: GP_FMT_BF16 / GP_FMT_F16
    assert rc == -1 and b"bad fmt 7" in lib.gp_last_error_string()
    br = (_hip.GpAttnBranch * 1)(_hip.GpAttnBranch(1024, 1, 16, 16, 2304, 0, 0, 16, 16))
    rc = lib.gp_dilated_attn_fwd_ex(16, 2304, 0, 1, 100, 16, 48, 50, 101, br, 1, 0.0, 0, 0, None)
    assert rc == -1 and b"bad window" in lib.gp_last_error_string()
    rc = lib.gp_dilated_sparsify(16, 2304, 768, 1536, 0, 10, 100, 16, 48, (ctypes.c_int32 * 1)(1024),
                                 (ctypes.c_int32 * 1)(3), 1, (ctypes.c_void_p * 1)(16), None, None)
    assert rc == -1 and b"H % r == 0" in lib.gp_last_error_string()
    rc = lib.gp_branch_merge_ln_window(None, None, None, None, 1, 1, 100, 90, 20, 16, 48, None, None, 1e-5, None, 0, None)
    assert rc == -1


def test_varlen_plan_host_side():
    """gp_varlen_plan is host-only: sizes of the packed per-branch outputs follow each slide's own
    schedule (runtime.branch_geometry), the plan header is checked before any launch."""
    _lib_path()
    from gigapath import _hip, runtime
    segs, ratios = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]
    Ls = [1025, 2897, 700, 70001, 6001]
    plan = _hip.VarlenPlan(Ls, 16, 48, segs, ratios)
    for b, (sl, r) in enumerate(zip(segs, ratios)):
        geo = [runtime.branch_geometry(L, sl, r) for L in Ls]
        assert plan.o_elems[b] == sum(n * m * 16 * 48 for _, n, m in geo)
        assert plan.lse_elems[b] == sum(n * 16 * m for _, n, m in geo)
    assert plan.tok_off == [0, 1025, 3922, 4622, 74623, 80624]
    assert plan.nbytes > 0 and plan.nbytes % 16 == 0
    lib = _hip.load_library()
    assert lib.gp_varlen_plan_bytes(0, 5) == -1
    fake = (ctypes.c_uint8 * 64)()
    rc = lib.gp_dilated_attn_fwd_varlen(fake, 16, 1, 0, None)
    assert rc == -1 and b"not a gp_varlen_plan" in lib.gp_last_error_string()
    L_bad = (ctypes.c_int64 * 1)(0)
    el = (ctypes.c_int64 * 5)()
    rc = lib.gp_varlen_plan(L_bad, 1, 16, 48, (ctypes.c_int32 * 5)(*segs), (ctypes.c_int32 * 5)(*ratios), 5,
                            None, 2304, None, None, None, 0, el, el)
    assert rc == -1 and b"L = 0" in lib.gp_last_error_string()


# ------------------------------------------------------------------ Python drop-in surface
@pytest.fixture(scope="module")
def model():
    from gigapath import slide_encoder
    return slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536)


def test_state_dict_matches_reference(model, golden_meta):
    sd = model.state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == golden_meta["state_dict"]
    assert sum(p.numel() for p in model.parameters()) == 86330880


def test_registered_architectures():
    from gigapath import slide_encoder
    assert slide_encoder.list_models() == ["gigapath_slide_enc12l1536d", "gigapath_slide_enc12l768d",
                                           "gigapath_slide_enc24l1024d"]
    with pytest.raises(RuntimeError):
        slide_encoder.create_model("", "no_such_model", 1536)


def test_segment_schedule_and_config(model, golden_meta):
    args = model.encoder.layers[0].self_attn.args
    assert args.segment_length == [1024, 5792, 32768, 185363, 1048576]
    assert args.dilated_ratio == [1, 2, 4, 8, 16]
    for mw, segs in golden_meta["schedules"].items():
        assert eval(model.get_optimal_segment_length(int(mw), 256)) == segs


def test_loads_seeded_weights_strict(model):
    import oracle
    W = oracle.make_weights(oracle.arch_config("gigapath_slide_enc12l768d"), seed=0)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)


def test_create_model_loads_checkpoint(tmp_path, capsys):
    import oracle
    from gigapath import slide_encoder
    W = oracle.make_weights(oracle.arch_config("gigapath_slide_enc12l768d"), seed=0)
    sd = {k: torch.from_numpy(v) for k, v in W.items()}
    sd.pop("norm.bias")
    sd["extra.key"] = torch.zeros(1)
    p = tmp_path / "slide_encoder.pth"
    torch.save({"model": sd}, p)
    m = slide_encoder.create_model(str(p), "gigapath_slide_enc12l768d", 1536)
    out = capsys.readouterr().out
    assert "Missing  norm.bias" in out and "Unexpected  extra.key" in out
    assert torch.equal(m.cls_token, sd["cls_token"])


def test_pos_table_product_bit_exact():
    from gigapath.pos_embed import axis_table
    import oracle
    g = load_golden("pos_embed_rows.npz")
    ours = oracle.pos_embed_rows(g["rows"], axis_table(768, 1000), 1000)
    assert np.array_equal(ours.view(np.uint32), g["values"].view(np.uint32))


def test_product_fails_loudly_on_cpu(model):
    model.eval()
    x = torch.zeros(1, 4, 1536)
    c = torch.zeros(1, 4, 2)
    with pytest.raises(RuntimeError, match="ROCm"):
        model(x, c)


def test_training_mode_is_rejected(model):
    model.train()
    with pytest.raises(RuntimeError, match="eval"):
        model(torch.zeros(1, 4, 1536), torch.zeros(1, 4, 2))
    model.eval()


def test_flops_model_matches_survey():
    from gigapath import runtime
    segs, ratios = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]
    att = 12 * runtime.attention_valid_flops(70001, segs, ratios, 16, 48)
    gemm = runtime.gemm_flops(1, 70000, 768, 3072, 1536, 12)
    assert abs(att / 1e12 - 14.868) < 0.01
    assert abs((att + gemm) / 1e12 - 26.924) < 0.01


def test_classification_head_surface():
    """The reference's slide-level caller (classification_head.py): same constructor, encoder
    frozen (inference-only engine), classifier over the selected layer embeddings."""
    from gigapath import classification_head
    head = classification_head.get_model(input_dim=1536, latent_dim=768, feat_layer="5-11", n_classes=3,
                                         model_arch="gigapath_slide_enc12l768d", pretrained="")
    assert head.feat_layer == [5, 11] and head.feat_dim == 1536
    assert head.classifier[0].weight.shape == (3, 1536)
    assert not any(p.requires_grad for p in head.slide_encoder.parameters())
    head.train()
    assert head.training and not head.slide_encoder.training
    assert sum(p.requires_grad for p in head.parameters()) == 2      # classifier weight + bias


def test_activation_format_selection():
    """runtime.call_act_dtype / compute_format: bf16 by default, fp16 for an fp16 model (the
    reference pipeline's autocast(float16) case is covered on the GPU, where autocast("cuda") is
    live); nested decorated calls keep the outer call's format; _hip.fmt_of maps the dtypes the C ABI
    accepts and rejects the rest."""
    _lib_path()
    import torch.nn as nn
    from gigapath import _hip, runtime
    lin = nn.Linear(4, 4)
    assert runtime.call_act_dtype(lin) == torch.bfloat16
    assert runtime.call_act_dtype(lin.half()) == torch.float16
    assert runtime.act_dtype() == torch.bfloat16                 # outside any decorated call

    class M(nn.Module):
        def __init__(self, half):
            super().__init__()
            self.p = nn.Parameter(torch.zeros(1, dtype=torch.float16 if half else torch.float32))

        @runtime.compute_format
        def forward(self, inner=None):
            seen = [runtime.act_dtype()]
            if inner is not None:
                seen += inner()
            return seen

    assert M(True)() == [torch.float16]
    assert M(True)(inner=M(False)) == [torch.float16, torch.float16]      # the outer call decides
    assert M(False)(inner=M(True)) == [torch.bfloat16, torch.bfloat16]
    assert runtime.act_dtype() == torch.bfloat16
    assert (_hip.fmt_of(torch.bfloat16), _hip.fmt_of(torch.float16)) == (_hip.FMT_BF16, _hip.FMT_F16)
    with pytest.raises(TypeError):
        _hip.fmt_of(torch.float32)


def test_graph_outputs_cloned_with_one_copy():
    """The graph replay's readouts (views of one [n_out, B, E] table) come back as views of ONE fresh copy
    (one copy launch instead of one per readout); independent outputs are cloned one by one."""
    from gigapath.slide_encoder import LongNetViT
    res = torch.randn(13, 2, 768)
    outs = [res[i] for i in range(13)]
    got = LongNetViT._clone_outputs(outs)
    assert all(torch.equal(a, b) for a, b in zip(got, outs))
    assert got[0].untyped_storage().data_ptr() == got[12].untyped_storage().data_ptr()
    assert got[0].untyped_storage().data_ptr() != res.untyped_storage().data_ptr()
    got[3].zero_()                      # the copies are disjoint views: the rest is untouched
    assert torch.equal(got[4], outs[4]) and not torch.equal(got[3], outs[3])
    loose = [torch.randn(2, 768) for _ in range(3)]
    got2 = LongNetViT._clone_outputs(loose)
    assert all(torch.equal(a, b) and a.data_ptr() != b.data_ptr() for a, b in zip(got2, loose))


def test_qkv_parts_views_v_in_its_stored_format():
    """PackedAttention.qkv_parts: under the fp16 caller's V-bf16 packing (ABI 8) the V third of the fp16 qkv
    buffer holds bf16 bits, and the helper hands it out as a bfloat16 view of the same memory; q / k stay
    fp16; without the flag (bf16 caller, or fp16 without V-bf16) every third keeps the buffer's dtype."""
    from gigapath import runtime
    E = 768
    pa = runtime.PackedAttention(E=E, H=16, D=48, segs=[1024], ratios=[1], w_qkv=None, b_qkv=None, w_o=None,
                                 b_o=None, b_o_act=None, ln_w=None, ln_b=None, ln_eps=1e-5, v_bf16=True)
    qkv = torch.zeros(5, 3 * E, dtype=torch.float16)
    vals = torch.randn(5, E)
    qkv[:, 2 * E:].view(torch.bfloat16).copy_(vals.to(torch.bfloat16))     # what the QKV GEMM writes
    q, k, v = pa.qkv_parts(qkv)
    assert (q.dtype, k.dtype, v.dtype) == (torch.float16, torch.float16, torch.bfloat16)
    assert v.data_ptr() == qkv.data_ptr() + 2 * E * 2
    assert torch.equal(v.float(), vals.to(torch.bfloat16).float())
    pa.v_bf16 = False
    assert pa.qkv_parts(qkv)[2].dtype == torch.float16
    pa.v_bf16 = True
    assert pa.qkv_parts(qkv.to(torch.bfloat16))[2].dtype == torch.bfloat16
