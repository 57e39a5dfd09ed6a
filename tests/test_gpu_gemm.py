"""The MFMA projection GEMMs and the fused FFN (csrc/gp_gemm.hip) against torch fp32 restatements of
the same ops on the same 16-bit inputs (run with -m gpu on an MI355X).

    gp_linear        nn.Linear (multihead_attention.py:43-48, feedforward_network.py:131-142)
    gp_ffn_fc1_gelu  fc1 + gelu(x.float()).type_as(x) + LN statistics (feedforward_network.py:131-135)
    gp_ffn_fc2_ln    ffn_layernorm + fc2 with the LN folded into the epilogue (:136-142)

Tolerances: outputs are 16-bit (one rounding: max |d| <= 1e-2 of max |ref|); h is compared
elementwise with the reference's two roundings (>= 97 % bit-identical, the rest within the propagation
of one 16-bit ulp of the pre-activation) and, for bf16, bit for bit with torch's GELU of the kernel's own
pre-activation (every bf16 input value included); the statistics to 1e-5 relative of the kernel's own h.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
ACTS = [torch.bfloat16, torch.float16]


def _hip():
    from gigapath import _hip
    _hip.load_library()
    return _hip


def _rand(shape, g, scale=1.0):
    return torch.randn(*shape, device=DEV, generator=g) * scale


def _rel(got, ref):
    return ((got.float() - ref).abs().max() / ref.abs().max()).item()


@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("M,N,K,bias", [(1, 256, 768, True), (17, 768, 768, False), (1000, 2304, 768, True),
                                        (4097, 768, 3072, False), (70001, 2304, 768, True),
                                        (70000, 768, 1536, True), (70001, 768, 3072, True)])
def test_linear_vs_fp32(act, M, N, K, bias):
    h = _hip()
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = _rand((M, K), g).to(act)
    w = _rand((N, K), g, K ** -0.5).to(act)
    b = _rand((N,), g, 0.1) if bias else None
    ref = a.float() @ w.float().t() + (b if bias else 0)
    nb = h.gemm_workspace_bytes(M, N, K)
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=DEV)
    for use_ws in (True, False):             # the split tail (workspace) and the all-data-parallel plan
        out = torch.full((M, N), float("nan"), dtype=act, device=DEV)
        h.linear(a, w, b, out, ws if use_ws else None)
        torch.cuda.synchronize()
        assert torch.isfinite(out.float()).all()
        assert _rel(out, ref) <= 1e-2, (use_ws, _rel(out, ref))


def test_linear_strided_rows_and_errors():
    """Row strides (a column window of a wider buffer), and the shape checks of the C ABI."""
    h = _hip()
    g = torch.Generator(device=DEV).manual_seed(3)
    base = _rand((300, 3 * 768), g).bfloat16()
    a = base[:, 768:1536]                     # lda = 2304
    w = _rand((768, 768), g, 768 ** -0.5).bfloat16()
    out_base = torch.zeros(300, 1024, dtype=torch.bfloat16, device=DEV)
    out = out_base[:, :768]                   # ldc = 1024
    h.linear(a, w, None, out)
    torch.cuda.synchronize()
    assert _rel(out, a.float() @ w.float().t()) <= 1e-2
    assert (out_base[:, 768:] == 0).all()     # nothing written past N
    with pytest.raises(RuntimeError, match="K=1000"):
        h.linear(_rand((10, 1000), g).bfloat16(), _rand((256, 1000), g).bfloat16(), None,
                 torch.empty(10, 256, dtype=torch.bfloat16, device=DEV))
    with pytest.raises(RuntimeError, match="multiple of 256"):
        h.linear(_rand((10, 768), g).bfloat16(), _rand((300, 768), g).bfloat16(), None,
                 torch.empty(10, 300, dtype=torch.bfloat16, device=DEV))


@pytest.mark.parametrize("M", [1, 17, 113, 300])
def test_no_writes_past_row_M(M):
    """Rows past M of a partial 256-row tile are dropped by the store descriptor: a sentinel region
    after the output (the next rows of the same allocation) stays untouched, for all three epilogues."""
    h = _hip()
    E, F = 768, 3072
    g = torch.Generator(device=DEV).manual_seed(M)
    a = _rand((M, E), g).bfloat16()
    w = _rand((E, E), g, E ** -0.5).bfloat16()
    base = torch.full((M + 256, E), 7.0, dtype=torch.bfloat16, device=DEV)
    h.linear(a, w, None, base[:M])
    w1 = _rand((F, E), g, E ** -0.5).bfloat16()
    fbase = torch.full((M + 256, F), 7.0, dtype=torch.bfloat16, device=DEV)
    stats = torch.empty((F // 256 + 1) * M * 2, device=DEV)
    h.ffn_fc1_gelu(a, w1, None, fbase[:M], stats)
    w2 = _rand((E, F), g, F ** -0.5).bfloat16()
    c = w2.float().sum(1)
    d = torch.zeros(E, device=DEV)
    ybase = torch.full((M + 256, E), 7.0, dtype=torch.bfloat16, device=DEV)
    h.ffn_fc2_ln(fbase[:M], w2, stats, c, d, 1e-5, ybase[:M])
    torch.cuda.synchronize()
    for t in (base, fbase, ybase):
        assert (t[M:] == 7.0).all()
        assert torch.isfinite(t[:M].float()).all() and not (t[:M] == 7.0).all()


@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("M", [1, 255, 1000, 70001])
def test_ffn_fc1_gelu_and_statistics(act, M):
    h = _hip()
    E, F = 768, 3072
    g = torch.Generator(device=DEV).manual_seed(M)
    a = _rand((M, E), g).to(act)
    w1 = _rand((F, E), g, E ** -0.5 * 1.5).to(act)
    b1 = _rand((F,), g, 0.2)
    hh = torch.empty(M, F, dtype=act, device=DEV)
    stats = torch.full(((F // 256 + 1) * M * 2,), float("nan"), device=DEV)
    h.ffn_fc1_gelu(a, w1, b1, hh, stats)
    torch.cuda.synchronize()
    x = a.float() @ w1.float().t() + b1
    ref = torch.nn.functional.gelu(x.to(act).float()).to(act)
    if act == torch.bfloat16:
        # bf16 h comes from torch's own GELU table: bit-identical to gelu(pre.float()).type_as(pre) of the
        # kernel's pre-activation, which gp_linear (same tiles, same accumulation order, no K split)
        # reproduces
        pre = torch.empty(M, F, dtype=act, device=DEV)
        h.linear(a, w1, b1, pre, None)
        torch.cuda.synchronize()
        # (torch's CPU GELU, the oracle's and the table's; the GPU build of F.gelu rounds ~0.4 % of bf16
        # inputs differently)
        exact = torch.nn.functional.gelu(pre.float().cpu()).to(act)
        assert torch.equal(hh.cpu(), exact), int((hh.cpu() != exact).sum())
    # the same two roundings as the reference: identical wherever the MFMA sums (accumulation order and
    # the matrix core's internal adds, as in any MFMA GEMM) and the fp32 sums of the restatement round the
    # pre-activation alike (measured ~98.8 %); elsewhere the pre-activation differs by one 16-bit ulp or by
    # the fp32 accumulation bound K u sum|a||w| (u = 2^-24; it dominates where the dot product cancels to
    # ~1e-4), so h moves by at most |gelu'| <= 1.13 of that plus its own rounding
    same = (hh == ref).float().mean().item()
    assert same >= 0.97, same
    ulp = 2.0 ** -7 if act == torch.bfloat16 else 2.0 ** -10
    mag = a.float().abs() @ w1.float().abs().t() + b1.abs()
    bound = 1.2 * (ulp * x.abs() + E * 2.0 ** -24 * mag) + ulp * ref.float().abs() + 1e-7
    bad = (hh.float() - ref.float()).abs() > bound
    assert not bad.any(), [(x[bad][:6].tolist()), ref[bad][:6].float().tolist(), hh[bad][:6].float().tolist(),
                           int(bad.sum())]
    st = stats[:(F // 256) * M * 2].view(F // 256, M, 2)
    hg = hh.float().view(M, F // 256, 256)
    mean = hg.mean(-1).t()
    m2 = ((hg - hg.mean(-1, keepdim=True)) ** 2).sum(-1).t()
    assert torch.allclose(st[..., 0], mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(st[..., 1], m2, rtol=1e-4, atol=1e-4)


def test_ffn_fc1_gelu_every_bf16_value():
    """Every finite normal bf16 pre-activation (and +-0) through the bf16 GELU epilogue -- the table, its
    clamped edges and the out-of-table rules (|x| < 2^-13, |x| > 5.53): A = the 768 x 768 identity (one
    exact product per output), so pre-activation (m, n) is W1[n, m], and the 65,536 bit patterns fill
    W1 [3072, 768]."""
    h = _hip()
    E, F = 768, 3072
    bits = torch.arange(0, 65536, dtype=torch.int32)
    mag = bits & 0x7FFF
    keep = ((mag >= 0x80) & (mag < 0x7F80)) | (mag == 0)          # normal finite, +-0
    vals = bits[keep].to(torch.int16).view(torch.bfloat16)
    w1 = vals.repeat((F * E) // vals.numel() + 1)[:F * E].view(F, E).to(DEV)
    a = torch.eye(E, dtype=torch.bfloat16, device=DEV)
    hh = torch.empty(E, F, dtype=torch.bfloat16, device=DEV)
    stats = torch.empty((F // 256 + 1) * E * 2, device=DEV)
    h.ffn_fc1_gelu(a, w1, None, hh, stats)
    pre = torch.empty(E, F, dtype=torch.bfloat16, device=DEV)
    h.linear(a, w1, None, pre, None)
    torch.cuda.synchronize()
    assert torch.equal(pre.float(), w1.t().float())                  # every pattern reached the epilogue
    exact = torch.nn.functional.gelu(pre.float().cpu()).to(torch.bfloat16)
    hh = hh.cpu()
    bad = hh.view(torch.int16) != exact.view(torch.int16)           # bit patterns: -0 is not +0
    assert not bad.any(), (pre.cpu()[bad][:8].float().tolist(), hh[bad][:8].float().tolist(), int(bad.sum()))


@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("M", [1, 300, 4097, 70001])
def test_ffn_fc2_layernorm_fold(act, M):
    """y = fc2(ffn_layernorm(h)) from gp_ffn_fc1_gelu's h and statistics, the LN folded into fc2 as the
    engine packs it (runtime.PackedLayer), against the reference order: LN in fp32, rounded to act,
    then fc2 (+ bias) in fp32."""
    from gigapath import runtime
    h = _hip()
    E, F = 768, 3072
    g = torch.Generator(device=DEV).manual_seed(M + 1)
    a = _rand((M, E), g).to(act)
    w1 = _rand((F, E), g, E ** -0.5 * 1.5).to(act)
    b1 = _rand((F,), g, 0.2)
    gamma = 1.0 + _rand((F,), g, 0.3)
    beta = _rand((F,), g, 0.1)
    w2 = _rand((E, F), g, F ** -0.5).to(act)
    b2 = _rand((E,), g, 0.1)
    hh = torch.empty(M, F, dtype=act, device=DEV)
    stats = torch.empty((F // 256 + 1) * M * 2, device=DEV)
    h.ffn_fc1_gelu(a, w1, b1, hh, stats)
    w2g = (w2.double() * gamma.double()[None]).to(act)
    c = w2g.double().sum(1).float()
    d = (w2.double() @ beta.double() + b2.double()).float()
    nb = h.gemm_workspace_bytes(M, E, F)
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=DEV)
    y = torch.full((M, E), float("nan"), dtype=act, device=DEV)
    h.ffn_fc2_ln(hh, w2g, stats, c, d, 1e-5, y, ws)
    torch.cuda.synchronize()
    ln = torch.nn.functional.layer_norm(hh.float(), (F,), gamma, beta, 1e-5).to(act).float()
    ref = ln @ w2.float().t() + b2
    assert torch.isfinite(y.float()).all()
    rel = _rel(y, ref)
    assert rel <= 1e-2, rel
    cos = torch.nn.functional.cosine_similarity(y.float().flatten(), ref.flatten(), dim=0).item()
    assert cos >= 0.99995, cos
    assert runtime.ffn_fusable(E, F)
