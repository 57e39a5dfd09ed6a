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


# ---------------------------------------------------------------------------------------------------
# The residual stream inside the GEMMs (ABI 7): gp_linear_resid / gp_ffn_fc2_ln_resid (producers: x += y,
# xb = act(gamma (x - s)), per-256-column statistics of x - s) and gp_linear_ln / gp_ffn_fc1_gelu_ln
# (consumers: the LayerNorm folded, statistics merged, shift carried).  Reference: encoder.py:141,147,159
# (residual adds), :126 / :147 (pre-LNs) -- restated in torch fp32/fp64 on the same 16-bit operands.
def _resid_inputs(g, M, N, shift_noise=0.05):
    x = _rand((M, N), g) + 0.7                       # a residual stream with a non-zero row mean
    s = x.mean(1) + _rand((M,), g, shift_noise)      # the shift: a stale row mean (the mean before the add)
    return x, s


def _stats_ref(v, s, N):
    dlt = (v.double() - s.double()[:, None]).view(v.shape[0], N // 256, 256)
    mean = dlt.mean(-1)
    return mean, ((dlt - mean[..., None]) ** 2).sum(-1)


def _check_resid(act, x_new, xb, xst, ref_x, s, gamma, N, M):
    # x: fp32 sum of the old stream and the GEMM output (accumulation-order differences only)
    err = (x_new.double() - ref_x.double()).abs().max().item()
    assert err <= 2e-4 * ref_x.abs().max().item(), err
    # xb = act(gamma (x - s)) of the kernel's own x, one 16-bit rounding
    want = ((x_new.double() - s.double()[:, None]) * gamma.double()[None]).to(act)
    assert (xb.float() - want.float()).abs().max().item() <= 1e-2 * want.float().abs().max().item()
    assert (xb == want).float().mean().item() >= 0.98
    mean, m2 = _stats_ref(x_new, s, N)
    st = xst.view(N // 256, M, 2).double()
    assert torch.allclose(st[..., 0], mean.t(), rtol=1e-4, atol=1e-5)
    assert torch.allclose(st[..., 1], m2.t(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("act", ACTS)
# 10,104 rows = the C5 packed batch's row count, where round 4's r04_y run (a split factor of 1 whose plan
# left the tail tiles uncomputed) produced garbage; launch() now refuses any plan its kernel would not complete
@pytest.mark.parametrize("M", [1, 17, 4097, 10104, 70001])
def test_linear_resid(act, M):
    """out-proj + residual (gp_linear_resid): x += a . w^T + b, xb, statistics; rows past M untouched; the
    split tail (70001 rows: 822 tiles) and the data-parallel plan; gamma = None updates x only."""
    h = _hip()
    N = K = 768
    g = torch.Generator(device=DEV).manual_seed(M + 7)
    a = _rand((M, K), g).to(act)
    w = _rand((N, K), g, K ** -0.5).to(act)
    b = _rand((N,), g, 0.1)
    gamma = 1.0 + _rand((N,), g, 0.3)
    x0, s = _resid_inputs(g, M, N)
    ref_x = x0 + (a.float() @ w.float().t() + b)
    nb = h.gemm_workspace_bytes(M, N, K)
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=DEV)
    for use_ws in (True, False):
        xbuf = torch.full((M + 8, N), 7.0, device=DEV)
        xbuf[:M] = x0
        xb = torch.full((M + 8, N), float("nan"), dtype=act, device=DEV)
        xst = torch.full((N // 256 + 1, M, 2), float("nan"), device=DEV)
        h.linear_resid(a, w, b, xbuf, s, gamma, xb, xst, ws if use_ws else None)
        torch.cuda.synchronize()
        assert (xbuf[M:] == 7.0).all() and torch.isnan(xb[M:].float()).all()   # nothing past row M
        _check_resid(act, xbuf[:M], xb[:M], xst[:N // 256], ref_x, s, gamma, N, M)
    xbuf = x0.clone()
    h.linear_resid(a, w, b, xbuf, None, None, None, None, ws)
    torch.cuda.synchronize()
    assert (xbuf.double() - ref_x.double()).abs().max().item() <= 2e-4 * ref_x.abs().max().item()


def _fold_setup(g, act, M, E, Nout):
    """x, shift, LN affine and the producer's xb / statistics planes (merged plane left to the consumer)."""
    x, s = _resid_inputs(g, M, E)
    gam = 1.0 + _rand((E,), g, 0.3)
    bet = _rand((E,), g, 0.1)
    xb = ((x.double() - s.double()[:, None]) * gam.double()[None]).to(act)
    mean, m2 = _stats_ref(x, s, E)
    st = torch.empty(E // 256 + 1, M, 2, device=DEV)
    st[:E // 256, :, 0] = mean.t().float()
    st[:E // 256, :, 1] = m2.t().float()
    return x, s, gam, bet, xb, st


@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("M", [1, 300, 10104, 70001])
def test_linear_ln_fold(act, M):
    """QKV with the pre-LN folded (gp_linear_ln): against the reference order LN(x) in fp32 rounded to act,
    then x . W^T + b; the merged statistics plane and the carried shift s_out = s_in + mean'."""
    h = _hip()
    E, N = 768, 2304
    g = torch.Generator(device=DEV).manual_seed(M + 11)
    x, s, gam, bet, xb, st = _fold_setup(g, act, M, E, N)
    w = _rand((N, E), g, E ** -0.5).to(act)
    b = _rand((N,), g, 0.1)
    c = (w.double() @ gam.double()).float()
    d = (w.double() @ bet.double() + b.double()).float()
    s_out = torch.full((M,), float("nan"), device=DEV)
    nb = h.gemm_workspace_bytes(M, N, E)
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=DEV)
    out = torch.full((M, N), float("nan"), dtype=act, device=DEV)
    h.linear_ln(xb, w, st, E // 256, c, d, 1e-5, s, s_out, out, ws)
    torch.cuda.synchronize()
    ln = torch.nn.functional.layer_norm(x, (E,), gam, bet, 1e-5)
    assert torch.allclose(s_out.double(), x.double().mean(1), rtol=1e-5, atol=1e-5)
    assert torch.allclose(st[E // 256, :, 1].double(), 1.0 / torch.sqrt(x.double().var(1, unbiased=False) + 1e-5),
                          rtol=1e-4)
    ref = ln.to(act).float() @ w.float().t() + b
    rel = _rel(out, ref)
    assert rel <= 1e-2, rel
    cos = torch.nn.functional.cosine_similarity(out.float().flatten(), ref.flatten(), dim=0).item()
    assert cos >= 0.99995, cos


@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("M", [1, 300, 10104, 70001])
def test_ffn_fc1_gelu_ln_fold(act, M):
    """fc1 + GELU with final_layer_norm folded (gp_ffn_fc1_gelu_ln) against LN(x) -> act -> fc1 -> act ->
    gelu -> act; its statistics against the kernel's own h."""
    h = _hip()
    E, F = 768, 3072
    g = torch.Generator(device=DEV).manual_seed(M + 13)
    x, s, gam, bet, xb, st = _fold_setup(g, act, M, E, F)
    w1 = _rand((F, E), g, E ** -0.5 * 1.5).to(act)
    b1 = _rand((F,), g, 0.2)
    c1 = (w1.double() @ gam.double()).float()
    d1 = (w1.double() @ bet.double() + b1.double()).float()
    hh = torch.full((M, F), float("nan"), dtype=act, device=DEV)
    hst = torch.full((F // 256 + 1, M, 2), float("nan"), device=DEV)
    s_out = torch.empty(M, device=DEV)
    h.ffn_fc1_gelu_ln(xb, w1, st, E // 256, c1, d1, 1e-5, s, s_out, hh, hst)
    torch.cuda.synchronize()
    ln = torch.nn.functional.layer_norm(x, (E,), gam, bet, 1e-5).to(act).float()
    pre = (ln @ w1.float().t() + b1).to(act).float()
    ref = torch.nn.functional.gelu(pre)
    rel = _rel(hh, ref)
    assert rel <= 1e-2, rel
    hf = hh.float().view(M, F // 256, 256).double()
    mean = hf.mean(-1)
    assert torch.allclose(hst[:F // 256, :, 0].double(), mean.t(), rtol=1e-5, atol=1e-6)
    assert torch.allclose(hst[:F // 256, :, 1].double(), ((hf - mean[..., None]) ** 2).sum(-1).t(), rtol=1e-4,
                          atol=1e-4)


@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("M", [1, 300, 10104, 70001])
def test_ffn_fc2_ln_resid(act, M):
    """fc2 with ffn_layernorm folded + residual (gp_ffn_fc2_ln_resid): x += LN(h) . W2^T + b2 in the
    reference order (LN in fp32 rounded to act, fp32 GEMM), the next layer's xb / statistics; gamma =
    None (the last layer) updates x only."""
    h = _hip()
    E, F = 768, 3072
    g = torch.Generator(device=DEV).manual_seed(M + 17)
    hh = torch.nn.functional.gelu(_rand((M, F), g)).to(act)
    hst = torch.empty(F // 256 + 1, M, 2, device=DEV)
    hf = hh.float().view(M, F // 256, 256).double()
    mean = hf.mean(-1)
    hst[:F // 256, :, 0] = mean.t().float()
    hst[:F // 256, :, 1] = ((hf - mean[..., None]) ** 2).sum(-1).t().float()
    gf = 1.0 + _rand((F,), g, 0.3)
    bf = _rand((F,), g, 0.1)
    w2 = _rand((E, F), g, F ** -0.5).to(act)
    b2 = _rand((E,), g, 0.1)
    w2g = (w2.double() * gf.double()[None]).to(act)
    c = w2g.double().sum(1).float()
    d = (w2.double() @ bf.double() + b2.double()).float()
    gam_next = 1.0 + _rand((E,), g, 0.3)
    x0, s = _resid_inputs(g, M, E)
    ln = torch.nn.functional.layer_norm(hh.float(), (F,), gf, bf, 1e-5).to(act).float()
    y_ref = ln @ w2.float().t() + b2
    nb = h.gemm_workspace_bytes(M, E, F)
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=DEV)
    xbuf = x0.clone()
    xb = torch.full((M, E), float("nan"), dtype=act, device=DEV)
    xst = torch.full((E // 256 + 1, M, 2), float("nan"), device=DEV)
    h.ffn_fc2_ln_resid(hh, w2g, hst, c, d, 1e-5, xbuf, s, gam_next, xb, xst, ws)
    torch.cuda.synchronize()
    y = xbuf.double() - x0.double()
    assert (y - y_ref.double()).abs().max().item() <= 1e-2 * y_ref.abs().max().item()
    _check_resid(act, xbuf, xb, xst[:E // 256], xbuf, s, gam_next, E, M)
    x2 = x0.clone()
    h.ffn_fc2_ln_resid(hh, w2g, hst, c, d, 1e-5, x2, None, None, None, None, ws)
    torch.cuda.synchronize()
    assert torch.equal(x2, xbuf)        # the same x whether or not the next LN's operands are written


def _consumer_merge(h, xst, nst, eps, s_in, M):
    """The merged plane and shift as the consumer's own merge computes them (gp_linear_ln, nst > 0), on a copy
    of the producer's planes: the reference the producer-side merge must equal bit for bit."""
    st = xst.clone()
    s_out = torch.full((M,), float("nan"), device=DEV)
    E = 256 * nst
    w = torch.zeros(256, E, dtype=torch.bfloat16, device=DEV)
    z = torch.zeros(256, device=DEV)
    out = torch.empty(M, 256, dtype=torch.bfloat16, device=DEV)
    xb = torch.zeros(M, E, dtype=torch.bfloat16, device=DEV)
    h.linear_ln(xb, w, st, nst, z, z, eps, s_in, s_out, out,
                torch.empty(max(h.gemm_workspace_bytes(M, 256, E), 16), dtype=torch.uint8, device=DEV))
    return st[nst], s_out


# 25,613 rows: 303 tiles, 256 data-parallel (not a multiple of 3: the first tail panel is part data-parallel,
# part split) + 47 split; 70,001: the C3 plan (822 tiles, whole tail panels); 1 and 10,104: no split (one merge
# launch after the GEMM)
@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("M", [1, 10104, 25613, 70001])
@pytest.mark.parametrize("producer", ["out_proj", "fc2"])
def test_resid_producer_merges_next_ln_stats(act, M, producer):
    """ABI 9: gp_linear_resid / gp_ffn_fc2_ln_resid with s_out merge the next LayerNorm's statistics planes
    themselves (in the split-tail reduce launch when the plan splits).  x, xb and the per-group planes equal
    the run without the merge, and the merged plane and s_out equal the consumer's own merge bit for bit."""
    h = _hip()
    E = 768
    eps = 1e-5 if producer == "out_proj" else 1e-6
    g = torch.Generator(device=DEV).manual_seed(M + 23)
    gam = 1.0 + _rand((E,), g, 0.3)
    x0, s = _resid_inputs(g, M, E)
    if producer == "out_proj":
        K = E
        a = _rand((M, K), g).to(act)
        w = _rand((E, K), g, K ** -0.5).to(act)
        b = _rand((E,), g, 0.1)

        def run(xbuf, xb, xst, ws, s_out):
            h.linear_resid(a, w, b, xbuf, s, gam, xb, xst, ws, eps_next=eps if s_out is not None else None,
                           s_out=s_out)
    else:
        K = 3072
        hh = torch.nn.functional.gelu(_rand((M, K), g)).to(act)
        hst = torch.empty(K // 256 + 1, M, 2, device=DEV)
        hf = hh.float().view(M, K // 256, 256).double()
        mean = hf.mean(-1)
        hst[:K // 256, :, 0] = mean.t().float()
        hst[:K // 256, :, 1] = ((hf - mean[..., None]) ** 2).sum(-1).t().float()
        w2g = _rand((E, K), g, K ** -0.5).to(act)
        c = w2g.double().sum(1).float()
        d = _rand((E,), g, 0.1)

        def run(xbuf, xb, xst, ws, s_out):
            h.ffn_fc2_ln_resid(hh, w2g, hst, c, d, 1e-5, xbuf, s, gam, xb, xst, ws,
                               eps_next=eps if s_out is not None else None, s_out=s_out)
    ws = torch.empty(max(h.gemm_workspace_bytes(M, E, K), 16), dtype=torch.uint8, device=DEV)
    outs = []
    for merge in (False, True):
        xbuf = x0.clone()
        xb = torch.full((M, E), float("nan"), dtype=act, device=DEV)
        xst = torch.full((E // 256 + 1, M, 2), float("nan"), device=DEV)
        s_out = torch.full((M,), float("nan"), device=DEV) if merge else None
        run(xbuf, xb, xst, ws, s_out)
        torch.cuda.synchronize()
        outs.append((xbuf, xb, xst, s_out))
    (x1, xb1, st1, _), (x2, xb2, st2, so2) = outs
    assert torch.equal(x1, x2) and torch.equal(xb1.view(torch.int16), xb2.view(torch.int16))
    assert torch.equal(st1[:E // 256], st2[:E // 256])
    ref_plane, ref_s = _consumer_merge(h, st1, E // 256, eps, s, M)
    assert torch.equal(st2[E // 256].view(torch.int32), ref_plane.view(torch.int32))
    assert torch.equal(so2.view(torch.int32), ref_s.view(torch.int32))


def test_resid_epilogue_errors():
    """The C ABI's checks of the residual entry points (no launch)."""
    h = _hip()
    g = torch.Generator(device=DEV).manual_seed(5)
    a = _rand((64, 768), g).bfloat16()
    w = _rand((768, 768), g).bfloat16()
    x = torch.zeros(64, 768, device=DEV)
    with pytest.raises(RuntimeError, match="K=3072"):   # the residual out-proj epilogue: K = E only
        h.linear_resid(_rand((64, 3072), g).bfloat16(), _rand((768, 3072), g).bfloat16(), None, x, None, None,
                       None, None)
    with pytest.raises(RuntimeError, match="xb"):
        lib = h.load_library()
        rc = lib.gp_linear_resid(a.data_ptr(), 768, w.data_ptr(), 768, None, x.data_ptr(), 768,
                                 x.data_ptr(), x.data_ptr(), None, 768, x.data_ptr(), 0.0, None, 64, 768, 768, None,
                                 0, 0, h._stream())
        h._check(rc, "gp_linear_resid")
    with pytest.raises(RuntimeError, match="statistics merge"):   # s_out needs gamma and eps_next > 0
        lib = h.load_library()
        rc = lib.gp_linear_resid(a.data_ptr(), 768, w.data_ptr(), 768, None, x.data_ptr(), 768, x.data_ptr(), None,
                                 None, 768, x.data_ptr(), 1e-5, x.data_ptr(), 64, 768, 768, None, 0, 0, h._stream())
        h._check(rc, "gp_linear_resid")


def test_runtime_linear_takes_strided_and_offset_operands():
    """runtime.linear (the engine's nn.Linear) accepts what torch.addmm accepts: an operand whose storage
    offset breaks gp_linear's 16-byte row alignment, a transposed-strided one, and a strided output are
    staged instead of refused; results equal the aligned call."""
    from gigapath import runtime
    _hip()
    g = torch.Generator(device=DEV).manual_seed(21)
    M, K, N = 333, 768, 768
    w = _rand((N, K), g, K ** -0.5).bfloat16()
    b = _rand((N,), g, 0.1)
    a = _rand((M, K), g).bfloat16()
    ref = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    runtime.linear(a, w, b.bfloat16(), b, ref)
    flat = torch.zeros(M * K + 4, dtype=torch.bfloat16, device=DEV)
    a_off = flat[4:].view(M, K)
    a_off.copy_(a)                                    # storage offset 4 elements = 8 bytes
    a_t = a.t().contiguous().t()                      # column-major view
    for aa in (a_off, a_t):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        runtime.linear(aa, w, b.bfloat16(), b, out)
        assert torch.equal(out, ref)
    big = torch.zeros(M, N + 4, dtype=torch.bfloat16, device=DEV)
    runtime.linear(a, w, b.bfloat16(), b, big[:, 4:])  # output rows 8 bytes off alignment
    assert torch.equal(big[:, 4:], ref)


@pytest.mark.parametrize("M", [1, 4097, 70001])
def test_fp16_qkv_with_bf16_v_third(M):
    """GP_FMT_F16_VBF16 (round 5): gp_linear / gp_linear_ln of an fp16 fused QKV write the V third (columns
    [2N/3, N)) in bf16 and the rest in fp16 -- each exactly the plain fp16 launch's fp32 result rounded to
    its format (bit-identical q / k columns; V = bf16 of the same accumulators); split tail and unsplit."""
    h = _hip()
    E, N = 768, 2304
    g = torch.Generator(device=DEV).manual_seed(M + 31)
    a = _rand((M, E), g).half()
    w = _rand((N, E), g, E ** -0.5).half()
    b = _rand((N,), g, 0.1)
    ref = a.float() @ w.float().t() + b
    nb = h.gemm_workspace_bytes(M, N, E)
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=DEV)
    for use_ws in (True, False):
        plain = torch.empty(M, N, dtype=torch.float16, device=DEV)
        h.linear(a, w, b, plain, ws if use_ws else None)
        out = torch.full((M, N), float("nan"), dtype=torch.float16, device=DEV)
        h.linear(a, w, b, out, ws if use_ws else None, v_bf16=True)
        torch.cuda.synchronize()
        assert torch.equal(out[:, :2 * E], plain[:, :2 * E])
        vb = out[:, 2 * E:].view(torch.bfloat16).float()
        assert torch.isfinite(vb).all()
        assert _rel(vb, ref[:, 2 * E:]) <= 1e-2
        # the V third is the bf16 rounding of the same accumulators the fp16 columns were rounded from
        assert (vb - plain[:, 2 * E:].float()).abs().max().item() <= 2 ** -8 * plain[:, 2 * E:].float().abs().max().item()
    # the LN-folded QKV (layers 1..): same split of formats
    x, s, gam, bet, xb, st = _fold_setup(g, torch.float16, M, E, N)
    c = (w.double() @ gam.double()).float()
    d = (w.double() @ bet.double() + b.double()).float()
    plain = torch.empty(M, N, dtype=torch.float16, device=DEV)
    h.linear_ln(xb, w, st, E // 256, c, d, 1e-5, s, torch.empty(M, device=DEV), plain, ws)
    out = torch.empty(M, N, dtype=torch.float16, device=DEV)
    h.linear_ln(xb, w, st, E // 256, c, d, 1e-5, s, torch.empty(M, device=DEV), out, ws, v_bf16=True)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :2 * E], plain[:, :2 * E])
    vb = out[:, 2 * E:].view(torch.bfloat16).float()
    assert (vb - plain[:, 2 * E:].float()).abs().max().item() <= 2 ** -8 * plain[:, 2 * E:].float().abs().max().item()
    with pytest.raises(RuntimeError, match="F16_VBF16"):        # N = 512: not a fused q | k | v (N % 3 != 0)
        h.linear(a, w[:512], b[:512], torch.empty(M, 512, dtype=torch.float16, device=DEV), ws, v_bf16=True)
