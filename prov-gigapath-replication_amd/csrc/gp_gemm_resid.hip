// GEMMs that update the fp32 residual stream (out-proj, fc2); kernels in gp_gemm_impl.h.
#include "gp_gemm_impl.h"

// s_out != NULL (round 5): also merge xstats' N/256 planes into plane N/256 with eps_next and write s_out = shift
// + the row mean -- what the next LN-folding GEMM's merge did (it is then called with nst < 0).  With a split
// tail the reduce launch does it; otherwise one row_stats_kernel launch here.
static int resid_merge_tail(const Plan& p, float* xstats, int64_t M, int64_t N, float eps_next, const float* shift,
                            float* s_out, hipStream_t s) {
  if (s_out != nullptr && p.S == 1) launch_row_stats(xstats, M, (int)(N / kBN), eps_next, shift, s_out, s);
  return 0;
}

extern "C" int gp_linear_resid(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, const float* bias,
                               float* x, int64_t ldx, const float* shift, const float* gamma, uint16_t* xb,
                               int64_t ldxb, float* xstats, float eps_next, float* s_out, int64_t M, int64_t N,
                               int64_t K, void* ws, int64_t ws_bytes, int fmt, void* stream) {
  if (int rc = check_shapes("gp_linear_resid", A, lda, W, ldw, x, ldx, M, N, K, fmt)) return rc;
  if (int rc = check_resid("gp_linear_resid", x, ldx, shift, gamma, xb, ldxb, xstats, N)) return rc;
  GP_REQUIRE(!bias || gp_aligned(bias, 16), "gp_linear_resid: misaligned bias");
  GP_REQUIRE(!s_out || (gamma && eps_next > 0.f && N / kBN <= kMaxTilesN),
             "gp_linear_resid: the statistics merge (s_out) needs gamma, eps_next > 0 and N <= %d", kMaxTilesN * kBN);
  const Plan p = make_plan(M, N, K, ws != nullptr);
  GP_REQUIRE(p.ws_bytes <= ws_bytes, "gp_linear_resid: workspace of %lld bytes, %lld needed", (long long)ws_bytes,
             (long long)p.ws_bytes);
  GP_REQUIRE(p.ws_bytes == 0 || gp_aligned(ws, 16), "gp_linear_resid: misaligned workspace");
  GemmArgs g = {};
  g.A = A; g.W = W; g.colp0 = bias; g.colp1 = gamma;
  g.C = gamma ? xb : nullptr; g.ostats = xstats; g.x = x; g.shift = shift;
  g.lda = lda; g.ldw = ldw; g.ldc = gamma ? ldxb : 8; g.ldx = ldx;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.ws = static_cast<float*>(ws);
  g.mrg_sout = s_out;
  g.mrg_eps = eps_next;
  const int lrc = fmt == GP_FMT_F16 ? launch<kEpiResid, true, kKE>(g, p, gp_stream(stream)) : launch<kEpiResid, false, kKE>(g, p, gp_stream(stream));
  if (lrc != 0) return lrc;
  resid_merge_tail(p, xstats, M, N, eps_next, shift, s_out, gp_stream(stream));
  return gp_check_launch("gp_linear_resid");
}

extern "C" int gp_ffn_fc2_ln_resid(const uint16_t* h, int64_t ldh, const uint16_t* W2g, int64_t ldw, float* hstats,
                                   const float* c, const float* d, float eps, float* x, int64_t ldx,
                                   const float* shift, const float* gamma, uint16_t* xb, int64_t ldxb, float* xstats,
                                   float eps_next, float* s_out, int64_t M, int64_t N, int64_t F, void* ws,
                                   int64_t ws_bytes, int fmt, void* stream) {
  if (int rc = check_shapes("gp_ffn_fc2_ln_resid", h, ldh, W2g, ldw, x, ldx, M, N, F, fmt)) return rc;
  if (int rc = check_fold("gp_ffn_fc2_ln_resid", hstats, F / kBN, c, d, N)) return rc;
  if (int rc = check_resid("gp_ffn_fc2_ln_resid", x, ldx, shift, gamma, xb, ldxb, xstats, N)) return rc;
  GP_REQUIRE(!s_out || (gamma && eps_next > 0.f && N / kBN <= kMaxTilesN),
             "gp_ffn_fc2_ln_resid: the statistics merge (s_out) needs gamma, eps_next > 0 and N <= %d",
             kMaxTilesN * kBN);
  const Plan p = make_plan(M, N, F, ws != nullptr);
  GP_REQUIRE(p.ws_bytes <= ws_bytes, "gp_ffn_fc2_ln_resid: workspace of %lld bytes, %lld needed",
             (long long)ws_bytes, (long long)p.ws_bytes);
  GP_REQUIRE(p.ws_bytes == 0 || gp_aligned(ws, 16), "gp_ffn_fc2_ln_resid: misaligned workspace");
  GemmArgs g = {};
  g.A = h; g.W = W2g; g.colp0 = c; g.colp1 = d; g.colp2 = gamma;
  g.C = gamma ? xb : nullptr; g.stats = hstats; g.ostats = xstats; g.x = x; g.shift = shift;
  g.lda = ldh; g.ldw = ldw; g.ldc = gamma ? ldxb : 8; g.ldx = ldx;
  g.M = (int)M; g.N = (int)N; g.K = (int)F;
  g.nst = (int)(F / kBN);
  g.eps = eps;
  g.ws = static_cast<float*>(ws);
  g.mrg_sout = s_out;
  g.mrg_eps = eps_next;
  launch_row_stats(hstats, M, g.nst, eps, nullptr, nullptr, gp_stream(stream));
  const int lrc = fmt == GP_FMT_F16 ? launch<kEpiLnFoldResid, true, kKF>(g, p, gp_stream(stream)) : launch<kEpiLnFoldResid, false, kKF>(g, p, gp_stream(stream));
  if (lrc != 0) return lrc;
  resid_merge_tail(p, xstats, M, N, eps_next, shift, s_out, gp_stream(stream));
  return gp_check_launch("gp_ffn_fc2_ln_resid");
}
