// fc1 + GELU (+ LN statistics), with or without the folded pre-LN; kernels in gp_gemm_impl.h.
#include "gp_gemm_impl.h"

extern "C" int gp_ffn_fc1_gelu(const uint16_t* A, int64_t lda, const uint16_t* W1, int64_t ldw, const float* b1,
                               uint16_t* h, int64_t ldh, float* stats, int64_t M, int64_t F, int64_t K, int fmt,
                               void* stream) {
  if (int rc = check_shapes("gp_ffn_fc1_gelu", A, lda, W1, ldw, h, ldh, M, F, K, fmt)) return rc;
  GP_REQUIRE(stats && gp_aligned(stats, 8), "gp_ffn_fc1_gelu: null or misaligned stats");
  GP_REQUIRE(!b1 || gp_aligned(b1, 16), "gp_ffn_fc1_gelu: misaligned bias");
  const Plan p = make_plan(M, F, K, false);
  GemmArgs g = {};
  g.A = A; g.W = W1; g.colp0 = b1; g.C = h; g.ostats = stats;
  g.lda = lda; g.ldw = ldw; g.ldc = ldh;
  g.M = (int)M; g.N = (int)F; g.K = (int)K;
  const int lrc = fmt == GP_FMT_F16 ? launch<kEpiGelu, true, kKE>(g, p, gp_stream(stream)) : launch<kEpiGelu, false, kKE>(g, p, gp_stream(stream));
  if (lrc != 0) return lrc;
  return gp_check_launch("gp_ffn_fc1_gelu");
}

extern "C" int gp_ffn_fc1_gelu_ln(const uint16_t* A, int64_t lda, const uint16_t* W1, int64_t ldw, float* xstats,
                                  int nst, const float* c1, const float* d1, float eps, const float* s_in,
                                  float* s_out, uint16_t* h, int64_t ldh, float* hstats, int64_t M, int64_t F,
                                  int64_t K, int fmt, void* stream) {
  if (int rc = check_shapes("gp_ffn_fc1_gelu_ln", A, lda, W1, ldw, h, ldh, M, F, K, fmt)) return rc;
  const bool merged = nst < 0;   // plane -nst merged by the producer (see gp_linear_ln)
  if (merged) nst = -nst;
  if (int rc = check_fold("gp_ffn_fc1_gelu_ln", xstats, nst, c1, d1, F)) return rc;
  GP_REQUIRE(hstats && gp_aligned(hstats, 8), "gp_ffn_fc1_gelu_ln: null or misaligned hstats");
  const Plan p = make_plan(M, F, K, false);
  GemmArgs g = {};
  g.A = A; g.W = W1; g.colp0 = c1; g.colp1 = d1; g.C = h; g.stats = xstats; g.ostats = hstats;
  g.lda = lda; g.ldw = ldw; g.ldc = ldh;
  g.M = (int)M; g.N = (int)F; g.K = (int)K;
  g.nst = nst;
  g.eps = eps;
  if (!merged) launch_row_stats(xstats, M, nst, eps, s_in, s_out, gp_stream(stream));
  const int lrc = fmt == GP_FMT_F16 ? launch<kEpiLnFoldGelu, true, kKE>(g, p, gp_stream(stream)) : launch<kEpiLnFoldGelu, false, kKE>(g, p, gp_stream(stream));
  if (lrc != 0) return lrc;
  return gp_check_launch("gp_ffn_fc1_gelu_ln");
}
