// Plain projections (gp_linear) and the split-K workspace query; kernels in gp_gemm_impl.h.
#include "gp_gemm_impl.h"

extern "C" int64_t gp_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0 || N % kBN) return 0;
  return make_plan(M, N, K, true).ws_bytes;
}

extern "C" int gp_linear(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, const float* bias,
                         uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K, void* ws, int64_t ws_bytes,
                         int fmt, void* stream) {
  if (int rc = check_shapes("gp_linear", A, lda, W, ldw, C, ldc, M, N, K, fmt, true)) return rc;
  GP_REQUIRE(!bias || gp_aligned(bias, 16), "gp_linear: misaligned bias");
  const Plan p = make_plan(M, N, K, ws != nullptr);
  GP_REQUIRE(p.ws_bytes <= ws_bytes, "gp_linear: workspace of %lld bytes, %lld needed", (long long)ws_bytes,
             (long long)p.ws_bytes);
  GP_REQUIRE(p.ws_bytes == 0 || gp_aligned(ws, 16), "gp_linear: misaligned workspace");
  GemmArgs g = {};
  g.A = A; g.W = W; g.colp0 = bias; g.C = C;
  g.lda = lda; g.ldw = ldw; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.ws = static_cast<float*>(ws);
  g.vcol0 = fmt == GP_FMT_F16_VBF16 ? (int)(2 * N / 3) : INT_MAX;
  const int lrc = fmt != GP_FMT_BF16 ? launch<kEpiLinear, true, kKE | kKF>(g, p, gp_stream(stream)) : launch<kEpiLinear, false, kKE | kKF>(g, p, gp_stream(stream));
  if (lrc != 0) return lrc;
  return gp_check_launch("gp_linear");
}
