// HBM-bound row kernels of the slide-encoder path: coords -> pos, pos-embed + CLS (+LN),
// residual + LN, GELU + LN, fp32 LN readout, token mean.  One 64-lane wave per row, each
// lane owning EPL = cols/64 contiguous values (16-byte fp32 / 8-byte bf16 accesses).
#include <math.h>

#include "gp_api.h"
#include "gp_common.h"

namespace {

constexpr int kRowsPerBlock = 4;  // 4 waves x 64 lanes

// ---------------------------------------------------------------------------------------
// coords -> pos  (slide_encoder.py:166-179).  Separate mul and add (no FMA contraction) so
// the float rounding matches torch's two elementwise kernels.
template <typename T>
__global__ void coords_to_pos_kernel(const T* __restrict__ coords, int64_t n, T tile, T grid,
                                     int64_t grid_rows, int64_t* __restrict__ pos,
                                     int32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  T fx, fy, p;
  if constexpr (sizeof(T) == 4) {
    fx = floorf(__fdiv_rn(coords[2 * i], tile));
    fy = floorf(__fdiv_rn(coords[2 * i + 1], tile));
    p = __fadd_rn(__fmul_rn(fx, grid), fy);
  } else {
    fx = floor(__ddiv_rn(coords[2 * i], tile));
    fy = floor(__ddiv_rn(coords[2 * i + 1], tile));
    p = __dadd_rn(__dmul_rn(fx, grid), fy);
  }
  bool bad = !(p == p) || p >= (T)9.2e18 || p <= (T)-9.2e18;
  const int64_t q = bad ? 0 : (int64_t)p + 1;
  bad = bad || q > grid_rows - 1 || q < -grid_rows;
  pos[i] = q;
  if (bad && err) atomicAdd(err, 1);
}

// ---------------------------------------------------------------------------------------
template <int EPL>
__global__ __launch_bounds__(256) void posembed_cls_ln_kernel(
    const uint16_t* __restrict__ xp, const int64_t* __restrict__ pos, const float* __restrict__ tab,
    const float* __restrict__ cls, int64_t B, int64_t N, int E, int G, const float* __restrict__ ln_w,
    const float* __restrict__ ln_b, float eps, float* __restrict__ x_out, uint16_t* __restrict__ ln_out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= B * (N + 1)) return;
  const int64_t b = row / (N + 1), t = row % (N + 1);
  const int col0 = lane * EPL;
  float v[EPL];
  if (t == 0) {
    load_f32<EPL>(cls + col0, v);
  } else {
    load_bf16<EPL>(xp + ((b * N + t - 1) * E + col0), v);
    int64_t p = pos[b * N + t - 1];
    const int64_t nrows = (int64_t)G * G + 1;
    if (p < 0) p += nrows;
    if (p > 0 && p < nrows) {  // p == 0 is the all-zero CLS row; out of range was reported upstream
      const int half = E / 2;
      const int64_t q = p - 1;
      const int64_t trow = (col0 < half) ? (q % G) : (q / G);
      const int tcol = (col0 < half) ? col0 : col0 - half;
      float tv[EPL];
      load_f32<EPL>(tab + trow * half + tcol, tv);
#pragma unroll
      for (int i = 0; i < EPL; ++i) v[i] += tv[i];
    }
  }
  store_f32<EPL>(x_out + row * E + col0, v);
  if (ln_w != nullptr) {
    wave_layernorm<EPL>(v, E, ln_w, ln_b, eps, col0);
    store_bf16<EPL>(ln_out + row * E + col0, v);
  }
}

// ---------------------------------------------------------------------------------------
template <int EPL>
__global__ __launch_bounds__(256) void residual_ln_kernel(float* __restrict__ x, const uint16_t* __restrict__ y,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ ln_w,
                                                          const float* __restrict__ ln_b, float eps,
                                                          uint16_t* __restrict__ out, int64_t rows,
                                                          int cols) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int col0 = lane * EPL;
  float v[EPL], yv[EPL];
  load_f32<EPL>(x + row * cols + col0, v);
  load_bf16<EPL>(y + row * cols + col0, yv);
  if (bias != nullptr) {
    float bv[EPL];
    load_f32<EPL>(bias + col0, bv);
#pragma unroll
    for (int i = 0; i < EPL; ++i) yv[i] += bv[i];
  }
#pragma unroll
  for (int i = 0; i < EPL; ++i) v[i] += yv[i];
  store_f32<EPL>(x + row * cols + col0, v);
  if (ln_w != nullptr) {
    wave_layernorm<EPL>(v, cols, ln_w, ln_b, eps, col0);
    store_bf16<EPL>(out + row * cols + col0, v);
  }
}

// ---------------------------------------------------------------------------------------
template <int EPL>
__global__ __launch_bounds__(256) void gelu_ln_kernel(const uint16_t* h, const float* __restrict__ ln_w,
                                                      const float* __restrict__ ln_b, float eps, uint16_t* out,
                                                      int64_t rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int col0 = lane * EPL;
  float v[EPL];
  load_bf16<EPL>(h + row * cols + col0, v);
#pragma unroll
  for (int i = 0; i < EPL; ++i) v[i] = 0.5f * v[i] * (1.0f + erff(v[i] * 0.70710678118654752440f));
  wave_layernorm<EPL>(v, cols, ln_w, ln_b, eps, col0);
  store_bf16<EPL>(out + row * cols + col0, v);
}

// ---------------------------------------------------------------------------------------
template <int EPL>
__global__ __launch_bounds__(256) void layernorm_f32_kernel(const float* __restrict__ x, int64_t row_stride,
                                                            const float* __restrict__ ln_w,
                                                            const float* __restrict__ ln_b, float eps,
                                                            float* __restrict__ out, int64_t rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int col0 = lane * EPL;
  float v[EPL];
  load_f32<EPL>(x + row * row_stride + col0, v);
  wave_layernorm<EPL>(v, cols, ln_w, ln_b, eps, col0);
  store_f32<EPL>(out + row * cols + col0, v);
}

// One block per (batch, 64-column group); 16 waves stride over tokens, LDS tree at the end.
__global__ __launch_bounds__(1024) void mean_tokens_kernel(const float* __restrict__ x, int64_t B, int64_t L,
                                                           int E, int64_t start, float* __restrict__ out) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ngrp = E / 64;
  const int64_t b = blockIdx.x / ngrp;
  const int col = (blockIdx.x % ngrp) * 64 + lane;
  float s = 0.f;
  for (int64_t t = start + w; t < L; t += 16) s += x[(b * L + t) * E + col];
  part[w][lane] = s;
  __syncthreads();
  if (w == 0) {
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) tot += part[i][lane];
    out[b * E + col] = tot / (float)(L - start);
  }
}

inline unsigned row_blocks(int64_t rows) { return (unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock); }

}  // namespace

// =========================================================================================
extern "C" int gp_coords_to_pos(const void* coords, int coords_is_f64, int64_t n_tiles, int grid,
                                double tile_size, int64_t* pos, int32_t* err_count, void* stream) {
  GP_REQUIRE(n_tiles >= 0 && grid > 0 && tile_size > 0, "gp_coords_to_pos: bad sizes");
  if (n_tiles == 0) return 0;
  GP_REQUIRE(coords && pos, "gp_coords_to_pos: null pointer");
  const unsigned nb = (unsigned)((n_tiles + 255) / 256);
  const int64_t grid_rows = (int64_t)grid * grid + 1;
  if (coords_is_f64)
    coords_to_pos_kernel<double><<<nb, 256, 0, gp_stream(stream)>>>(
        (const double*)coords, n_tiles, tile_size, (double)grid, grid_rows, pos, err_count);
  else
    coords_to_pos_kernel<float><<<nb, 256, 0, gp_stream(stream)>>>(
        (const float*)coords, n_tiles, (float)tile_size, (float)grid, grid_rows, pos, err_count);
  return gp_check_launch("gp_coords_to_pos");
}

static bool epl_ok(int cols) {
  return cols % 64 == 0 && (cols / 64 == 12 || cols / 64 == 16 || cols / 64 == 24);
}

extern "C" int gp_posembed_cls_ln(const uint16_t* xp, const int64_t* pos, const float* tab, const float* cls,
                                  int64_t B, int64_t N, int E, int G, const float* ln_w, const float* ln_b,
                                  float eps, float* x_out, uint16_t* ln_out, void* stream) {
  GP_REQUIRE(epl_ok(E), "gp_posembed_cls_ln: E=%d unsupported (64*{12,16,24})", E);
  GP_REQUIRE(B > 0 && N >= 0 && G > 0, "gp_posembed_cls_ln: bad sizes");
  GP_REQUIRE(cls && tab && x_out && (N == 0 || (xp && pos)), "gp_posembed_cls_ln: null pointer");
  GP_REQUIRE(ln_w == nullptr || (ln_b && ln_out), "gp_posembed_cls_ln: LN needs ln_b and ln_out");
  const int64_t rows = B * (N + 1);
  hipStream_t s = gp_stream(stream);
  switch (E / 64) {
    case 12: posembed_cls_ln_kernel<12><<<row_blocks(rows), 256, 0, s>>>(xp, pos, tab, cls, B, N, E, G, ln_w, ln_b, eps, x_out, ln_out); break;
    case 16: posembed_cls_ln_kernel<16><<<row_blocks(rows), 256, 0, s>>>(xp, pos, tab, cls, B, N, E, G, ln_w, ln_b, eps, x_out, ln_out); break;
    case 24: posembed_cls_ln_kernel<24><<<row_blocks(rows), 256, 0, s>>>(xp, pos, tab, cls, B, N, E, G, ln_w, ln_b, eps, x_out, ln_out); break;
  }
  return gp_check_launch("gp_posembed_cls_ln");
}

extern "C" int gp_residual_layernorm(float* x, const uint16_t* y, const float* bias, const float* ln_w,
                                     const float* ln_b, float eps, uint16_t* ln_out, int64_t rows, int cols,
                                     void* stream) {
  GP_REQUIRE(epl_ok(cols), "gp_residual_layernorm: cols=%d unsupported (64*{12,16,24})", cols);
  GP_REQUIRE(rows >= 0, "gp_residual_layernorm: bad rows");
  if (rows == 0) return 0;
  GP_REQUIRE(x && y, "gp_residual_layernorm: null pointer");
  GP_REQUIRE(ln_w == nullptr || (ln_b && ln_out), "gp_residual_layernorm: LN needs ln_b and ln_out");
  hipStream_t s = gp_stream(stream);
  switch (cols / 64) {
    case 12: residual_ln_kernel<12><<<row_blocks(rows), 256, 0, s>>>(x, y, bias, ln_w, ln_b, eps, ln_out, rows, cols); break;
    case 16: residual_ln_kernel<16><<<row_blocks(rows), 256, 0, s>>>(x, y, bias, ln_w, ln_b, eps, ln_out, rows, cols); break;
    case 24: residual_ln_kernel<24><<<row_blocks(rows), 256, 0, s>>>(x, y, bias, ln_w, ln_b, eps, ln_out, rows, cols); break;
  }
  return gp_check_launch("gp_residual_layernorm");
}

extern "C" int gp_gelu_layernorm(const uint16_t* h, const float* ln_w, const float* ln_b, float eps,
                                 uint16_t* out, int64_t rows, int cols, void* stream) {
  GP_REQUIRE(cols % 64 == 0 && (cols / 64 == 48 || cols / 64 == 64 || cols / 64 == 96),
             "gp_gelu_layernorm: cols=%d unsupported (64*{48,64,96})", cols);
  GP_REQUIRE(rows >= 0, "gp_gelu_layernorm: bad rows");
  if (rows == 0) return 0;
  GP_REQUIRE(h && ln_w && ln_b && out, "gp_gelu_layernorm: null pointer");
  hipStream_t s = gp_stream(stream);
  switch (cols / 64) {
    case 48: gelu_ln_kernel<48><<<row_blocks(rows), 256, 0, s>>>(h, ln_w, ln_b, eps, out, rows, cols); break;
    case 64: gelu_ln_kernel<64><<<row_blocks(rows), 256, 0, s>>>(h, ln_w, ln_b, eps, out, rows, cols); break;
    case 96: gelu_ln_kernel<96><<<row_blocks(rows), 256, 0, s>>>(h, ln_w, ln_b, eps, out, rows, cols); break;
  }
  return gp_check_launch("gp_gelu_layernorm");
}

extern "C" int gp_layernorm_f32(const float* x, int64_t row_stride, const float* ln_w, const float* ln_b,
                                float eps, float* out, int64_t rows, int cols, void* stream) {
  GP_REQUIRE(epl_ok(cols), "gp_layernorm_f32: cols=%d unsupported (64*{12,16,24})", cols);
  GP_REQUIRE(rows >= 0 && row_stride >= cols && row_stride % 4 == 0, "gp_layernorm_f32: bad sizes");
  if (rows == 0) return 0;
  GP_REQUIRE(x && ln_w && ln_b && out, "gp_layernorm_f32: null pointer");
  hipStream_t s = gp_stream(stream);
  switch (cols / 64) {
    case 12: layernorm_f32_kernel<12><<<row_blocks(rows), 256, 0, s>>>(x, row_stride, ln_w, ln_b, eps, out, rows, cols); break;
    case 16: layernorm_f32_kernel<16><<<row_blocks(rows), 256, 0, s>>>(x, row_stride, ln_w, ln_b, eps, out, rows, cols); break;
    case 24: layernorm_f32_kernel<24><<<row_blocks(rows), 256, 0, s>>>(x, row_stride, ln_w, ln_b, eps, out, rows, cols); break;
  }
  return gp_check_launch("gp_layernorm_f32");
}

extern "C" int gp_mean_tokens(const float* x, int64_t B, int64_t L, int E, int64_t start, float* out,
                              void* stream) {
  GP_REQUIRE(B > 0 && E % 64 == 0 && start >= 0 && L > start, "gp_mean_tokens: bad sizes");
  GP_REQUIRE(x && out, "gp_mean_tokens: null pointer");
  mean_tokens_kernel<<<(unsigned)(B * (E / 64)), 1024, 0, gp_stream(stream)>>>(x, B, L, E, start, out);
  return gp_check_launch("gp_mean_tokens");
}
