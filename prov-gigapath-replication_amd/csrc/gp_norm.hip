// HBM-bound row kernels of the slide-encoder path: coords -> pos, pos-embed + CLS (+LN),
// residual + LN, GELU + LN, fp32 LN readout, token mean.  One 64-lane wave per row, each
// lane owning EPL = cols/64 contiguous values (16-byte fp32 / 8-byte bf16 accesses).
#include <math.h>

#include <atomic>

#include <stdlib.h>

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
// Row kernels: one wave per row, "x4"/"x8" coalesced lane mappings (gp_common.h), grid-stride
// over rows with the per-column parameters (LN affine, biases) held in registers.
constexpr int kMaxRowBlocks = 1 << 20;   // one row per wave: loads of many rows in flight

inline unsigned row_grid(int64_t rows) {
  const int64_t nb = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
  return (unsigned)(nb < kMaxRowBlocks ? nb : kMaxRowBlocks);
}

template <int EPL, bool kH>
__global__ __launch_bounds__(256) void posembed_cls_ln_kernel(
    const uint16_t* __restrict__ xp, const int64_t* __restrict__ pos, const float* __restrict__ tab,
    const float* __restrict__ cls, int64_t B, int64_t N, int E, int G, const float* __restrict__ ln_w,
    const float* __restrict__ ln_b, float eps, float* __restrict__ x_out, uint16_t* __restrict__ ln_out,
    float* __restrict__ row_mean) {
  const int lane = threadIdx.x & 63;
  const int half = E / 2;
  float wv[EPL], bv[EPL];
  if (ln_w != nullptr) {
    ld_x4_f32<EPL>(ln_w, lane, wv);
    ld_x4_f32<EPL>(ln_b, lane, bv);
  }
  const int has_cls = cls != nullptr;        // no CLS row: a sequence-parallel shard
  const int64_t per = N + has_cls;
  const int64_t rows = B * per;
  for (int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6); row < rows;
       row += (int64_t)gridDim.x * kRowsPerBlock) {
    const int64_t b = row / per, t = row % per - has_cls;   // t = tile index, -1 = CLS
    float v[EPL];
    if (t < 0) {
      ld_x4_f32<EPL>(cls, lane, v);
    } else {
      ld_x4_e<kH, EPL>(xp + (b * N + t) * E, lane, v);
      int64_t p = pos[b * N + t];
      const int64_t nrows = (int64_t)G * G + 1;
      if (p < 0) p += nrows;
      if (p > 0 && p < nrows) {  // p == 0 is the all-zero CLS row; out of range was reported upstream
        const int64_t q = p - 1;
        const float* ty = tab + (q % G) * half;   // first E/2 columns: y index
        const float* tx = tab + (q / G) * half - half;   // last E/2 columns: x index
#pragma unroll
        for (int k = 0; k < EPL / 4; ++k) {
          const int e = k * 256 + 4 * lane;     // 4 columns, never straddling E/2
          const float4 u = *reinterpret_cast<const float4*>((e < half ? ty : tx) + e);
          v[4 * k] += u.x; v[4 * k + 1] += u.y; v[4 * k + 2] += u.z; v[4 * k + 3] += u.w;
        }
      }
    }
    st_x4_f32<EPL>(x_out + row * E, lane, v);
    if (row_mean != nullptr) {   // the first residual epilogue's row shift (gp_linear_resid)
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < EPL; ++i) sm += v[i];
      sm = wave_sum(sm) / (float)E;
      if (lane == 0) row_mean[row] = sm;
    }
    if (ln_w != nullptr) {
      wave_layernorm_regs<EPL>(v, E, wv, bv, eps);
      st_x4_e<kH, EPL>(ln_out + row * E, lane, v);
    }
  }
}

// ---------------------------------------------------------------------------------------
template <int EPL, bool kH>
__global__ __launch_bounds__(256) void residual_ln_kernel(float* __restrict__ x, const uint16_t* __restrict__ y,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ ln_w,
                                                          const float* __restrict__ ln_b, float eps,
                                                          uint16_t* __restrict__ out, int64_t rows,
                                                          int cols) {
  const int lane = threadIdx.x & 63;
  float bb[EPL], wv[EPL], bv[EPL];
  if (bias != nullptr) ld_x4_f32<EPL>(bias, lane, bb);
  else
#pragma unroll
    for (int i = 0; i < EPL; ++i) bb[i] = 0.f;
  if (ln_w != nullptr) {
    ld_x4_f32<EPL>(ln_w, lane, wv);
    ld_x4_f32<EPL>(ln_b, lane, bv);
  }
  for (int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6); row < rows;
       row += (int64_t)gridDim.x * kRowsPerBlock) {
    float v[EPL], yv[EPL];
    // the fp32 residual stream is read and written back once per half-layer and not touched again until
    // the next one (~15 ms later at 70k): non-temporal both ways, the caches keep y and the LN output
    // the next GEMM reads (−13 % per launch in isolation, profiles/r03_y_resid_ab.json)
    ld_x4_f32_nt<EPL>(x + row * cols, lane, v);
    ld_x4_e<kH, EPL>(y + row * cols, lane, yv);
#pragma unroll
    for (int i = 0; i < EPL; ++i) v[i] += yv[i] + bb[i];
    st_x4_f32_nt<EPL>(x + row * cols, lane, v);
    if (ln_w != nullptr) {
      wave_layernorm_regs<EPL>(v, cols, wv, bv, eps);
      st_x4_e<kH, EPL>(out + row * cols, lane, v);
    }
  }
}

// ---------------------------------------------------------------------------------------
// The layer's two residual adds without the mid-layer write of the fp32 residual stream (encoder.py:141,159;
// round 6): the first call computes x1 = x + (y1 + b1) and LN2(x1) but leaves x as it was, the second
// recomputes x1 the same way (same fp32 operations, so the same bits) from the still-live out-proj output
// y1, adds (y2 + b2) and writes x2 and LN(x2).  Per element 8 + 14 bytes instead of 12 + 12: the x1 store
// and reload (8 B) traded for a second read of x and y1 (6 B).
// 16-bit row loads, non-temporal (the GEMM outputs the residual pair reads are dead after it, and cached they
// would push the LN output the next GEMM reads out of the MALL)
typedef uint32_t gp_u2v __attribute__((ext_vector_type(2)));
template <bool kH, int EPL>
GP_DEV void ld_x4_e_nt(const uint16_t* row, int lane, float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 4; ++k) {
    const gp_u2v u = __builtin_nontemporal_load(reinterpret_cast<const gp_u2v*>(row + k * 256 + 4 * lane));
    v[4 * k + 0] = e2f<kH>(u.x);
    v[4 * k + 1] = e2f_hi<kH>(u.x);
    v[4 * k + 2] = e2f<kH>(u.y);
    v[4 * k + 3] = e2f_hi<kH>(u.y);
  }
}

template <int EPL, bool kH, bool kY2>
__global__ __launch_bounds__(256) void residual2_ln_kernel(float* __restrict__ x, const uint16_t* __restrict__ y1,
                                                           const float* __restrict__ b1, const uint16_t* __restrict__ y2,
                                                           const float* __restrict__ b2, const float* __restrict__ ln_w,
                                                           const float* __restrict__ ln_b, float eps,
                                                           uint16_t* __restrict__ out, int64_t rows, int cols) {
  const int lane = threadIdx.x & 63;
  float c1[EPL], c2[EPL], wv[EPL], bv[EPL];
#pragma unroll
  for (int i = 0; i < EPL; ++i) c1[i] = c2[i] = 0.f;
  if (b1 != nullptr) ld_x4_f32<EPL>(b1, lane, c1);
  if (kY2 && b2 != nullptr) ld_x4_f32<EPL>(b2, lane, c2);
  if (ln_w != nullptr) {
    ld_x4_f32<EPL>(ln_w, lane, wv);
    ld_x4_f32<EPL>(ln_b, lane, bv);
  }
  for (int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6); row < rows;
       row += (int64_t)gridDim.x * kRowsPerBlock) {
    float v[EPL], yv[EPL];
    ld_x4_f32_nt<EPL>(x + row * cols, lane, v);
    ld_x4_e_nt<kH, EPL>(y1 + row * cols, lane, yv);
#pragma unroll
    for (int i = 0; i < EPL; ++i) v[i] += yv[i] + c1[i];        // x1, as residual_ln_kernel rounds it
    if constexpr (kY2) {
      ld_x4_e_nt<kH, EPL>(y2 + row * cols, lane, yv);
#pragma unroll
      for (int i = 0; i < EPL; ++i) v[i] += yv[i] + c2[i];      // x2
      st_x4_f32_nt<EPL>(x + row * cols, lane, v);
    }
    if (ln_w != nullptr) {
      wave_layernorm_regs<EPL>(v, cols, wv, bv, eps);
      st_x4_e<kH, EPL>(out + row * cols, lane, v);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Exact-erf GELU, x * Phi(x) = 0.5 x (1 + erf(x / sqrt 2)) (feedforward_network.py:135, torch's
// F.gelu default), with erf from Abramowitz & Stegun 7.1.26: |erf error| <= 1.5e-7, i.e. GELU
// within 0.75e-7 |x| of the libm value -- far below the bf16 rounding of the output, at a
// fraction of erff's instruction count (one v_rcp, one v_exp, ~10 FMA-class ops).
GP_DEV float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  poly *= t;
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.44269504088896340736f);
  const float erf_x = copysignf(fmaf(-poly, e, 1.0f), x);
  const float hx = 0.5f * x;
  return fmaf(hx, erf_x, hx);
}

// ---------------------------------------------------------------------------------------
// GELU + LN v2, one wave per row, grid-stride over rows with the NEXT row's 16-byte loads
// issued before the current row's math (memory-level parallelism at the occupancy the
// registers allow).  The GELU outputs are rounded to bf16 in place -- as the reference's
// gelu(x.float()).type_as(x) does before ffn_layernorm (feedforward_network.py:135-137) -- so
// a row lives in EPL/2 registers, and the LN statistics are taken over those rounded values.
template <bool kH>
GP_DEV void unpack8(const uint4 u, float* v) {
  const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = e2f<kH>(w4[i]);
    v[2 * i + 1] = e2f_hi<kH>(w4[i]);
  }
}
template <bool kH>
GP_DEV uint4 pack8(const float* v) {
  return make_uint4(pack2e<kH>(v[0], v[1]), pack2e<kH>(v[2], v[3]), pack2e<kH>(v[4], v[5]), pack2e<kH>(v[6], v[7]));
}

template <int EPL, bool kH>
__global__ __launch_bounds__(256) void gelu_ln_wave2_kernel(const uint16_t* h, const float* __restrict__ ln_w,
                                                            const float* __restrict__ ln_b, float eps,
                                                            uint16_t* out, int64_t rows) {
  constexpr int C = 64 * EPL, NK = EPL / 8;
  // LN weights in LDS once per block (in registers they would be loop-invariant across the
  // grid-stride loop: 2*EPL VGPRs held for the whole kernel)
  __shared__ __attribute__((aligned(16))) float sw[C], sb[C];
  for (int i = threadIdx.x * 4; i < C; i += 256 * 4) {
    *reinterpret_cast<float4*>(sw + i) = *reinterpret_cast<const float4*>(ln_w + i);
    *reinterpret_cast<float4*>(sb + i) = *reinterpret_cast<const float4*>(ln_b + i);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  uint4 cur[NK], nxt[NK];
  if (row < rows) {
#pragma unroll
    for (int k = 0; k < NK; ++k) cur[k] = *reinterpret_cast<const uint4*>(h + row * C + k * 512 + 8 * lane);
  }
  for (; row < rows; row += stride) {
    if (row + stride < rows) {
#pragma unroll
      for (int k = 0; k < NK; ++k)
        nxt[k] = *reinterpret_cast<const uint4*>(h + (row + stride) * C + k * 512 + 8 * lane);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      float v[8];
      unpack8<kH>(cur[k], v);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = gelu_erf(v[i]);
      cur[k] = pack8<kH>(v);
      unpack8<kH>(cur[k], v);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[i];
      __builtin_amdgcn_sched_barrier(0);   // one chunk's GELU temporaries live at a time
    }
    const float mean = wave_sum(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      float v[8];
      unpack8<kH>(cur[k], v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[i] - mean;
        q += d * d;
      }
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      float v[8], wv[8], bv[8];
      unpack8<kH>(cur[k], v);
      *reinterpret_cast<float4*>(wv) = *reinterpret_cast<const float4*>(sw + k * 512 + 8 * lane);
      *reinterpret_cast<float4*>(wv + 4) = *reinterpret_cast<const float4*>(sw + k * 512 + 8 * lane + 4);
      *reinterpret_cast<float4*>(bv) = *reinterpret_cast<const float4*>(sb + k * 512 + 8 * lane);
      *reinterpret_cast<float4*>(bv + 4) = *reinterpret_cast<const float4*>(sb + k * 512 + 8 * lane + 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (v[i] - mean) * rstd * wv[i] + bv[i];
      *reinterpret_cast<uint4*>(out + row * C + k * 512 + 8 * lane) = pack8<kH>(v);
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) cur[k] = nxt[k];
  }
}

// ---------------------------------------------------------------------------------------
// GELU+LN through a lookup table (default for F = 3072 / 4096): the input is bf16 and the GELU output
// is rounded to bf16 before the LN, so GELU is a function of the 16 input bits.  Each block first
// fills a 65536-entry table in LDS with exactly bf16(gelu_erf(x)) (the v2 arithmetic, so the output is
// bit-identical to gelu_ln_wave2_kernel), then its 16 waves walk rows grid-stride with the v2 LN
// arithmetic, one ds_read_u16 per element instead of ~13 VALU operations with a v_rcp and a v_exp
// (v2 is VALU-issue bound at ~1130 instructions per row per wave).  128 KiB table + the LN weights:
// one block per CU, launched once per CU; 8 waves (16 waves and deeper row prefetch measured slower).
// kCopy: the table is copied into LDS from g_gelu_tab (filled once per device by gelu_tab_fill_kernel,
// the same arithmetic, so the entries are bit-identical) -- 128 KiB from L2 instead of 65,536 gelu_erf
// evaluations per block (~8 % of the launch at 70k rows).  Without kCopy each block evaluates the table.
// GP_GELU_NW: waves per block of the lookup-table kernel (one block per CU: the table fills the LDS)
#ifndef GP_GELU_NW
#define GP_GELU_NW 8
#endif
// One table per format (index: the input's 16 bits; entry: gelu_erf rounded to the same format).
__device__ __attribute__((aligned(16))) uint16_t g_gelu_tab[2][65536];

template <bool kH>
__global__ __launch_bounds__(256) void gelu_tab_fill_kernel() {
  const int g = (int)blockIdx.x * 256 + (int)threadIdx.x;   // 8192 groups of 8 consecutive entries
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = gelu_erf(e2f<kH>((uint32_t)(8 * g + i)));
  *reinterpret_cast<uint4*>(g_gelu_tab[kH] + 8 * g) = pack8<kH>(v);
}

template <int EPL, int NW, bool kCopy, bool kH>
__global__ __launch_bounds__(NW * 64) void gelu_ln_lut_kernel(const uint16_t* h, const float* __restrict__ ln_w,
                                                          const float* __restrict__ ln_b, float eps,
                                                          uint16_t* out, int64_t rows) {
  constexpr int C = 64 * EPL, NK = EPL / 8;
  __shared__ __attribute__((aligned(16))) uint16_t tab[65536];
  __shared__ __attribute__((aligned(16))) float sw[C], sb[C];
  if constexpr (kCopy) {
    for (int g = threadIdx.x; g < 65536 / 8; g += NW * 64)
      *reinterpret_cast<uint4*>(tab + 8 * g) = *reinterpret_cast<const uint4*>(g_gelu_tab[kH] + 8 * g);
  } else {
    for (int g = threadIdx.x; g < 65536 / 8; g += NW * 64) {   // 8 consecutive entries per step
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = gelu_erf(e2f<kH>((uint32_t)(8 * g + i)));
      *reinterpret_cast<uint4*>(tab + 8 * g) = pack8<kH>(v);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  for (int i = threadIdx.x * 4; i < C; i += NW * 64 * 4) {
    *reinterpret_cast<float4*>(sw + i) = *reinterpret_cast<const float4*>(ln_w + i);
    *reinterpret_cast<float4*>(sb + i) = *reinterpret_cast<const float4*>(ln_b + i);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * NW;
  int64_t row = (int64_t)blockIdx.x * NW + (threadIdx.x >> 6);
  uint4 cur[NK], nxt[NK];
  if (row < rows) {
#pragma unroll
    for (int k = 0; k < NK; ++k) cur[k] = *reinterpret_cast<const uint4*>(h + row * C + k * 512 + 8 * lane);
  }
  auto look2 = [&](uint32_t w) -> uint32_t {   // two 16-bit inputs -> two GELU outputs
    return (uint32_t)tab[w & 0xffffu] | ((uint32_t)tab[w >> 16] << 16);
  };
  for (; row < rows; row += stride) {
    if (row + stride < rows) {
#pragma unroll
      for (int k = 0; k < NK; ++k)
        nxt[k] = *reinterpret_cast<const uint4*>(h + (row + stride) * C + k * 512 + 8 * lane);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      cur[k] = make_uint4(look2(cur[k].x), look2(cur[k].y), look2(cur[k].z), look2(cur[k].w));
      float v[8];
      unpack8<kH>(cur[k], v);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[i];
      __builtin_amdgcn_sched_barrier(0);   // bounds the lookups in flight (registers: 1024-thread block)
    }
    const float mean = wave_sum(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      float v[8];
      unpack8<kH>(cur[k], v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[i] - mean;
        q += d * d;
      }
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
    const int wo = 8 * lane;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      float v[8], wv[8], bv[8];
      unpack8<kH>(cur[k], v);
      *reinterpret_cast<float4*>(wv) = *reinterpret_cast<const float4*>(sw + k * 512 + wo);
      *reinterpret_cast<float4*>(wv + 4) = *reinterpret_cast<const float4*>(sw + k * 512 + wo + 4);
      *reinterpret_cast<float4*>(bv) = *reinterpret_cast<const float4*>(sb + k * 512 + wo);
      *reinterpret_cast<float4*>(bv + 4) = *reinterpret_cast<const float4*>(sb + k * 512 + wo + 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (v[i] - mean) * rstd * wv[i] + bv[i];
      *reinterpret_cast<uint4*>(out + row * C + k * 512 + 8 * lane) = pack8<kH>(v);
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) cur[k] = nxt[k];
  }
}

// the device a stream's work runs on (the null stream: the current device)
static int stream_device(hipStream_t s) {
  hipDevice_t dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess) return -1;
  return (int)dev;
}

static int gp_num_cus(hipStream_t s) {       // per-device cache of the CU count (LUT kernel: one block per CU)
  static int cache[64] = {0};
  const int dev = stream_device(s);
  if (dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// g_gelu_tab of the stream's device is filled (once: a fill launch on the caller's stream, then a
// synchronize of that stream, so no other stream can see the flag before the table is complete).  The
// flag is keyed by the device the stream runs on, not the current device.  While
// the stream is being captured into a graph the fill cannot be synchronised: the caller then takes the
// self-filling kernel until an eager call has filled the table.  Two threads filling at once write the
// same bytes.
static bool gelu_tab_ready(hipStream_t s, bool kh) {
  static std::atomic<bool> ready[2][64];
  const int dev = stream_device(s);
  if (dev < 0 || dev >= 64) return false;
  if (ready[kh][dev].load(std::memory_order_acquire)) return true;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
  // a launch error here is reported by this call only (hipPeekAtLastError leaves earlier errors
  // pending for the caller's own check)
  if (kh) gelu_tab_fill_kernel<true><<<65536 / 8 / 256, 256, 0, s>>>();
  else gelu_tab_fill_kernel<false><<<65536 / 8 / 256, 256, 0, s>>>();
  if (hipPeekAtLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) return false;
  ready[kh][dev].store(true, std::memory_order_release);
  return true;
}

// ---------------------------------------------------------------------------------------
template <int EPL>
__global__ __launch_bounds__(256) void layernorm_f32_kernel(const float* __restrict__ x, int64_t row_stride,
                                                            const float* __restrict__ ln_w,
                                                            const float* __restrict__ ln_b, float eps,
                                                            float* out, int64_t rows, int cols) {
  const int lane = threadIdx.x & 63;
  float wv[EPL], bv[EPL];
  ld_x4_f32<EPL>(ln_w, lane, wv);
  ld_x4_f32<EPL>(ln_b, lane, bv);
  for (int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6); row < rows;
       row += (int64_t)gridDim.x * kRowsPerBlock) {
    float v[EPL];
    ld_x4_f32<EPL>(x + row * row_stride, lane, v);
    wave_layernorm_regs<EPL>(v, cols, wv, bv, eps);
    st_x4_f32<EPL>(out + row * cols, lane, v);
  }
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

// fmt (every entry with 16-bit activations): GP_FMT_BF16 or GP_FMT_F16
#define GP_FMT_DISPATCH(fmt, KERNEL_CALL_H, KERNEL_CALL_B) \
  do {                                                    \
    if (fmt == GP_FMT_F16) { KERNEL_CALL_H; } else { KERNEL_CALL_B; } \
  } while (0)

extern "C" int gp_posembed_cls_ln(const uint16_t* xp, const int64_t* pos, const float* tab, const float* cls,
                                  int64_t B, int64_t N, int E, int G, const float* ln_w, const float* ln_b,
                                  float eps, float* x_out, uint16_t* ln_out, float* row_mean, int fmt,
                                  void* stream) {
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16, "gp_posembed_cls_ln: bad fmt %d", fmt);
  GP_REQUIRE(epl_ok(E), "gp_posembed_cls_ln: E=%d unsupported (64*{12,16,24})", E);
  GP_REQUIRE(B > 0 && N >= 0 && G > 0, "gp_posembed_cls_ln: bad sizes");
  GP_REQUIRE(tab && x_out && (N == 0 || (xp && pos)), "gp_posembed_cls_ln: null pointer");
  GP_REQUIRE(ln_w == nullptr || (ln_b && ln_out), "gp_posembed_cls_ln: LN needs ln_b and ln_out");
  const int64_t rows = B * (N + (cls != nullptr));
  if (rows == 0) return 0;
  hipStream_t s = gp_stream(stream);
#define GP_POSEMB(EPL, KH) posembed_cls_ln_kernel<EPL, KH><<<row_grid(rows), 256, 0, s>>>(xp, pos, tab, cls, B, N, E, G, ln_w, ln_b, eps, x_out, ln_out, row_mean)
  switch (E / 64) {
    case 12: GP_FMT_DISPATCH(fmt, GP_POSEMB(12, true), GP_POSEMB(12, false)); break;
    case 16: GP_FMT_DISPATCH(fmt, GP_POSEMB(16, true), GP_POSEMB(16, false)); break;
    case 24: GP_FMT_DISPATCH(fmt, GP_POSEMB(24, true), GP_POSEMB(24, false)); break;
  }
#undef GP_POSEMB
  return gp_check_launch("gp_posembed_cls_ln");
}

extern "C" int gp_residual_layernorm(float* x, const uint16_t* y, const float* bias, const float* ln_w,
                                     const float* ln_b, float eps, uint16_t* ln_out, int64_t rows, int cols,
                                     int fmt, void* stream) {
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16, "gp_residual_layernorm: bad fmt %d", fmt);
  GP_REQUIRE(epl_ok(cols), "gp_residual_layernorm: cols=%d unsupported (64*{12,16,24})", cols);
  GP_REQUIRE(rows >= 0, "gp_residual_layernorm: bad rows");
  if (rows == 0) return 0;
  GP_REQUIRE(x && y, "gp_residual_layernorm: null pointer");
  GP_REQUIRE(ln_w == nullptr || (ln_b && ln_out), "gp_residual_layernorm: LN needs ln_b and ln_out");
  hipStream_t s = gp_stream(stream);
#define GP_RESLN(EPL, KH) residual_ln_kernel<EPL, KH><<<row_grid(rows), 256, 0, s>>>(x, y, bias, ln_w, ln_b, eps, ln_out, rows, cols)
  switch (cols / 64) {
    case 12: GP_FMT_DISPATCH(fmt, GP_RESLN(12, true), GP_RESLN(12, false)); break;
    case 16: GP_FMT_DISPATCH(fmt, GP_RESLN(16, true), GP_RESLN(16, false)); break;
    case 24: GP_FMT_DISPATCH(fmt, GP_RESLN(24, true), GP_RESLN(24, false)); break;
  }
#undef GP_RESLN
  return gp_check_launch("gp_residual_layernorm");
}

extern "C" int gp_residual2_layernorm(float* x, const uint16_t* y1, const float* b1, const uint16_t* y2,
                                      const float* b2, const float* ln_w, const float* ln_b, float eps,
                                      uint16_t* ln_out, int64_t rows, int cols, int fmt, void* stream) {
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16, "gp_residual2_layernorm: bad fmt %d", fmt);
  GP_REQUIRE(epl_ok(cols), "gp_residual2_layernorm: cols=%d unsupported (64*{12,16,24})", cols);
  GP_REQUIRE(rows >= 0, "gp_residual2_layernorm: bad rows");
  if (rows == 0) return 0;
  GP_REQUIRE(x && y1, "gp_residual2_layernorm: null pointer");
  GP_REQUIRE(ln_w == nullptr || (ln_b && ln_out), "gp_residual2_layernorm: LN needs ln_b and ln_out");
  GP_REQUIRE(y2 != nullptr || ln_w != nullptr, "gp_residual2_layernorm: without y2 the call only writes ln_out");
  hipStream_t s = gp_stream(stream);
#define GP_RES2(EPL, KH)                                                                                        \
  do {                                                                                                          \
    if (y2) residual2_ln_kernel<EPL, KH, true><<<row_grid(rows), 256, 0, s>>>(x, y1, b1, y2, b2, ln_w, ln_b, eps, ln_out, rows, cols); \
    else residual2_ln_kernel<EPL, KH, false><<<row_grid(rows), 256, 0, s>>>(x, y1, b1, y2, b2, ln_w, ln_b, eps, ln_out, rows, cols); \
  } while (0)
  switch (cols / 64) {
    case 12: GP_FMT_DISPATCH(fmt, GP_RES2(12, true), GP_RES2(12, false)); break;
    case 16: GP_FMT_DISPATCH(fmt, GP_RES2(16, true), GP_RES2(16, false)); break;
    case 24: GP_FMT_DISPATCH(fmt, GP_RES2(24, true), GP_RES2(24, false)); break;
  }
#undef GP_RES2
  return gp_check_launch("gp_residual2_layernorm");
}

extern "C" int gp_gelu_layernorm(const uint16_t* h, const float* ln_w, const float* ln_b, float eps,
                                 uint16_t* out, int64_t rows, int cols, int fmt, void* stream) {
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16, "gp_gelu_layernorm: bad fmt %d", fmt);
  GP_REQUIRE(cols % 64 == 0 && (cols / 64 == 48 || cols / 64 == 64 || cols / 64 == 96),
             "gp_gelu_layernorm: cols=%d unsupported (64*{48,64,96})", cols);
  GP_REQUIRE(rows >= 0, "gp_gelu_layernorm: bad rows");
  if (rows == 0) return 0;
  GP_REQUIRE(h && ln_w && ln_b && out, "gp_gelu_layernorm: null pointer");
  hipStream_t s = gp_stream(stream);
  GP_REQUIRE(rows < (int64_t)0x7fffffff, "gp_gelu_layernorm: too many rows");
  if (cols == 3072 || cols == 4096) {
    // GELU by lookup table (the table + LN weights fit in LDS): one block per CU, the table copied
    // from g_gelu_tab, or evaluated per block while a graph capture runs before any eager call
    const int64_t want = (rows + GP_GELU_NW - 1) / GP_GELU_NW;
    const int cus = gp_num_cus(s);
    const unsigned nb = (unsigned)(want < cus ? want : cus);
    const bool copy = gelu_tab_ready(s, fmt == GP_FMT_F16);
#define GP_LUT(EPL, CP, KH) gelu_ln_lut_kernel<EPL, GP_GELU_NW, CP, KH><<<nb, 64 * GP_GELU_NW, 0, s>>>(h, ln_w, ln_b, eps, out, rows)
    if (cols == 3072) {
      if (copy) GP_FMT_DISPATCH(fmt, GP_LUT(48, true, true), GP_LUT(48, true, false));
      else GP_FMT_DISPATCH(fmt, GP_LUT(48, false, true), GP_LUT(48, false, false));
    } else {
      if (copy) GP_FMT_DISPATCH(fmt, GP_LUT(64, true, true), GP_LUT(64, true, false));
      else GP_FMT_DISPATCH(fmt, GP_LUT(64, false, true), GP_LUT(64, false, false));
    }
#undef GP_LUT
  } else {
    // v2 (F = 6144): wave per row, grid-stride with next-row prefetch, bf16-rounded GELU
    const int64_t want = (rows + 3) / 4;
    const unsigned nb = (unsigned)(want < 1024 ? want : 1024);
    GP_FMT_DISPATCH(fmt, (gelu_ln_wave2_kernel<96, true><<<nb, 256, 0, s>>>(h, ln_w, ln_b, eps, out, rows)),
                    (gelu_ln_wave2_kernel<96, false><<<nb, 256, 0, s>>>(h, ln_w, ln_b, eps, out, rows)));
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
    case 12: layernorm_f32_kernel<12><<<row_grid(rows), 256, 0, s>>>(x, row_stride, ln_w, ln_b, eps, out, rows, cols); break;
    case 16: layernorm_f32_kernel<16><<<row_grid(rows), 256, 0, s>>>(x, row_stride, ln_w, ln_b, eps, out, rows, cols); break;
    case 24: layernorm_f32_kernel<24><<<row_grid(rows), 256, 0, s>>>(x, row_stride, ln_w, ln_b, eps, out, rows, cols); break;
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
