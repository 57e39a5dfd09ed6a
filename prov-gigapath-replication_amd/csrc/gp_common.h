// Shared device helpers for the gfx950 slide-encoder kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GP_DEV __device__ __forceinline__

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// bf16 <-> fp32 on raw bit patterns.  f2bf is round-to-nearest-even (keeps NaN a NaN).
GP_DEV float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
GP_DEV uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}

// 16-bit activation formats: kH = false is bf16 (BASELINE's dtype), kH = true is fp16 (the compute
// format under the reference pipeline's torch.cuda.amp.autocast(float16), pipeline.py:186-187).
// Raw 16-bit patterns in and out; conversions round to nearest even.
template <bool kH>
GP_DEV float e2f(uint32_t b16) {                 // the low 16 bits of b16
  if constexpr (kH) return (float)__builtin_bit_cast(_Float16, (uint16_t)b16);
  else return __uint_as_float(b16 << 16);
}
template <bool kH>
GP_DEV float e2f_hi(uint32_t w) {                // the high 16 bits of w
  if constexpr (kH) return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
  else return __uint_as_float(w & 0xffff0000u);
}
template <bool kH>
GP_DEV uint16_t f2e(float f) {
  if constexpr (kH) return __builtin_bit_cast(uint16_t, (_Float16)f);
  else return f2bf(f);
}
// two values rounded (to nearest even) and packed by one v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32
typedef __bf16 gp_bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 gp_f16x2 __attribute__((ext_vector_type(2)));
typedef float gp_f32x2 __attribute__((ext_vector_type(2)));
template <bool kH>
GP_DEV uint32_t pack2e(float lo, float hi) {
  const gp_f32x2 v = {lo, hi};
  if constexpr (kH) return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, gp_f16x2));
  else return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, gp_bf16x2));
}

template <bool kH, int N>
GP_DEV void load_e(const uint16_t* p, float* out) {
  static_assert(N % 4 == 0, "");
  const uint2* q = reinterpret_cast<const uint2*>(p);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    const uint2 u = q[i];
    out[4 * i + 0] = e2f<kH>(u.x);
    out[4 * i + 1] = e2f_hi<kH>(u.x);
    out[4 * i + 2] = e2f<kH>(u.y);
    out[4 * i + 3] = e2f_hi<kH>(u.y);
  }
}
template <bool kH, int N>
GP_DEV void store_e(uint16_t* p, const float* v) {
  static_assert(N % 4 == 0, "");
  uint2* q = reinterpret_cast<uint2*>(p);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) q[i] = make_uint2(pack2e<kH>(v[4 * i], v[4 * i + 1]), pack2e<kH>(v[4 * i + 2], v[4 * i + 3]));
}

GP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
GP_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Load / store N consecutive bf16 (N % 4 == 0, 8-byte aligned) as fp32.
template <int N>
GP_DEV void load_bf16(const uint16_t* p, float* out) {
  static_assert(N % 4 == 0, "");
  const uint2* q = reinterpret_cast<const uint2*>(p);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    uint2 u = q[i];
    out[4 * i + 0] = __uint_as_float(u.x << 16);
    out[4 * i + 1] = __uint_as_float(u.x & 0xffff0000u);
    out[4 * i + 2] = __uint_as_float(u.y << 16);
    out[4 * i + 3] = __uint_as_float(u.y & 0xffff0000u);
  }
}
template <int N>
GP_DEV void store_bf16(uint16_t* p, const float* v) {
  static_assert(N % 4 == 0, "");
  uint2* q = reinterpret_cast<uint2*>(p);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    uint2 u;
    u.x = (uint32_t)f2bf(v[4 * i + 0]) | ((uint32_t)f2bf(v[4 * i + 1]) << 16);
    u.y = (uint32_t)f2bf(v[4 * i + 2]) | ((uint32_t)f2bf(v[4 * i + 3]) << 16);
    q[i] = u;
  }
}
template <int N>
GP_DEV void load_f32(const float* p, float* out) {
  static_assert(N % 4 == 0, "");
  const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    float4 u = q[i];
    out[4 * i + 0] = u.x; out[4 * i + 1] = u.y; out[4 * i + 2] = u.z; out[4 * i + 3] = u.w;
  }
}
template <int N>
GP_DEV void store_f32(float* p, const float* v) {
  static_assert(N % 4 == 0, "");
  float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) q[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}

// Coalesced row mappings for one 64-lane wave.
//   "x4":  lane owns elements k*256 + 4*lane + {0..3}, k < EPL/4 (fp32: 16-B, bf16: 8-B accesses;
//          every wave-instruction touches one contiguous 1 KiB / 512 B span)
//   "x8":  lane owns elements k*512 + 8*lane + {0..7}, k < EPL/8 (bf16: 16-B accesses)
template <int EPL>
GP_DEV void ld_x4_f32(const float* row, int lane, float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 4; ++k) {
    const float4 u = *reinterpret_cast<const float4*>(row + k * 256 + 4 * lane);
    v[4 * k] = u.x; v[4 * k + 1] = u.y; v[4 * k + 2] = u.z; v[4 * k + 3] = u.w;
  }
}
template <int EPL>
GP_DEV void st_x4_f32(float* row, int lane, const float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 4; ++k)
    *reinterpret_cast<float4*>(row + k * 256 + 4 * lane) = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
}
// non-temporal variants (streamed rows that the next kernels do not read back soon)
typedef float gp_f4v __attribute__((ext_vector_type(4)));
template <int EPL>
GP_DEV void ld_x4_f32_nt(const float* row, int lane, float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 4; ++k) {
    const gp_f4v u = __builtin_nontemporal_load(reinterpret_cast<const gp_f4v*>(row + k * 256 + 4 * lane));
    v[4 * k] = u.x; v[4 * k + 1] = u.y; v[4 * k + 2] = u.z; v[4 * k + 3] = u.w;
  }
}
template <int EPL>
GP_DEV void st_x4_f32_nt(float* row, int lane, const float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 4; ++k) {
    const gp_f4v u = {v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
    __builtin_nontemporal_store(u, reinterpret_cast<gp_f4v*>(row + k * 256 + 4 * lane));
  }
}
template <int EPL>
GP_DEV void ld_x4_bf16(const uint16_t* row, int lane, float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 4; ++k) load_bf16<4>(row + k * 256 + 4 * lane, v + 4 * k);
}
template <int EPL>
GP_DEV void st_x4_bf16(uint16_t* row, int lane, const float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 4; ++k) store_bf16<4>(row + k * 256 + 4 * lane, v + 4 * k);
}
template <bool kH, int EPL>
GP_DEV void ld_x4_e(const uint16_t* row, int lane, float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 4; ++k) load_e<kH, 4>(row + k * 256 + 4 * lane, v + 4 * k);
}
template <bool kH, int EPL>
GP_DEV void st_x4_e(uint16_t* row, int lane, const float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 4; ++k) store_e<kH, 4>(row + k * 256 + 4 * lane, v + 4 * k);
}
template <int EPL>
GP_DEV void ld_x8_bf16(const uint16_t* row, int lane, float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 8; ++k) {
    const uint4 u = *reinterpret_cast<const uint4*>(row + k * 512 + 8 * lane);
    const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[8 * k + 2 * i] = __uint_as_float(w4[i] << 16);
      v[8 * k + 2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
    }
  }
}
template <int EPL>
GP_DEV void st_x8_bf16(uint16_t* row, int lane, const float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 8; ++k) {
    uint4 u;
    u.x = (uint32_t)f2bf(v[8 * k + 0]) | ((uint32_t)f2bf(v[8 * k + 1]) << 16);
    u.y = (uint32_t)f2bf(v[8 * k + 2]) | ((uint32_t)f2bf(v[8 * k + 3]) << 16);
    u.z = (uint32_t)f2bf(v[8 * k + 4]) | ((uint32_t)f2bf(v[8 * k + 5]) << 16);
    u.w = (uint32_t)f2bf(v[8 * k + 6]) | ((uint32_t)f2bf(v[8 * k + 7]) << 16);
    *reinterpret_cast<uint4*>(row + k * 512 + 8 * lane) = u;
  }
}
template <int EPL>
GP_DEV void ld_x8_f32(const float* row, int lane, float* v) {
#pragma unroll
  for (int k = 0; k < EPL / 8; ++k) {
    const float4 a = *reinterpret_cast<const float4*>(row + k * 512 + 8 * lane);
    const float4 b = *reinterpret_cast<const float4*>(row + k * 512 + 8 * lane + 4);
    v[8 * k] = a.x; v[8 * k + 1] = a.y; v[8 * k + 2] = a.z; v[8 * k + 3] = a.w;
    v[8 * k + 4] = b.x; v[8 * k + 5] = b.y; v[8 * k + 6] = b.z; v[8 * k + 7] = b.w;
  }
}

// LayerNorm statistics + affine on register-resident values (any lane mapping; w/b in the
// same mapping as v).  torch semantics: biased variance, two-pass, fp32.
template <int EPL>
GP_DEV void wave_layernorm_regs(float* v, int cols, const float* w, const float* b, float eps) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) s += v[i];
  const float mean = wave_sum(s) / (float)cols;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)cols + eps);
#pragma unroll
  for (int i = 0; i < EPL; ++i) v[i] = (v[i] - mean) * rstd * w[i] + b[i];
}

// Per-branch geometry of the dilated schedule (dilated_attention.py:16-31, 76-98).
struct GpBranch {
  int32_t s;      // min(sl, L)
  int32_t r;      // dilation ratio
  int32_t m;      // ceil(s / r) sparse rows per segment
  int32_t nseg;   // ceil(L / s) segments per batch
  int32_t g;      // m * r: dense length per segment after sparse_to_dense
  int32_t hpg;    // heads per dilation group: (H rounded up to r) / r
};

inline GpBranch gp_make_branch(int64_t L, int sl, int r, int H) {
  GpBranch b;
  b.s = (int32_t)(sl < L ? sl : L);
  b.r = r;
  b.m = (b.s + r - 1) / r;
  b.nseg = (int32_t)((L + b.s - 1) / b.s);
  b.g = b.m * r;
  const int hp = H + ((H % r) ? (r - H % r) : 0);
  b.hpg = hp / r;
  return b;
}

// Number of valid (non-pad) sparse rows of segment n for head group j.
GP_DEV int gp_valid_rows(const GpBranch& br, int64_t L, int n, int j) {
  const int64_t rem = L - (int64_t)n * br.s;
  const int64_t lim = (rem < br.s ? rem : br.s) - j;
  return lim > 0 ? (int)((lim + br.r - 1) / br.r) : 0;
}
