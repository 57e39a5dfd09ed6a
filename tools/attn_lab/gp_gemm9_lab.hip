// LAB BUILD (not the product): GEMM v9 -- TWO independent workgroups per CU, so that one workgroup's
// epilogue (the fused FFN's GELU + statistics: ~16 VALU per output element with the MFMA pipe idle in the
// product's one-workgroup-per-CU v8 kernel) overlaps the other workgroup's MFMAs.  Same C ABI and
// epilogues as csrc/gp_gemm.hip (gp_linear, gp_ffn_fc1_gelu, gp_ffn_fc2_ln, gp_gemm_workspace_bytes);
// A/B with  python tools/ffn_bench.py --lab tools/attn_lab/liblab_gemm9.so
//
//   * 128 x 256 output tile per workgroup of 4 waves (1 M x 4 N, one wave per SIMD), a wave owning 128 x 64
//     = 8 x 4 v_mfma_f32_16x16x32 tiles (128 fp32 accumulators per lane, as in v8); BK = 32;
//   * a 3-stage LDS ring of [A 128 x 32 | W 256 x 32] (24 KiB per stage, 64-byte rows whose 16-byte chunk c
//     sits at c ^ ((row >> 2) & 3): the 16 rows of every ds_read_b128 lane group on 16 distinct bank slots),
//     staged by LDS-DMA, 6 one-KiB pieces per wave per stage; per K-tile: counted vmcnt(6) (the next stage
//     stays in flight) | s_barrier | the DMA of stage kt+2 into the slot read at kt-1 | 12 fragment reads |
//     32 MFMAs -- one barrier per K-tile, the other workgroup on the same SIMDs filling its gaps;
//   * ~78 KiB of LDS per workgroup (ring 72 + per-tile column parameters and row exchange): 2 per CU;
//   * persistent over tiles with the next tile's first two stages streaming in during the current tile's
//     last two K-tiles; the per-tile column parameters (bias, or c | d of the LN fold) and the fold's row
//     statistics come by LDS-DMA too, two tiles' slots;
//   * the last, partial round of tiles split in K as in v8.
#include <math.h>

#include <type_traits>

#include "gp_api.h"
#include "gp_common.h"

namespace {

constexpr int kBM = 128, kBN = 256, kBK = 32, kNS = 3;
constexpr int kThreads = 256;
constexpr int kRowB = kBK * 2;           // 64-byte LDS rows
constexpr int kAT = kBM * kRowB;         // 8 KiB
constexpr int kWT = kBN * kRowB;         // 16 KiB
constexpr int kST = kAT + kWT;           // 24 KiB per stage
constexpr int kMaxN = 3072;

enum { kEpiLinear = 0, kEpiGelu = 1, kEpiLnFold = 2 };

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8g __attribute__((ext_vector_type(8)));

__shared__ __attribute__((aligned(1024))) char s_ring[kNS * kST];
__shared__ __attribute__((aligned(1024))) float s_bias[2][kBN];        // linear / GELU
__shared__ __attribute__((aligned(1024))) float s_cd[2][2 * kBN];      // LN fold: c | d
__shared__ __attribute__((aligned(1024))) float2 s_rowst[2][kBM];      // LN fold: (mean, rstd)
__shared__ __attribute__((aligned(16))) float s_rsum[kBM * 4];         // GELU row exchange
__shared__ __attribute__((aligned(16))) float s_rsq[kBM * 4];

template <int I, int N, typename F>
GP_DEV void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>());
    static_for<I + 1, N>(f);
  }
}

GP_DEV int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

struct GemmArgs {
  const uint16_t* A;
  const uint16_t* W;
  const float* colp0;   // bias (linear / gelu, may be null) or c (LN fold)
  const float* colp1;   // d (LN fold)
  uint16_t* C;
  float* stats;         // gelu: written [N/256][M] float2; LN fold: (mean, rstd) [M] float2 (plane nst)
  int64_t lda, ldw, ldc;
  int M, N, K;
  int nst;
  float eps;
  int n_dp;
  int split;
  float* ws;
};

template <int n>
GP_DEV void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}

GP_DEV void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  __builtin_amdgcn_sched_barrier(0);
}

GP_DEV float gelu_g(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(0.5307027145f, t, -0.7265760135f);
  p = fmaf(p, t, 0.7107068705f);
  p = fmaf(p, t, -0.142248368f);
  p = fmaf(p, t, 0.127414796f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f((x * -0.72134752044448170368f) * x);
  return fmaf(-fabsf(x) * p, e, fmaxf(x, 0.f));
}

GP_DEV float2 merge_row_stats(const float2* st, int64_t stride, int nst, float eps) {
  float msum = 0.f;
  for (int g = 0; g < nst; ++g) msum += st[g * stride].x;
  const float mean = msum / (float)nst;
  float m2 = 0.f;
  for (int g = 0; g < nst; ++g) {
    const float2 p = st[g * stride];
    const float dm = p.x - mean;
    m2 += p.y + 256.f * dm * dm;
  }
  return make_float2(mean, rsqrtf(m2 / (float)(256 * nst) + eps));
}

__global__ __launch_bounds__(256) void row_stats_kernel(float* stats, int M, int nst, float eps) {
  const int row = (int)blockIdx.x * 256 + (int)threadIdx.x;
  if (row >= M) return;
  float2* st = reinterpret_cast<float2*>(stats);
  st[(int64_t)nst * M + row] = merge_row_stats(st + row, M, nst, eps);
}

// NK = K / 32 K-tiles (a multiple of 3, so the ring slot of K-tile kt is kt % 3 in every tile)
template <int NK, int S, int EPI, bool kH>
__global__ __launch_bounds__(kThreads, 2) void gemm9_kernel(const GemmArgs g) {
  static_assert(NK % 3 == 0 && NK >= 3 && (S == 1 || (NK % (3 * S) == 0)), "");
  const int tiles_n = g.N / kBN;
  const int ntiles = ((g.M + kBM - 1) / kBM) * tiles_n;
  const int G = (int)gridDim.x;
  const int sid = xcd_remap((int)blockIdx.x, G);
  const int n_dp = g.n_dp;
  const int n_my = sid < n_dp ? (n_dp - 1 - sid) / G + 1 : 0;
  const bool tail = S > 1 && g.split && sid < (ntiles - n_dp) * S;
  if (n_my == 0 && !tail) return;
  const int lane = threadIdx.x & 63;
  const int wn = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int r16 = lane & 15, q = lane >> 4;

  auto rsrc_a = [&](int T) {
    const int m0 = (T / tiles_n) * kBM;
    const int64_t a_bytes = (int64_t)(g.M - m0) * g.lda * 2;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(g.A + (int64_t)m0 * g.lda), (short)0,
                                             (int)(a_bytes < 0x7fffffff ? a_bytes : 0x7fffffff), 0x00020000);
  };
  auto rsrc_w = [&](int T) {
    const int n0 = (T % tiles_n) * kBN;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(g.W + (int64_t)n0 * g.ldw), (short)0,
                                             (int)((int64_t)kBN * g.ldw * 2), 0x00020000);
  };
  // DMA pieces: piece p (0..23; A 0..7, W 8..23) covers 16 rows; wave wn issues p = wn + 4j, j < 6 (2 A, 4 W).
  // Lane l writes row p*16 + l/4, physical chunk l%4 = logical chunk (l%4) ^ ((l >> 4) & 3).
  const int lrow = lane >> 2, lch = (lane & 3) ^ ((lane >> 4) & 3);
  const int voff_a = (int)((int64_t)lrow * g.lda * 2) + lch * 16;
  const int voff_w = (int)((int64_t)lrow * g.ldw * 2) + lch * 16;
  int pa[2] = {(int)((int64_t)wn * 16 * g.lda * 2), (int)((int64_t)(wn + 4) * 16 * g.lda * 2)};
  int pw[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) pw[j] = (int)((int64_t)(wn + 4 * j) * 16 * g.ldw * 2);
  auto issue_stage = [&](auto slotc, const __amdgpu_buffer_rsrc_t& ra, const __amdgpu_buffer_rsrc_t& rw, int kt) {
    constexpr int SL = decltype(slotc)::value;
    char* base = s_ring + SL * kST;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(base + (wn + 4 * j) * 1024),
                                               16, voff_a, kt * kRowB + pa[j], 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rw, (__attribute__((address_space(3))) void*)(base + kAT + (wn + 4 * j) * 1024), 16, voff_w,
          kt * kRowB + pw[j], 0, 0);
  };
  // per-tile column parameters / row statistics (wave 0, one or two 1-KiB pieces), issued at the tile's
  // first K-tile right before that K-tile's stage DMA (so the counted waits retire it with the stage)
  auto issue_tile_params = [&](int T, int slot) {
    if (wn != 0) return;
    const int n0 = (T % tiles_n) * kBN;
    if constexpr (EPI == kEpiLnFold) {
      const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)(g.colp0 + n0), (short)0, 1024, 0x00020000);
      const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(g.colp1 + n0), (short)0, 1024, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (__attribute__((address_space(3))) void*)(&s_cd[slot][0]), 16, lane * 16, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (__attribute__((address_space(3))) void*)(&s_cd[slot][kBN]), 16, lane * 16, 0, 0, 0);
      const int m0 = (T / tiles_n) * kBM;
      const int64_t nb = (int64_t)(g.M - m0) * 8;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(reinterpret_cast<const float2*>(g.stats) + (int64_t)g.nst * g.M + m0), (short)0,
          (int)(nb < 1024 ? nb : 1024), 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(&s_rowst[slot][0]), 16, lane * 16, 0, 0, 0);
    } else {
      if (g.colp0 != nullptr) {
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)(g.colp0 + n0), (short)0, 1024, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)(&s_bias[slot][0]), 16, lane * 16, 0, 0, 0);
      }
    }
  };

  // fragment reads: lane (r16, q) reads row R0 + r16, logical chunk q = physical q ^ ((r16 >> 2) & 3)
  const int lo = r16 * kRowB + ((q ^ ((r16 >> 2) & 3)) << 4);
  bf16x8 af[8], wf[4];
  f32x4v acc[8][4];
  auto mfma = [](const bf16x8& a, const bf16x8& b, const f32x4v& c) -> f32x4v {
    if constexpr (kH)
      return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8g, a), __builtin_bit_cast(f16x8g, b), c,
                                                    0, 0, 0);
    else
      return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  };
  auto compute = [&](auto slotc) {
    constexpr int SL = decltype(slotc)::value;
    const char* base = s_ring + SL * kST;
#pragma unroll
    for (int e = 0; e < 4; ++e) wf[e] = *reinterpret_cast<const bf16x8*>(base + kAT + (wn * 64 + e * 16) * kRowB + lo);
#pragma unroll
    for (int f = 0; f < 8; ++f) af[f] = *reinterpret_cast<const bf16x8*>(base + f * 16 * kRowB + lo);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[f][e] = mfma(wf[e], af[f], acc[f][e]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto zero_acc = [&]() {
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[f][e] = f32x4v{0.f, 0.f, 0.f, 0.f};
  };

  // epilogue of tile T (slot = its parameter slot): lane (r16, q) of wave wn holds rows m0 + 16 f + r16,
  // columns n0 + 64 wn + 16 e + 4 q .. +3
  auto epilogue_tile = [&](int T, int slot) {
    const int tn = T % tiles_n;
    const int m0 = (T / tiles_n) * kBM;
    const int nw = tn * kBN + wn * 64;
    uint32_t hp[8][4][2];
    if constexpr (EPI == kEpiLinear) {
      if (g.colp0 != nullptr) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float4 b = *reinterpret_cast<const float4*>(&s_bias[slot][wn * 64 + e * 16 + 4 * q]);
#pragma unroll
          for (int f = 0; f < 8; ++f) acc[f][e] += f32x4v{b.x, b.y, b.z, b.w};
        }
      }
    } else if constexpr (EPI == kEpiGelu) {
      float bb[4][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
        if (g.colp0 != nullptr) b = *reinterpret_cast<const float4*>(&s_bias[slot][wn * 64 + e * 16 + 4 * q]);
        bb[e][0] = b.x; bb[e][1] = b.y; bb[e][2] = b.z; bb[e][3] = b.w;
      }
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        float s = 0.f, s2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t xp = pack2e<kH>(acc[f][e][2 * h] + bb[e][2 * h], acc[f][e][2 * h + 1] + bb[e][2 * h + 1]);
            hp[f][e][h] = pack2e<kH>(gelu_g(e2f<kH>(xp)), gelu_g(e2f_hi<kH>(xp)));
            const float h0 = e2f<kH>(hp[f][e][h]), h1 = e2f_hi<kH>(hp[f][e][h]);
            s += h0 + h1;
            s2 = fmaf(h0, h0, fmaf(h1, h1, s2));
          }
        }
        s += __shfl_xor(s, 16, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s += __shfl_xor(s, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (q == 0) {
          s_rsum[(f * 16 + r16) * 4 + wn] = s;
          s_rsq[(f * 16 + r16) * 4 + wn] = s2;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      lds_barrier();
      if (threadIdx.x < kBM) {
        const int row = m0 + (int)threadIdx.x;
        if (row < g.M) {
          const float4 s4 = *reinterpret_cast<const float4*>(s_rsum + threadIdx.x * 4);
          const float4 q4 = *reinterpret_cast<const float4*>(s_rsq + threadIdx.x * 4);
          const float sum = (s4.x + s4.y) + (s4.z + s4.w), sq = (q4.x + q4.y) + (q4.z + q4.w);
          const float mean = sum * (1.f / 256.f);
          reinterpret_cast<float2*>(g.stats)[(int64_t)tn * g.M + row] = make_float2(mean, fmaxf(fmaf(-sum, mean, sq), 0.f));
        }
      }
    } else {   // LN fold
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        const float2 rs = s_rowst[slot][f * 16 + r16];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float4 c = *reinterpret_cast<const float4*>(&s_cd[slot][wn * 64 + e * 16 + 4 * q]);
          const float4 d = *reinterpret_cast<const float4*>(&s_cd[slot][kBN + wn * 64 + e * 16 + 4 * q]);
          const float cc[4] = {c.x, c.y, c.z, c.w}, dd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[f][e][j] = fmaf(rs.y, fmaf(-rs.x, cc[j], acc[f][e][j]), dd[j]);
        }
      }
    }
    const int64_t c_rows = g.M - m0 < kBM ? (g.M - m0 > 0 ? g.M - m0 : 0) : kBM;
    const uint64_t cp = reinterpret_cast<uint64_t>(g.C + (int64_t)m0 * g.ldc + nw);
    const uint64_t cpu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(cp >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)cp);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(cpu), (short)0, __builtin_amdgcn_readfirstlane((int)(c_rows * g.ldc * 2)),
        0x00020000);
    const int c_lane = (int)((r16 * g.ldc + 16 * (q & 1) + 8 * (q >> 1)) * 2);
    const int c_f = (int)(16 * g.ldc * 2);
#pragma unroll
    for (int f = 0; f < 8; ++f) {
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        uint32_t pk[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = 2 * pr + h;
          if constexpr (EPI == kEpiGelu) {
            pk[h][0] = hp[f][e][0];
            pk[h][1] = hp[f][e][1];
          } else {
            pk[h][0] = pack2e<kH>(acc[f][e][0], acc[f][e][1]);
            pk[h][1] = pack2e<kH>(acc[f][e][2], acc[f][e][3]);
          }
        }
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto r = __builtin_amdgcn_permlane16_swap(pk[0][d], pk[1][d], false, false);
          pk[0][d] = r[0];
          pk[1][d] = r[1];
        }
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        const i32x4 v4 = {(int)pk[0][0], (int)pk[0][1], (int)pk[1][0], (int)pk[1][1]};
        __builtin_amdgcn_raw_buffer_store_b128(v4, rc, c_lane + pr * 64, f * c_f, 0);
      }
    }
  };
  auto store_partial = [&](int u) {
    float* base = g.ws + (int64_t)u * (kBM * kBN);
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = f * 16 + r16, col = wn * 64 + e * 16 + 4 * q;
        *reinterpret_cast<f32x4v*>(base + row * kBN + col) = acc[f][e];
      }
  };

  // one sequence of `count` tiles of nk K-tiles each (K-tiles kt0 ..), the DMA of tile i+1's first two
  // stages issued during tile i's last two K-tiles; with_params: the per-tile parameter DMA + epilogue
  auto run_seq = [&](auto nkc, int count, int kt0, auto&& tile_of, auto&& epilogue, bool with_params) {
    constexpr int nk = decltype(nkc)::value;
    int T = tile_of(0);
    __amdgpu_buffer_rsrc_t ra = rsrc_a(T), rw = rsrc_w(T);
    if (with_params) issue_tile_params(T, 0);
    issue_stage(std::integral_constant<int, 0>(), ra, rw, kt0);
    issue_stage(std::integral_constant<int, 1>(), ra, rw, kt0 + 1);
    for (int i = 0; i < count; ++i) {
      const bool has_next = i + 1 < count;
      const int Tn = has_next ? tile_of(i + 1) : T;
      const __amdgpu_buffer_rsrc_t ran = rsrc_a(Tn), rwn = rsrc_w(Tn);
      asm volatile("" : "+s"(pa[0]), "+s"(pa[1]), "+s"(pw[0]), "+s"(pw[1]), "+s"(pw[2]), "+s"(pw[3]));
      zero_acc();
      auto step = [&](auto ktc) {
        constexpr int kt = decltype(ktc)::value;
        constexpr int SL = kt % kNS;
        constexpr int SN = (kt + 2) % kNS;
        if (kt + 1 < nk || has_next) wait_vmcnt<6>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (kt + 2 < nk) {
          issue_stage(std::integral_constant<int, SN>(), ra, rw, kt0 + kt + 2);
        } else {
          if (has_next) {
            if (kt + 2 == nk && with_params) issue_tile_params(Tn, (i + 1) & 1);
            issue_stage(std::integral_constant<int, SN>(), ran, rwn, kt0 + kt + 2 - nk);
          }
        }
        compute(std::integral_constant<int, SL>());
      };
      static_for<0, nk>(step);
      epilogue(i, T);
      ra = ran;
      rw = rwn;
      T = Tn;
    }
    wait_vmcnt<0>();
  };

  if (n_my > 0)
    run_seq(std::integral_constant<int, NK>(), n_my, 0, [&](int i) { return sid + i * G; },
            [&](int i, int T) { epilogue_tile(T, i & 1); }, true);
  if constexpr (S > 1) {
    if (tail) {
      constexpr int NKS = NK / S;
      __builtin_amdgcn_s_barrier();   // every wave done with the ring of the data-parallel tiles
      const int T = n_dp + sid / S, part = sid % S;
      run_seq(std::integral_constant<int, NKS>(), 1, part * NKS, [&](int) { return T; },
              [&](int, int) { store_partial(sid); }, false);
    }
  }
}

// split tail: sum of the S partials + the linear / LN-fold epilogue; one thread per 8 columns of a row
template <int EPI, bool kH>
__global__ __launch_bounds__(256) void gemm9_reduce_kernel(const GemmArgs g, int S) {
  const int tiles_n = g.N / kBN;
  constexpr int kPer = kBM * kBN / 8 / 256;
  const int unit = blockIdx.x / kPer;
  const int idx = (blockIdx.x % kPer) * 256 + threadIdx.x;
  const int row = idx / (kBN / 8), col = (idx % (kBN / 8)) * 8;
  const int T = g.n_dp + unit;
  const int m = (T / tiles_n) * kBM + row, n = (T % tiles_n) * kBN + col;
  if (m >= g.M) return;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const float* p = g.ws + (int64_t)(unit * S + s) * (kBM * kBN) + row * kBN + col;
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
  if constexpr (EPI == kEpiLinear) {
    if (g.colp0 != nullptr)
      for (int e = 0; e < 8; ++e) v[e] += g.colp0[n + e];
  } else {
    const float2 mr = reinterpret_cast<const float2*>(g.stats)[(int64_t)g.nst * g.M + m];
    for (int e = 0; e < 8; ++e) v[e] = fmaf(mr.y, fmaf(-mr.x, g.colp0[n + e], v[e]), g.colp1[n + e]);
  }
  uint4 o;
  o.x = pack2e<kH>(v[0], v[1]);
  o.y = pack2e<kH>(v[2], v[3]);
  o.z = pack2e<kH>(v[4], v[5]);
  o.w = pack2e<kH>(v[6], v[7]);
  *reinterpret_cast<uint4*>(g.C + (int64_t)m * g.ldc + n) = o;
}

int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

struct Plan {
  int G, S, n_dp;
  int64_t rem, ws_bytes;
};

Plan make_plan(int64_t M, int64_t N, int64_t K, bool allow_split) {
  Plan p;
  const int64_t tiles = ((M + kBM - 1) / kBM) * (N / kBN);
  const int slots = 2 * device_cus();
  p.G = (int)(tiles < slots ? tiles : slots);
  p.S = 1;
  p.n_dp = (int)tiles;
  p.rem = 0;
  p.ws_bytes = 0;
  const int S = K == 768 ? 2 : 4;
  const int64_t rem = tiles % p.G;
  if (allow_split && tiles > p.G && rem > 0 && rem * S <= p.G && rem * 2 <= p.G) {
    p.S = S;
    p.n_dp = (int)(tiles - rem);
    p.rem = rem;
    p.ws_bytes = rem * S * kBM * kBN * (int64_t)sizeof(float);
  }
  return p;
}

int check_shapes(const char* who, const void* A, int64_t lda, const void* W, int64_t ldw, const void* C, int64_t ldc,
                 int64_t M, int64_t N, int64_t K, int fmt) {
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16, "%s: bad fmt %d", who, fmt);
  GP_REQUIRE(A && W && C, "%s: null pointer", who);
  GP_REQUIRE(M > 0 && M < (int64_t)0x7fffffff && N > 0 && K > 0, "%s: bad sizes", who);
  GP_REQUIRE(N % kBN == 0 && N <= kMaxN, "%s: N=%lld must be a multiple of %d, at most %d", who, (long long)N, kBN,
             kMaxN);
  GP_REQUIRE(K == 768 || K == 1536 || K == 3072, "%s: K=%lld not instantiated (768 / 1536 / 3072)", who,
             (long long)K);
  GP_REQUIRE(lda >= K && ldw >= K && ldc >= N && lda % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0,
             "%s: bad leading dimensions", who);
  GP_REQUIRE(gp_aligned(A, 16) && gp_aligned(W, 16) && gp_aligned(C, 16), "%s: misaligned operand", who);
  GP_REQUIRE((int64_t)kBM * lda * 2 < 0x7fffffff && (int64_t)kBN * ldw * 2 < 0x7fffffff &&
                 (int64_t)kBM * ldc * 2 < 0x7fffffff,
             "%s: leading dimension too large for 32-bit tile offsets", who);
  return 0;
}

template <int EPI, bool kH>
int launch(GemmArgs g, const Plan& p, hipStream_t s) {
  g.n_dp = p.n_dp;
  g.split = p.S > 1;
  const dim3 grid((unsigned)p.G), block(kThreads);
  constexpr bool kSplit = EPI != kEpiGelu;
  switch (g.K) {
    case 768:
      if (kSplit && p.S > 1) gemm9_kernel<24, kSplit ? 2 : 1, EPI, kH><<<grid, block, 0, s>>>(g);
      else gemm9_kernel<24, 1, EPI, kH><<<grid, block, 0, s>>>(g);
      break;
    case 1536:
      if (kSplit && p.S > 1) gemm9_kernel<48, kSplit ? 4 : 1, EPI, kH><<<grid, block, 0, s>>>(g);
      else gemm9_kernel<48, 1, EPI, kH><<<grid, block, 0, s>>>(g);
      break;
    default:
      if (kSplit && p.S > 1) gemm9_kernel<96, kSplit ? 4 : 1, EPI, kH><<<grid, block, 0, s>>>(g);
      else gemm9_kernel<96, 1, EPI, kH><<<grid, block, 0, s>>>(g);
      break;
  }
  if constexpr (EPI != kEpiGelu) {
    if (p.S > 1) gemm9_reduce_kernel<EPI, kH><<<(unsigned)(p.rem * (kBM * kBN / 8 / 256)), 256, 0, s>>>(g, p.S);
  }
  return 0;
}

}  // namespace

extern "C" int64_t gp_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0 || N % kBN) return 0;
  return make_plan(M, N, K, true).ws_bytes;
}

extern "C" int gp_linear(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, const float* bias,
                         uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K, void* ws, int64_t ws_bytes,
                         int fmt, void* stream) {
  if (int rc = check_shapes("gp_linear", A, lda, W, ldw, C, ldc, M, N, K, fmt)) return rc;
  GP_REQUIRE(!bias || gp_aligned(bias, 16), "gp_linear: misaligned bias");
  const Plan p = make_plan(M, N, K, ws != nullptr);
  GP_REQUIRE(p.ws_bytes <= ws_bytes, "gp_linear: workspace of %lld bytes, %lld needed", (long long)ws_bytes,
             (long long)p.ws_bytes);
  GemmArgs g = {};
  g.A = A; g.W = W; g.colp0 = bias; g.C = C;
  g.lda = lda; g.ldw = ldw; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.ws = static_cast<float*>(ws);
  if (fmt == GP_FMT_F16) launch<kEpiLinear, true>(g, p, gp_stream(stream));
  else launch<kEpiLinear, false>(g, p, gp_stream(stream));
  return gp_check_launch("gp_linear");
}

extern "C" int gp_ffn_fc1_gelu(const uint16_t* A, int64_t lda, const uint16_t* W1, int64_t ldw, const float* b1,
                               uint16_t* h, int64_t ldh, float* stats, int64_t M, int64_t F, int64_t K, int fmt,
                               void* stream) {
  if (int rc = check_shapes("gp_ffn_fc1_gelu", A, lda, W1, ldw, h, ldh, M, F, K, fmt)) return rc;
  GP_REQUIRE(stats && gp_aligned(stats, 8), "gp_ffn_fc1_gelu: null or misaligned stats");
  const Plan p = make_plan(M, F, K, false);
  GemmArgs g = {};
  g.A = A; g.W = W1; g.colp0 = b1; g.C = h; g.stats = stats;
  g.lda = lda; g.ldw = ldw; g.ldc = ldh;
  g.M = (int)M; g.N = (int)F; g.K = (int)K;
  if (fmt == GP_FMT_F16) launch<kEpiGelu, true>(g, p, gp_stream(stream));
  else launch<kEpiGelu, false>(g, p, gp_stream(stream));
  return gp_check_launch("gp_ffn_fc1_gelu");
}

extern "C" int gp_ffn_fc2_ln(const uint16_t* h, int64_t ldh, const uint16_t* W2g, int64_t ldw, float* stats,
                             const float* c, const float* d, float eps, uint16_t* y, int64_t ldy, int64_t M, int64_t N,
                             int64_t F, void* ws, int64_t ws_bytes, int fmt, void* stream) {
  if (int rc = check_shapes("gp_ffn_fc2_ln", h, ldh, W2g, ldw, y, ldy, M, N, F, fmt)) return rc;
  GP_REQUIRE(stats && c && d, "gp_ffn_fc2_ln: null stats / c / d");
  const Plan p = make_plan(M, N, F, ws != nullptr);
  GP_REQUIRE(p.ws_bytes <= ws_bytes, "gp_ffn_fc2_ln: workspace of %lld bytes, %lld needed", (long long)ws_bytes,
             (long long)p.ws_bytes);
  GemmArgs g = {};
  g.A = h; g.W = W2g; g.colp0 = c; g.colp1 = d; g.C = y; g.stats = stats;
  g.lda = ldh; g.ldw = ldw; g.ldc = ldy;
  g.M = (int)M; g.N = (int)N; g.K = (int)F;
  g.nst = (int)(F / kBN);
  g.eps = eps;
  g.ws = static_cast<float*>(ws);
  row_stats_kernel<<<(unsigned)((M + 255) / 256), 256, 0, gp_stream(stream)>>>(g.stats, g.M, g.nst, eps);
  if (fmt == GP_FMT_F16) launch<kEpiLnFold, true>(g, p, gp_stream(stream));
  else launch<kEpiLnFold, false>(g, p, gp_stream(stream));
  return gp_check_launch("gp_ffn_fc2_ln");
}
