// (the implementation shared by the gp_gemm*.hip translation units: every entry point instantiates only the
// kernels of its own epilogue, so `make -j` compiles them in parallel)
#pragma once
// The slide encoder's projection GEMMs on gfx950 MFMAs, with the FFN's row passes fused into them.
//
//   gp_linear        C = A . W^T (+ bias)                               nn.Linear
//   gp_ffn_fc1_gelu  h = act(gelu(act(A . W1^T + b1))) + per-row LN statistics of h
//                    (feedforward_network.py:131-135: fc1, gelu(x.float()).type_as(x))
//   gp_ffn_fc2_ln    y = act(LayerNorm_F(h) . W2^T + b2) with the LN folded into the epilogue
//                    (feedforward_network.py:136-142: ffn_layernorm, fc2)
//
// A [M, K] and W [N, K] are both K-contiguous 16-bit (bf16, or fp16 under the caller's fp16 autocast),
// fp32 accumulation.  The FFN pair replaces hipBLASLt fc1 + gp_gelu_layernorm + hipBLASLt fc2: the
// GELU+LN pass (one read and one write of the [M, F] activation) disappears.
//
// LN fold (fc2).  With per-row mean mu and rstd s of h, gamma/beta the ffn_layernorm affine:
//   LN(h) . W2^T + b2 = s * (h . W2g^T - mu * c) + d,   W2g = W2 * gamma (column-scaled, act),
//   c[n] = sum_k W2g[n, k] (of the rounded W2g),        d[n] = sum_k W2[n, k] beta[k] + b2[n]
// -- packed once per weight version (runtime.PackedLayer).  The reference rounds LN(h) to act before
// fc2; here the rounding sits on W2g instead (one act rounding per product term either way).
//
// Statistics.  fc1's epilogue writes, for every 256-column group g of h and every row m,
// stats[g][m] = (mean, M2) of the 256 act-rounded GELU values; fc2 first merges the F/256 groups (Chan et
// al.'s pairwise update, row_stats_kernel) into plane F/256: the row's mean and 1/sqrt(biased variance +
// eps), as torch's LayerNorm computes them in fp32; its epilogue reads them from LDS, where an LDS-DMA
// issued at the tile's start has put them.
//
// GEMM structure (cdna_hip_programming.md §5, "the 256² 8-phase template"):
//   * 256 x 256 output tile per workgroup of 8 waves as 2 (M) x 4 (N); a wave owns 128 x 64 = 8 x 4
//     v_mfma_f32_16x16x32 tiles (128 fp32 accumulators per lane); BK = 64;
//   * LDS: two K-tile buffers (distinct __shared__ objects, so the compiler sees that a fragment read of
//     one never aliases the LDS-DMA in flight into the other) of [A 256 x 64 | W 256 x 64], rows of
//     128 B whose 16-byte chunk c sits at c ^ ((row >> 1) & 7): the 16 rows x 4 chunks of every
//     ds_read_b128 lane group land on 16 distinct bank slots;
//   * staging by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction, lane-linear; the
//     swizzle lives in the per-lane SOURCE address), rows past M read as zero through the descriptor;
//   * a K-tile = 4 phases, one C quadrant (4 m-frags x 2 n-frags x K 64 = 16 MFMAs) each; each phase is
//     fragment reads + DMA issue | s_barrier | 16 MFMAs at s_setprio 1 | s_barrier, and waves 4-7 run
//     one barrier behind waves 0-3: on each SIMD one wave's MFMAs overlap the other's reads and issue;
//   * persistent: one workgroup per CU walks its tiles, the next tile's first K-tiles streaming in
//     during the current tile's last phases; XCD-grouped tile order (one A row panel's N-tiles on one
//     XCD's L2); the last partial round of tiles split in K when it is at most half full (fp32
//     partials in the caller's workspace, summed by gemm_reduce_kernel with the same epilogue).
#include <limits.h>
#include <math.h>

#include <type_traits>

#include "gp_api.h"
#include "gp_common.h"
#include "gp_gelu_lut.h"

namespace {

// GP_LAB_EPI (lab builds only, tools/attn_lab `make full`; 0 in the product): timing-only ablations of the
// epilogues, results deliberately wrong -- 1: no residual x loads (x = 0), 2: no x stores, 4: no 16-bit
// output stores (xb / h / C; a plain epilogue's MFMAs are then dead code), 8: no GELU evaluation (h = the
// packed pre-activation), 16: the 16-bit output stores skipped by a run-time test (MFMAs stay live),
// 32 / 64: no W / A K-tile staging past K-tile 1 (the MFMAs read stale tiles)
#ifndef GP_LAB_EPI
#define GP_LAB_EPI 0
#endif
// GP_GEMM_GELU_EARLY_STORE (round 6, product 1): the GELU epilogue stores each m-frag's h right after computing
// it -- its stores drain under the remaining m-frags' GELU work -- instead of all 8 m-frags after the statistics
// barrier: fc1 + GELU 351 -> 315 us per 70k launch, the eager forward 31.03 -> 30.50 ms, bit-identical
// (profiles/r06_gelu_*)
#ifndef GP_GEMM_GELU_EARLY_STORE
#define GP_GEMM_GELU_EARLY_STORE 1
#endif
constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kThreads = 512;
constexpr int kRowB = kBK * 2;                // 128-byte LDS rows
constexpr int kOpT = 256 * kRowB;             // one operand's K-tile: 32 KiB
constexpr int kHalf = 128 * kRowB;            // one operand half-tile: 16 KiB

// Epilogues.  kEpiResid / kEpiLnFoldResid carry the residual add (encoder.py:141,147 / :159): the fp32
// residual stream x is read, updated and written in the epilogue, and the NEXT sub-layer's pre-LN input is
// written as xb = act(gamma_next * (x - s)) with per-256-column statistics of x - s (s = a per-row shift,
// the row mean before the add, so the 16-bit rounding sees a nearly centred row); the next GEMM folds that
// LayerNorm (kEpiLnFold = QKV, kEpiLnFoldGelu = fc1).  The residual_layernorm pass disappears.
enum { kEpiLinear = 0, kEpiGelu = 1, kEpiLnFold = 2, kEpiResid = 3, kEpiLnFoldResid = 4, kEpiLnFoldGelu = 5 };
template <int EPI>
constexpr bool epi_fold = EPI == kEpiLnFold || EPI == kEpiLnFoldResid || EPI == kEpiLnFoldGelu;
template <int EPI>
constexpr bool epi_gelu = EPI == kEpiGelu || EPI == kEpiLnFoldGelu;
template <int EPI>
constexpr bool epi_res = EPI == kEpiResid || EPI == kEpiLnFoldResid;
// per-tile column parameters LDS-DMA'd at the tile's start (g_colt): linear / GELU bias; LN fold c | d;
// residual bias | gamma; LN fold + residual c | d | gamma.  Every epilogue starts its accumulators at zero
// and applies them at the end (no N limit, no whole-N staging).
template <int EPI>
constexpr int epi_ncol = EPI == kEpiLnFoldResid ? 3 : (EPI >= kEpiLnFold ? 2 : 1);

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8g __attribute__((ext_vector_type(8)));

__shared__ __attribute__((aligned(1024))) char g_buf0[2 * kOpT];   // K-tiles 0, 2, 4, ...
__shared__ __attribute__((aligned(1024))) char g_buf1[2 * kOpT];   // K-tiles 1, 3, 5, ...
template <int B>
GP_DEV char* bufp() {
  if constexpr (B == 0) return g_buf0;
  else return g_buf1;
}
// epilogue row exchange: GELU statistics (sums, then M2) per (tile row, wave column) / LN-fold (mean, rstd)
__shared__ __attribute__((aligned(16))) float g_rsum[kBM * 4];
__shared__ __attribute__((aligned(16))) float g_rm2[kBM * 4];
// LN fold: (mean, rstd) of the tile's 256 rows, LDS-DMA'd at the tile's start, two tiles in flight
__shared__ __attribute__((aligned(1024))) float2 g_rowst[2][kBM];
// per-tile column parameters (epi_ncol vectors of the tile's 256 columns) and the residual's row shift,
// LDS-DMA'd at the tile's start like g_rowst
__shared__ __attribute__((aligned(1024))) float g_colt[2][3 * kBN];
__shared__ __attribute__((aligned(1024))) float g_shift[2][kBM];

GP_DEV int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

struct GemmArgs {
  const uint16_t* A;
  const uint16_t* W;
  const float* colp0;   // bias (linear / gelu / resid, may be null) or c (LN fold)
  const float* colp1;   // d (LN fold) or gamma_next (resid)
  const float* colp2;   // gamma_next (LN fold + resid)
  uint16_t* C;          // act output (resid: xb; may be null there -- no xb, no statistics)
  float* stats;         // LN fold input: (mean, rstd) [M] float2 at plane nst
  float* ostats;        // gelu / resid output statistics: [N/256][M] float2 (mean, M2)
  float* x;             // resid: fp32 residual stream [M, ldx], updated in place
  const float* shift;   // resid: per-row shift s [M]
  int64_t lda, ldw, ldc, ldx;
  int M, N, K;
  int nst;              // LN fold: statistics groups per row (F / 256)
  float eps;
  int vcol0 = INT_MAX;  // fp16 (kH) plain / LN-fold outputs: columns >= vcol0 are stored in bf16 instead (the
                        // V third of the fp16 caller's fused QKV, GP_FMT_F16_VBF16); INT_MAX: none
  int n_dp;             // tiles run data-parallel
  int split;            // 1: the remaining tiles are split in K (workspace ws)
  float* ws;
  // resid producers (round 5): merge the N/256 statistics planes of ostats into plane N/256 (mean, rstd with
  // mrg_eps) and write mrg_sout = shift + mean in the split-tail reduce launch -- the next LN-folding GEMM's
  // row_stats_kernel, without its launch.  Null: no merge here.
  float* mrg_sout;
  float mrg_eps;
};

template <int n>
GP_DEV void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}

// the wave's LDS writes visible to the workgroup, then a workgroup barrier (no wait on the LDS-DMA /
// global loads in flight: an LDS-only release)
GP_DEV void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  __builtin_amdgcn_sched_barrier(0);
}

template <bool kH>
GP_DEV float round_act(float v) { return e2f<kH>(f2e<kH>(v)); }

// v + v[lane ^ 16] and v + v[lane ^ 32] by v_permlane16_swap / v_permlane32_swap: VALU, no LDS round trip (the
// ds_bpermute of __shfl_xor put two dependent LDS latencies into every m-frag of the statistics epilogues).  Same
// lane pairs as __shfl_xor(v, 16 / 32) + v, and IEEE addition commutes: the same bits.
GP_DEV float add_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
GP_DEV float add_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Exact-erf GELU (torch's F.gelu default), x Phi(x) = max(x, 0) - |x|/2 erfc(|x|/sqrt 2), with erfc from
// Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7 exp(-z^2)-relative; the arithmetic of gp_norm.hip's
// gelu_erf rearranged to 13 operations with one v_rcp and one v_exp: the 1/2 folded into the polynomial)
GP_DEV float gelu_g(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(0.5307027145f, t, -0.7265760135f);
  p = fmaf(p, t, 0.7107068705f);
  p = fmaf(p, t, -0.142248368f);
  p = fmaf(p, t, 0.127414796f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f((x * -0.72134752044448170368f) * x);   // exp(-x^2 / 2)
  return fmaf(-fabsf(x) * p, e, fmaxf(x, 0.f));
}

// bf16 GELU by table (gp_gelu_lut.h): h = bf16(gelu(float(x))) is a function of x's 16 bits, so the bf16
// epilogue looks it up in LDS instead of evaluating gelu_g -- the reference's own fp32 GELU bit for bit
// (the table is torch's F.gelu) and ~11 VALU per pair of elements (packed 16-bit index arithmetic, two
// ds_read_u16) instead of ~26.  LDS copy: x = sign | m at byte 8192 sign + 2 (m - LO) -- the sign bit
// shifted right by 2 is that offset in both 16-bit halves -- the table first in LDS (largest alignment),
// so the ds_read address is the offset itself.  Halves outside [LO, HI] read a clamped entry and raise
// `bad`; gelu_fix then applies the generator-checked rules to them.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
constexpr int kLutNegB = 8192;
static_assert(2 * kGeluLutN <= kLutNegB, "");
__shared__ __attribute__((aligned(16384))) uint16_t g_lut[(kLutNegB + 2 * kGeluLutN) / 2];

GP_DEV uint32_t gelu_lut_pair(uint32_t xp, bool& bad) {
  const uint32_t m = xp & 0x7fff7fffu;
  const u16x2 t = __builtin_bit_cast(u16x2, m) - (u16x2)kGeluLutLo;   // wraps for m < LO
  const u16x2 tc = __builtin_elementwise_min(t, (u16x2)(kGeluLutN - 1));
  bad |= __builtin_bit_cast(uint32_t, tc) != __builtin_bit_cast(uint32_t, t);
  // byte offsets of both halves (2 tc < 2^12: no carry into the high half)
  const uint32_t off = (__builtin_bit_cast(uint32_t, tc) << 1) | ((xp ^ m) >> 2);
  const uint32_t lo = *reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(g_lut) + (off & 0xffff));
  const uint32_t hi = *reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(g_lut) + (off >> 16));
  return lo | (hi << 16);
}

// the halves of xp outside the table: |x| < 2^-16 -> x / 2 (half: the pair's fp32 accumulators halved and
// rounded, = bf16(x) / 2 exactly), x > HI -> x (+inf from 2^127 up, as torch's formula overflows there),
// x < -HI -> -0 (NaN for -inf / NaN)
GP_DEV uint32_t gelu_fix(uint32_t xp, uint32_t hv, uint32_t half) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t b = (xp >> (16 * j)) & 0xffff, m = b & 0x7fff;
    const uint32_t big = (b & 0x8000) ? (m >= 0x7f80 ? 0x7fc0u : 0x8000u) : (m - 0x7f00u < 0x80u ? 0x7f80u : b);
    uint32_t v = (hv >> (16 * j)) & 0xffff;
    v = m > (uint32_t)kGeluLutHi ? big : v;
    v = m < (uint32_t)kGeluLutLo ? (half >> (16 * j)) & 0xffff : v;
    r |= v << (16 * j);
  }
  return r;
}

// Chan merge of nst (mean, M2) groups of 256 values -> (mean, rstd) of the row (biased variance + eps);
// plane(g) yields group g.  ONE arithmetic for row_stats_kernel and the reduce kernel's merge below, so both
// produce the same bits.
template <class Plane>
GP_DEV float2 merge_row_stats_f(Plane plane, int nst, float eps) {
  float msum = 0.f;
  for (int g = 0; g < nst; ++g) msum += plane(g).x;
  const float mean = msum / (float)nst;
  float m2 = 0.f;
  for (int g = 0; g < nst; ++g) {
    const float2 p = plane(g);
    const float dm = p.x - mean;
    m2 += p.y + 256.f * dm * dm;
  }
  return make_float2(mean, rsqrtf(m2 / (float)(256 * nst) + eps));
}
GP_DEV float2 merge_row_stats(const float2* st, int64_t stride, int nst, float eps) {
  return merge_row_stats_f([&](int g) { return st[g * stride]; }, nst, eps);
}

// plane nst of the statistics = (mean, rstd) of each row, merged from planes 0 .. nst-1 (one thread per row).
// Residual statistics (of x - s_in): s_out = s_in + mean = the row's mean of x, the next residual
// epilogue's shift.
__global__ __launch_bounds__(256) void row_stats_kernel(float* stats, int M, int nst, float eps, const float* s_in,
                                                        float* s_out) {
  const int row = (int)blockIdx.x * 256 + (int)threadIdx.x;
  if (row >= M) return;
  float2* st = reinterpret_cast<float2*>(stats);
  const float2 r = merge_row_stats(st + row, M, nst, eps);
  st[(int64_t)nst * M + row] = r;
  if (s_out != nullptr) s_out[row] = (s_in != nullptr ? s_in[row] : 0.f) + r.x;
}

// NK = K / 64 as a template constant: the K loop is unrolled completely, so no loop header merges the
// LDS-DMA state of two paths (hipcc's wait insertion then put a vmcnt(0) before every iteration's first
// fragment read although the pending DMA targets the other buffer).
//
// Work: persistent, one workgroup per CU (G = grid).  Tiles [0, n_dp) run data-parallel: workgroup sid
// takes sid, sid + G, ...  Tiles [n_dp, ntiles) -- the last, partial round -- are split S ways in K when
// the host asks for it (n_dp a multiple of G, (ntiles - n_dp) * S <= G): unit u = sid takes tile
// n_dp + u / S, K-tiles [(u % S) NK/S, +NK/S), and writes its fp32 partial tile to the workspace.
template <int NK, int S, int EPI, bool kH, bool NT = false>
__global__ __launch_bounds__(kThreads, 1) void gemm_kernel(const GemmArgs g) {
  static_assert(NK % 2 == 0 && NK >= 2 && (S == 1 || (NK % (2 * S) == 0)), "");
  const int tiles_n = g.N / kBN;
  const int ntiles = ((g.M + kBM - 1) / kBM) * tiles_n;
  const int G = (int)gridDim.x;
  const int sid = xcd_remap((int)blockIdx.x, G);
  const int n_dp = g.n_dp;
  const int n_my = sid < n_dp ? (n_dp - 1 - sid) / G + 1 : 0;
  const bool tail = S > 1 && g.split && sid < (ntiles - n_dp) * S;
  if (n_my == 0 && !tail) return;
#ifdef GP_LAB_STAGGER
  // lab: half of each XCD's workgroups start ~GP_LAB_STAGGER x 0.25 us late (desynchronises the CUs' tile
  // boundaries, so their epilogue HBM bursts stop coinciding); GP_LAB_STAGGER_EPI: only for the fc1 (GELU)
  // and fc2 (residual) epilogues
#ifdef GP_LAB_STAGGER_EPI
  if constexpr (EPI == kEpiLnFoldGelu || EPI == kEpiLnFoldResid)
#endif
  if (((int)blockIdx.x >> 3) & 1)
    for (int z = 0; z < GP_LAB_STAGGER; ++z) __builtin_amdgcn_s_sleep(8);
#endif
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;

  constexpr bool kFold = epi_fold<EPI>, kGelu = epi_gelu<EPI>, kRes = epi_res<EPI>;
  constexpr int kNCol = epi_ncol<EPI>;
  if constexpr (kGelu && !kH) {   // the GELU table (published by run_seq's first barrier)
    static_assert(kGeluLutN % 2 == 0, "");
    for (int i = threadIdx.x; i < kGeluLutN; i += kThreads) {   // dword i: entries 2i, 2i+1
      const int half = i >= kGeluLutN / 2;
      reinterpret_cast<uint32_t*>(g_lut)[i - half * (kGeluLutN / 2) + half * (kLutNegB / 4)] =
          reinterpret_cast<const uint32_t*>(gp_gelu_lut_bf16)[i];
    }
  }

  // buffer descriptors of tile T: A rows past M read as zero (record count ends at row M)
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

  // LDS-DMA: instruction j of wave w for half h covers rows h*128 + (2w + j)*8 .. +7; lane l writes row
  // + l/8, physical chunk l%8, which holds logical chunk (l%8) ^ ((row >> 1) & 7) (the half's 128-row
  // offset leaves that XOR unchanged: it rides in the scalar offset)
  int voff[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = (2 * w + j) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    voff[0][j] = (int)((int64_t)r * g.lda * 2) + c * 16;
    voff[1][j] = (int)((int64_t)r * g.ldw * 2) + c * 16;
  }
  int hoff[2] = {(int)(128 * g.lda * 2), (int)(128 * g.ldw * 2)};
  auto issue = [&](auto opc, auto hc, auto bc, const __amdgpu_buffer_rsrc_t& rs, int kt) {
    constexpr int OP = decltype(opc)::value, H = decltype(hc)::value, B = decltype(bc)::value;
    char* dst = bufp<B>() + OP * kOpT + H * kHalf;
    if constexpr ((GP_LAB_EPI & (OP == 0 ? 64 : 32)) != 0) {   // lab: no re-staging past K-tile 1
      if (kt >= 2) return;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + (2 * w + j) * 1024),
                                               16, voff[OP][j], kt * kRowB + H * hoff[OP], 0, 0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  // fragment reads: lane (r16 = lane & 15, q = lane >> 4) reads row R0 + r16, logical chunk 4 ks + q,
  // physical (q ^ (r16 >> 1)) ^ 4 ks  (R0 a multiple of 16)
  const int r16 = lane & 15, q = lane >> 4;
  const int lo0 = r16 * kRowB + ((q ^ (r16 >> 1)) << 4);
  const int lo1 = r16 * kRowB + (((q ^ (r16 >> 1)) ^ 4) << 4);
  bf16x8 as[4][2], ws[2][2][2];     // one A m-half (8 frags), both W n-halves (16-bit patterns)
  auto read_a = [&](auto bc, auto mqc) {
    constexpr int B = decltype(bc)::value, MQ = decltype(mqc)::value;
    const char* base = bufp<B>() + (wm * 128 + MQ * 64) * kRowB;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      as[f][0] = *reinterpret_cast<const bf16x8*>(base + f * 16 * kRowB + lo0);
      as[f][1] = *reinterpret_cast<const bf16x8*>(base + f * 16 * kRowB + lo1);
    }
  };
  auto read_w = [&](auto bc, auto nqc) {
    constexpr int B = decltype(bc)::value, NQ = decltype(nqc)::value;
    const char* base = bufp<B>() + kOpT + (wn * 64 + NQ * 32) * kRowB;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      ws[NQ][f][0] = *reinterpret_cast<const bf16x8*>(base + f * 16 * kRowB + lo0);
      ws[NQ][f][1] = *reinterpret_cast<const bf16x8*>(base + f * 16 * kRowB + lo1);
    }
  };

  f32x4v acc[8][4];
  auto mfma = [](const bf16x8& a, const bf16x8& b, const f32x4v& c) -> f32x4v {
    if constexpr (kH)
      return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8g, a), __builtin_bit_cast(f16x8g, b), c,
                                                    0, 0, 0);
    else
      return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  };
  auto quadrant = [&](auto mqc, auto nqc) {
    constexpr int MQ = decltype(mqc)::value, NQ = decltype(nqc)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[MQ * 4 + f][NQ * 2 + e] = mfma(ws[NQ][e][ks], as[f][ks], acc[MQ * 4 + f][NQ * 2 + e]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((GP_LAB_EPI & 256) == 0) __builtin_amdgcn_s_barrier();   // (lab 256: no K-loop barriers)
    __builtin_amdgcn_sched_barrier(0);
  };

  // Epilogue of tile T.  Lane (r16, q) of wave (wm, wn) holds, for m-frag mi and n-frag ni, row
  // mw + 16 mi + r16 and columns nw + 16 ni + 4q .. +3 (v_mfma_f32_16x16x32 D layout with W as srcA).
  // Stores are 16 bytes (T21 with v_permlane16_swap): for each n-frag pair (2p, 2p+1) one swap per dword
  // gives lane groups q = 0 / 2 the 8 columns 8(q>>1) .. +7 of n-frag 2p and q = 1 / 3 those of n-frag
  // 2p+1; through a per-wave buffer descriptor whose record count ends at row M (rows past it are
  // dropped by the hardware), the row group in the scalar offset.
  auto epilogue_tile = [&](int i_tile, int T) {
    const int tm = T / tiles_n, tn = T % tiles_n;
    const int m0 = tm * kBM;
    const int mw = m0 + wm * 128, nw = tn * kBN + wn * 64;
    const int slot = i_tile & 1;
    const float* colt = g_colt[slot] + wn * 64 + 4 * q;   // per-tile column params: + 256 v + 16 ni
    uint32_t hp[8][4][2];            // GELU: h as packed 16-bit pairs
    const int64_t c_rows = g.M - mw < 128 ? (g.M - mw > 0 ? g.M - mw : 0) : 128;
    // (readfirstlane: wave-uniform values the compiler cannot prove uniform would put every store in a
    // waterfall loop over the descriptor)
    const uint64_t cp = reinterpret_cast<uint64_t>((g.C != nullptr ? g.C : reinterpret_cast<uint16_t*>(g.x)) + (int64_t)mw * g.ldc + nw);
    const uint64_t cpu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(cp >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)cp);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(cpu), (short)0, __builtin_amdgcn_readfirstlane((int)(c_rows * g.ldc * 2)),
        0x00020000);
    // Full-line stores: after the v_permlane16_swap below, lane (r16, q) holds for m-frag mi two 16-byte
    // column chunks of row r16 (V[0]: the wave's columns 0-31, V[1]: 32-63).  One DPP row_ror:8 per dword
    // hands rows 8-15's V[0] to lanes 0-7 and rows 0-7's V[1] to lanes 8-15 of every 16-lane row, so each
    // 16-byte store then writes 8 rows x the whole 128-byte line of the wave's 64 columns (8 lanes per
    // row) instead of 16 rows x half lines -- half-line non-temporal writes cost 1.5x the bytes in HBM
    // (PMC r03_z: QKV WRITE_SIZE 488 MB for a 322 MB output).
    const int c_lane = (int)(((r16 & 7) * g.ldc + 16 * (q & 1) + 8 * (q >> 1) + 32 * (r16 >> 3)) * 2);
    const int c_mi = (int)(16 * g.ldc * 2);
    const int c_hi = (int)(8 * g.ldc * 2);
    const bool lo8 = r16 < 8;
    // the 16-bit output of m-frag mi: pk[ni] = act pairs (columns 16 ni + 4 q .. +3 of row 16 mi + r16)
    auto store_mfrag = [&](int mi, const uint32_t (&pkin)[4][2]) {
      typedef int i32x4 __attribute__((ext_vector_type(4)));
      i32x4 V[2];
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        uint32_t pk[2][2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          pk[e][0] = pkin[2 * pr + e][0];
          pk[e][1] = pkin[2 * pr + e][1];
        }
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto r = __builtin_amdgcn_permlane16_swap(pk[0][d], pk[1][d], false, false);
          pk[0][d] = r[0];
          pk[1][d] = r[1];
        }
        V[pr] = i32x4{(int)pk[0][0], (int)pk[0][1], (int)pk[1][0], (int)pk[1][1]};
      }
      i32x4 X, Y;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int r0 = __builtin_amdgcn_update_dpp(0, V[0][d], 0x128, 0xf, 0xf, false);   // row_ror:8
        const int r1 = __builtin_amdgcn_update_dpp(0, V[1][d], 0x128, 0xf, 0xf, false);
        X[d] = lo8 ? V[0][d] : r1;   // rows 0-7
        Y[d] = lo8 ? r0 : V[1][d];   // rows 8-15
      }
      // Store-data hazard: hipcc spaces a VALU write of a store's data registers from a b128 store only
      // when soffset is not an SGPR, yet on gfx950 the store can still read such a register after the
      // next instruction has rewritten it (measured: the GELU epilogue's m-frag 1 store, 4 rows of every
      // tile wrong, timing-dependent).  Two wait states after every store, as the model
      // gives the other case.  (NT: non-temporal stores for wide, short-K outputs, see launch().)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if constexpr ((GP_LAB_EPI & 4) != 0) continue;
        if constexpr ((GP_LAB_EPI & 16) != 0) {   // stores predicated on a run-time-false test: no DCE
          if (g.K >= 0) continue;
        }
        __builtin_amdgcn_raw_buffer_store_b128(hh ? Y : X, rc, c_lane, mi * c_mi + hh * c_hi, NT ? 2 : 0);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 1");
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if constexpr (kFold) {   // s * (acc - mu c) + d.  (mean, rstd) and c | d landed during the K loop
                             // (init_tile's DMA, retired by the issuing waves' first counted waits,
                             // published by the barriers after them)
      float2 rs[8];
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) rs[mi] = g_rowst[slot][wm * 128 + mi * 16 + r16];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const float4 c = *reinterpret_cast<const float4*>(colt + ni * 16);
        const float4 d = *reinterpret_cast<const float4*>(colt + kBN + ni * 16);
        const float cc[4] = {c.x, c.y, c.z, c.w}, dd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[mi][ni][j] = fmaf(rs[mi].y, fmaf(-rs[mi].x, cc[j], acc[mi][ni][j]), dd[j]);
      }
    }
    if constexpr (EPI == kEpiLinear || EPI == kEpiGelu) {   // + bias (landed with the tile's column parameters)
      if (g.colp0 != nullptr) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const f32x4v b = *reinterpret_cast<const f32x4v*>(colt + ni * 16);
#pragma unroll
          for (int mi = 0; mi < 8; ++mi) acc[mi][ni] += b;
        }
      }
    }
    const bool has_c = !kRes || g.C != nullptr;   // resid without a next LN (last layer): x only
    if constexpr (kRes) {
      // x += acc (+ bias); xb = act(gamma * (x - s)); per-row sums of d = x - s and d^2 over the lane's 16
      // columns.  The fp32 x tile is read and written in the accumulator layout (16 B per lane and n-frag,
      // rows past M dropped / read as zero by the descriptor), two m-frags of loads in flight.
      const int64_t x_rows = g.M - mw < 128 ? (g.M - mw > 0 ? g.M - mw : 0) : 128;
      const uint64_t xp_ = reinterpret_cast<uint64_t>(g.x + (int64_t)mw * g.ldx + nw);
      const uint64_t xpu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(xp_ >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xp_);
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void*>(xpu), (short)0, __builtin_amdgcn_readfirstlane((int)(x_rows * g.ldx * 4)), 0x00020000);
      const int x_lane = (int)((r16 * g.ldx + 4 * q) * 4);
      const int x_mi = (int)(16 * g.ldx * 4);
      constexpr int vb = EPI == kEpiLnFoldResid ? -1 : 0;   // bias vector (resid only)
      constexpr int vg = EPI == kEpiLnFoldResid ? 2 : 1;    // gamma_next vector
      const bool has_bias = vb >= 0 && g.colp0 != nullptr;
      f32x4v xv[2][4];
      auto load_x = [&](int mi) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          if constexpr ((GP_LAB_EPI & 1) != 0) xv[mi & 1][ni] = f32x4v{0.f, 0.f, 0.f, 0.f};
          else xv[mi & 1][ni] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rx, x_lane, mi * x_mi + ni * 64, 0));
        }
      };
      load_x(0);
      load_x(1);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const float sh = g_shift[slot][wm * 128 + mi * 16 + r16];
        float s = 0.f, s2 = 0.f;
        uint32_t hq[4][2];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          // (bias / gamma re-read from LDS per m-frag: held in registers they cost 32 VGPRs across the loop)
          f32x4v yv = acc[mi][ni];
          if constexpr (vb >= 0) {
            if (has_bias) yv += *reinterpret_cast<const f32x4v*>(colt + vb * kBN + ni * 16);
          }
          const f32x4v v = xv[mi & 1][ni] + yv;   // the reference's order: x + (y + b), y kept in fp32
          typedef int i32x4 __attribute__((ext_vector_type(4)));
          if constexpr ((GP_LAB_EPI & 2) == 0) {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rx, x_lane, mi * x_mi + ni * 64, 0);
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_nop 1");   // the store-data hazard (see the C stores below)
            __builtin_amdgcn_sched_barrier(0);
          }
          const f32x4v dv = v - sh;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            s += dv[j];
            s2 = fmaf(dv[j], dv[j], s2);
          }
          const f32x4v gv = dv * *reinterpret_cast<const f32x4v*>(colt + vg * kBN + ni * 16);
          hq[ni][0] = pack2e<kH>(gv[0], gv[1]);
          hq[ni][1] = pack2e<kH>(gv[2], gv[3]);
        }
        if (has_c) store_mfrag(mi, hq);   // xb of this m-frag (nothing of it stays live)
        if (mi + 2 < 8) load_x(mi + 2);
        s = add_xor32(add_xor16(s));
        s2 = add_xor32(add_xor16(s2));
        if (q == 0) {
          g_rsum[(wm * 128 + mi * 16 + r16) * 4 + wn] = s;
          g_rm2[(wm * 128 + mi * 16 + r16) * 4 + wn] = s2;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (has_c) {
        lds_barrier();
        if (threadIdx.x < kBM) {
          const int row = m0 + (int)threadIdx.x;
          if (row < g.M) {
            const float4 s4 = *reinterpret_cast<const float4*>(g_rsum + threadIdx.x * 4);
            const float4 q4 = *reinterpret_cast<const float4*>(g_rm2 + threadIdx.x * 4);
            const float sum = (s4.x + s4.y) + (s4.z + s4.w), sq = (q4.x + q4.y) + (q4.z + q4.w);
            const float mean = sum * (1.f / 256.f);
            reinterpret_cast<float2*>(g.ostats)[(int64_t)tn * g.M + row] = make_float2(mean, fmaxf(fmaf(-sum, mean, sq), 0.f));
          }
        }
      }
    }
    if constexpr (kGelu) {
      // GELU (of the biased / LN-folded accumulators) and the row sums of h and h^2 over the lane's
      // 16 columns, one m-frag at a time (the GELU temporaries of only one are live); h is kept as
      // packed 16-bit pairs (64 registers: an m-frag's accumulators die as it is converted).  Per tile
      // and row, M2 = sum h^2 - (sum h)^2 / 256 over 256 bounded activation values: the fp32
      // cancellation is ~1e-7 * (1 + mean^2 / var), far below the act rounding of h itself.
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        float s = 0.f, s2 = 0.f;
        if constexpr (!kH) {   // bf16: table lookup, sums by v_dot2 (exact bf16 products, fp32 adds)
          uint32_t xp[4][2];
          bool bad = false;
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              xp[ni][e] = pack2e<false>(acc[mi][ni][2 * e], acc[mi][ni][2 * e + 1]);
              if constexpr ((GP_LAB_EPI & 8) != 0) hp[mi][ni][e] = xp[ni][e];
              else hp[mi][ni][e] = gelu_lut_pair(xp[ni][e], bad);
            }
          if (__builtin_amdgcn_ballot_w64(bad) != 0) {   // a |x| < 2^-16 or > 5.53 in this m-frag (rare)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
#pragma unroll
              for (int e = 0; e < 2; ++e)
                hp[mi][ni][e] = gelu_fix(xp[ni][e], hp[mi][ni][e],
                                         pack2e<false>(acc[mi][ni][2 * e] * 0.5f, acc[mi][ni][2 * e + 1] * 0.5f));
          }
          typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
          const bf16x2v one2 = __builtin_bit_cast(bf16x2v, 0x3f803f80u);
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const bf16x2v hv = __builtin_bit_cast(bf16x2v, hp[mi][ni][e]);
              s = __builtin_amdgcn_fdot2_f32_bf16(hv, one2, s, false);
              s2 = __builtin_amdgcn_fdot2_f32_bf16(hv, hv, s2, false);
            }
        } else {
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const uint32_t xp = pack2e<kH>(acc[mi][ni][2 * e], acc[mi][ni][2 * e + 1]);
              hp[mi][ni][e] = pack2e<kH>(gelu_g(e2f<kH>(xp)), gelu_g(e2f_hi<kH>(xp)));
              const float h0 = e2f<kH>(hp[mi][ni][e]), h1 = e2f_hi<kH>(hp[mi][ni][e]);
              s += h0 + h1;
              s2 = fmaf(h0, h0, fmaf(h1, h1, s2));
            }
          }
        }
        s = add_xor32(add_xor16(s));
        s2 = add_xor32(add_xor16(s2));
        if (q == 0) {
          g_rsum[(wm * 128 + mi * 16 + r16) * 4 + wn] = s;
          g_rm2[(wm * 128 + mi * 16 + r16) * 4 + wn] = s2;
        }
        if constexpr (GP_GEMM_GELU_EARLY_STORE != 0) store_mfrag(mi, hp[mi]);
        __builtin_amdgcn_sched_barrier(0);
      }
      lds_barrier();
      if (threadIdx.x < kBM) {
        const int row = m0 + (int)threadIdx.x;
        if (row < g.M) {
          const float4 s4 = *reinterpret_cast<const float4*>(g_rsum + threadIdx.x * 4);
          const float4 q4 = *reinterpret_cast<const float4*>(g_rm2 + threadIdx.x * 4);
          const float sum = (s4.x + s4.y) + (s4.z + s4.w), sq = (q4.x + q4.y) + (q4.z + q4.w);
          const float mean = sum * (1.f / 256.f);
          reinterpret_cast<float2*>(g.ostats)[(int64_t)tn * g.M + row] = make_float2(mean, fmaxf(fmaf(-sum, mean, sq), 0.f));
        }
      }
    }
    if constexpr (kRes) return;   // (xb stored per m-frag above)
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      if constexpr (kGelu) {
        if constexpr (GP_GEMM_GELU_EARLY_STORE == 0) store_mfrag(mi, hp[mi]);
      } else {
        uint32_t pk[4][2];
        if (kH && tn * kBN >= g.vcol0) {   // (wave-uniform) the bf16 V columns of an fp16 QKV
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
            pk[ni][0] = pack2e<false>(acc[mi][ni][0], acc[mi][ni][1]);
            pk[ni][1] = pack2e<false>(acc[mi][ni][2], acc[mi][ni][3]);
          }
        } else {
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
            pk[ni][0] = pack2e<kH>(acc[mi][ni][0], acc[mi][ni][1]);
            pk[ni][1] = pack2e<kH>(acc[mi][ni][2], acc[mi][ni][3]);
          }
        }
        store_mfrag(mi, pk);
      }
    }
  };
  // the VMEM instructions EVERY wave issues in epilogue_tile: 8 m-frags x 2 stores (waves 0-3 of the GELU
  // epilogue add a statistics store, wave 0 of the LN fold two LDS-DMA pieces in init_tile: a wait
  // counted with the minimum is only stricter for them)
  // (resid: 32 x stores + 16 xb stores, the x loads interleaved with them already consumed; a count below the
  // true one only makes the next tile's first wait stricter)
  constexpr int kEpiVmem = kRes ? 48 : 16;
  // VMEM instructions EVERY wave issues in init_tile (the per-tile parameters' LDS-DMA pieces, padded with
  // stores through an empty descriptor): one compile-time count, so K-tile 0's counted wait can leave them
  // and the previous epilogue's stores in flight (uncounted, they made that wait drain the first stores)
  constexpr int kInitVmem = 2;
  // accumulators start at zero (the epilogue applies the bias / the LN fold)
  auto zero_acc = [&]() {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4v{0.f, 0.f, 0.f, 0.f};
  };
  // (the column offset of a workgroup's tiles changes from tile to tile unless G % tiles_n == 0, so the
  // bias is read per tile from LDS: 4 ds_read_b128 per lane)
  auto init_tile = [&](int i_tile, int T) {
    {
      zero_acc();
      const int m0 = (T / tiles_n) * kBM, n0 = (T % tiles_n) * kBN;
      const int slot = i_tile & 1;
      int issued = 0;   // (wave-uniform)
      // LN fold: (mean, rstd) of the tile's 256 rows -> g_rowst[slot]: 2 KiB, two 1-KiB LDS-DMA pieces of
      // wave 0 (lane l: rows 2l, 2l+1 of the piece); rows past M read as zero
      if constexpr (kFold) {
        if (w == 0) {
          const int64_t nb = (int64_t)(g.M - m0) * 8;
          const __amdgpu_buffer_rsrc_t rs_ = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(reinterpret_cast<const float2*>(g.stats) + (int64_t)g.nst * g.M + m0), (short)0,
              (int)(nb < 2048 ? nb : 2048), 0x00020000);
#pragma unroll
          for (int j = 0; j < 2; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs_, (__attribute__((address_space(3))) void*)((char*)g_rowst[slot] + j * 1024), 16, lane * 16,
                j * 1024, 0, 0);
          issued = 2;
        }
      }
      // column vector v (the tile's 256 columns, 1 KiB) by wave 1 + v; a null vector (no bias, no next LN)
      // loads nothing
      if (w >= 1 && w <= kNCol) {
        const float* src = w == 1 ? g.colp0 : (w == 2 ? g.colp1 : g.colp2);
        if (src != nullptr) {
          const __amdgpu_buffer_rsrc_t rc_ = __builtin_amdgcn_make_buffer_rsrc((void*)(src + n0), (short)0, 1024,
                                                                              0x00020000);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rc_, (__attribute__((address_space(3))) void*)(g_colt[slot] + (w - 1) * kBN), 16, lane * 16, 0, 0, 0);
          issued = 1;
        }
      }
      // residual: the row shift s of the tile's 256 rows (wave 7; none without a next LN: no xb, no
      // statistics, and the shift may be null)
      if constexpr (kRes) {
        if (w == 7 && g.shift != nullptr) {
          const int64_t nb = (int64_t)(g.M - m0) * 4;
          const __amdgpu_buffer_rsrc_t rh_ = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(g.shift + m0), (short)0, (int)(nb < 1024 ? nb : 1024), 0x00020000);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rh_, (__attribute__((address_space(3))) void*)(g_shift[slot]), 16,
                                                   lane * 16, 0, 0, 0);
          issued = 1;
        }
      }
      const __amdgpu_buffer_rsrc_t none_ = __builtin_amdgcn_make_buffer_rsrc(g.ws, (short)0, 0, 0x00020000);
#pragma unroll
      for (int j = 0; j < kInitVmem; ++j)
        if (j >= issued) __builtin_amdgcn_raw_buffer_store_b32(0, none_, 0, 0, 0);
    }
  };

  // fp32 partial of split unit u: [256][256] floats at ws + u * 65536, lane's 4 columns as one 16-B store
  auto store_partial = [&](int u) {
    float* base = g.ws + (int64_t)u * (kBM * kBN);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int row = wm * 128 + mi * 16 + r16, col = wn * 64 + ni * 16 + 4 * q;
        *reinterpret_cast<f32x4v*>(base + row * kBN + col) = acc[mi][ni];
      }
  };

  // One sequence of `count` tiles of nk K-tiles each (K-tiles kt0 .. kt0 + nk - 1), tile_of(i) giving
  // the i-th; the DMA of tile i+1's first K-tiles runs during tile i's last phases.
  auto run_seq = [&](auto nkc, int count, int kt0, auto&& tile_of, auto&& epilogue, auto&& init_acc) {
    constexpr int nk = decltype(nkc)::value;
    __amdgpu_buffer_rsrc_t ra = rsrc_a(tile_of(0)), rw = rsrc_w(tile_of(0));
    bool has_next = false;
    int i_cur = 0;
    // stage half H of operand OP of the tile-local K-tile vv (vv >= nk: the next tile's K-tile vv - nk)
    auto stage = [&](auto opc, auto hc, auto bc, int vv) {
      constexpr int OP = decltype(opc)::value;
      // (unconditional: past the last tile the descriptors still name the current one and the pieces
      // re-load consumed K-tiles -- a DMA issued on one path only made hipcc put a vmcnt(0) before
      // later LDS reads)
      issue(opc, hc, bc, OP == 0 ? ra : rw, kt0 + (vv < nk ? vv : vv - nk));
    };
    // one K-tile v of the current output tile, in buffer B (v even: B = 0).  Phases (quadrant; fragments
    // read; DMA issued): Q0 (m0, n0; A m-half 0 + W n-half 0; A half 0 of K-tile v+1), Q1 (m0, n1; W
    // n-half 1; A half 1 of v+1), Q2 (m1, n1; A m-half 1; none), Q3 (m1, n0; none; both W halves of
    // v+2).  A halves are last read in Q2, W halves in Q1, so every restage comes >= 2 phases after the
    // last read of its buffer half; one counted vmcnt(4) in Q3 retires all of K-tile v+1, which is read
    // one phase later (the weights of K-tile v+2 stay in flight: 4 phases of lead)
    auto ktile = [&](auto bc, int v) {
      constexpr int B = decltype(bc)::value;
      using BN_ = std::integral_constant<int, 1 - B>;
      const bool pre = v == 0;   // K-tile 1's A halves are already in flight (see the tile loop)
      read_a(bc, I0());
      read_w(bc, I0());
      if (!pre) stage(I0(), I0(), BN_(), v + 1);   // (pre: compile-time after the unroll)
      sync();
      quadrant(I0(), I0());
      sync();
      read_w(bc, I1());
      if (!pre) stage(I0(), I1(), BN_(), v + 1);
      sync();
      quadrant(I0(), I1());
      sync();
      read_a(bc, I1());
      sync();
      quadrant(I1(), I1());
      sync();
      if (v + 2 == nk) {   // every DMA of this tile is issued: switch to the next tile's (if any)
        const int Tn = tile_of(has_next ? i_cur + 1 : i_cur);
        ra = rsrc_a(Tn);
        rw = rsrc_w(Tn);
      }
      stage(I1(), I0(), bc, v + 2);
      stage(I1(), I1(), bc, v + 2);
      // retire K-tile v+1 (the weights of v+2 stay in flight); at v = 0 K-tile 1's A halves are older
      // than the previous tile's epilogue stores (or the prologue's stand-ins), which may stay in flight
      if (pre) wait_vmcnt<4 + kEpiVmem + kInitVmem>();
      else wait_vmcnt<4>();
      sync();
      quadrant(I1(), I0());
      sync();
    };
    // prologue: K-tile 0 whole, K-tile 1 whole, then kEpiVmem stores through an empty descriptor
    // (dropped by the hardware) standing in for an epilogue's: every tile then starts in the same
    // VMEM state, and K-tile 0's counted wait is one compile-time constant
    issue(I0(), I0(), I0(), ra, kt0);
    issue(I0(), I1(), I0(), ra, kt0);
    issue(I1(), I0(), I0(), rw, kt0);
    issue(I1(), I1(), I0(), rw, kt0);
    issue(I1(), I0(), I1(), rw, kt0 + 1);
    issue(I1(), I1(), I1(), rw, kt0 + 1);
    issue(I0(), I0(), I1(), ra, kt0 + 1);
    issue(I0(), I1(), I1(), ra, kt0 + 1);
    {
      const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(g.ws, (short)0, 0, 0x00020000);
#pragma unroll
      for (int j = 0; j < kEpiVmem; ++j) __builtin_amdgcn_raw_buffer_store_b32(0, none, 0, 0, 0);
    }
    wait_vmcnt<8 + kEpiVmem>();     // K-tile 0 landed
    lds_barrier();                  // (also publishes the column parameters)
    for (int i = 0; i < count; ++i) {
      has_next = i + 1 < count;
      i_cur = i;
      // opaque per tile: the DMA scalar offsets derived from these are then computed where they are used
      // instead of being hoisted out of the tile loop (~100 loop-invariant SGPRs for K = 3072 -> spills)
      asm volatile("" : "+s"(hoff[0]), "+s"(hoff[1]));
      init_acc(i, tile_of(i));
      if (wm == 1) sync();          // waves 4-7 one barrier behind
#pragma unroll
      for (int v = 0; v < nk; v += 2) {
        ktile(I0(), v);
        ktile(I1(), v + 1);
      }
      if (wm == 0) sync();          // realign
      // The next tile's K-tile 1 A halves go out BEFORE this tile's stores.  vmcnt counts stores too and
      // retires in order, so a wait for a load issued after the stores waits for the stores; issued
      // before them, the next tile's first wait (K-tile 0's Q3) can leave the stores in flight, and they
      // drain behind a whole K-tile of MFMAs instead of stalling it.  (Buffer 1's A halves were last read
      // in this tile's last Q2; every wave is past its last MFMA here.)
      issue(I0(), I0(), I1(), ra, kt0 + 1);
      issue(I0(), I1(), I1(), ra, kt0 + 1);
      epilogue(i);
    }
    wait_vmcnt<0>();   // no LDS-DMA in flight past the sequence (LDS reuse, hand-off)
  };

  if (n_my > 0)
    run_seq(std::integral_constant<int, NK>(), n_my, 0, [&](int i) { return sid + i * G; },
            [&](int i) { epilogue_tile(i, sid + i * G); }, [&](int i, int T) { init_tile(i, T); });
  if constexpr (S > 1) {
    if (tail) {
      constexpr int NKS = NK / S;
      if (n_my > 0) sync();         // every wave done reading the last data-parallel tile's buffers
      const int T = n_dp + sid / S, part = sid % S;
      run_seq(std::integral_constant<int, NKS>(), 1, part * NKS, [&](int) { return T; },
              [&](int) { store_partial(sid); }, [&](int, int) { zero_acc(); });
    }
  }
}

// Split tail: sum of the S fp32 partials of each tail tile, then the tile epilogue (linear, LN fold,
// residual) -> act C.  One thread per 8 columns of a row: a row's 256 tile columns are 32 consecutive lanes,
// so the residual statistics reduce by shuffles (the GELU epilogue is never split).
template <int EPI, bool kH>
__global__ __launch_bounds__(256) void gemm_reduce_kernel(const GemmArgs g, int S) {
  static_assert(!epi_gelu<EPI>, "");
  constexpr bool kFold = epi_fold<EPI>, kRes = epi_res<EPI>;
  const int tiles_n = g.N / kBN;
  const int unit = blockIdx.x / (kBM * kBN / 8 / 256);          // tail tile ordinal
  const int idx = (blockIdx.x % (kBM * kBN / 8 / 256)) * 256 + threadIdx.x;
  const int row = idx / (kBN / 8), col = (idx % (kBN / 8)) * 8;
  const int T = g.n_dp + unit;
  const int tn = T % tiles_n;
  const int m = (T / tiles_n) * kBM + row, n = tn * kBN + col;
  if (m >= g.M) return;   // (all 32 lanes of a row together)
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const float* p = g.ws + (int64_t)(unit * S + s) * (kBM * kBN) + row * kBN + col;
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
  if constexpr (kFold) {
    const float2 mr = reinterpret_cast<const float2*>(g.stats)[(int64_t)g.nst * g.M + m];
    for (int e = 0; e < 8; ++e) v[e] = fmaf(mr.y, fmaf(-mr.x, g.colp0[n + e], v[e]), g.colp1[n + e]);
  } else {
    if (g.colp0 != nullptr)
      for (int e = 0; e < 8; ++e) v[e] += g.colp0[n + e];
  }
  if constexpr (kRes) {
    float* xr = g.x + (int64_t)m * g.ldx + n;
    const float4 a = *reinterpret_cast<const float4*>(xr), b = *reinterpret_cast<const float4*>(xr + 4);
    const float xo[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    for (int e = 0; e < 8; ++e) v[e] = xo[e] + v[e];
    *reinterpret_cast<float4*>(xr) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(xr + 4) = make_float4(v[4], v[5], v[6], v[7]);
    if (g.C == nullptr) return;
    const float* gam = EPI == kEpiLnFoldResid ? g.colp2 : g.colp1;
    const float sh = g.shift[m];
    float s = 0.f, s2 = 0.f;
    for (int e = 0; e < 8; ++e) {
      const float d = v[e] - sh;
      s += d;
      s2 = fmaf(d, d, s2);
      v[e] = d * gam[n + e];
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      s += __shfl_xor(s, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    if (col == 0) {
      const float mean = s * (1.f / 256.f);
      reinterpret_cast<float2*>(g.ostats)[(int64_t)tn * g.M + m] = make_float2(mean, fmaxf(fmaf(-s, mean, s2), 0.f));
    }
  }
  uint4 o;
  if (kH && !kRes && n >= g.vcol0) {   // the bf16 V columns of an fp16 QKV (see GemmArgs::vcol0)
    o.x = pack2e<false>(v[0], v[1]);
    o.y = pack2e<false>(v[2], v[3]);
    o.z = pack2e<false>(v[4], v[5]);
    o.w = pack2e<false>(v[6], v[7]);
  } else {
    o.x = pack2e<kH>(v[0], v[1]);
    o.y = pack2e<kH>(v[2], v[3]);
    o.z = pack2e<kH>(v[4], v[5]);
    o.w = pack2e<kH>(v[6], v[7]);
  }
  *reinterpret_cast<uint4*>(g.C + (int64_t)m * g.ldc + n) = o;
}

// Split tail of a residual producer that also merges the next LayerNorm's statistics (g.mrg_sout, round 5).
// Blocks [0, nmb): the rows of the row panels whose tiles all ran data-parallel (their planes are final: the
// GEMM kernel completed before this launch), one thread per row as row_stats_kernel.  Blocks [nmb, nmb +
// 32 * tail panels): 8 rows of one tail panel each, through every tail tile of that panel in turn -- the
// split sum and residual epilogue of gemm_reduce_kernel, same thread layout -- keeping the rows' per-tile
// (mean, M2) in LDS, then merging them with the panel's data-parallel tiles' planes in plane order: the
// values and the arithmetic of row_stats_kernel, so plane N/256 and mrg_sout come out bit-identical to the
// separate launch this replaces.  No block depends on another (no atomics, no flags).
constexpr int kMaxTilesN = 8;   // N / 256 of the residual producers (E = 768 / 1024 / 1536)
template <int EPI, bool kH>
__global__ __launch_bounds__(256) void gemm_reduce_merge_kernel(const GemmArgs g, int S, int nmb) {
  static_assert(epi_res<EPI>, "");
  constexpr bool kFold = epi_fold<EPI>;
  const int tiles_n = g.N / kBN;
  float2* st = reinterpret_cast<float2*>(g.ostats);
  const int p0 = g.n_dp / tiles_n;               // first panel with a tail tile
  if ((int)blockIdx.x < nmb) {
    const int m = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (m >= p0 * kBM || m >= g.M) return;
    const float2 r = merge_row_stats(st + m, g.M, tiles_n, g.mrg_eps);
    st[(int64_t)tiles_n * g.M + m] = r;
    g.mrg_sout[m] = g.shift[m] + r.x;
    return;
  }
  __shared__ float2 pst[kMaxTilesN][8];
  const int b = (int)blockIdx.x - nmb;
  const int pnl = p0 + b / 32, rg = b % 32;
  const int row = rg * 8 + (int)threadIdx.x / 32, col = ((int)threadIdx.x % 32) * 8;
  const int m = pnl * kBM + row;
  const float* gam = EPI == kEpiLnFoldResid ? g.colp2 : g.colp1;
  for (int tn = 0; tn < tiles_n; ++tn) {
    const int T = pnl * tiles_n + tn;
    if (T < g.n_dp || m >= g.M) continue;        // (data-parallel tile / rows past M: all 32 lanes of a row)
    const int unit = T - g.n_dp, n = tn * kBN + col;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) {
      const float* pp = g.ws + (int64_t)(unit * S + s) * (kBM * kBN) + row * kBN + col;
      const float4 a = *reinterpret_cast<const float4*>(pp), c = *reinterpret_cast<const float4*>(pp + 4);
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += c.x; v[5] += c.y; v[6] += c.z; v[7] += c.w;
    }
    if constexpr (kFold) {
      const float2 mr = reinterpret_cast<const float2*>(g.stats)[(int64_t)g.nst * g.M + m];
      for (int e = 0; e < 8; ++e) v[e] = fmaf(mr.y, fmaf(-mr.x, g.colp0[n + e], v[e]), g.colp1[n + e]);
    } else {
      if (g.colp0 != nullptr)
        for (int e = 0; e < 8; ++e) v[e] += g.colp0[n + e];
    }
    float* xr = g.x + (int64_t)m * g.ldx + n;
    const float4 a = *reinterpret_cast<const float4*>(xr), c = *reinterpret_cast<const float4*>(xr + 4);
    const float xo[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
    for (int e = 0; e < 8; ++e) v[e] = xo[e] + v[e];
    *reinterpret_cast<float4*>(xr) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(xr + 4) = make_float4(v[4], v[5], v[6], v[7]);
    const float sh = g.shift[m];
    float s = 0.f, s2 = 0.f;
    for (int e = 0; e < 8; ++e) {
      const float d = v[e] - sh;
      s += d;
      s2 = fmaf(d, d, s2);
      v[e] = d * gam[n + e];
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      s += __shfl_xor(s, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    if (col == 0) {
      const float mean = s * (1.f / 256.f);
      const float2 ms = make_float2(mean, fmaxf(fmaf(-s, mean, s2), 0.f));
      st[(int64_t)tn * g.M + m] = ms;
      pst[tn][row % 8] = ms;
    }
    uint4 o;
    o.x = pack2e<kH>(v[0], v[1]);
    o.y = pack2e<kH>(v[2], v[3]);
    o.z = pack2e<kH>(v[4], v[5]);
    o.w = pack2e<kH>(v[6], v[7]);
    *reinterpret_cast<uint4*>(g.C + (int64_t)m * g.ldc + n) = o;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    const int r8 = (int)threadIdx.x, mm = pnl * kBM + rg * 8 + r8;
    if (mm < g.M) {
      const float2 r = merge_row_stats_f(
          [&](int tn) { return pnl * tiles_n + tn < g.n_dp ? st[(int64_t)tn * g.M + mm] : pst[tn][r8]; }, tiles_n,
          g.mrg_eps);
      st[(int64_t)tiles_n * g.M + mm] = r;
      g.mrg_sout[mm] = g.shift[mm] + r.x;
    }
  }
}

// ----------------------------------------------------------------------------------------------------
// host side
int device_cus() {                 // per-device cache of the CU count (one persistent workgroup per CU)
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
  int G;          // persistent workgroups
  int S;          // K split of the tail round (1: none)
  int n_dp;       // data-parallel tiles
  int64_t rem;    // tail tiles
  int64_t ws_bytes;
};

#ifndef GP_GEMM_SPLIT_SHORT
#define GP_GEMM_SPLIT_SHORT 2
#endif
#ifndef GP_GEMM_SPLIT_LONG
#define GP_GEMM_SPLIT_LONG 4
#endif
// K-split factor of the tail round for a K loop of nk K-tiles: ONE definition, used by make_plan and by
// launch's kernel choice (round 4 had two, and a plan whose split the launched kernel did not share left
// its tail tiles uncomputed: DESIGN §10, "r04_y")
constexpr int split_for_nk(int nk) { return nk == 12 ? GP_GEMM_SPLIT_SHORT : (nk == 48 ? GP_GEMM_SPLIT_LONG : 4); }

// the last partial round split in K when it is at most half full (S = 4, or 2 for K = 768)
Plan make_plan(int64_t M, int64_t N, int64_t K, bool allow_split) {
  Plan p;
  const int64_t tiles = ((M + kBM - 1) / kBM) * (N / kBN);
  const int cus = device_cus();
  p.G = (int)(tiles < cus ? tiles : cus);
  p.S = 1;
  p.n_dp = (int)tiles;
  p.rem = 0;
  p.ws_bytes = 0;
  const int S = split_for_nk((int)(K / kBK));
  const int64_t rem = tiles % p.G;
  if (allow_split && S > 1 && tiles > p.G && rem > 0 && rem * S <= p.G && rem * 2 <= p.G) {
    p.S = S;
    p.n_dp = (int)(tiles - rem);
    p.rem = rem;
    p.ws_bytes = rem * S * kBM * kBN * (int64_t)sizeof(float);
  }
  return p;
}

// K of the slide encoder's three registered archs (slide_encoder.py:261-270): E in {768, 1024, 1536},
// F = 4E, patch in_chans 1536; one fully unrolled K loop (NK = K / 64) each
bool gemm_k_supported(int64_t K) {
  return K == 768 || K == 1024 || K == 1536 || K == 3072 || K == 4096 || K == 6144;
}

int check_shapes(const char* who, const void* A, int64_t lda, const void* W, int64_t ldw, const void* C, int64_t ldc,
                 int64_t M, int64_t N, int64_t K, int fmt, bool qkv_fmt_ok = false) {
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16 || (qkv_fmt_ok && fmt == GP_FMT_F16_VBF16), "%s: bad fmt %d", who,
             fmt);
  GP_REQUIRE(fmt != GP_FMT_F16_VBF16 || (N % 3 == 0 && (2 * N / 3) % kBN == 0),
             "%s: fmt F16_VBF16 needs a fused [q | k | v] output, N = 3E with 2E a multiple of %d (N=%lld)", who, kBN,
             (long long)N);
  GP_REQUIRE(A && W && C, "%s: null pointer", who);
  GP_REQUIRE(M > 0 && M < (int64_t)0x7fffffff && N > 0 && K > 0, "%s: bad sizes", who);
  GP_REQUIRE(N % kBN == 0, "%s: N=%lld must be a multiple of %d", who, (long long)N, kBN);
  GP_REQUIRE(gemm_k_supported(K), "%s: K=%lld not instantiated (768 / 1024 / 1536 / 3072 / 4096 / 6144)", who,
             (long long)K);
  GP_REQUIRE(lda >= K && ldw >= K && ldc >= N && lda % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0,
             "%s: bad leading dimensions", who);
  GP_REQUIRE(gp_aligned(A, 16) && gp_aligned(W, 16) && gp_aligned(C, 16), "%s: misaligned operand", who);
  GP_REQUIRE((int64_t)kBM * lda * 2 < 0x7fffffff && (int64_t)kBN * ldw * 2 < 0x7fffffff &&
                 (int64_t)128 * ldc * 2 < 0x7fffffff,
             "%s: leading dimension too large for 32-bit tile offsets", who);
  return 0;
}

// K instantiations per epilogue: the projections of E-wide inputs (QKV, out-proj, fc1: K = E) and of the
// F-wide FFN hidden (fc2: K = F = 4E) -- one translation unit per entry-point pair keeps the build parallel
enum { kKE = 1, kKF = 2 };
template <int EPI, bool kH, int KSET>
int launch(GemmArgs g, const Plan& p, hipStream_t s) {
  g.n_dp = p.n_dp;
  g.split = p.S > 1;
  // Output stores: every CU finishes a tile at about the same moment, so each round of tiles writes
  // G x 128 KiB at once (a whole XCD's L2 per round).  For wide, short-K outputs (QKV 2304 x 768, fc1
  // 3072 x 768) non-temporal stores drain that burst faster: -14 % per launch; for N = 768 or K = 3072
  // they are 4-10 % slower (r03_w probe).
#ifndef GP_NT_MIN_N
#define GP_NT_MIN_N 2048   // (lab builds probe other thresholds)
#endif
  const bool nt = g.N >= GP_NT_MIN_N && g.K <= 1536;
  const dim3 grid((unsigned)p.G), block(kThreads);
  constexpr bool kSplit = !epi_gelu<EPI>;   // (the GELU plan never splits)
  // nt only for the epilogues whose output is a plain wide activation (QKV / fc1 / their LN-fold forms)
  constexpr bool kNtOk = !epi_res<EPI> && EPI != kEpiLnFoldResid;
  // The plan must be one the launched kernel computes completely: unsplit (every tile data-parallel), or
  // split by exactly the factor the kernel instantiation carries for this K -- a tail outside the
  // data-parallel range with no matching split kernel would be skipped silently (round 4's r04_y failure).
  const int64_t ntiles = ((int64_t)(g.M + kBM - 1) / kBM) * (g.N / kBN);
  GP_REQUIRE(p.S == 1 ? (p.rem == 0 && p.n_dp == ntiles)
                      : (kSplit && g.K % kBK == 0 && p.S == split_for_nk(g.K / kBK) && p.rem > 0 &&
                         p.n_dp + p.rem == ntiles && p.rem * p.S <= p.G && p.n_dp % p.G == 0),
             "GEMM epilogue %d: inconsistent tile plan (S=%d, n_dp=%d, rem=%lld, tiles=%lld, K=%d)", EPI, p.S, p.n_dp,
             (long long)p.rem, (long long)ntiles, g.K);
  auto go = [&](auto nkc, auto ntc) {
    constexpr int NKc = decltype(nkc)::value;
    constexpr bool NTc = decltype(ntc)::value && kNtOk;
    constexpr int Sc = split_for_nk(NKc);
    if constexpr (kSplit && Sc > 1) {
      if (p.S > 1) {   // (== Sc: checked above)
        gemm_kernel<NKc, Sc, EPI, kH, NTc><<<grid, block, 0, s>>>(g);
        return;
      }
    }
    gemm_kernel<NKc, 1, EPI, kH, NTc><<<grid, block, 0, s>>>(g);
  };
  auto go_nt = [&](auto nkc) {
    if (nt) go(nkc, std::true_type());
    else go(nkc, std::false_type());
  };
  bool done = false;
  if constexpr ((KSET & kKE) != 0) {
    done = true;
    switch (g.K) {
      case 768: go_nt(std::integral_constant<int, 12>()); break;
      case 1024: go_nt(std::integral_constant<int, 16>()); break;
      case 1536: go_nt(std::integral_constant<int, 24>()); break;
      default: done = false;
    }
  }
  if constexpr ((KSET & kKF) != 0) {
    if (!done) {
      done = true;
      switch (g.K) {
        case 3072: go(std::integral_constant<int, 48>(), std::false_type()); break;
        case 4096: go(std::integral_constant<int, 64>(), std::false_type()); break;
        case 6144: go(std::integral_constant<int, 96>(), std::false_type()); break;
        default: done = false;
      }
    }
  }
  GP_REQUIRE(done, "GEMM epilogue %d: K=%d not instantiated (K = E in {768, 1024, 1536} or F = 4E)", EPI, g.K);
  if constexpr (kSplit) {
    if constexpr (epi_res<EPI>) {
      if (p.S > 1 && g.mrg_sout != nullptr) {   // the tail's reduce + the next LN's statistics merge (see above)
        const int tiles_n = g.N / kBN;
        const int64_t ntile = ((int64_t)(g.M + kBM - 1) / kBM) * tiles_n;
        const int p0 = p.n_dp / tiles_n, pend = (int)((ntile + tiles_n - 1) / tiles_n);
        GP_REQUIRE(tiles_n <= kMaxTilesN && g.C != nullptr, "GEMM epilogue %d: bad statistics merge", EPI);
        const int nmb = (int)(((int64_t)p0 * kBM + 255) / 256);
        gemm_reduce_merge_kernel<EPI, kH><<<(unsigned)(nmb + 32 * (pend - p0)), 256, 0, s>>>(g, p.S, nmb);
        return 0;
      }
    }
    if (p.S > 1) gemm_reduce_kernel<EPI, kH><<<(unsigned)(p.rem * (kBM * kBN / 8 / 256)), 256, 0, s>>>(g, p.S);
  }
  return 0;
}


// the LN fold's inputs: nst statistics planes of M (mean, M2) pairs + the merged plane; c, d [N] fp32
int check_fold(const char* who, const float* stats, int64_t nst, const float* c, const float* d, int64_t N) {
  GP_REQUIRE(stats && c && d && gp_aligned(stats, 8) && gp_aligned(c, 16) && gp_aligned(d, 16),
             "%s: null or misaligned stats / c / d", who);
  GP_REQUIRE(nst >= 1 && nst <= 64, "%s: bad statistics group count %lld", who, (long long)nst);
  (void)N;
  return 0;
}
// the residual epilogue's operands: x [M, ldx] fp32, shift [M], gamma [N], xb [M, ldxb] act, xstats [N/256][M]
int check_resid(const char* who, const float* x, int64_t ldx, const float* shift, const float* gamma,
                const uint16_t* xb, int64_t ldxb, const float* xstats, int64_t N) {
  GP_REQUIRE(x && gp_aligned(x, 16) && ldx >= N && ldx % 4 == 0 && (int64_t)128 * ldx * 4 < 0x7fffffff,
             "%s: null, misaligned or badly strided x", who);
  if (gamma != nullptr) {
    GP_REQUIRE(shift && gp_aligned(shift, 16) && gp_aligned(gamma, 16), "%s: null or misaligned shift / gamma", who);
    GP_REQUIRE(xb && gp_aligned(xb, 16) && ldxb >= N && ldxb % 8 == 0 && (int64_t)128 * ldxb * 2 < 0x7fffffff,
               "%s: null, misaligned or badly strided xb", who);
    GP_REQUIRE(xstats && gp_aligned(xstats, 8), "%s: null or misaligned xstats", who);
  }
  return 0;
}
void launch_row_stats(float* stats, int64_t M, int nst, float eps, const float* s_in, float* s_out, hipStream_t s) {
  row_stats_kernel<<<(unsigned)((M + 255) / 256), 256, 0, s>>>(stats, (int)M, nst, eps, s_in, s_out);
}

}  // namespace
