// Dilated attention for gfx950: sparsify (gather), per-segment flash attention with MFMA,
// and the LSE-weighted branch merge.  Replaces DilatedAttention.gathering / flash_attn_func /
// scattering (torchscale/component/dilated_attention.py:16-131, flash_attention.py:13-16).
//
// Attention kernel design (one launch covers every branch of a layer):
//   * work item = (branch, batch*segment, head, q-block of NW*32 rows); items ordered heaviest
//     branch first (LPT) and regrouped so that 8 consecutive q-blocks of one (segment, head)
//     run on one XCD and share its L2 for K/V;
//   * NW waves x 32 query rows (8 for the LDS-DMA kernels, 4 for the register-staged kModeGen);
//     K/V tiles of 64 keys staged in LDS, double buffered (one barrier per tile).  The dilated
//     gather is folded into the addressing: sparse row i of (segment n, head h) is token
//     n*s + i*r + h/(Hp/r);
//   * D = 48 / 64 (v2 kernel, dilated_attn32_kernel): S^T = K.Q^T and O^T += V^T.P^T with
//     v_mfma_f32_32x32x16_bf16; D = 96 (dilated_attn_kernel): v_mfma_f32_16x16x32_bf16;
//   * the reference's zero-padded keys (dilated_attention.py:85-91, unmasked in flash-attn)
//     are added analytically at the end: n_pad * exp(0 - max) in the denominator.
// Every launch configuration is fixed at compile time (no run-time variant switches); measured
// alternatives live in tools/attn_lab/ (a separate build target).
#include <math.h>
#include <type_traits>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "gp_api.h"
#include "gp_common.h"

namespace {

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// 16-bit element format of q / k / v / o: kH = false is bf16 (BASELINE's dtype), kH = true is fp16
// (the forward and the operator seam under the reference pipeline's fp16 autocast,
// pipeline.py:186-187, whose flash-attn computes in fp16).  Operands travel as raw 16-bit containers
// (bf16x8); only the MFMA opcode, the P rounding and the output rounding depend on the format.
template <bool kH>
GP_DEV f32x16 mfma_32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  if constexpr (kH)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <bool kH>
GP_DEV f32x4 mfma_16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (kH)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <bool kH>
GP_DEV __bf16 f2e_slot(float f) { return __builtin_bit_cast(__bf16, f2e<kH>(f)); }
// Exact unsigned division by a launch constant d < 2^31 via a multiply-high: the merge kernel's
// per-token divisions are wave-uniform, so they run on the scalar unit instead of ~25 VALU
// instructions each.  With m = floor(2^32 (2^l - d) / d) + 1, l = ceil(log2 d), the quotient is
// (mulhi(n, m) + n) >> l for every n < 2^31 (mulhi(n, m) < n, so the sum cannot wrap); d == 1 is
// m = 0, l = 0 -- no branch, so a chain of divisions does not split the scalar argument loads
// into one wait per division.
struct DivMagic {
  uint32_t m;
  int32_t l;     // 0: d == 1
};
inline DivMagic make_div_magic(uint32_t d) {
  DivMagic r{0, 0};
  if (d <= 1) return r;
  int l = 0;
  while ((1ull << l) < d) ++l;                                   // ceil(log2 d)
  r.m = (uint32_t)(((((uint64_t)1 << l) - d) << 32) / d + 1);
  r.l = l;
  return r;
}
GP_DEV uint32_t div_magic(uint32_t n, DivMagic mg) {   // n < 2^31
  return (__umulhi(n, mg.m) + n) >> mg.l;
}


struct AttnBranch {
  GpBranch g;
  int32_t nqb;          // q-blocks per (batch-segment, head)
  int32_t n_lo;         // first segment whose dense slots meet the query window
  int32_t nseg_w;       // segments meeting the window
  int32_t kv_sparse;    // 0: head h at columns h*D of a k/v row; 1: at (h % hpg)*D (sparsified rows)
  int64_t item_begin;   // first work item of this branch
  const uint16_t* k;    // key rows: token t of batch b at row (b*L + t - kv_tok_base)
  const uint16_t* v;
  int64_t kv_stride;    // elements between consecutive k / v rows
  int64_t kv_tok_base;
  uint16_t* o;          // [B*nseg, m, H, D]
  float* lse;           // [B*nseg, H, m]
  int32_t kpart, kparts;   // key part kpart of kparts (<= 1: all keys; see GpAttnBranch.key_parts)
  // varlen table entries only (one per (slide, branch); B = 1, window = the whole slide)
  const uint16_t* q;    // the slide's first query row
  int64_t L;            // the slide's length (CLS + tiles)
  DivMagic d_nqb, d_nsegw, d_hpg, d_r;   // the work-item decode's divisors (scalar multiply-high)
};
inline void attn_branch_magic(AttnBranch& e) {
  e.d_nqb = make_div_magic((uint32_t)e.nqb);
  e.d_nsegw = make_div_magic((uint32_t)e.nseg_w);
  e.d_hpg = make_div_magic((uint32_t)e.g.hpg);
  e.d_r = make_div_magic((uint32_t)e.g.r);
}

struct AttnArgs {
  const uint16_t* q;    // query rows: token t of batch b at row (b*L + t - q_tok_base)
  int64_t q_stride;
  int64_t q_tok_base;
  int64_t L;
  int64_t win_lo, win_hi;   // dense-slot window of every batch: rows the merge reads there
  int32_t H;
  int32_t nbranch;
  float c_log2;         // softmax_scale * log2(e)
  int64_t total_items;
  AttnBranch br[GP_MAX_BRANCHES];   // work order (heaviest first)
  const AttnBranch* tab;            // varlen: ntab (slide, branch) entries in device memory
  int32_t ntab;
  DivMagic d_H;
};

// Work item -> (branch, batch, segment, head, query-row range).  Rows [i_lo, i_hi) of
// (segment n, head group j) are those whose sparse_to_dense slot n*g + i*r + j lies in the
// window (dilated_attention.py:33-53 places sparse row i of head group j at that slot).
struct WorkItem {
  int bi, bn, bidx, n, hh, j, c, i_lo, i_hi, qb;
};

GP_DEV int ceil_div_pos(int64_t a, int r) { return a > 0 ? (int)((a + r - 1) / r) : 0; }

// The decode's divisions are wave-uniform: multiply-high by host-computed magic numbers (32-bit
// operands: every quantity here is below 2^31) instead of VALU integer-division emulation.
GP_DEV void decode_core(const AttnBranch& br, int local, int H, DivMagic dH, int64_t L, int64_t win_lo,
                        int64_t win_hi, WorkItem& w) {
  const GpBranch& g = br.g;
  const int q1 = (int)div_magic((uint32_t)local, br.d_nqb);
  w.qb = local - q1 * br.nqb;
  const int bnw = (int)div_magic((uint32_t)q1, dH);
  w.hh = q1 - bnw * H;
  w.bidx = (int)div_magic((uint32_t)bnw, br.d_nsegw);
  w.n = br.n_lo + (bnw - w.bidx * br.nseg_w);
  w.bn = w.bidx * g.nseg + w.n;
  w.j = (int)div_magic((uint32_t)w.hh, br.d_hpg);
  const int rem = (int)(L - (int64_t)w.n * g.s);
  const int lim = (rem < g.s ? rem : g.s) - w.j;
  w.c = lim > 0 ? (int)div_magic((uint32_t)(lim + g.r - 1), br.d_r) : 0;
  const int base = w.n * g.g + w.j;
  const int alo = (int)(win_lo - base), ahi = (int)(win_hi - base);
  w.i_lo = alo > 0 ? (int)div_magic((uint32_t)(alo + g.r - 1), br.d_r) : 0;
  const int hi = ahi > 0 ? (int)div_magic((uint32_t)(ahi + g.r - 1), br.d_r) : 0;
  w.i_hi = hi < g.m ? hi : g.m;
}

GP_DEV void decode_item(const AttnArgs& a, int item, WorkItem& w) {
  int bi = 0;
#pragma unroll
  for (int t = 1; t < GP_MAX_BRANCHES; ++t)
    if (t < a.nbranch && item >= (int)a.br[t].item_begin) bi = t;
  w.bi = bi;
  decode_core(a.br[bi], item - (int)a.br[bi].item_begin, a.H, a.d_H, a.L, a.win_lo, a.win_hi, w);
}

// Varlen (packed slides): entry = (slide, branch), items ordered by entry (heaviest first);
// binary search on item_begin (wave-uniform), then the B = 1, whole-slide decode.
GP_DEV void decode_item_tab(const AttnArgs& a, int item, WorkItem& w, AttnBranch& e) {
  int lo = 0, hi = a.ntab - 1;
  while (lo < hi) {                    // last entry with item_begin <= item
    const int mid = (lo + hi + 1) >> 1;
    if ((int64_t)item >= a.tab[mid].item_begin) lo = mid; else hi = mid - 1;
  }
  // the entry by scalar loads (uniform index, constant address space) instead of flat loads into VGPRs
  lo = __builtin_amdgcn_readfirstlane(lo);
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(sizeof(AttnBranch) % 4 == 0, "");
  uint32_t words[sizeof(AttnBranch) / 4];
  const __attribute__((address_space(4))) uint32_t* src =
      (const __attribute__((address_space(4))) uint32_t*)(uintptr_t)(a.tab + lo);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(AttnBranch) / 4); ++i) words[i] = src[i];
  __builtin_memcpy(&e, words, sizeof(AttnBranch));
#else
  e = a.tab[lo];
#endif
  w.bi = lo;
  decode_core(e, item - (int)e.item_begin, a.H, a.d_H, e.L, 0, e.L, w);
}

constexpr int kWaves = 4;
constexpr int kQT = 2;                       // 16-row q-tiles per wave
constexpr int kQB = kWaves * kQT * 16;       // 128 query rows per workgroup
constexpr int kKB = 64;                      // keys per K/V tile

// Blocks b, b+8, b+16, ... share an XCD (round-robin dispatch).  Within each chunk of 8*G blocks
// give the blocks of one XCD G consecutive work items (q-blocks of one segment and head), so they
// read the same K/V rows from that XCD's L2.  G is a compile-time tunable (tools/attn_lab).
#ifndef GP_ATTN_XCDG
#define GP_ATTN_XCDG 8
#endif
// GP_ATTN_WIDE_STORE: the epilogue pairs the two half-waves' 4-element groups with
// v_permlane32_swap so every lane stores 16 contiguous bytes (3 stores instead of 6 per row)
#ifndef GP_ATTN_WIDE_STORE
#define GP_ATTN_WIDE_STORE 1
#endif
GP_DEV int64_t xcd_group(int64_t bid, int64_t nb) {
  constexpr int64_t G = GP_ATTN_XCDG, C = 8 * G;
  const int64_t full = nb - nb % C;
  if (bid >= full) return bid;
  const int64_t base = bid - bid % C;
  const int64_t in = bid % C;
  return base + (in & 7) * G + (in >> 3);
}

template <int D, bool kH = false>
__global__ __launch_bounds__(256, 2) void dilated_attn_kernel(const AttnArgs a) {
  constexpr int KS = (D + 31) / 32;          // 32-deep k-steps of Q.K (zero-padded d)
  constexpr int DT = D / 16;                 // 16-wide d tiles of P.V
  constexpr int ROWB = D * 2;                // LDS bytes per K/V row
  constexpr int TILEB = kKB * ROWB;
  constexpr int CH = D / 8;                  // 16-byte chunks per row
  constexpr int LPT = 2 * kKB * CH / 256;    // K+V chunks per thread per tile
  static_assert((2 * kKB * CH) % 256 == 0, "tile must split evenly over 256 threads");
  // [K0 | V0 | K1 | V1] + slack: the zero-weight d>=D lanes of the last K row read into V.
  __shared__ __attribute__((aligned(16))) char smem[4 * TILEB + 64];

  WorkItem wi;
  decode_item(a, (int)xcd_group(blockIdx.x, gridDim.x), wi);
  const GpBranch g = a.br[wi.bi].g;
  const int hh = wi.hh, j = wi.j, c = wi.c;
  const int64_t bn = wi.bn;
  const int q0 = wi.i_lo + wi.qb * kQB;
  const int rows_needed = wi.i_hi;
  if (q0 >= rows_needed) return;
  // q rows past the window are neither computed nor (in a shard) resident: load only real rows
  // of the window (rows >= c are the reference's zero-padded queries)
  const int qvalid = c < rows_needed ? c : rows_needed;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l16 = lane & 15, g4 = lane >> 4;
  const AttnBranch& brr = a.br[wi.bi];
  const int64_t tok0 = (int64_t)wi.bidx * a.L + (int64_t)wi.n * g.s + j;     // token of sparse row 0
  const int64_t qstride = (int64_t)g.r * a.q_stride;                        // elements between sparse rows
  const int64_t kvstride = (int64_t)g.r * brr.kv_stride;
  const int kcol = brr.kv_sparse ? (hh % g.hpg) * D : hh * D;
  const uint16_t* qbase = a.q + (tok0 - a.q_tok_base) * a.q_stride + hh * D;
  const uint16_t* kbase = brr.k + (tok0 - brr.kv_tok_base) * brr.kv_stride + kcol;
  const uint16_t* vbase = brr.v + (tok0 - brr.kv_tok_base) * brr.kv_stride + kcol;

  // ---- Q fragments (B operand of S^T = K.Q^T): lane holds Q[row l16][d = 32ks + 8g4 .. +7]
  bf16x8 qf[kQT][KS];
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    const int i = q0 + w * 32 + qt * 16 + l16;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = ks * 32 + g4 * 8;
      bf16x8 z = {};
      if (i < qvalid && d0 < D) z = *reinterpret_cast<const bf16x8*>(qbase + (int64_t)i * qstride + d0);
      qf[qt][ks] = z;
    }
  }

  // ---- K/V tile staging (global -> registers -> LDS), chunk u of this thread
  uint4 stage[LPT];
  auto load_tile = [&](int kv0) {
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int idx = threadIdx.x + 256 * u;
      const int tsel = idx / (kKB * CH);
      const int rem = idx % (kKB * CH);
      const int row = rem / CH, ch = rem % CH;
      const int key = kv0 + row;
      uint4 z = make_uint4(0, 0, 0, 0);
      if (key < c) z = *reinterpret_cast<const uint4*>((tsel ? vbase : kbase) + (int64_t)key * kvstride + ch * 8);
      stage[u] = z;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int idx = threadIdx.x + 256 * u;
      const int tsel = idx / (kKB * CH);
      const int rem = idx % (kKB * CH);
      const int row = rem / CH, ch = rem % CH;
      *reinterpret_cast<uint4*>(smem + (2 * buf + tsel) * TILEB + row * ROWB + ch * 16) = stage[u];
    }
  };

  float m_run[kQT], l_run[kQT];
  f32x4 oacc[kQT][DT];
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    m_run[qt] = -INFINITY;
    l_run[qt] = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) oacc[qt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int ntiles = (c + kKB - 1) / kKB;
  if (ntiles > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int kv0 = t * kKB;
    if (t + 1 < ntiles) load_tile(kv0 + kKB);
    const char* Kb = smem + (2 * (t & 1)) * TILEB;
    const char* Vb = Kb + TILEB;

    // S^T[key][q] for 4 key sub-tiles of 16: lane holds keys 16kt + 4g4 + reg of query l16
    f32x4 sacc[kQT][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      bf16x8 kf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        kf[ks] = *reinterpret_cast<const bf16x8*>(Kb + (kt * 16 + l16) * ROWB + ks * 64 + g4 * 16);
#pragma unroll
      for (int qt = 0; qt < kQT; ++qt) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acc = mfma_16x16x32<kH>(kf[ks], qf[qt][ks], acc);
        sacc[qt][kt] = acc;
      }
    }
    if (kv0 + kKB > c) {   // last partial tile: keys >= c are zero pads, handled analytically
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kv0 + kt * 16 + g4 * 4 + r >= c)
#pragma unroll
            for (int qt = 0; qt < kQT; ++qt) sacc[qt][kt][r] = -INFINITY;
    }

    // online softmax (log2 domain), one query per lane; 4 lanes (g4) share a query
    bf16x8 pf[kQT][2];
#pragma unroll
    for (int qt = 0; qt < kQT; ++qt) {
      float mx = sacc[qt][0][0];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sacc[qt][kt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m_run[qt], mx * a.c_log2);
      const float alpha = exp2f(m_run[qt] - mnew);
      m_run[qt] = mnew;
      float ps = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(fmaf(sacc[qt][kt][r], a.c_log2, -mnew));
          sacc[qt][kt][r] = p;
          ps += p;
        }
      l_run[qt] = l_run[qt] * alpha + ps;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) oacc[qt][dt] *= alpha;
      // B operand of O^T += V^T.P^T: element e<4 = key 32u+4g4+e, e>=4 = key 32u+16+4g4+e-4
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pf[qt][u][e] = f2e_slot<kH>(sacc[qt][2 * u][e]);
          pf[qt][u][4 + e] = f2e_slot<kH>(sacc[qt][2 * u + 1][e]);
        }
    }

    // O^T[d][q] += V^T[d][key] . P^T[key][q]; V^T fragment by transposed LDS reads
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const char* base = Vb + (32 * u + 4 * g4 + (l16 >> 2)) * ROWB + (16 * dt + 4 * (l16 & 3)) * 2;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 16 * ROWB));
        const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int qt = 0; qt < kQT; ++qt)
          oacc[qt][dt] = mfma_16x16x32<kH>(vf, pf[qt][u], oacc[qt][dt]);
      }
    }

    if (t + 1 < ntiles) store_tile((t + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: analytic zero-pad keys, normalise, store O rows and LSE
  const int npad = g.m - c;
  const AttnBranch& br = a.br[wi.bi];
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    float l = l_run[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    float mr = m_run[qt];
    float so = 1.f;
    if (npad > 0) {
      const float mf = fmaxf(mr, 0.f);
      so = exp2f(mr - mf);
      l = l * so + (float)npad * exp2f(-mf);
      mr = mf;
    }
    const float inv = so / l;
    const int i = q0 + w * 32 + qt * 16 + l16;
    if (i < rows_needed) {
      uint16_t* orow = br.o + ((bn * g.m + i) * a.H + hh) * (int64_t)D;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        float vv[4] = {oacc[qt][dt][0] * inv, oacc[qt][dt][1] * inv, oacc[qt][dt][2] * inv, oacc[qt][dt][3] * inv};
        store_e<kH, 4>(orow + 16 * dt + 4 * g4, vv);
      }
      if (g4 == 0) br.lse[(bn * a.H + hh) * (int64_t)g.m + i] = (mr + log2f(l)) * 0.69314718055994530942f;
    }
  }
}

// ---------------------------------------------------------------------------------------
// v2: 32x32x16 MFMA formulation (D in {48, 64}).
//   * S^T[32 keys][32 q] = K.Q^T in D/16 k-steps of v_mfma_f32_32x32x16_bf16 (no d padding);
//     a lane owns 16 scores of ONE query per 32-key sub-tile, so the row max needs one
//     v_permlane32_swap per tile and no LDS traffic;
//   * O^T[d][q] += V^T[d][key] . P^T[key][q], P^T taken straight from the S^T accumulator
//     registers (k-step s = registers 8s..8s+7), V^T from two ds_read_b64_tr_b16 per k-step;
//     the d-tile is 64 rows: for D = 48 rows 48..63 read a constant block of bf16 ones that the
//     V image carries, so the MFMA also produces the softmax row sum (no VALU adds);
//   * lazy rescale (defer-max): O is rescaled only when a query's running max grows by more
//     than 2^8 (log2 domain), so P stays <= 256 (exact in fp32 sums, bf16 relative precision);
//   * V image: 128-byte rows of four 32-byte blocks, block b of row r stored at b ^ (r & 3),
//     which makes the transposed reads bank-conflict free; K image: 16-byte row padding
//     (112 / 144-byte rows) makes the 32-row ds_read_b128 fragment reads conflict free.
GP_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// lse bit pattern (a quiet NaN no real row produces) that flags a row for the fixup pass
constexpr uint32_t kLseRedo = 0x7fc0dead;

// Builds of the v2 kernel (NW waves x 32 queries per workgroup -- 8 for the LDS-DMA modes, 4 for kModeGen --
// sharing each 64-key K/V tile, one barrier per tile):
//   kModeFast (D = 48, q pre-scaled by D^-0.5*log2 e; the product launch): K/V tiles staged by
//     LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction, lane-linear) straight into the
//     padded K image and the swizzled V image through a per-tile buffer descriptor whose record
//     count ends at the last valid key row (rows past c read as zero in hardware); tile loop
//     unrolled by two so each tile's LDS buffer is a compile-time constant; NO row max and NO
//     offset: S starts from C = 0 and p = exp2(s).  Valid while a row's real-key sum l stays in
//     [2^-100, 2^100]; outside it (or not finite) the row's lse gets the kLseRedo marker;
//   kModeFix: the exact kernel run right after kModeFast on the same stream (the fixup pass):
//     kFixItems work items per block, the block reads the lse of every row of all of them and
//     exits unless one holds the marker, else recomputes the flagged items with a running row
//     max (tile 0 sets it exactly; lazy rescale when a row's max grows by > kThr log2 units),
//     the -m start block of S from one extra MFMA of an exact hi + lo bf16 pair;
//   kModeGen (D = 48 / 64, q pre-scaled or not): the same exact arithmetic with register-staged
//     K/V tiles (global loads, addresses computed once), for k / v layouts the descriptor cannot
//     cover (the operator seam's separate q / k / v tensors) and for D = 64.
//   kModeExact (D = 48, q pre-scaled): the LDS-DMA staging and work decomposition of kModeFast with the
//     exact running-max arithmetic, the -m start as the accumulator's initial value: fp16 q / k / v
//     (GP_FMT_F16; the reference pipeline's fp16 caller when its V is fp16).
// kH (fp16 operands) with kModeFast / kModeFix: the fp16 caller's product pair (GP_FMT_F16_VBF16): q and k
//   fp16, S = K.Q^T on the fp16 MFMA, but V bf16 (the QKV GEMM writes the V third of qkv in bf16) so P
//   and P.V are bf16 exactly as in the bf16 kernel -- the no-max p = 2^s needs bf16's range (fp16's ends at
//   2^16), and the exact fp16 kernel's running max costs ~15 % of the launch.
enum AttnMode { kModeFast = 0, kModeFix = 1, kModeGen = 2, kModeExact = 3 };
// work items per fixup-pass block: the block reads the lse rows of kFixItems consecutive (LPT-ordered)
// items and recomputes the flagged ones in turn.  4 (round 3): no-flag cost 1.2506 ms per 70k launch
// (fast + fixup) vs 1.2548 with 32 and 1.2652 with 1 (profiles/r03_g_ab_fixup_items.json); with sharp
// attention the flagged items run nearly in parallel: 0.3 % flagged rows 2.69 ms, 96 % 3.19 ms, vs 7.2 /
// 8.1 ms with round 2's 32 items per block, whose blocks ran up to 32 long items serially
// (profiles/r03_g_flag_rate_bf16_fixup_items.json).  1 = one block per item.
#ifndef GP_ATTN_FIX_ITEMS
#define GP_ATTN_FIX_ITEMS 4
#endif
constexpr int kFixItems = GP_ATTN_FIX_ITEMS;

// Waves per workgroup of the LDS-DMA kernels (each wave 32 queries; the K/V tile is shared by all):
// a compile-time tunable (tools/attn_lab); the register-staged kernel always runs 4 waves.
#ifndef GP_ATTN_NW
#define GP_ATTN_NW 8
#endif
constexpr int kNWFast = GP_ATTN_NW;
// GP_ATTN_PRIO: the second-dispatched half of the workgroup's waves (w >= NW/2, the arbitration
// losers of each SIMD pair) runs at s_setprio 1 for the whole kernel (MI355X_MICROARCH.md §Two waves
// per SIMD, item 4)
#ifndef GP_ATTN_PRIO
#define GP_ATTN_PRIO 1
#endif
// the fast kernel at three workgroups per CU (GP_ATTN_FAST_WPS, round 5): no static priority -- with six
// waves per SIMD arbitration by age alone measured 1.1-1.8 % faster (profiles/r05_occ6b_*, r05_occ6c_*)
#ifndef GP_ATTN_PRIO_FAST
#define GP_ATTN_PRIO_FAST 0
#endif
static_assert(kNWFast == 4 || kNWFast == 8 || kNWFast == 16, "GP_ATTN_NW must be 4, 8 or 16");
#ifndef GP_ATTN_SKIP_IDLE
#define GP_ATTN_SKIP_IDLE 1
#endif
// GP_ATTN_ONES_SPARSE: the V image's spare d-block carries 1.0 only in the two rows the epilogue reads
// (d = 48 and 52) and 0 elsewhere: same outputs, fewer toggling MFMA operand bits (same-box A/B
// 1.276 -> 1.262 ms per 70k layer, profiles/r02_s6_ab_ones.json)
#ifndef GP_ATTN_ONES_SPARSE
#define GP_ATTN_ONES_SPARSE 1
#endif
// fp16 formats of the LDS-DMA launch: GP_FMT_F16 (v fp16) runs kModeExact, the exact running-max kernel
// (lazy rescale), no fixup pass; GP_FMT_F16_VBF16 (v bf16: the fp16 caller's fused QKV, round 5) runs the
// bf16 product pair with fp16 S (kModeFast + kModeFix with kH).  Round 2's fp16 fast mode (p = 2^(s - m0),
// m0 = tile 0's max, in fp16) is gone: with sharp attention its overflowing rows made it 2.6-4.6x slower
// than the exact kernel (profiles/r03_b_fp16_flag_rate.json); P in bf16 has no such overflow.
// GP_ATTN_NOFIX (lab only) skips the fixup pass, so flagged rows keep the kLseRedo marker for the count.
#ifndef GP_ATTN_NOFIX
#define GP_ATTN_NOFIX 0
#endif
// GP_ATTN_FAST_WPS (round 5): waves per SIMD the fast kernel's registers are sized for -- 6 = three 8-wave
// workgroups per CU (<= 80 VGPRs, LDS 3 x 30 KiB), which needs the one-sub-tile-at-a-time order of its tile
// body (S, exps and P.V of keys 0-31, then of keys 32-63: half the live S / P registers of the interleaved
// order).  Against round 4's two workgroups per CU with both sub-tiles' S first: the new order at four waves
// per SIMD is 6 % slower, at six 1.2-2.3 % faster per 70k launch (fp16 V-bf16 pair 1.5 %), bit-identical
// (profiles/r05_occ6*_attn_ab_*.json, r05_occ6h_forward_ab_product_vs_r4order.json); the interleaved order
// squeezed into 80 VGPRs spills 25 registers inside the loop (1.6x slower).  4 = round 4's kernel.
#ifndef GP_ATTN_FAST_WPS
#define GP_ATTN_FAST_WPS 6
#endif
// the same for the packed (varlen, work-table) fast kernel: 6 since its table entry comes by scalar loads
// (decode_item_tab); with the entry in VGPRs the 80-register budget spilled 12 and the C5 launch ran 7 % slower
// (profiles/r05_occ6v_varlen_ab.json); with scalar loads 10.61 vs 11.00 ms per C5 launch, bit-identical
// (profiles/r05_tab6_varlen_ab.json)
#ifndef GP_ATTN_FAST_WPS_TAB
#define GP_ATTN_FAST_WPS_TAB 6
#endif
// minimum waves per SIMD the kernel instantiation is sized for (HIP launch-bounds semantics; 2: no register
// constraint at these sizes -- the fixup / exact / register-staged kernels, 104-138 VGPRs)
// (the 4-wave fast kernel of under-filled launches keeps the interleaved body, no register cap)
template <int MODE, bool kTab, int NW>
constexpr int attn_wps() { return MODE == 0 && NW == 8 ? (kTab ? GP_ATTN_FAST_WPS_TAB : GP_ATTN_FAST_WPS) : 2; }
// Measured lab variants of this kernel (the 16x16x32 P.V GP_ATTN_PV16, the 3-slot ring GP_ATTN_RING3) build
// from round 3's source in git (make -C tools/attn_lab r3lab).

template <int D, bool kPre, int MODE, bool kTab, int NW, bool kH, bool kParts = false>
__device__ __forceinline__ void attn32_item(const AttnArgs& a, const int item_idx) {
  static_assert(!kH || D == 48 || MODE == kModeGen, "fp16 LDS-DMA modes: D = 48");
  static_assert(!kParts || (MODE != kModeGen && !kTab), "key parts: LDS-DMA modes, branch launches");
  static_assert(D == 48 || D == 64, "v2 kernel covers D = 48 and 64");
  static_assert(MODE == kModeGen || (D == 48 && kPre), "LDS-DMA modes need D = 48 and a pre-scaled q");
  static_assert(NW == 4 || ((NW == 8 || NW == 16) && MODE != kModeGen), "8 / 16 waves: LDS-DMA modes only");
  constexpr int NT = NW * 64;
  constexpr int QB = NW * 32;                // query rows per workgroup
  constexpr int KT = 64;                     // keys per staged tile
  constexpr int KS = D / 16;                 // k-steps of Q.K^T
  constexpr bool kOnes = (D % 32) != 0;      // spare d rows carry the row-sum ones
  constexpr bool kDMA = MODE != kModeGen;
  constexpr bool kZM = MODE == kModeFast;          // no max, no offset (P in bf16 for both formats)
  constexpr bool kFlag = MODE == kModeFast;        // flag rows for the fixup pass
  constexpr bool kMI = MODE == kModeFix;           // -m start block from one MFMA (bf16 hi + lo pair)
  // format of V, P and the P.V MFMA: fp16 only for the exact / register-staged fp16 kernels; the fp16
  // caller's fast / fixup pair reads a bf16 V (GP_FMT_F16_VBF16)
  constexpr bool kVH = kH && (MODE == kModeExact || MODE == kModeGen);
  constexpr int KROWB = D * 2 + 16;          // K image row bytes (padded)
  constexpr int VROWB = 128;                 // V image row bytes (64 bf16, swizzled 32-B blocks)
  constexpr int KTILE = KT * KROWB;
  constexpr int VTILE = KT * VROWB;
  constexpr int BUF = KTILE + VTILE;
  constexpr int CH = D / 8;                  // 16-byte chunks per K/V row in HBM
  constexpr int TOT = 2 * KT * CH;           // 16-byte chunks of one K tile + one V tile
  constexpr int LPT = (MODE == kModeGen) ? TOT / NT : 1;
  static_assert(MODE != kModeGen || TOT % NT == 0, "");
  constexpr float kThr = 8.0f;               // lazy-rescale threshold (log2 units)
  constexpr int NBUF = 2;                    // K/V tile buffers (double-buffered)
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF];
  auto bufc = [&](auto bc) -> char* {        // tile buffer B (compile time)
    return smem + decltype(bc)::value * BUF;
  };
  using IB0 = std::integral_constant<int, 0>;

  // ---- work item (32-bit index math: items < 2^31, checked on the host)
  WorkItem wi;
  AttnBranch te;                             // kTab: this item's table entry
  if constexpr (kTab) decode_item_tab(a, item_idx, wi, te);
  else decode_item(a, item_idx, wi);
  const AttnBranch& brr = kTab ? te : a.br[wi.bi];
  const GpBranch g = brr.g;
  const int hh = wi.hh, c = wi.c, bn = wi.bn;
  const int rows_needed = wi.i_hi;
  const int q0 = wi.i_lo + wi.qb * QB;
  if (q0 >= rows_needed) return;
  // rows >= c are zero-padded queries (their q is 0): load nothing for them
  const int qvalid = c < rows_needed ? c : rows_needed;
  if constexpr (MODE == kModeFix) {          // only blocks the fast kernel flagged are recomputed
    const int i = q0 + (int)threadIdx.x;
    bool flagged = false;
    if (threadIdx.x < QB && i < rows_needed)
      flagged = __float_as_uint(brr.lse[((int64_t)wi.bn * a.H + wi.hh) * g.m + i]) == kLseRedo;
    if (!__syncthreads_or(flagged)) return;
  }
  // kModeFix rewrites ONLY the rows the fast kernel flagged (each query's own lse still holds the
  // marker here: only this block writes it), so an unflagged row keeps the fast kernel's bits whatever
  // items share its fixup block -- a packed (varlen) slide's rows never depend on a neighbour's overflow
  bool fixrow = true;
  if constexpr (MODE == kModeFix) {
    const int iq = q0 + (int)(threadIdx.x >> 6) * 32 + (int)(threadIdx.x & 31);
    fixrow = iq < rows_needed &&
             __float_as_uint(brr.lse[((int64_t)wi.bn * a.H + wi.hh) * g.m + iq]) == kLseRedo;
  }

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int64_t tok0 = (int64_t)wi.bidx * a.L + (int64_t)wi.n * g.s + wi.j;
  const int64_t qstride = (int64_t)g.r * a.q_stride;
  const int64_t kvstride = (int64_t)g.r * brr.kv_stride;
  const int kcol = brr.kv_sparse ? (hh % g.hpg) * D : hh * D;
  const uint16_t* qbase = kTab ? brr.q + tok0 * a.q_stride + hh * D
                               : a.q + (tok0 - a.q_tok_base) * a.q_stride + hh * D;
  const uint16_t* kbase = brr.k + (tok0 - brr.kv_tok_base) * brr.kv_stride + kcol;
  const uint16_t* vbase = brr.v + (tok0 - brr.kv_tok_base) * brr.kv_stride + kcol;

  // V images: the d-columns >= D of every row (block 3 for D = 48) hold bf16 1.0
  // (GP_ATTN_ONES_SPARSE: only d = 48 and 52, the two rows the epilogue reads; the rest 0)
  if constexpr (kOnes) {
    for (int idx = threadIdx.x; idx < NBUF * KT * 2; idx += NT) {   // NBUF bufs x KT rows x 2 chunks
      const int buf = idx / (2 * KT), rem = idx % (2 * KT), row = rem >> 1, half = rem & 1;
      char* const bb = smem + buf * BUF;
#if GP_ATTN_ONES_SPARSE
      constexpr uint32_t one = kVH ? 0x3C00u : 0x3F80u;   // 1.0 in V's format
      const uint4 ones = half ? make_uint4(0u, 0u, 0u, 0u) : make_uint4(one, 0u, one, 0u);
#else
      constexpr uint32_t one2 = kVH ? 0x3C003C00u : 0x3F803F80u;
      const uint4 ones = make_uint4(one2, one2, one2, one2);
#endif
      *reinterpret_cast<uint4*>(bb + KTILE + row * VROWB + 32 * (3 ^ (row & 3)) + 16 * half) = ones;
    }
  }

  // Q fragments (B operand): lane holds Q[q = l32][d = 16ks + 8h .. +7]
  bf16x8 qf[KS];
  {
    const int i = q0 + w * 32 + l32;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 z = {};
      if (i < qvalid) z = *reinterpret_cast<const bf16x8*>(qbase + (int64_t)i * qstride + 16 * ks + 8 * h);
      qf[ks] = z;
    }
  }

  // ---- K/V staging
  const int64_t kv_dv = (int64_t)((const char*)vbase - (const char*)kbase);   // V row = K row + kv_dv bytes
  // kModeGen: per-thread staging chunks (source of key 0, row, LDS offset), computed once
  const uint16_t* lsrc[LPT];
  int lrow[LPT], loff[LPT];
  uint4 stage[LPT];
  // kDMA: piece p of the 15 (7 K + 8 V) goes to wave p % NW; lane-linear 16-B units.  K image:
  // 112-B rows = 6 chunks + 1 pad unit (pad lanes off); V image: 128-B rows, swizzled 32-B blocks
  // (the lanes of the bf16-ones block are off: the prologue wrote it)
  constexpr int kPieces = (KT * KROWB + KT * VROWB) / 1024;
  constexpr int PPW = (kPieces + NW - 1) / NW;   // pieces per wave
  int dvo[PPW];
  unsigned dmask = 0;
  if constexpr (kDMA) {
#pragma unroll
    for (int sl = 0; sl < PPW; ++sl) {
      const int pc = w + NW * sl;
      dvo[sl] = 0;
      if (pc >= kPieces) continue;
      if (pc < KTILE / 1024) {
        const int unit = pc * 64 + lane, row = unit / 7, ch = unit % 7;
        dvo[sl] = (int)((int64_t)row * kvstride * 2 + (ch < 6 ? ch : 0) * 16);
        if (ch < 6) dmask |= 1u << sl;
      } else {
        const int unit = (pc - KTILE / 1024) * 64 + lane, row = unit / 8, slot = unit % 8;
        const int b = (slot >> 1) ^ (row & 3);
        dvo[sl] = (int)(kv_dv + (int64_t)row * kvstride * 2 + (2 * (b < 3 ? b : 0) + (slot & 1)) * 16);
        if (b < 3) dmask |= 1u << sl;
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int idx = threadIdx.x + NT * u;
      const int tsel = idx / (KT * CH);
      const int rem = idx % (KT * CH);
      const int row = rem / CH, ch = rem % CH;
      lsrc[u] = (tsel ? vbase : kbase) + (int64_t)row * kvstride + ch * 8;
      lrow[u] = row;
      loff[u] = tsel ? KTILE + row * VROWB + 32 * ((ch >> 1) ^ (row & 3)) + 16 * (ch & 1) : row * KROWB + ch * 16;
    }
  }
  // kDMA: tile kv0 / KT goes to buffer (kv0 / KT) % 2 = the compile-time bc
  auto load_tile = [&](int kv0, auto bc) {
    if constexpr (kDMA) {
      const int64_t tb = (int64_t)kv0 * kvstride * 2;
      const int64_t nrec = (int64_t)(c - kv0 - 1) * kvstride * 2 + kv_dv + 2 * D;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((const char*)kbase + tb), (short)0, (int)(nrec < 0x7fffffff ? nrec : 0x7fffffff), 0x00020000);
      char* bufp = bufc(bc);
#pragma unroll
      for (int sl = 0; sl < PPW; ++sl) {
        const int pc = w + NW * sl;
        if (pc < kPieces && ((dmask >> sl) & 1u))
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rs, (__attribute__((address_space(3))) void*)(bufp + (pc < KTILE / 1024 ? pc * 1024 : KTILE + (pc - KTILE / 1024) * 1024)),
              16, dvo[sl], 0, 0, 0);
      }
    } else {
      const int64_t toff = (int64_t)kv0 * kvstride;      // wave-uniform
      if (kv0 + KT <= c) {                                // full tile: no per-key bound checks
#pragma unroll
        for (int u = 0; u < LPT; ++u) stage[u] = *reinterpret_cast<const uint4*>(lsrc[u] + toff);
      } else {
#pragma unroll
        for (int u = 0; u < LPT; ++u) {
          uint4 z = make_uint4(0, 0, 0, 0);
          if (kv0 + lrow[u] < c) z = *reinterpret_cast<const uint4*>(lsrc[u] + toff);
          stage[u] = z;
        }
      }
    }
  };
  auto store_tile = [&](int buf) {
    if constexpr (!kDMA) {
#pragma unroll
      for (int u = 0; u < LPT; ++u) *reinterpret_cast<uint4*>(smem + buf * BUF + loff[u]) = stage[u];
    }
  };

  bf16x8 onesA = {}, mqB = {};    // kMI operands: [1, 1, 0 ...] x [hi, lo, 0 ...] = -m_run
  if constexpr (kMI) {
    if (h == 0) { onesA[0] = (__bf16)1.0f; onesA[1] = (__bf16)1.0f; }
  }
  float m_run = -INFINITY;   // running max, log2 domain, of query l32
  float lsum = 0.f;          // row sum (VALU path, D % 32 == 0 only)
  f32x16 oacc[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[mt][r] = 0.f;

  // key tiles of this item: all of them, or key part kpart of kparts (round 5: an under-filled launch splits a
  // long branch's keys over several branch entries; each writes a softmax over its keys (o, lse) and the merge
  // combines them as it combines branches).  The reference's zero-pad keys belong to the last part.  A kernel
  // instantiation of its own (kParts): the product kernel keeps its fixed key loop (a variable start costs it
  // spills inside the loop).
  const int ntiles_all = (c + KT - 1) / KT;
  const bool split = kParts && brr.kparts > 1;
  const int t_lo = split ? (int)((int64_t)ntiles_all * brr.kpart / brr.kparts) : 0;
  const int t_hi = split ? (int)((int64_t)ntiles_all * (brr.kpart + 1) / brr.kparts) : ntiles_all;
  const bool last_part = !split || brr.kpart == brr.kparts - 1;
  if (t_hi > t_lo) {
    load_tile(t_lo * KT, IB0());
    store_tile(0);
  }
  __syncthreads();
  // every vector load so far (Q fragments, tile 0) is complete here; saying so with a real
  // s_waitcnt (vmcnt 0) lets the compiler's wait insertion drop its "Q may still be in flight"
  // state at the loop head, which otherwise forces vmcnt(0) -- a wait on the next tile's
  // prefetch -- before the first MFMA of every tile
  __builtin_amdgcn_s_waitcnt(0x0f70);

  if constexpr ((attn_wps<MODE, kTab, NW>() >= 6 ? GP_ATTN_PRIO_FAST : GP_ATTN_PRIO) != 0 && NW >= 8) {
    if (__builtin_amdgcn_readfirstlane((int)threadIdx.x) >= NT / 2) __builtin_amdgcn_s_setprio(1);
  }
  // one 64-key tile; SET = the tile's LDS buffer when the loop is unrolled by two (kDMA), so the
  // buffer offsets fold into the ds_read immediates
  // GP_ATTN_SKIP_IDLE: a wave whose 32 queries all lie at or past the last needed row (the tail
  // q-block of a segment) skips the MFMAs and the softmax -- its outputs are never stored -- and
  // only issues its share of the K/V staging and the barriers (~2 % of the wave-tiles at 70k)
  const bool wact = !GP_ATTN_SKIP_IDLE || __builtin_amdgcn_readfirstlane(q0 + w * 32) < rows_needed;
  auto tile_step = [&](int t, auto setc) {
    constexpr int SET = decltype(setc)::value;
    if (t + 1 < t_hi) load_tile((t + 1) * KT, std::integral_constant<int, 1 - SET>());
    const int kv0 = t * KT;
    const char* Kb = kDMA ? (const char*)bufc(setc) : smem + (t & 1) * BUF;
    const char* Vb = Kb + KTILE;
    if constexpr (attn_wps<MODE, kTab, NW>() >= 6) {
      // the fast kernel (GP_ATTN_FAST_WPS): one 32-key sub-tile at a time -- S, exps and P.V of sub-tile u before
      // sub-tile u + 1's S -- so the body fits 80 VGPRs and three workgroups share each CU
      if (wact) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          f32x16 acc;
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            const bf16x8 kk = *reinterpret_cast<const bf16x8*>(Kb + (32 * u + l32) * KROWB + 32 * ks + 16 * h);
            acc = mfma_32x32x16<kH>(kk, qf[ks], acc);
          }
          if (kv0 + 64 > c) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (kv0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * h >= c) acc[r] = -INFINITY;
          }
          bf16x8 pu[2];
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) pu[s][e] = f2e_slot<kVH>(fast_exp2(acc[8 * s + e]));
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const int row = 32 * u + 16 * s + 4 * (lane >> 5) + ((lane >> 2) & 3);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
              const int blk = 2 * mt + ((lane >> 4) & 1);
              const char* p0 = Vb + row * VROWB + 32 * (blk ^ (row & 3)) + 8 * (lane & 3);
              const char* p1 = p0 + 8 * VROWB;
              const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
              const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
              const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
              oacc[mt] = mfma_32x32x16<kVH>(vf, pu[s], oacc[mt]);
            }
          }
        }
      }
    } else if (wact) {   // (GP_ATTN_SKIP_IDLE) waves with no needed query only stage K/V and join the barriers
      // ---- S^T for two 32-key sub-tiles.  kPre (q pre-multiplied by scale*log2 e): the
      // accumulator starts at -m_run, so it already holds log2-domain scores minus the max.
      f32x16 sacc[2];
      f32x16 ini;
      if constexpr (kMI) {
        f32x16 zero;
#pragma unroll
        for (int r = 0; r < 16; ++r) zero[r] = 0.f;
        ini = __builtin_amdgcn_mfma_f32_32x32x16_bf16(onesA, mqB, zero, 0, 0, 0);
      }
      const float init = (kPre && !kZM && !kMI && t > t_lo) ? -m_run : 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f32x16 acc;
        if constexpr (kMI) {
          acc = ini;
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] = init;
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 kk = *reinterpret_cast<const bf16x8*>(Kb + (32 * u + l32) * KROWB + 32 * ks + 16 * h);
          acc = mfma_32x32x16<kH>(kk, qf[ks], acc);
        }
        sacc[u] = acc;
      }
      if (kv0 + 64 > c) {      // keys >= c are zero pads (added analytically at the end)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kv0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * h >= c) sacc[u][r] = -INFINITY;
      }

      // ---- online softmax with deferred rescale (two independent max chains)
      float mx = 0.f;
      if (!kZM) {
        float mxa = sacc[0][0], mxb = sacc[1][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) {
          mxa = fmaxf(mxa, sacc[0][r]);
          mxb = fmaxf(mxb, sacc[1][r]);
        }
        mx = fmaxf(mxa, mxb);
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      }
      bf16x8 pf[2][2];
      if constexpr (kPre) {
        if constexpr (!kZM) {
          // scores are s*c - m_run; rescale only when a query's max moved up by > kThr
          // (the first tile: always, which sets m_run to that tile's exact max)
          const bool need = (t == t_lo) || mx > kThr;
          if (__builtin_amdgcn_ballot_w64(need)) {
            if constexpr (kMI) {
              // m kept as an exact hi + lo pair of bf16 values (two rows of the init MFMA), so it
              // tracks the max to ~2^-16 relative and numerator and denominator stay consistent
              const float m_old = (t == t_lo) ? 0.f : m_run;
              float m_new = m_old;
              if (need) {
                const float tt = -(m_old + mx);
                const __bf16 hi = (__bf16)tt;
                const __bf16 lo = (__bf16)(tt - (float)hi);
                m_new = -((float)hi + (float)lo);
              }
              const float d = m_new - m_old;
              if (t > t_lo) {
                const float alpha = fast_exp2(-d);
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                  for (int r = 0; r < 16; ++r) oacc[mt][r] *= alpha;
                lsum *= alpha;
              }
              m_run = m_new;
#pragma unroll
              for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 16; ++r) sacc[u][r] -= d;
              if (h == 0) {
                const __bf16 hi = (__bf16)(-m_run);
                mqB[0] = hi;
                mqB[1] = (__bf16)(-m_run - (float)hi);
              }
            } else {
              const float delta = need ? mx : 0.f;
              const float alpha = fast_exp2(-delta);
              if (t > t_lo) {
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                  for (int r = 0; r < 16; ++r) oacc[mt][r] *= alpha;
                lsum *= alpha;
              }
              m_run = (t == t_lo) ? delta : m_run + delta;
#pragma unroll
              for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 16; ++r) sacc[u][r] -= delta;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float p = fast_exp2(sacc[u][8 * s + e]);
              if constexpr (!kOnes) lsum += p;
              pf[u][s][e] = f2e_slot<kVH>(p);
            }
      } else {
        const float tm = mx * a.c_log2;
        const bool need = tm > m_run + kThr;
        if (__builtin_amdgcn_ballot_w64(need)) {
          const float m_new = need ? tm : m_run;
          const float alpha = fast_exp2(m_run - m_new);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[mt][r] *= alpha;
          lsum *= alpha;
          m_run = m_new;
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float p = fast_exp2(fmaf(sacc[u][8 * s + e], a.c_log2, -m_run));
              if constexpr (!kOnes) lsum += p;
              pf[u][s][e] = f2e_slot<kVH>(p);
            }
      }

      // ---- O^T += V^T . P^T  (2 sub-tiles x 2 k-steps x 2 d-tiles)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int row = 32 * u + 16 * s + 4 * (lane >> 5) + ((lane >> 2) & 3);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const int blk = 2 * mt + ((lane >> 4) & 1);
            const char* p0 = Vb + row * VROWB + 32 * (blk ^ (row & 3)) + 8 * (lane & 3);
            const char* p1 = p0 + 8 * VROWB;   // rows + 8 keep (row & 3)
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
            const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            oacc[mt] = mfma_32x32x16<kVH>(vf, pf[u][s], oacc[mt]);
          }
        }

    }
    if (t + 1 < t_hi) store_tile((t + 1) & 1);
    if constexpr (kDMA) __builtin_amdgcn_s_waitcnt(0x0f70);   // this wave's DMA pieces landed
    __syncthreads();
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if constexpr (kDMA) {
    for (int t = t_lo; t < t_hi; t += 2) {
      tile_step(t, S0());
      if (t + 1 < t_hi) tile_step(t + 1, S1());
    }
  } else {
    for (int t = t_lo; t < t_hi; ++t) tile_step(t, S0());
  }

  // ---- epilogue
  float l;
  if constexpr (kOnes) {
    l = oacc[1][8];                       // d-row 48 (+4h): the ones row = sum_k P
  } else {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(lsum), __float_as_uint(lsum), false, false);
    l = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  const int npad = last_part ? g.m - c : 0;
  // a key part with no keys at all (a short last segment split in parts): an empty softmax -- o = 0,
  // lse = -inf, which the merge weighs 0 -- not a flagged row
  const bool empty = kParts && t_hi <= t_lo && npad == 0;
  bool zm_bad = false;
  if constexpr (kFlag) {
    if constexpr (kZM) m_run = 0.f;
    const uint32_t eb = __float_as_uint(l) & 0x7f800000u;
    // with zero-pad keys (p = 1 each) a tiny real-key sum is not flagged: the pads then dominate
    // exactly as in the reference
    zm_bad = !empty && (eb == 0x7f800000u || !(l <= 0x1p100f) || (npad == 0 && !(l >= 0x1p-100f)));
  }
  // the reference's unmasked zero-padded keys (dilated_attention.py:85-91): npad keys of score 0
  float mr = m_run, so = 1.f;
  if (npad > 0) {
    const float mf = fmaxf(mr, 0.f);
    so = fast_exp2(mr - mf);
    l = l * so + (float)npad * fast_exp2(-mf);
    mr = mf;
  }
  const float inv = empty ? 0.f : so / l;
  const int i = q0 + w * 32 + l32;
  if constexpr (GP_ATTN_WIDE_STORE != 0) {
    // lane (q, h) holds d = 8k + 4h .. +3 for the D/8 groups k.  For each pair of groups (k, k+1)
    // one permlane32_swap per dword gives lanes 0-31 d = 8k .. 8k+7 and lanes 32-63 d = 8k+8 .. 8k+15
    // (T21): one 16-byte store per pair.  The swap needs EXEC full: it runs before the row check.
    uint2 pk[D / 8];
#pragma unroll
    for (int k = 0; k < D / 8; ++k) {
      const int mt = k / 4, rg = k % 4;
      pk[k].x = (uint32_t)f2e<kH>(oacc[mt][4 * rg] * inv) | ((uint32_t)f2e<kH>(oacc[mt][4 * rg + 1] * inv) << 16);
      pk[k].y = (uint32_t)f2e<kH>(oacc[mt][4 * rg + 2] * inv) | ((uint32_t)f2e<kH>(oacc[mt][4 * rg + 3] * inv) << 16);
    }
#pragma unroll
    for (int k = 0; k < D / 8; k += 2) {
      const auto rx = __builtin_amdgcn_permlane32_swap(pk[k].x, pk[k + 1].x, false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(pk[k].y, pk[k + 1].y, false, false);
      pk[k].x = rx[0]; pk[k + 1].x = rx[1];
      pk[k].y = ry[0]; pk[k + 1].y = ry[1];
    }
    if (i < rows_needed && fixrow) {
      uint16_t* orow = brr.o + (((int64_t)bn * g.m + i) * a.H + hh) * (int64_t)D + 8 * h;
#pragma unroll
      for (int k = 0; k < D / 8; k += 2)
        *reinterpret_cast<uint4*>(orow + 8 * k) = make_uint4(pk[k].x, pk[k].y, pk[k + 1].x, pk[k + 1].y);
    }
  } else if (i < rows_needed && fixrow) {
    uint16_t* orow = brr.o + (((int64_t)bn * g.m + i) * a.H + hh) * (int64_t)D;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int d0 = 32 * mt + 8 * rg + 4 * h;
        if (d0 < D) {
          float vv[4] = {oacc[mt][4 * rg] * inv, oacc[mt][4 * rg + 1] * inv, oacc[mt][4 * rg + 2] * inv,
                         oacc[mt][4 * rg + 3] * inv};
          store_e<kH, 4>(orow + d0, vv);
        }
      }
  }
  if (i < rows_needed && fixrow) {
    float lse = empty ? -INFINITY : (mr + __builtin_amdgcn_logf(l)) * 0.69314718055994530942f;
    if constexpr (kFlag) {   // overflowed / out of range: flag the row for the fixup pass
      if (!empty && ((__float_as_uint(l) & 0x7f800000u) == 0x7f800000u || !(l > 0.f) || zm_bad))
        lse = __uint_as_float(kLseRedo);
    }
    if (h == 0) brr.lse[((int64_t)bn * a.H + hh) * g.m + i] = lse;
  }
}

// One work item per block (XCD-grouped order).  The fixup pass (kModeFix), product layout kFixItems = 4
// (GP_ATTN_FIX_ITEMS): a block reads the lse of every needed row of its kFixItems consecutive items at
// once (independent loads per lane), exits unless one holds the kLseRedo marker, and recomputes the
// flagged items in turn; kFixItems = 1 (lab builds) is one item per block in item order.
template <int D, bool kPre, int MODE, bool kTab = false, int NW = 4, bool kH = false, bool kParts = false>
__global__ __launch_bounds__(NW * 64, (attn_wps<MODE, kTab, NW>())) void dilated_attn32_kernel(const AttnArgs a) {
  if constexpr (MODE == kModeFix && kFixItems == 1) {
    attn32_item<D, kPre, MODE, kTab, NW, kH, kParts>(a, (int)blockIdx.x);   // its own flagged-row check first
  } else if constexpr (MODE == kModeFix) {
    constexpr int QB = NW * 32;
    const int it0 = (int)blockIdx.x * kFixItems;
    // wave index made provably uniform: the item decode then runs on the scalar unit (s_load from
    // the kernel arguments), not as a chain of dependent per-lane global loads
    const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = (int)threadIdx.x & 63;
    // slot s = 64 rows of one item (item s / (QB / 64)); wave w reads slots w, w + NW, ...; every load is
    // issued before any is compared (clamped in-bounds indices, masked after), so they are in flight together
    constexpr int SLOTS = kFixItems * (QB / 64);
    constexpr int NV = (SLOTS + NW - 1) / NW;
    uint32_t vals[NV];
    bool use[NV];
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const int sl = w + NW * n;
      const int it = it0 + sl / (QB / 64), hf = sl % (QB / 64);
      const bool live = sl < SLOTS && it < a.total_items;
      WorkItem wi;
      AttnBranch te;
      const int itc = live ? it : (int)a.total_items - 1;
      if constexpr (kTab) decode_item_tab(a, itc, wi, te);
      else decode_item(a, itc, wi);
      const AttnBranch& brr = kTab ? te : a.br[wi.bi];
      const int q0 = wi.i_lo + wi.qb * QB;
      const float* lrow = brr.lse + ((int64_t)wi.bn * a.H + wi.hh) * brr.g.m;
      const int i = q0 + 64 * hf + lane;
      use[n] = live && i < wi.i_hi;
      vals[n] = __float_as_uint(lrow[use[n] ? i : 0]);
    }
    bool flagged = false;
#pragma unroll
    for (int n = 0; n < NV; ++n) flagged |= use[n] && vals[n] == kLseRedo;
    if (!__syncthreads_or(flagged)) return;
    for (int k = 0; k < kFixItems && it0 + k < a.total_items; ++k) attn32_item<D, kPre, MODE, kTab, NW, kH, kParts>(a, it0 + k);
  } else {
    attn32_item<D, kPre, MODE, kTab, NW, kH, kParts>(a, (int)xcd_group(blockIdx.x, gridDim.x));
  }
}
// ---------------------------------------------------------------------------------------
struct MergeBranch {
  GpBranch g;
  const uint16_t* o;
  const float* lse;
  DivMagic dg, dr;   // division by g.g and by g.r
};
inline void merge_branch_magic(MergeBranch& m) {
  m.dg = make_div_magic((uint32_t)m.g.g);
  m.dr = make_div_magic((uint32_t)m.g.r);
}

struct MergeArgs {
  int64_t B, L;
  int64_t tok_lo, ntok;   // window of tokens [tok_lo, tok_lo + ntok) of every batch; out row = b*ntok + t
  int32_t H, D, E, nbranch;
  MergeBranch br[GP_MAX_BRANCHES];
  const float* ln_w;
  const float* ln_b;
  float eps;
  uint16_t* out;
  // varlen (packed slides): slide i owns packed tokens [tok_off[i], tok_off[i+1]); its branch b
  // geometry and o/lse regions are mtab[i * nbranch + b]
  const MergeBranch* mtab;
  const int64_t* tok_off;
  int32_t nslide;
  DivMagic dnt;        // division by ntok (the batch index of a row)
};

// One wave per run of kTPW consecutive tokens; lane l owns the EPL = E/64 contiguous elements
// [l*EPL, (l+1)*EPL) of head l*EPL/D (EPL divides D).  The sparse_to_dense position of the
// token in every branch -- segment n, dense slot t = p mod g, sparse row i = t / r, phase
// jj = t mod r -- is wave-uniform: divided out once per run, then stepped token by token.  The
// lanes a branch covers for phase jj are the contiguous range [jj*LPH, (jj+1)*LPH), LPH = lanes
// per head group.  Math per token is that of dilated_attention.py:100-131 (fp32 weights,
// branch-order accumulation) followed by inner_attn_ln.
constexpr int kTPW = 1;

// NBR < GP_MAX_BRANCHES: the launch guarantees a.nbranch == NBR, so the branch loops have a
// compile-time trip count (the 5-branch schedule of every registered arch: 3 dead branches of
// position stepping, address math and exp fewer per token)
template <int EPL, int D, bool kTab = false, int NBR = GP_MAX_BRANCHES, bool kH = false>
__global__ __launch_bounds__(256) void branch_merge_kernel(const MergeArgs a) {
  const int nbr = NBR < GP_MAX_BRANCHES ? NBR : a.nbranch;
  const int lane = threadIdx.x & 63;
  const int run = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
  const int total = (int)(a.B * a.ntok);
  const int r0 = run * kTPW;
  if (r0 >= total) return;
  // kTab: the token's slide (binary search, wave-uniform) and that slide's branch entries
  MergeBranch tb[kTab ? GP_MAX_BRANCHES : 1];
  int64_t slide_tok0 = 0;
  if constexpr (kTab) {
    int lo = 0, hi = a.nslide - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((int64_t)r0 >= a.tok_off[mid]) lo = mid; else hi = mid - 1;
    }
    slide_tok0 = a.tok_off[lo];
#pragma unroll
    for (int b = 0; b < NBR; ++b)
      if (b < nbr) tb[b] = a.mtab[lo * a.nbranch + b];
  }
  const int nt = (int)a.ntok;
  const int E = 64 * EPL;
  const int col0 = lane * EPL;
  int pn[GP_MAX_BRANCHES], pt[GP_MAX_BRANCHES], pi[GP_MAX_BRANCHES], pj[GP_MAX_BRANCHES];
  int bidx = 0, p = 0;
  for (int k = 0; k < kTPW; ++k) {
    const int row = r0 + k;
    if (row >= total) break;
    if (k == 0 || p + 1 >= (int)a.tok_lo + nt) {   // (re)derive positions: run start / next batch
      if constexpr (kTab) {
        bidx = 0;
        p = (int)(row - slide_tok0);
      } else {
        bidx = (int)div_magic((uint32_t)row, a.dnt);
        p = (int)a.tok_lo + (row - bidx * nt);
      }
#pragma unroll
      for (int b = 0; b < NBR; ++b)
        if (b < nbr) {
          const MergeBranch& mb = kTab ? tb[b] : a.br[b];
          pn[b] = (int)div_magic((uint32_t)p, mb.dg);
          pt[b] = p - pn[b] * mb.g.g;
          pi[b] = (int)div_magic((uint32_t)pt[b], mb.dr);
          pj[b] = pt[b] - pi[b] * mb.g.r;
        }
    } else {
      ++p;
#pragma unroll
      for (int b = 0; b < NBR; ++b)
        if (b < nbr) {
          const GpBranch& g = (kTab ? tb[b] : a.br[b]).g;
          if (++pt[b] == g.g) { pt[b] = 0; ++pn[b]; pi[b] = 0; pj[b] = 0; }
          else if (++pj[b] == g.r) { pj[b] = 0; ++pi[b]; }
        }
    }
    // Every branch's loads are issued before any wait, with no exec-mask region around them: a
    // lane outside the branch's head group reads the group's first lane's o / lse (the same
    // cache lines, no extra traffic) and its weight is forced to zero below.  (Loads guarded by
    // `if (covered)` compiled to one wait per branch -- five serial memory latencies per token.)
    float lse[GP_MAX_BRANCHES];
    bool cov[GP_MAX_BRANCHES];
    uint2 ob[GP_MAX_BRANCHES][EPL / 4];
#pragma unroll
    for (int b = 0; b < NBR; ++b) {
      lse[b] = -1e8f;
      cov[b] = false;
      if (b < nbr) {
        const MergeBranch& mb = kTab ? tb[b] : a.br[b];
        const int lph = mb.g.hpg * (D / EPL);     // lanes per head group
        const int l0 = pj[b] * lph;
        cov[b] = lane >= l0 && lane < l0 + lph;
        const int ln = cov[b] ? lane : l0;
        const int64_t rb = (int64_t)(bidx * mb.g.nseg + pn[b]);
        lse[b] = mb.lse[(rb * a.H + ln * EPL / D) * mb.g.m + pi[b]];
        const uint2* src = reinterpret_cast<const uint2*>(mb.o + (rb * mb.g.m + pi[b]) * E + ln * EPL);
#pragma unroll
        for (int q = 0; q < EPL / 4; ++q) ob[b][q] = src[q];
      }
    }
    float wv[EPL], bv[EPL];
    if (a.ln_w != nullptr) {   // LN affine via L1, in flight with the o rows (-5 % vs loading after the sums)
      load_f32<EPL>(a.ln_w + col0, wv);
      load_f32<EPL>(a.ln_b + col0, bv);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int b = 0; b < NBR; ++b)
      if (b < nbr) {
        if (!cov[b] || lse[b] == 0.f) lse[b] = -1e8f;   // dilated_attention.py:46
        mx = fmaxf(mx, lse[b]);
      }
    float wsum = 0.f;
#pragma unroll
    for (int b = 0; b < NBR; ++b)
      if (b < nbr) {
        // v_exp_f32 / v_rcp_f32 (1 ulp) instead of the libm expf and the IEEE division sequence: the
        // weights are fp32 (the reference rounds them to the activation dtype, dilated_attention.py:128)
        lse[b] = fast_exp2((lse[b] - mx) * 1.44269504088896340736f);
        wsum += lse[b];
      }
    const float inv = __builtin_amdgcn_rcpf(wsum);
    float acc[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
#pragma unroll
    for (int b = 0; b < NBR; ++b) {
      if (b < nbr) {
        const float wb = cov[b] ? lse[b] * inv : 0.f;   // + 0 * finite leaves acc unchanged
#pragma unroll
        for (int q = 0; q < EPL / 4; ++q) {
          // explicit fma: every instantiation (and the varlen path) rounds identically
          acc[4 * q + 0] = __builtin_fmaf(e2f<kH>(ob[b][q].x), wb, acc[4 * q + 0]);
          acc[4 * q + 1] = __builtin_fmaf(e2f_hi<kH>(ob[b][q].x), wb, acc[4 * q + 1]);
          acc[4 * q + 2] = __builtin_fmaf(e2f<kH>(ob[b][q].y), wb, acc[4 * q + 2]);
          acc[4 * q + 3] = __builtin_fmaf(e2f_hi<kH>(ob[b][q].y), wb, acc[4 * q + 3]);
        }
      }
    }
    if (a.ln_w != nullptr) wave_layernorm_regs<EPL>(acc, E, wv, bv, a.eps);
    store_e<kH, EPL>(a.out + (int64_t)row * E + col0, acc);
  }
}

// ---------------------------------------------------------------------------------------
// Merge for E = 768, D = 48 (H = 16: every registered 768-wide arch, the product path), one token per
// wave as branch_merge_kernel, with fewer vector instructions per token (that kernel issues ~380 VALU
// per token-wave, ~70 of them 64-bit per-lane address arithmetic, and 12 dependent ds_bpermute for the
// LN sums):
//  * a lane owns two column chunks: 8 columns (one 16-byte access) and 4 columns (one 8-byte access)
//    instead of three 8-byte accesses of 12 contiguous columns.  kMap 1 ("x8", the default): [8l, 8l + 8)
//    of head l / 6 and [512 + 4l, 516 + 4l) of head (128 + l) / 12, so each wave-instruction covers one
//    contiguous span (two heads per lane: twice the softmax VALU, yet measured faster: the kernel is bound
//    by memory requests, not issue); kMap 0: both chunks in head l / 4 (lane k of a head: columns 8k..
//    and 32 + 4k.. of the head, one softmax per lane);
//  * loads address a wave-uniform row base plus a 32-bit lane offset (no per-lane 64-bit math);
//  * the LN row sums are xor-butterflies (DPP quad_perm / row_half_mirror / row_ror:8, then
//    v_permlane16/32_swap): the same sum in every lane, no LDS round trips.
// Per (token, head) the branch weights and the fp32 accumulation are branch_merge_kernel's bit for bit
// (dilated_attention.py:100-131).
#ifndef GP_MERGE_MAP
#define GP_MERGE_MAP 1
#endif
// waves (tokens) per block of the v2 merge: consecutive tokens of one block share their lse / o lines in L1
#ifndef GP_MERGE_WPB
#define GP_MERGE_WPB 4
#endif

// A 32-bit lane offset the compiler may not re-associate with constants: keeps a uniform-base + lane-offset
// load in its SGPR-base (saddr) form instead of a per-lane 64-bit address.
GP_DEV uint32_t opaque_u32(uint32_t x) {
  __asm__("" : "+v"(x));
  return x;
}

GP_DEV float wave_sum_xor(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false));   // quad_perm 1,0,3,2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false));   // quad_perm 2,3,0,1
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xf, 0xf, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));  // row_ror:8
  const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
  const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
}

template <int NBR, bool kTab, bool kH, int kMap = GP_MERGE_MAP>
__global__ __launch_bounds__(64 * GP_MERGE_WPB) void branch_merge_v2_kernel(const MergeArgs a) {
  // no implicit contraction: the compiler fused v - s * (1/E) into one fma in some instantiations only, so the
  // packed (varlen) and single-slide merges differed in the last bit; every fma below is explicit
#pragma clang fp contract(off)
  constexpr int E = 768, H = 16, D = 48;
  constexpr bool k1h = kMap == 0;          // one head per lane
  const int nbr = NBR < GP_MAX_BRANCHES ? NBR : a.nbranch;
  const int lane = threadIdx.x & 63;
  const int row = __builtin_amdgcn_readfirstlane((int)blockIdx.x * GP_MERGE_WPB + (int)(threadIdx.x >> 6));
  const int total = (int)(a.B * a.ntok);
  if (row >= total) return;
  // the lane's chunks: columns c0 .. c0 + 7 (head h0) and c1 .. c1 + 3 (head h1)
  const int kq = lane & 3;
  const int h0 = k1h ? lane >> 2 : lane / 6;
  const int h1 = k1h ? h0 : (128 + lane) / 12;
  const int c0 = k1h ? D * h0 + 8 * kq : 8 * lane;
  const int c1 = k1h ? D * h0 + 32 + 4 * kq : 512 + 4 * lane;
  // LN affine (L1-resident): issued with the branch loads; a null ln_w reads the output row's own
  // location instead (valid memory, unused) so the registers need no zero-fill
  const bool ln = a.ln_w != nullptr;
  const float* lw = ln ? a.ln_w : reinterpret_cast<const float*>(a.out);
  const float* lb = ln ? a.ln_b : reinterpret_cast<const float*>(a.out);
  float w0[8], w1[4], b0[8], b1[4];
  load_f32<8>(lw + c0, w0);
  load_f32<4>(lw + c1, w1);
  load_f32<8>(lb + c0, b0);
  load_f32<4>(lb + c1, b1);
  int bidx = 0, p;
  MergeBranch tb[kTab ? GP_MAX_BRANCHES : 1];
  if constexpr (kTab) {
    int lo = 0, hi = a.nslide - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((int64_t)row >= a.tok_off[mid]) lo = mid; else hi = mid - 1;
    }
    p = (int)(row - a.tok_off[lo]);
#pragma unroll
    for (int b = 0; b < NBR; ++b)
      if (b < nbr) tb[b] = a.mtab[lo * a.nbranch + b];
  } else {
    bidx = (int)div_magic((uint32_t)row, a.dnt);
    p = (int)a.tok_lo + (row - bidx * (int)a.ntok);
  }
  // every branch's loads before any wait; a lane outside the branch's head group reads the group's
  // first head (same cache lines as the covered lanes) and gets weight 0
  uint4 o0[NBR];
  uint2 o1[NBR];
  float l0[NBR], l1[NBR];
  bool cv0[NBR], cv1[NBR];
#pragma unroll
  for (int b = 0; b < NBR; ++b) {
    cv0[b] = cv1[b] = false;
    l0[b] = l1[b] = -1e8f;
    o0[b] = make_uint4(0, 0, 0, 0);
    o1[b] = make_uint2(0, 0);
    if (b < nbr) {
      const MergeBranch& mb = kTab ? tb[b] : a.br[b];
      const int pn = (int)div_magic((uint32_t)p, mb.dg);
      const int pt = p - pn * mb.g.g;
      const int pi = (int)div_magic((uint32_t)pt, mb.dr);
      const int pj = pt - pi * mb.g.r;
      const int hpg = mb.g.hpg;
      const int hf = pj * hpg;                                 // the covered group's first head
      // 32-bit byte offsets: the launch checks every branch's o / lse buffer is below 4 GiB
      const uint32_t rb = (uint32_t)(bidx * mb.g.nseg + pn);
      const char* orow = reinterpret_cast<const char*>(mb.o) + (rb * (uint32_t)mb.g.m + (uint32_t)pi) * (uint32_t)(E * 2);
      const char* lrow = reinterpret_cast<const char*>(mb.lse) + (rb * (uint32_t)(H * mb.g.m) + (uint32_t)pi) * 4u;
      const uint32_t m4 = (uint32_t)mb.g.m * 4u;
      cv0[b] = (unsigned)(h0 - hf) < (unsigned)hpg;
      const int s0 = cv0[b] ? h0 : hf;
      // (m < 2^22 for any segment of the schedule: 24-bit multiplies)
      l0[b] = *reinterpret_cast<const float*>(lrow + opaque_u32(__umul24((uint32_t)s0, m4)));
      if constexpr (k1h) {
        cv1[b] = cv0[b];
        const uint32_t off0 = __umul24((uint32_t)s0, 2u * D) + 16u * kq;   // head s0, lane kq's columns
        const uint32_t off1 = off0 + (uint32_t)(64 - 8 * kq);
        o0[b] = *reinterpret_cast<const uint4*>(orow + opaque_u32(off0));
        o1[b] = *reinterpret_cast<const uint2*>(orow + opaque_u32(off1));
      } else {
        cv1[b] = (unsigned)(h1 - hf) < (unsigned)hpg;
        l1[b] = *reinterpret_cast<const float*>(lrow + opaque_u32(__umul24((uint32_t)(cv1[b] ? h1 : hf), m4)));
        o0[b] = *reinterpret_cast<const uint4*>(orow + opaque_u32(cv0[b] ? 2 * c0 : 2 * D * hf));
        o1[b] = *reinterpret_cast<const uint2*>(orow + opaque_u32(cv1[b] ? 2 * c1 : 2 * D * hf));
      }
    }
  }
  // per-head softmax over the branches (k1h: one head per lane)
  float mx0 = -INFINITY, mx1 = -INFINITY;
#pragma unroll
  for (int b = 0; b < NBR; ++b)
    if (b < nbr) {
      if (!cv0[b] || l0[b] == 0.f) l0[b] = -1e8f;   // dilated_attention.py:46
      mx0 = fmaxf(mx0, l0[b]);
      if constexpr (!k1h) {
        if (!cv1[b] || l1[b] == 0.f) l1[b] = -1e8f;
        mx1 = fmaxf(mx1, l1[b]);
      }
    }
  float ws0 = 0.f, ws1 = 0.f;
#pragma unroll
  for (int b = 0; b < NBR; ++b)
    if (b < nbr) {
      l0[b] = fast_exp2((l0[b] - mx0) * 1.44269504088896340736f);
      ws0 += l0[b];
      if constexpr (!k1h) {
        l1[b] = fast_exp2((l1[b] - mx1) * 1.44269504088896340736f);
        ws1 += l1[b];
      }
    }
  const float inv0 = __builtin_amdgcn_rcpf(ws0), inv1 = k1h ? inv0 : __builtin_amdgcn_rcpf(ws1);
  float v[12];
#pragma unroll
  for (int e = 0; e < 12; ++e) v[e] = 0.f;
#pragma unroll
  for (int b = 0; b < NBR; ++b)
    if (b < nbr) {
      const float wb0 = cv0[b] ? l0[b] * inv0 : 0.f;   // + 0 * finite leaves v unchanged
      const float wb1 = k1h ? wb0 : (cv1[b] ? l1[b] * inv1 : 0.f);
      const uint32_t u0[4] = {o0[b].x, o0[b].y, o0[b].z, o0[b].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] = __builtin_fmaf(e2f<kH>(u0[k]), wb0, v[2 * k]);
        v[2 * k + 1] = __builtin_fmaf(e2f_hi<kH>(u0[k]), wb0, v[2 * k + 1]);
      }
      v[8] = __builtin_fmaf(e2f<kH>(o1[b].x), wb1, v[8]);
      v[9] = __builtin_fmaf(e2f_hi<kH>(o1[b].x), wb1, v[9]);
      v[10] = __builtin_fmaf(e2f<kH>(o1[b].y), wb1, v[10]);
      v[11] = __builtin_fmaf(e2f_hi<kH>(o1[b].y), wb1, v[11]);
    }
  if (ln) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 12; ++e) s += v[e];
    const float mean = wave_sum_xor(s) * (1.0f / E);
    // explicit fmas: every instantiation (the varlen one included) rounds the LN identically
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 12; ++e) {
      const float d = v[e] - mean;
      q = __builtin_fmaf(d, d, q);
    }
    const float rstd = rsqrtf(__builtin_fmaf(wave_sum_xor(q), 1.0f / E, a.eps));
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = __builtin_fmaf((v[e] - mean) * rstd, w0[e], b0[e]);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[8 + e] = __builtin_fmaf((v[8 + e] - mean) * rstd, w1[e], b1[e]);
  }
  char* orow = reinterpret_cast<char*>(a.out) + (int64_t)row * (E * 2);
  *reinterpret_cast<uint4*>(orow + 2 * c0) =
      make_uint4(pack2e<kH>(v[0], v[1]), pack2e<kH>(v[2], v[3]), pack2e<kH>(v[4], v[5]), pack2e<kH>(v[6], v[7]));
  *reinterpret_cast<uint2*>(orow + 2 * c1) = make_uint2(pack2e<kH>(v[8], v[9]), pack2e<kH>(v[10], v[11]));
}

// GP_MERGE_V3 (round 6, product 1): the v2 merge with the LSEs staged per block of up to kV3Tok consecutive tokens.  The
// [B * nseg, H, m] lse layout puts one token's covered heads in 16 / r different cache lines, and the v2 kernel's
// one-token waves fetch them token by token (~16 of its ~42 L2 read requests per token, at the per-CU cap of
// outstanding requests, §3.5).  Here the block's four waves first load every lse its 64 tokens need -- lane t =
// token t, so one wave-instruction reads up to 64 consecutive rows of a head -- into LDS, then each wave merges
// a quarter of the tokens (t = wave + 4k) exactly as branch_merge_v2_kernel does, reading the weights' LSEs from
// LDS.  Same arithmetic per token, so the same bits (the varlen merge too, GP_MERGE_V3_TAB).  Same-process A/B
// (profiles/r06_mv3e_merge_ab_*): 70k 73.5 vs 84.2 us, 256k 238 vs 284 us per launch, bit-identical; up to 64
// tokens per block 82.5 / 246 us, 16: 82.0 / 272 us.
#ifndef GP_MERGE_V3
#define GP_MERGE_V3 1
#endif
// GP_MERGE_V3_TAB (product 1): the packed-slide (varlen) merge on the v3 kernel too, when every slide holds at least a
// block's tokens: C5 batch (675,619 tokens) 0.625 vs 0.868 ms per launch, bit-identical (profiles/r06_mv3tab2_*)
#ifndef GP_MERGE_V3_TAB
#define GP_MERGE_V3_TAB 1
#endif
#ifndef GP_MERGE_V3_TOK
#define GP_MERGE_V3_TOK 32
#endif
constexpr int kV3Tok = GP_MERGE_V3_TOK;    // most tokens per block (4 waves, up to kV3Tok / 4 tokens each); <= 64

// A MergeBranch table entry by scalar loads (uniform index, constant address space): the entries then live in
// SGPRs even when the load follows the kernel's global stores (the compiler's uniform-load analysis would
// otherwise fall back to per-lane loads into VGPRs)
GP_DEV MergeBranch merge_entry_scalar(const MergeBranch* tab, int idx) {
  MergeBranch e;
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(sizeof(MergeBranch) % 4 == 0, "");
  uint32_t words[sizeof(MergeBranch) / 4];
  const __attribute__((address_space(4))) uint32_t* src =
      (const __attribute__((address_space(4))) uint32_t*)(uintptr_t)(tab + __builtin_amdgcn_readfirstlane(idx));
#pragma unroll
  for (int i = 0; i < (int)(sizeof(MergeBranch) / 4); ++i) words[i] = src[i];
  __builtin_memcpy(&e, words, sizeof(MergeBranch));
#else
  e = tab[idx];
#endif
  return e;
}

template <int NBR, bool kH, bool kTab = false>
__global__ __launch_bounds__(256) void branch_merge_v3_kernel(const MergeArgs a, const int tpb) {
#pragma clang fp contract(off)
  constexpr int E = 768, H = 16, D = 48;
  constexpr int LS = NBR * 16 + 1;           // LDS floats per token (16 per branch entry; +1: bank spread)
  __shared__ float lse_s[kV3Tok * LS];
  const int nbr = NBR < GP_MAX_BRANCHES ? NBR : a.nbranch;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int total = (int)(a.B * a.ntok);
  const int row0 = (int)blockIdx.x * tpb;    // tpb <= kV3Tok tokens of this block (the launch balances them)
  // kTab (packed slides): the slide of the block's first token (wave-uniform binary search); a block of at most
  // kV3Tok tokens meets at most two slides (every slide holds more tokens than that, checked by the launch)
  int slide0 = 0;
  if constexpr (kTab) {
    int lo = 0, hi = a.nslide - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((int64_t)row0 >= a.tok_off[mid]) lo = mid; else hi = mid - 1;
    }
    slide0 = __builtin_amdgcn_readfirstlane(lo);
  }
  // ---- stage: lane t loads, for token row0 + t, the covered heads' lse of every branch (wave w: heads h' = w mod 4)
  if constexpr (!kTab) {
    if (lane < tpb) {
      const int tl = lane;
      const int row = row0 + tl;
      const bool live = row < total;
      const int rr = live ? row : total - 1;
      const int bidx = (int)div_magic((uint32_t)rr, a.dnt);
      const int p = (int)a.tok_lo + (rr - bidx * (int)a.ntok);
#pragma unroll
      for (int b = 0; b < NBR; ++b) {
        if (b < nbr) {
          const MergeBranch& mb = a.br[b];
          const int pn = (int)div_magic((uint32_t)p, mb.dg);
          const int pt = p - pn * mb.g.g;
          const int pi = (int)div_magic((uint32_t)pt, mb.dr);
          const int pj = pt - pi * mb.g.r;
          const int hpg = mb.g.hpg;
          const uint32_t rb = (uint32_t)(bidx * mb.g.nseg + pn);
          const float* lrow = mb.lse + (size_t)rb * (uint32_t)(H * mb.g.m) + (uint32_t)pi;
          for (int hq = wv; hq < hpg; hq += 4) {
            const float v = lrow[(size_t)(uint32_t)(pj * hpg + hq) * (uint32_t)mb.g.m];
            lse_s[tl * LS + b * 16 + hq] = v;
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int pass = 0; pass < (kTab ? 2 : 1); ++pass) {
      int s_lo = 0, s_hi = total;
      MergeBranch tb[kTab ? NBR : 1];
      if constexpr (kTab) {
        const int sl = slide0 + pass;
        if (sl >= a.nslide) break;
        s_lo = (int)a.tok_off[sl];
        s_hi = (int)a.tok_off[sl + 1];
#pragma unroll
        for (int b = 0; b < NBR; ++b)
          if (b < nbr) tb[b] = a.mtab[sl * a.nbranch + b];
      }
      const int tl = lane;
      const int row = row0 + tl;
      if (tl < tpb && row < total && row >= s_lo && row < s_hi) {
        int bidx = 0, p;
        if constexpr (kTab) {
          p = row - s_lo;
        } else {
          bidx = (int)div_magic((uint32_t)row, a.dnt);
          p = (int)a.tok_lo + (row - bidx * (int)a.ntok);
        }
#pragma unroll
        for (int b = 0; b < NBR; ++b) {
          if (b < nbr) {
            const MergeBranch& mb = kTab ? tb[b] : a.br[b];
            const int pn = (int)div_magic((uint32_t)p, mb.dg);
            const int pt = p - pn * mb.g.g;
            const int pi = (int)div_magic((uint32_t)pt, mb.dr);
            const int pj = pt - pi * mb.g.r;
            const int hpg = mb.g.hpg;
            const uint32_t rb = (uint32_t)(bidx * mb.g.nseg + pn);
            const float* lrow = mb.lse + (size_t)rb * (uint32_t)(H * mb.g.m) + (uint32_t)pi;
            for (int hq = wv; hq < hpg; hq += 4) {
              const float v = lrow[(size_t)(uint32_t)(pj * hpg + hq) * (uint32_t)mb.g.m];
              lse_s[tl * LS + b * 16 + hq] = v;
            }
          }
        }
      }
    }
  }
  __syncthreads();
  // ---- merge: wave wv takes tokens wv, wv + 4, ..., as branch_merge_v2_kernel (kMap 1, "x8") does one token
  const int kq = lane & 3;
  (void)kq;
  const int h0 = lane / 6, h1 = (128 + lane) / 12;
  const int c0 = 8 * lane, c1 = 512 + 4 * lane;
  const bool ln = a.ln_w != nullptr;
  const float* lw = ln ? a.ln_w : reinterpret_cast<const float*>(a.out);
  const float* lb = ln ? a.ln_b : reinterpret_cast<const float*>(a.out);
  float w0[8], w1[4], b0[8], b1[4];
  load_f32<8>(lw + c0, w0);
  load_f32<4>(lw + c1, w1);
  load_f32<8>(lb + c0, b0);
  load_f32<4>(lb + c1, b1);
  // kTab: the first slide's entries, loaded once for the wave's tokens (its tokens ascend, so a crossing into
  // the next slide happens at most once)
  MergeBranch tb[kTab ? NBR : 1];
  int t_sl = 0, t_base = 0, t_bnd = INT_MAX;
  if constexpr (kTab) {
    t_sl = slide0;
    t_base = (int)a.tok_off[slide0];
    t_bnd = slide0 + 1 < a.nslide ? (int)a.tok_off[slide0 + 1] : INT_MAX;
#pragma unroll
    for (int b = 0; b < NBR; ++b)
      if (b < nbr) tb[b] = merge_entry_scalar(a.mtab, slide0 * a.nbranch + b);
  }
  for (int k = 0; k < kV3Tok / 4; ++k) {
    const int t = wv + 4 * k;
    const int row = row0 + t;
    if (t >= tpb || row >= total) break;
    int bidx = 0, p;
    if constexpr (kTab) {
      if (row >= t_bnd) {                    // this wave's tokens crossed into the next slide (rare): switch tables
        t_sl += 1;
        t_base = t_bnd;
        t_bnd = t_sl + 1 < a.nslide ? (int)a.tok_off[t_sl + 1] : INT_MAX;
#pragma unroll
        for (int b = 0; b < NBR; ++b)
          if (b < nbr) tb[b] = merge_entry_scalar(a.mtab, t_sl * a.nbranch + b);
      }
      p = row - t_base;
    } else {
      bidx = (int)div_magic((uint32_t)row, a.dnt);
      p = (int)a.tok_lo + (row - bidx * (int)a.ntok);
    }
    uint4 o0[NBR];
    uint2 o1[NBR];
    float l0[NBR], l1[NBR];
    bool cv0[NBR], cv1[NBR];
#pragma unroll
    for (int b = 0; b < NBR; ++b) {
      cv0[b] = cv1[b] = false;
      l0[b] = l1[b] = -1e8f;
      o0[b] = make_uint4(0, 0, 0, 0);
      o1[b] = make_uint2(0, 0);
      if (b < nbr) {
        const MergeBranch& mb = kTab ? tb[b] : a.br[b];
        const int pn = (int)div_magic((uint32_t)p, mb.dg);
        const int pt = p - pn * mb.g.g;
        const int pi = (int)div_magic((uint32_t)pt, mb.dr);
        const int pj = pt - pi * mb.g.r;
        const int hpg = mb.g.hpg;
        const int hf = pj * hpg;
        const uint32_t rb = (uint32_t)(bidx * mb.g.nseg + pn);
        const char* orow = reinterpret_cast<const char*>(mb.o) + (rb * (uint32_t)mb.g.m + (uint32_t)pi) * (uint32_t)(E * 2);
        cv0[b] = (unsigned)(h0 - hf) < (unsigned)hpg;
        cv1[b] = (unsigned)(h1 - hf) < (unsigned)hpg;
        l0[b] = lse_s[t * LS + b * 16 + (cv0[b] ? h0 - hf : 0)];
        l1[b] = lse_s[t * LS + b * 16 + (cv1[b] ? h1 - hf : 0)];
        o0[b] = *reinterpret_cast<const uint4*>(orow + opaque_u32(cv0[b] ? 2 * c0 : 2 * D * hf));
        o1[b] = *reinterpret_cast<const uint2*>(orow + opaque_u32(cv1[b] ? 2 * c1 : 2 * D * hf));
      }
    }
    float mx0 = -INFINITY, mx1 = -INFINITY;
#pragma unroll
    for (int b = 0; b < NBR; ++b)
      if (b < nbr) {
        if (!cv0[b] || l0[b] == 0.f) l0[b] = -1e8f;   // dilated_attention.py:46
        mx0 = fmaxf(mx0, l0[b]);
        if (!cv1[b] || l1[b] == 0.f) l1[b] = -1e8f;
        mx1 = fmaxf(mx1, l1[b]);
      }
    float ws0 = 0.f, ws1 = 0.f;
#pragma unroll
    for (int b = 0; b < NBR; ++b)
      if (b < nbr) {
        l0[b] = fast_exp2((l0[b] - mx0) * 1.44269504088896340736f);
        ws0 += l0[b];
        l1[b] = fast_exp2((l1[b] - mx1) * 1.44269504088896340736f);
        ws1 += l1[b];
      }
    const float inv0 = __builtin_amdgcn_rcpf(ws0), inv1 = __builtin_amdgcn_rcpf(ws1);
    float v[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) v[e] = 0.f;
#pragma unroll
    for (int b = 0; b < NBR; ++b)
      if (b < nbr) {
        const float wb0 = cv0[b] ? l0[b] * inv0 : 0.f;
        const float wb1 = cv1[b] ? l1[b] * inv1 : 0.f;
        const uint32_t u0[4] = {o0[b].x, o0[b].y, o0[b].z, o0[b].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[2 * q] = __builtin_fmaf(e2f<kH>(u0[q]), wb0, v[2 * q]);
          v[2 * q + 1] = __builtin_fmaf(e2f_hi<kH>(u0[q]), wb0, v[2 * q + 1]);
        }
        v[8] = __builtin_fmaf(e2f<kH>(o1[b].x), wb1, v[8]);
        v[9] = __builtin_fmaf(e2f_hi<kH>(o1[b].x), wb1, v[9]);
        v[10] = __builtin_fmaf(e2f<kH>(o1[b].y), wb1, v[10]);
        v[11] = __builtin_fmaf(e2f_hi<kH>(o1[b].y), wb1, v[11]);
      }
    if (ln) {
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 12; ++e) s += v[e];
      const float mean = wave_sum_xor(s) * (1.0f / E);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 12; ++e) {
        const float d = v[e] - mean;
        q = __builtin_fmaf(d, d, q);
      }
      const float rstd = rsqrtf(__builtin_fmaf(wave_sum_xor(q), 1.0f / E, a.eps));
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = __builtin_fmaf((v[e] - mean) * rstd, w0[e], b0[e]);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[8 + e] = __builtin_fmaf((v[8 + e] - mean) * rstd, w1[e], b1[e]);
    }
    char* orow = reinterpret_cast<char*>(a.out) + (int64_t)row * (E * 2);
    *reinterpret_cast<uint4*>(orow + 2 * c0) =
        make_uint4(pack2e<kH>(v[0], v[1]), pack2e<kH>(v[2], v[3]), pack2e<kH>(v[4], v[5]), pack2e<kH>(v[6], v[7]));
    *reinterpret_cast<uint2*>(orow + 2 * c1) = make_uint2(pack2e<kH>(v[8], v[9]), pack2e<kH>(v[10], v[11]));
  }
}

// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dilated_gather_kernel(const uint16_t* __restrict__ src, int64_t row_stride,
                                                             int64_t col_off, int64_t L, int H, int D, GpBranch g,
                                                             int64_t total_rows, uint16_t* __restrict__ dst) {
  const int CH = D / 8;
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = id / CH;
  if (row >= total_rows) return;
  const int ch = (int)(id % CH);
  const int i = (int)(row % g.m);
  const int64_t t = row / g.m;
  const int hh = (int)(t % H);
  const int64_t bn = t / H;
  const int64_t bidx = bn / g.nseg;
  const int n = (int)(bn % g.nseg);
  const int j = hh / g.hpg;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (i < gp_valid_rows(g, L, n, j)) {
    const int64_t tok = bidx * L + (int64_t)n * g.s + j + (int64_t)i * g.r;
    v = *reinterpret_cast<const uint4*>(src + tok * row_stride + col_off + hh * D + ch * 8);
  }
  *reinterpret_cast<uint4*>(dst + row * D + ch * 8) = v;
}

}  // namespace

// =========================================================================================
extern "C" int gp_dilated_gather(const uint16_t* src, int64_t row_stride, int64_t col_off, int64_t B, int64_t L,
                                 int H, int D, int sl, int r, uint16_t* dst, void* stream) {
  GP_REQUIRE(B > 0 && L > 0 && H > 0 && D > 0 && sl > 0 && r > 0, "gp_dilated_gather: bad sizes");
  GP_REQUIRE(D % 8 == 0 && row_stride % 8 == 0 && col_off % 8 == 0 && row_stride >= col_off + (int64_t)H * D,
             "gp_dilated_gather: D, row_stride and col_off must be multiples of 8 elements");
  GP_REQUIRE(src && dst && gp_aligned(src, 16) && gp_aligned(dst, 16), "gp_dilated_gather: pointers must be 16-byte aligned");
  const GpBranch g = gp_make_branch(L, sl, r, H);
  const int64_t rows = B * g.nseg * (int64_t)H * g.m;
  const int64_t chunks = rows * (D / 8);
  dilated_gather_kernel<<<(unsigned)((chunks + 255) / 256), 256, 0, gp_stream(stream)>>>(src, row_stride, col_off, L,
                                                                                         H, D, g, rows, dst);
  return gp_check_launch("gp_dilated_gather");
}

static int attn_num_cus(hipStream_t s) {     // per-device cache of the CU count
  static int cache[64] = {0};
  int dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// An LDS-DMA launch whose 8-wave work items cannot fill the GPU (fewer items than the 3 per CU that are
// resident at once: the long-branch launch of a sequence-parallel rank holds ~384 for 768 slots) runs 4-wave
// workgroups of 128 queries instead -- twice the items, each K/V tile shared by half as many queries.  Same
// per-query arithmetic: bit-identical outputs (round 5).  0 disables.
#ifndef GP_ATTN_SMALL_LAUNCH_NW4
#define GP_ATTN_SMALL_LAUNCH_NW4 1
#endif
// (8-wave items per CU below which a launch counts as under-filled)
#ifndef GP_ATTN_SMALL_LAUNCH_PER_CU
#define GP_ATTN_SMALL_LAUNCH_PER_CU 3
#endif

extern "C" int gp_attn_launch_params(int32_t* params, int n) {
  GP_REQUIRE(params && n >= 0, "gp_attn_launch_params: null params");
  const int32_t v[4] = {32 * kNWFast, GP_ATTN_FAST_WPS * 4 / kNWFast,
                        GP_ATTN_SMALL_LAUNCH_NW4 ? GP_ATTN_SMALL_LAUNCH_PER_CU : 0, 64};
  for (int i = 0; i < n && i < 4; ++i) params[i] = v[i];
  return 0;
}

// fmt: GP_FMT_BF16, GP_FMT_F16 (fp16 q / k / v) or GP_FMT_F16_VBF16 (fp16 q / k, bf16 v; o fp16)
static int attn_fwd_impl(const uint16_t* q, int64_t q_row_stride, int64_t q_tok_base, int64_t B, int64_t L, int H,
                         int D, int64_t win_lo, int64_t win_hi, const GpAttnBranch* branches, int nbranch,
                         float softmax_scale, int q_log2_prescaled, int fmt, void* stream) {
  const bool kh = fmt != GP_FMT_BF16;
  // bf16: the no-max LDS-DMA kernel + fixup pass (kModeFast / kModeFix) when the layout allows LDS-DMA
  // staging, else the register-staged exact kernel; fp16 likewise (its fast mode offsets p by the
  // row max of tile 0)
  GP_REQUIRE(D == 48 || D == 64 || D == 96, "gp_dilated_attn_fwd: head dim %d unsupported (48, 64, 96)", D);
  GP_REQUIRE(nbranch >= 1 && nbranch <= GP_MAX_BRANCHES, "gp_dilated_attn_fwd: nbranch must be 1..%d", GP_MAX_BRANCHES);
  GP_REQUIRE(B > 0 && L > 0 && H > 0 && q_row_stride >= (int64_t)H * D && q_row_stride % 8 == 0,
             "gp_dilated_attn_fwd: bad sizes");
  GP_REQUIRE(B * L < (int64_t)0x7fffffff, "gp_dilated_attn_fwd: B*L too large");
  GP_REQUIRE(0 <= win_lo && win_lo <= win_hi && win_hi <= L, "gp_dilated_attn_fwd: bad window [%lld, %lld) for L=%lld",
             (long long)win_lo, (long long)win_hi, (long long)L);
  GP_REQUIRE(q && branches, "gp_dilated_attn_fwd: null pointer");
  GP_REQUIRE(gp_aligned(q, 16), "gp_dilated_attn_fwd: q must be 16-byte aligned");
  if (win_lo == win_hi) return 0;
  AttnArgs a;
  a.q = q;
  a.q_stride = q_row_stride;
  a.q_tok_base = q_tok_base;
  a.L = L;
  a.win_lo = win_lo;
  a.win_hi = win_hi;
  a.H = H;
  a.nbranch = nbranch;
  const float scale = softmax_scale > 0.f ? softmax_scale : 1.0f / sqrtf((float)D);
  a.c_log2 = q_log2_prescaled ? 1.0f : scale * 1.44269504088896340736f;
  GP_REQUIRE(!q_log2_prescaled || D != 96, "gp_dilated_attn_fwd: q_log2_prescaled needs D in {48, 64}");
  // LDS-DMA staging addresses V as K + dv inside one buffer descriptor whose record count ends at
  // the last valid row: needs v at or after k in memory, a row stride that covers dv + one head
  // (rows past c then fall outside the records) and 32-bit tile offsets
  bool kv_desc_ok = true;
  for (int b = 0; b < nbranch; ++b) {
    const GpAttnBranch& d = branches[b];
    const int64_t dv = (int64_t)((const char*)d.v - (const char*)d.k);
    const int64_t rs2 = 2 * d.kv_row_stride;
    kv_desc_ok = kv_desc_ok && dv >= 0 && rs2 >= dv + 2 * D && dv + 64 * (int64_t)d.ratio * rs2 < 0x7fffffff;
  }
  const bool fast = D == 48 && q_log2_prescaled && kv_desc_ok;   // LDS-DMA staging (8 waves x 32 queries)
  GP_REQUIRE(fmt != GP_FMT_F16_VBF16 || fast,
             "gp_dilated_attn_fwd: fmt F16_VBF16 needs D = 48, a pre-scaled q and k / v in one row layout");
  hipStream_t s = gp_stream(stream);
  // query rows per workgroup; an under-filled 8-wave LDS-DMA launch of the bf16 / V-bf16 pair goes to 4 waves
  // (the item count is computed for 8 first, below)
  const bool small_ok = GP_ATTN_SMALL_LAUNCH_NW4 && fast && kNWFast == 8 && (fmt == GP_FMT_BF16 || fmt == GP_FMT_F16_VBF16);
  int qblk = fast ? 32 * kNWFast : 128;
  // order branches by keys per work item (descending) so the longest items start first
  int order[GP_MAX_BRANCHES];
  GpBranch geo[GP_MAX_BRANCHES];
  for (int b = 0; b < nbranch; ++b) {
    const GpAttnBranch& d = branches[b];
    GP_REQUIRE(d.seg_len > 0 && d.ratio > 0, "gp_dilated_attn_fwd: branch %d has sl=%d r=%d", b, d.seg_len, d.ratio);
    GP_REQUIRE(d.key_parts <= 1 || (d.key_part >= 0 && d.key_part < d.key_parts && d.key_parts <= 64 && D != 96),
               "gp_dilated_attn_fwd: branch %d key part %d of %d (0 <= part < parts <= 64, D != 96)", b, d.key_part,
               d.key_parts);
    GP_REQUIRE(d.o && d.lse && gp_aligned(d.o, 8), "gp_dilated_attn_fwd: branch %d output null/misaligned", b);
    GP_REQUIRE(d.k && d.v && gp_aligned(d.k, 16) && gp_aligned(d.v, 16) && d.kv_row_stride % 8 == 0,
               "gp_dilated_attn_fwd: branch %d k/v must be 16-byte aligned with a row stride multiple of 8", b);
    geo[b] = gp_make_branch(L, d.seg_len, d.ratio, H);
    GP_REQUIRE(!d.kv_sparse_cols || H % d.ratio == 0, "gp_dilated_attn_fwd: sparse k/v columns need H %% r == 0");
    GP_REQUIRE(d.kv_row_stride >= (int64_t)(d.kv_sparse_cols ? geo[b].hpg : H) * D,
               "gp_dilated_attn_fwd: branch %d k/v row stride too small", b);
    order[b] = b;
  }
  for (int x = 1; x < nbranch; ++x)
    for (int y = x; y > 0 && geo[order[y]].m > geo[order[y - 1]].m; --y) {
      int tmp = order[y]; order[y] = order[y - 1]; order[y - 1] = tmp;
    }
  int64_t items = 0;
  auto plan_items = [&]() {
  items = 0;
  for (int x = 0; x < nbranch; ++x) {
    const int b = order[x];
    const GpBranch& g = geo[b];
    const GpAttnBranch& d = branches[b];
    AttnBranch& e = a.br[x];
    e.g = g;
    e.n_lo = (int32_t)(win_lo / g.g);
    const int32_t n_hi = (int32_t)((win_hi - 1) / g.g);
    e.nseg_w = n_hi - e.n_lo + 1;
    // q-blocks per (segment, head): the largest window row count over the segments and phases
    int most = 0;
    for (int32_t n = e.n_lo; n <= n_hi; ++n) {
      for (int j = 0; j < g.r; ++j) {
        const int64_t base = (int64_t)n * g.g + j;
        const int64_t lo = win_lo > base ? (win_lo - base + g.r - 1) / g.r : 0;
        int64_t hi = win_hi > base ? (win_hi - base + g.r - 1) / g.r : 0;
        if (hi > g.m) hi = g.m;
        if (hi - lo > most) most = (int)(hi - lo);
      }
      if (n > e.n_lo + 1 && n < n_hi - 1) n = n_hi - 2;   // interior segments are all full: skip ahead
    }
    e.nqb = (most + qblk - 1) / qblk;
    if (e.nqb == 0) e.nqb = 1;
    e.item_begin = items;
    e.k = d.k;
    e.v = d.v;
    e.kv_stride = d.kv_row_stride;
    e.kv_tok_base = d.kv_tok_base;
    e.kv_sparse = d.kv_sparse_cols ? 1 : 0;
    e.o = d.o;
    e.lse = d.lse;
    e.kpart = d.key_parts > 1 ? d.key_part : 0;
    e.kparts = d.key_parts > 1 ? d.key_parts : 1;
    attn_branch_magic(e);
    items += B * (int64_t)e.nseg_w * H * e.nqb;
  }
  };
  plan_items();
  bool parts = false;
  for (int b = 0; b < nbranch; ++b) parts = parts || branches[b].key_parts > 1;
  GP_REQUIRE(!parts || (fast && kNWFast == 8 && (fmt == GP_FMT_BF16 || fmt == GP_FMT_F16_VBF16)),
             "gp_dilated_attn_fwd: key parts need the LDS-DMA bf16 pair (D = 48, pre-scaled q, k / v in one layout)");
  bool nw4 = false;
  if (small_ok && !parts && items < GP_ATTN_SMALL_LAUNCH_PER_CU * (int64_t)attn_num_cus(s)) {
    qblk = 128;
    nw4 = true;
    plan_items();
  }
  for (int x = nbranch; x < GP_MAX_BRANCHES; ++x) a.br[x] = a.br[nbranch - 1];
  a.total_items = items;
  a.d_H = make_div_magic((uint32_t)H);
  a.tab = nullptr;
  a.ntab = 0;
  GP_REQUIRE(items < (int64_t)0x7fffffff, "gp_dilated_attn_fwd: too many work items");
  if (parts) {   // key parts (sequence-parallel under-filled launches): the 8-wave pair built with parts
    if (fmt == GP_FMT_F16_VBF16) {
      dilated_attn32_kernel<48, true, kModeFast, false, 8, true, true><<<(unsigned)items, 512, 0, s>>>(a);
      if constexpr (GP_ATTN_NOFIX == 0)
        dilated_attn32_kernel<48, true, kModeFix, false, 8, true, true><<<(unsigned)((items + kFixItems - 1) / kFixItems), 512, 0, s>>>(a);
    } else {
      dilated_attn32_kernel<48, true, kModeFast, false, 8, false, true><<<(unsigned)items, 512, 0, s>>>(a);
      if constexpr (GP_ATTN_NOFIX == 0)
        dilated_attn32_kernel<48, true, kModeFix, false, 8, false, true><<<(unsigned)((items + kFixItems - 1) / kFixItems), 512, 0, s>>>(a);
    }
    return gp_check_launch("gp_dilated_attn_fwd");
  }
  if (nw4) {   // the under-filled launch in 4-wave workgroups (fast pair only)
    if (fmt == GP_FMT_F16_VBF16) {
      dilated_attn32_kernel<48, true, kModeFast, false, 4, true><<<(unsigned)items, 256, 0, s>>>(a);
      if constexpr (GP_ATTN_NOFIX == 0)
        dilated_attn32_kernel<48, true, kModeFix, false, 4, true><<<(unsigned)((items + kFixItems - 1) / kFixItems), 256, 0, s>>>(a);
    } else {
      dilated_attn32_kernel<48, true, kModeFast, false, 4><<<(unsigned)items, 256, 0, s>>>(a);
      if constexpr (GP_ATTN_NOFIX == 0)
        dilated_attn32_kernel<48, true, kModeFix, false, 4><<<(unsigned)((items + kFixItems - 1) / kFixItems), 256, 0, s>>>(a);
    }
    return gp_check_launch("gp_dilated_attn_fwd");
  }
  if (fmt == GP_FMT_F16_VBF16) {
    // fp16 q / k, bf16 v: the bf16 product pair with the fp16 S MFMA (no max; fixup pass)
    dilated_attn32_kernel<48, true, kModeFast, false, kNWFast, true><<<(unsigned)items, 64 * kNWFast, 0, s>>>(a);
    if constexpr (GP_ATTN_NOFIX == 0)
      dilated_attn32_kernel<48, true, kModeFix, false, kNWFast, true>
          <<<(unsigned)((items + kFixItems - 1) / kFixItems), 64 * kNWFast, 0, s>>>(a);
  } else if (kh) {
    if (fast) {        // fp16 v: the exact running-max kernel
      dilated_attn32_kernel<48, true, kModeExact, false, kNWFast, true><<<(unsigned)items, 64 * kNWFast, 0, s>>>(a);
    } else if (D == 96) dilated_attn_kernel<96, true><<<(unsigned)items, 256, 0, s>>>(a);
    else if (D == 48 && q_log2_prescaled) dilated_attn32_kernel<48, true, kModeGen, false, 4, true><<<(unsigned)items, 256, 0, s>>>(a);
    else if (D == 48) dilated_attn32_kernel<48, false, kModeGen, false, 4, true><<<(unsigned)items, 256, 0, s>>>(a);
    else if (q_log2_prescaled) dilated_attn32_kernel<64, true, kModeGen, false, 4, true><<<(unsigned)items, 256, 0, s>>>(a);
    else dilated_attn32_kernel<64, false, kModeGen, false, 4, true><<<(unsigned)items, 256, 0, s>>>(a);
  } else if (D == 96) {
    dilated_attn_kernel<96><<<(unsigned)items, 256, 0, s>>>(a);
  } else if (fast) {
    // the product launch: no-max kernel, then the fixup pass (exits at once unless a row was flagged)
    dilated_attn32_kernel<48, true, kModeFast, false, kNWFast><<<(unsigned)items, 64 * kNWFast, 0, s>>>(a);
    if constexpr (GP_ATTN_NOFIX == 0)
      dilated_attn32_kernel<48, true, kModeFix, false, kNWFast>
          <<<(unsigned)((items + kFixItems - 1) / kFixItems), 64 * kNWFast, 0, s>>>(a);
  } else if (D == 48) {
    if (q_log2_prescaled) dilated_attn32_kernel<48, true, kModeGen><<<(unsigned)items, 256, 0, s>>>(a);
    else dilated_attn32_kernel<48, false, kModeGen><<<(unsigned)items, 256, 0, s>>>(a);
  } else {
    if (q_log2_prescaled) dilated_attn32_kernel<64, true, kModeGen><<<(unsigned)items, 256, 0, s>>>(a);
    else dilated_attn32_kernel<64, false, kModeGen><<<(unsigned)items, 256, 0, s>>>(a);
  }
  return gp_check_launch("gp_dilated_attn_fwd");
}

extern "C" int gp_dilated_attn_fwd_ex(const uint16_t* q, int64_t q_row_stride, int64_t q_tok_base, int64_t B,
                                      int64_t L, int H, int D, int64_t win_lo, int64_t win_hi,
                                      const GpAttnBranch* branches, int nbranch, float softmax_scale,
                                      int q_log2_prescaled, int fmt, void* stream) {
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16 || fmt == GP_FMT_F16_VBF16, "gp_dilated_attn_fwd: bad fmt %d", fmt);
  return attn_fwd_impl(q, q_row_stride, q_tok_base, B, L, H, D, win_lo, win_hi, branches, nbranch, softmax_scale,
                       q_log2_prescaled, fmt, stream);
}

extern "C" int gp_dilated_attn_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, int64_t row_stride,
                                   int64_t B, int64_t L, int H, int D, const int32_t* seg_len, const int32_t* ratios,
                                   int nbranch, uint16_t* const* o_out, float* const* lse_out, float softmax_scale,
                                   int q_log2_prescaled, int fmt, void* stream) {
  GP_REQUIRE(D == 48 || D == 64 || D == 96, "gp_dilated_attn_fwd: head dim %d unsupported (48, 64, 96)", D);
  GP_REQUIRE(nbranch >= 1 && nbranch <= GP_MAX_BRANCHES, "gp_dilated_attn_fwd: nbranch must be 1..%d", GP_MAX_BRANCHES);
  GP_REQUIRE(k && v && seg_len && ratios && o_out && lse_out, "gp_dilated_attn_fwd: null pointer");
  GpAttnBranch br[GP_MAX_BRANCHES] = {};
  for (int b = 0; b < nbranch; ++b) {
    br[b].seg_len = seg_len[b];
    br[b].ratio = ratios[b];
    br[b].k = k;
    br[b].v = v;
    br[b].kv_row_stride = row_stride;
    br[b].kv_tok_base = 0;
    br[b].kv_sparse_cols = 0;
    br[b].o = o_out[b];
    br[b].lse = lse_out[b];
  }
  return gp_dilated_attn_fwd_ex(q, row_stride, 0, B, L, H, D, 0, L, br, nbranch, softmax_scale, q_log2_prescaled,
                                fmt, stream);
}

static int seg_attn(const uint16_t* q, const uint16_t* k, const uint16_t* v, int64_t nbatch, int64_t seqlen, int H,
                    int D, float softmax_scale, uint16_t* o, float* lse, bool kh, void* stream) {
  GP_REQUIRE(seqlen > 0 && seqlen < (int64_t)0x7fffffff, "gp_seg_attn_fwd: bad seqlen");
  GP_REQUIRE(k && v && o && lse, "gp_seg_attn_fwd: null pointer");
  GpAttnBranch br = {};
  br.seg_len = (int32_t)seqlen;
  br.ratio = 1;
  br.k = k;
  br.v = v;
  br.kv_row_stride = (int64_t)H * D;
  br.kv_tok_base = 0;
  br.kv_sparse_cols = 0;
  br.o = o;
  br.lse = lse;
  return attn_fwd_impl(q, (int64_t)H * D, 0, nbatch, seqlen, H, D, 0, seqlen, &br, 1, softmax_scale, 0,
                       kh ? GP_FMT_F16 : GP_FMT_BF16, stream);
}

extern "C" int gp_seg_attn_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, int64_t nbatch,
                               int64_t seqlen, int H, int D, float softmax_scale, uint16_t* o, float* lse,
                               void* stream) {
  return seg_attn(q, k, v, nbatch, seqlen, H, D, softmax_scale, o, lse, false, stream);
}

extern "C" int gp_seg_attn_fwd_f16(const uint16_t* q, const uint16_t* k, const uint16_t* v, int64_t nbatch,
                                   int64_t seqlen, int H, int D, float softmax_scale, uint16_t* o, float* lse,
                                   void* stream) {
  return seg_attn(q, k, v, nbatch, seqlen, H, D, softmax_scale, o, lse, true, stream);
}

extern "C" int gp_branch_merge_ln(const uint16_t* const* o_in, const float* const* lse_in, const int32_t* seg_len,
                                  const int32_t* ratios, int nbranch, int64_t B, int64_t L, int H, int D,
                                  const float* ln_w, const float* ln_b, float eps, uint16_t* out, int fmt,
                                  void* stream) {
  return gp_branch_merge_ln_window(o_in, lse_in, seg_len, ratios, nbranch, B, L, 0, L, H, D, ln_w, ln_b, eps, out,
                                   fmt, stream);
}

// the E = 768 / D = 48 merge: one token per wave, 4 waves per block
static unsigned merge_v2_grid(int64_t tokens) { return (unsigned)((tokens + GP_MERGE_WPB - 1) / GP_MERGE_WPB); }
// its 32-bit byte offsets: every branch's o rows (B * nseg * m rows of 1,536 B) below 4 GiB
static bool merge_v2_fits(const MergeArgs& a) {
  for (int b = 0; b < a.nbranch; ++b)
    if ((uint64_t)a.B * a.br[b].g.nseg * a.br[b].g.m * 1536u >= (1ull << 32)) return false;
  return true;
}

template <bool kH>
static void launch_merge(const MergeArgs& a, int E, int D, int nbranch, unsigned nb, hipStream_t s) {
  switch (E) {
    case 768:
      // (5 entries only: the 7 / 8-entry instantiations need 134-145 VGPRs and spill SGPRs; they keep the v2 kernel)
      if (GP_MERGE_V3 != 0 && D == 48 && nbranch == 5 && merge_v2_fits(a)) {
        // tokens per block: the blocks spread evenly over the CUs -- the kernel is bound per CU (outstanding L2
        // requests), so a CU holding one block more than another finishes a block's time later (70k: 9 blocks of
        // 31 tokens per CU; 256k: 32 blocks of 32)
        const int64_t T = a.B * a.ntok;
        const int64_t ncu = attn_num_cus(s);
        const int64_t per_cu = (T + ncu * kV3Tok - 1) / (ncu * kV3Tok);
        const int tpb = (int)std::max<int64_t>(1, (T + ncu * per_cu - 1) / (ncu * per_cu));
        const unsigned g = (unsigned)((T + tpb - 1) / tpb);
        branch_merge_v3_kernel<5, kH><<<g, 256, 0, s>>>(a, tpb);
      } else if (D == 48 && merge_v2_fits(a)) {
        const unsigned g = merge_v2_grid(a.B * a.ntok);
        if (nbranch == 5) branch_merge_v2_kernel<5, false, kH><<<g, 64 * GP_MERGE_WPB, 0, s>>>(a);
        // (5 branches, two of them in two key parts: the sequence-parallel long-branch split, seqpar.plan_key_parts)
        else if (nbranch == 7) branch_merge_v2_kernel<7, false, kH><<<g, 64 * GP_MERGE_WPB, 0, s>>>(a);
        else branch_merge_v2_kernel<GP_MAX_BRANCHES, false, kH><<<g, 64 * GP_MERGE_WPB, 0, s>>>(a);
      } else if (D == 96) branch_merge_kernel<12, 96, false, GP_MAX_BRANCHES, kH><<<nb, 256, 0, s>>>(a);
      else branch_merge_kernel<12, 12, false, GP_MAX_BRANCHES, kH><<<nb, 256, 0, s>>>(a);
      break;
    case 1024:
      if (D == 64) branch_merge_kernel<16, 64, false, GP_MAX_BRANCHES, kH><<<nb, 256, 0, s>>>(a);
      else branch_merge_kernel<16, 16, false, GP_MAX_BRANCHES, kH><<<nb, 256, 0, s>>>(a);
      break;
    case 1536:
      if (D == 96) branch_merge_kernel<24, 96, false, GP_MAX_BRANCHES, kH><<<nb, 256, 0, s>>>(a);
      else if (D == 48) branch_merge_kernel<24, 48, false, GP_MAX_BRANCHES, kH><<<nb, 256, 0, s>>>(a);
      else branch_merge_kernel<24, 24, false, GP_MAX_BRANCHES, kH><<<nb, 256, 0, s>>>(a);
      break;
  }
}

extern "C" int gp_branch_merge_ln_window(const uint16_t* const* o_in, const float* const* lse_in,
                                         const int32_t* seg_len, const int32_t* ratios, int nbranch, int64_t B,
                                         int64_t L, int64_t tok_lo, int64_t n_tok, int H, int D, const float* ln_w,
                                         const float* ln_b, float eps, uint16_t* out, int fmt, void* stream) {
  const int E = H * D;
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16, "gp_branch_merge_ln: bad fmt %d", fmt);
  GP_REQUIRE(nbranch >= 1 && nbranch <= GP_MAX_BRANCHES, "gp_branch_merge_ln: nbranch must be 1..%d", GP_MAX_BRANCHES);
  GP_REQUIRE((E == 768 && (D == 48 || D == 96 || D == 12)) || (E == 1024 && (D == 64 || D == 16)) ||
                 (E == 1536 && (D == 96 || D == 48 || D == 24)),
             "gp_branch_merge_ln: H*D=%d with D=%d unsupported", E, D);
  GP_REQUIRE(B * L < (int64_t)0x7fffffff, "gp_branch_merge_ln: B*L too large");
  GP_REQUIRE(B > 0 && L > 0 && tok_lo >= 0 && n_tok >= 0 && tok_lo + n_tok <= L, "gp_branch_merge_ln: bad sizes");
  if (n_tok == 0) return 0;
  GP_REQUIRE(o_in && lse_in && seg_len && ratios && out, "gp_branch_merge_ln: null pointer");
  GP_REQUIRE(ln_w == nullptr || ln_b != nullptr, "gp_branch_merge_ln: ln_w without ln_b");
  MergeArgs a;
  a.B = B; a.L = L; a.H = H; a.D = D; a.E = E; a.nbranch = nbranch;
  a.tok_lo = tok_lo; a.ntok = n_tok;
  a.dnt = make_div_magic((uint32_t)n_tok);
  for (int b = 0; b < nbranch; ++b) {
    GP_REQUIRE(seg_len[b] > 0 && ratios[b] > 0 && o_in[b] && lse_in[b], "gp_branch_merge_ln: bad branch %d", b);
    a.br[b].g = gp_make_branch(L, seg_len[b], ratios[b], H);
    a.br[b].o = o_in[b];
    a.br[b].lse = lse_in[b];
    merge_branch_magic(a.br[b]);
  }
  for (int b = nbranch; b < GP_MAX_BRANCHES; ++b) a.br[b] = a.br[nbranch - 1];
  a.ln_w = ln_w; a.ln_b = ln_b; a.eps = eps; a.out = out;
  const unsigned nb = (unsigned)((B * n_tok + 4 * kTPW - 1) / (4 * kTPW));   // kTPW tokens per wave
  if (fmt == GP_FMT_F16) launch_merge<true>(a, E, D, nbranch, nb, gp_stream(stream));
  else launch_merge<false>(a, E, D, nbranch, nb, gp_stream(stream));
  return gp_check_launch("gp_branch_merge_ln");
}

// =========================================================================================
// Varlen packing (config C5): several slides concatenated token-major in one [T, 3E] qkv buffer
// (slide i at rows [tok_off[i], tok_off[i] + L_i)), one attention launch and one merge launch
// for all of them.  Every slide keeps its own segment schedule (s = min(sl, L_i), ...) and no
// query attends across slides, so each slide's outputs are those of its own B = 1 forward.
// The plan (host bytes, copied by the caller to device memory) holds the work table.
namespace {
constexpr int32_t kVarlenMagic = 0x47505631;   // "GPV1"
struct VarlenHdr {
  int32_t magic, nslide, nbranch, H, D, ntab;
  int64_t T, total_items, qkv_stride;
  int64_t tab_off, mtab_off, tok_off_off, bytes;
};
inline int64_t gp_align16(int64_t x) { return (x + 15) & ~int64_t(15); }
inline void varlen_layout(int nslide, int nbranch, VarlenHdr& h) {
  h.tab_off = gp_align16(sizeof(VarlenHdr));
  h.mtab_off = gp_align16(h.tab_off + (int64_t)nslide * nbranch * sizeof(AttnBranch));
  h.tok_off_off = gp_align16(h.mtab_off + (int64_t)nslide * nbranch * sizeof(MergeBranch));
  h.bytes = gp_align16(h.tok_off_off + (int64_t)(nslide + 1) * sizeof(int64_t));
}
}  // namespace

extern "C" int64_t gp_varlen_plan_bytes(int nslide, int nbranch) {
  if (nslide < 1 || nbranch < 1 || nbranch > GP_MAX_BRANCHES) return -1;
  VarlenHdr h;
  varlen_layout(nslide, nbranch, h);
  return h.bytes;
}

extern "C" int gp_varlen_plan(const int64_t* L, int nslide, int H, int D, const int32_t* seg_len,
                              const int32_t* ratios, int nbranch, const uint16_t* qkv, int64_t qkv_row_stride,
                              uint16_t* const* o_out, float* const* lse_out, void* plan_host, int64_t plan_bytes,
                              int64_t* o_elems, int64_t* lse_elems) {
  GP_REQUIRE(nslide >= 1 && L && seg_len && ratios && o_elems && lse_elems, "gp_varlen_plan: bad arguments");
  GP_REQUIRE(nbranch >= 1 && nbranch <= GP_MAX_BRANCHES, "gp_varlen_plan: nbranch must be 1..%d", GP_MAX_BRANCHES);
  GP_REQUIRE(H > 0 && D > 0 && qkv_row_stride >= 3LL * H * D && qkv_row_stride % 8 == 0, "gp_varlen_plan: bad sizes");
  int64_t T = 0;
  for (int i = 0; i < nslide; ++i) {
    GP_REQUIRE(L[i] > 0, "gp_varlen_plan: slide %d has L = %lld", i, (long long)L[i]);
    T += L[i];
  }
  GP_REQUIRE(T < (int64_t)0x7fffffff, "gp_varlen_plan: %lld packed tokens is too many", (long long)T);
  const int qblk = 32 * kNWFast;                   // query rows per work item (the LDS-DMA kernel)
  for (int b = 0; b < nbranch; ++b) { o_elems[b] = 0; lse_elems[b] = 0; }
  // per (slide, branch) output region offsets, in slide order
  std::vector<int64_t> ooff((size_t)nslide * nbranch), loff((size_t)nslide * nbranch);
  std::vector<GpBranch> geo((size_t)nslide * nbranch);
  for (int i = 0; i < nslide; ++i)
    for (int b = 0; b < nbranch; ++b) {
      GP_REQUIRE(seg_len[b] > 0 && ratios[b] > 0, "gp_varlen_plan: branch %d has sl=%d r=%d", b, seg_len[b], ratios[b]);
      const GpBranch g = gp_make_branch(L[i], seg_len[b], ratios[b], H);
      geo[(size_t)i * nbranch + b] = g;
      ooff[(size_t)i * nbranch + b] = o_elems[b];
      loff[(size_t)i * nbranch + b] = lse_elems[b];
      o_elems[b] += (int64_t)g.nseg * g.m * H * D;
      lse_elems[b] += (int64_t)g.nseg * H * g.m;
    }
  if (plan_host == nullptr) return 0;               // sizing call
  VarlenHdr h;
  varlen_layout(nslide, nbranch, h);
  GP_REQUIRE(plan_bytes >= h.bytes, "gp_varlen_plan: plan buffer %lld < %lld bytes", (long long)plan_bytes,
             (long long)h.bytes);
  GP_REQUIRE(qkv && o_out && lse_out, "gp_varlen_plan: null device pointer");
  for (int b = 0; b < nbranch; ++b) GP_REQUIRE(o_out[b] && lse_out[b], "gp_varlen_plan: branch %d output null", b);
  char* base = static_cast<char*>(plan_host);
  memset(base, 0, (size_t)h.bytes);
  AttnBranch* tab = reinterpret_cast<AttnBranch*>(base + h.tab_off);
  MergeBranch* mtab = reinterpret_cast<MergeBranch*>(base + h.mtab_off);
  int64_t* tok_off = reinterpret_cast<int64_t*>(base + h.tok_off_off);
  tok_off[0] = 0;
  for (int i = 0; i < nslide; ++i) tok_off[i + 1] = tok_off[i] + L[i];
  // attention entries heaviest first (keys per item), stable
  std::vector<int> order((size_t)nslide * nbranch);
  for (size_t x = 0; x < order.size(); ++x) order[x] = (int)x;
  std::stable_sort(order.begin(), order.end(), [&](int u, int v) { return geo[u].m > geo[v].m; });
  const int E = H * D;
  int64_t items = 0;
  for (size_t x = 0; x < order.size(); ++x) {
    const int id = order[x], i = id / nbranch, b = id % nbranch;
    const GpBranch& g = geo[id];
    AttnBranch& e = tab[x];
    e.g = g;
    e.nqb = (g.m + qblk - 1) / qblk;
    e.n_lo = 0;
    e.nseg_w = g.nseg;
    e.kv_sparse = 0;
    e.item_begin = items;
    const uint16_t* row0 = qkv + tok_off[i] * qkv_row_stride;
    e.q = row0;
    e.k = row0 + E;
    e.v = row0 + 2 * E;
    e.kv_stride = qkv_row_stride;
    e.kv_tok_base = 0;
    e.o = o_out[b] + ooff[id];
    e.lse = lse_out[b] + loff[id];
    e.L = L[i];
    attn_branch_magic(e);
    items += (int64_t)g.nseg * H * e.nqb;
  }
  for (int i = 0; i < nslide; ++i)
    for (int b = 0; b < nbranch; ++b) {
      MergeBranch& m = mtab[(size_t)i * nbranch + b];
      m.g = geo[(size_t)i * nbranch + b];
      m.o = o_out[b] + ooff[(size_t)i * nbranch + b];
      m.lse = lse_out[b] + loff[(size_t)i * nbranch + b];
      merge_branch_magic(m);
    }
  GP_REQUIRE(items < (int64_t)0x7fffffff, "gp_varlen_plan: too many work items");
  VarlenHdr* hp = reinterpret_cast<VarlenHdr*>(base);
  *hp = h;
  hp->magic = kVarlenMagic;
  hp->nslide = nslide;
  hp->nbranch = nbranch;
  hp->H = H;
  hp->D = D;
  hp->ntab = nslide * nbranch;
  hp->T = T;
  hp->total_items = items;
  hp->qkv_stride = qkv_row_stride;
  return 0;
}

static int varlen_header(const void* plan_host, const void* plan_dev, const char* who, VarlenHdr& h) {
  GP_REQUIRE(plan_host && plan_dev && gp_aligned(plan_dev, 16), "%s: null/misaligned plan", who);
  h = *static_cast<const VarlenHdr*>(plan_host);
  GP_REQUIRE(h.magic == kVarlenMagic, "%s: not a gp_varlen_plan buffer", who);
  return 0;
}

extern "C" int gp_dilated_attn_fwd_varlen(const void* plan_host, const void* plan_dev, int q_log2_prescaled,
                                          int fmt, void* stream) {
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16 || fmt == GP_FMT_F16_VBF16, "gp_dilated_attn_fwd_varlen: bad fmt %d",
             fmt);
  VarlenHdr h;
  if (int rc = varlen_header(plan_host, plan_dev, "gp_dilated_attn_fwd_varlen", h)) return rc;
  GP_REQUIRE(h.D == 48 && q_log2_prescaled, "gp_dilated_attn_fwd_varlen: needs D = 48 and a pre-scaled q (D=%d)", h.D);
  if (h.total_items == 0) return 0;
  AttnArgs a;
  memset(&a, 0, sizeof(a));
  a.q_stride = h.qkv_stride;
  a.H = h.H;
  a.nbranch = h.nbranch;
  a.c_log2 = 1.0f;
  a.total_items = h.total_items;
  a.tab = reinterpret_cast<const AttnBranch*>(static_cast<const char*>(plan_dev) + h.tab_off);
  a.ntab = h.ntab;
  a.d_H = make_div_magic((uint32_t)h.H);
  // the single-slide default's variant, so each packed slide's outputs equal its own launch's
  if (fmt == GP_FMT_F16) {
    dilated_attn32_kernel<48, true, kModeExact, true, kNWFast, true>
        <<<(unsigned)h.total_items, 64 * kNWFast, 0, gp_stream(stream)>>>(a);
    return gp_check_launch("gp_dilated_attn_fwd_varlen");
  }
  if (fmt == GP_FMT_F16_VBF16) {
    dilated_attn32_kernel<48, true, kModeFast, true, kNWFast, true>
        <<<(unsigned)h.total_items, 64 * kNWFast, 0, gp_stream(stream)>>>(a);
    dilated_attn32_kernel<48, true, kModeFix, true, kNWFast, true>
        <<<(unsigned)((h.total_items + kFixItems - 1) / kFixItems), 64 * kNWFast, 0, gp_stream(stream)>>>(a);
    return gp_check_launch("gp_dilated_attn_fwd_varlen");
  }
  dilated_attn32_kernel<48, true, kModeFast, true, kNWFast><<<(unsigned)h.total_items, 64 * kNWFast, 0, gp_stream(stream)>>>(a);
  dilated_attn32_kernel<48, true, kModeFix, true, kNWFast>
      <<<(unsigned)((h.total_items + kFixItems - 1) / kFixItems), 64 * kNWFast, 0, gp_stream(stream)>>>(a);
  return gp_check_launch("gp_dilated_attn_fwd_varlen");
}

extern "C" int gp_branch_merge_ln_varlen(const void* plan_host, const void* plan_dev, const float* ln_w,
                                         const float* ln_b, float eps, uint16_t* out, int fmt, void* stream) {
  GP_REQUIRE(fmt == GP_FMT_BF16 || fmt == GP_FMT_F16, "gp_branch_merge_ln_varlen: bad fmt %d", fmt);
  VarlenHdr h;
  if (int rc = varlen_header(plan_host, plan_dev, "gp_branch_merge_ln_varlen", h)) return rc;
  GP_REQUIRE(h.H * h.D == 768 && h.D == 48, "gp_branch_merge_ln_varlen: needs H*D = 768, D = 48");
  GP_REQUIRE(out && (ln_w == nullptr || ln_b != nullptr), "gp_branch_merge_ln_varlen: bad output / LN arguments");
  MergeArgs a;
  memset(&a, 0, sizeof(a));
  a.B = 1; a.L = h.T; a.tok_lo = 0; a.ntok = h.T;
  a.H = h.H; a.D = h.D; a.E = h.H * h.D; a.nbranch = h.nbranch;
  a.ln_w = ln_w; a.ln_b = ln_b; a.eps = eps; a.out = out;
  a.mtab = reinterpret_cast<const MergeBranch*>(static_cast<const char*>(plan_dev) + h.mtab_off);
  a.tok_off = reinterpret_cast<const int64_t*>(static_cast<const char*>(plan_dev) + h.tok_off_off);
  a.nslide = h.nslide;
  // (the v2 kernel's 32-bit offsets run from each slide's own o / lse region: a slide's branch rows
  // are at most 2 L_i, below 4 GiB for any slide the 1000 x 1000 position grid admits)
  const unsigned nb = merge_v2_grid(h.T);
  hipStream_t s = gp_stream(stream);
  if constexpr (GP_MERGE_V3_TAB != 0 && GP_MERGE_V3 != 0) if (h.nbranch == 5) {
    // the v3 merge over the packed tokens when every slide holds at least a block's tokens (a block then meets at
    // most two slides); tokens per block as the single-slide launch
    const int64_t* toh = reinterpret_cast<const int64_t*>(static_cast<const char*>(plan_host) + h.tok_off_off);
    int64_t shortest = INT64_MAX;
    for (int i = 0; i < h.nslide; ++i) shortest = std::min<int64_t>(shortest, toh[i + 1] - toh[i]);
    const int64_t ncu = attn_num_cus(s);
    const int64_t per_cu = (h.T + ncu * kV3Tok - 1) / (ncu * kV3Tok);
    const int tpb = (int)std::max<int64_t>(1, (h.T + ncu * per_cu - 1) / (ncu * per_cu));
    if (shortest >= tpb) {
      const unsigned g = (unsigned)((h.T + tpb - 1) / tpb);
      if (fmt == GP_FMT_F16) branch_merge_v3_kernel<5, true, true><<<g, 256, 0, s>>>(a, tpb);
      else branch_merge_v3_kernel<5, false, true><<<g, 256, 0, s>>>(a, tpb);
      return gp_check_launch("gp_branch_merge_ln_varlen");
    }
  }
  if (h.nbranch == 5) {   // every registered arch's schedule: compile-time branch loops
    if (fmt == GP_FMT_F16) branch_merge_v2_kernel<5, true, true><<<nb, 64 * GP_MERGE_WPB, 0, s>>>(a);
    else branch_merge_v2_kernel<5, true, false><<<nb, 64 * GP_MERGE_WPB, 0, s>>>(a);
  } else if (fmt == GP_FMT_F16) {
    branch_merge_v2_kernel<GP_MAX_BRANCHES, true, true><<<nb, 64 * GP_MERGE_WPB, 0, s>>>(a);
  } else {
    branch_merge_v2_kernel<GP_MAX_BRANCHES, true, false><<<nb, 64 * GP_MERGE_WPB, 0, s>>>(a);
  }
  return gp_check_launch("gp_branch_merge_ln_varlen");
}

// =========================================================================================
// Token-major sparsified K/V rows for sequence parallelism (the per-rank half of
// DilatedAttention.gathering, dilated_attention.py:16-31,76-98): for branch b, token p of
// segment n = p / s sits at offset t = p % s, in head group j = t % r (sparse row t / r).  Its
// row of dst[b] keeps only that group's hpg*D = C columns: [K cols j*C .. | V cols j*C ..], so a
// contiguous token range of dst[b] is exactly what another rank's queries need from it.
namespace {
struct SparsifyArgs {
  const uint16_t* src;
  int64_t src_stride, k_col, v_col;
  int64_t tok_lo, ntok, L;
  int32_t nbranch, per_tok;            // 16-byte chunks per token over all branches
  int32_t s[GP_MAX_BRANCHES], r[GP_MAX_BRANCHES], C[GP_MAX_BRANCHES], cbeg[GP_MAX_BRANCHES + 1];
  int32_t ndest[GP_MAX_BRANCHES];
  int64_t lo[GP_MAX_BRANCHES][GP_MAX_DESTS], hi[GP_MAX_BRANCHES][GP_MAX_DESTS];
  uint16_t* dst[GP_MAX_BRANCHES][GP_MAX_DESTS];   // row of token lo
};

__global__ __launch_bounds__(256) void dilated_sparsify_kernel(const SparsifyArgs a) {
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t t = id / a.per_tok;
  if (t >= a.ntok) return;
  int rem = (int)(id - t * a.per_tok);
  int b = 0;
#pragma unroll
  for (int x = 1; x < GP_MAX_BRANCHES; ++x)
    if (x < a.nbranch && rem >= a.cbeg[x]) b = x;
  rem -= a.cbeg[b];
  const int C = a.C[b];
  const int half = C / 8;                      // chunks per K (or V) part
  const int kv = rem >= half;
  const int ch = rem - kv * half;
  const int64_t p = a.tok_lo + t;
  const int j = (int)(p % a.s[b]) % a.r[b];
  const uint4 v = *reinterpret_cast<const uint4*>(a.src + t * a.src_stride + (kv ? a.v_col : a.k_col) + (int64_t)j * C + ch * 8);
  for (int d = 0; d < a.ndest[b]; ++d)
    if (p >= a.lo[b][d] && p < a.hi[b][d])
      *reinterpret_cast<uint4*>(a.dst[b][d] + (p - a.lo[b][d]) * (2 * (int64_t)C) + kv * C + ch * 8) = v;
}
}  // namespace

extern "C" int gp_dilated_sparsify_dests(const uint16_t* src, int64_t src_row_stride, int64_t k_col, int64_t v_col,
                                         int64_t tok_lo, int64_t n_tok, int64_t L, int H, int D,
                                         const int32_t* seg_len, const int32_t* ratios, int nbranch,
                                         const GpRowDest* dests, const int32_t* ndest, void* stream) {
  GP_REQUIRE(nbranch >= 1 && nbranch <= GP_MAX_BRANCHES, "gp_dilated_sparsify: nbranch must be 1..%d", GP_MAX_BRANCHES);
  GP_REQUIRE(L > 0 && H > 0 && D > 0 && D % 8 == 0 && tok_lo >= 0 && n_tok >= 0 && tok_lo + n_tok <= L,
             "gp_dilated_sparsify: bad sizes");
  GP_REQUIRE(src_row_stride % 8 == 0 && k_col % 8 == 0 && v_col % 8 == 0, "gp_dilated_sparsify: strides must be multiples of 8");
  if (n_tok == 0) return 0;
  GP_REQUIRE(src && seg_len && ratios && dests && ndest && gp_aligned(src, 16), "gp_dilated_sparsify: null or misaligned pointer");
  SparsifyArgs a;
  a.src = src; a.src_stride = src_row_stride; a.k_col = k_col; a.v_col = v_col;
  a.tok_lo = tok_lo; a.ntok = n_tok; a.L = L; a.nbranch = nbranch;
  int cb = 0;
  for (int b = 0; b < GP_MAX_BRANCHES; ++b) {
    a.ndest[b] = 0;
    for (int d = 0; d < GP_MAX_DESTS; ++d) { a.lo[b][d] = 0; a.hi[b][d] = 0; a.dst[b][d] = nullptr; }
  }
  for (int b = 0; b < nbranch; ++b) {
    GP_REQUIRE(seg_len[b] > 0 && ratios[b] > 0 && H % ratios[b] == 0, "gp_dilated_sparsify: branch %d needs H %% r == 0", b);
    GP_REQUIRE(ndest[b] >= 0 && ndest[b] <= GP_MAX_DESTS, "gp_dilated_sparsify: branch %d has %d destinations (max %d)",
               b, ndest[b], GP_MAX_DESTS);
    a.s[b] = (int32_t)(seg_len[b] < L ? seg_len[b] : L);
    a.r[b] = ratios[b];
    a.C[b] = (H / ratios[b]) * D;
    a.ndest[b] = ndest[b];
    for (int d = 0; d < ndest[b]; ++d) {
      const GpRowDest& e = dests[b * GP_MAX_DESTS + d];
      GP_REQUIRE(e.tok_lo <= e.tok_hi && (e.tok_lo == e.tok_hi || (e.dst && gp_aligned(e.dst, 16))),
                 "gp_dilated_sparsify: branch %d destination %d null/misaligned or empty range", b, d);
      a.lo[b][d] = e.tok_lo;
      a.hi[b][d] = e.tok_hi;
      a.dst[b][d] = e.dst;
    }
    a.cbeg[b] = cb;
    cb += 2 * a.C[b] / 8;
  }
  for (int b = nbranch; b < GP_MAX_BRANCHES; ++b) { a.s[b] = 1; a.r[b] = 1; a.C[b] = 8; a.cbeg[b] = cb; }
  a.cbeg[GP_MAX_BRANCHES] = cb;
  a.per_tok = cb;
  const int64_t work = n_tok * cb;
  GP_REQUIRE(work / 256 < (int64_t)0x7fffffff, "gp_dilated_sparsify: too much work");
  dilated_sparsify_kernel<<<(unsigned)((work + 255) / 256), 256, 0, gp_stream(stream)>>>(a);
  return gp_check_launch("gp_dilated_sparsify");
}

extern "C" int gp_dilated_sparsify(const uint16_t* src, int64_t src_row_stride, int64_t k_col, int64_t v_col,
                                   int64_t tok_lo, int64_t n_tok, int64_t L, int H, int D, const int32_t* seg_len,
                                   const int32_t* ratios, int nbranch, uint16_t* const* dst,
                                   const int64_t* dst_tok_base, void* stream) {
  GP_REQUIRE(nbranch >= 1 && nbranch <= GP_MAX_BRANCHES, "gp_dilated_sparsify: nbranch must be 1..%d", GP_MAX_BRANCHES);
  GP_REQUIRE(dst && seg_len && ratios, "gp_dilated_sparsify: null pointer");
  GpRowDest dests[GP_MAX_BRANCHES * GP_MAX_DESTS];
  int32_t nd[GP_MAX_BRANCHES];
  for (int b = 0; b < nbranch; ++b) {
    GP_REQUIRE(ratios[b] > 0 && H > 0 && H % ratios[b] == 0, "gp_dilated_sparsify: branch %d needs H %% r == 0", b);
    const int64_t base = dst_tok_base ? dst_tok_base[b] : 0;
    GP_REQUIRE(base <= tok_lo, "gp_dilated_sparsify: branch %d dst_tok_base beyond tok_lo", b);
    const int64_t C = (int64_t)(H / ratios[b]) * D;
    dests[b * GP_MAX_DESTS].tok_lo = tok_lo;
    dests[b * GP_MAX_DESTS].tok_hi = tok_lo + n_tok;
    dests[b * GP_MAX_DESTS].dst = dst[b] ? dst[b] + (tok_lo - base) * 2 * C : nullptr;
    nd[b] = 1;
  }
  return gp_dilated_sparsify_dests(src, src_row_stride, k_col, v_col, tok_lo, n_tok, L, H, D, seg_len, ratios,
                                   nbranch, dests, nd, stream);
}
