// LAB BUILD (not the product yet): bf16 GEMM v8 for the slide encoder's projections on gfx950 -- the
// 256 x 256 "8-phase" ping-pong structure (cdna_hip_programming.md §5, "The 256² 8-phase template"),
// written for these shapes.  Measured against hipBLASLt with
//   python tools/gemm_bench.py --lib tools/attn_lab/liblab_gemm8.so
// C[M, N] = A[M, K] . W[N, K]^T (+ bias[N]), fp32 accumulation, bf16 output: the nn.Linear of the QKV /
// out-proj / fc1 / fc2 / patch layers (torchscale/component/multihead_attention.py:43-48,
// feedforward_network.py:131-142, gigapath/slide_encoder.py:47-51); A and W both K-contiguous.
//
// Structure:
//   * 256 x 256 output tile per workgroup of 8 waves as 2 (M) x 4 (N); a wave owns 128 x 64 = 8 x 4
//     v_mfma_f32_16x16x32_bf16 tiles (128 fp32 accumulators per lane); BK = 64;
//   * LDS: two K-tile buffers (distinct __shared__ objects, so the compiler sees that a fragment read of
//     one never aliases the LDS-DMA in flight into the other) of [A 256 x 64 | W 256 x 64] bf16, rows of
//     128 B whose 16-byte chunk c sits at c ^ ((row >> 1) & 7): the 16 rows x 4 chunks of every
//     ds_read_b128 lane group land on 16 distinct bank slots;
//   * staging by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction, lane-linear; the
//     swizzle lives in the per-lane SOURCE address), one operand half-tile (128 rows x 64 k = 16 KiB,
//     2 instructions per wave) per phase, rows past M read as zero through the buffer descriptor;
//   * a K-tile = 4 phases, one C quadrant (4 m-frags x 2 n-frags x K 64 = 16 MFMAs) each, with one A
//     m-half and both W n-halves in registers (ktile() below has the phase table); one counted
//     s_waitcnt vmcnt(2) per K-tile retires the next K-tile's DMA, read one phase later;
//   * each phase: fragment reads + LDS-DMA issue | s_barrier | 16 MFMAs at s_setprio 1 | s_barrier, and
//     waves 4-7 run one barrier behind waves 0-3 (one extra s_barrier before the loop, one more for waves
//     0-3 after it): on each SIMD one wave's MFMAs overlap the other's reads and DMA issue;
//   * XCD-grouped tile order: consecutive tile ids (the N-tiles of one A row panel) on one XCD's L2.
#include "gp_api.h"
#include "gp_common.h"

namespace {

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kThreads = 512;
constexpr int kRowB = kBK * 2;                // 128-byte LDS rows
constexpr int kOpT = 256 * kRowB;             // one operand's K-tile: 32 KiB
constexpr int kHalf = 128 * kRowB;            // one operand half-tile: 16 KiB

typedef float f32x4v __attribute__((ext_vector_type(4)));

__shared__ __attribute__((aligned(1024))) char g_buf0[2 * kOpT];   // K-tiles 0, 2, 4, ...
__shared__ __attribute__((aligned(1024))) char g_buf1[2 * kOpT];   // K-tiles 1, 3, 5, ...
template <int B>
GP_DEV char* bufp() {
  if constexpr (B == 0) return g_buf0;
  else return g_buf1;
}

GP_DEV int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

struct GemmArgs {
  const uint16_t* A;
  const uint16_t* W;
  const void* bias;
  uint16_t* C;
  int64_t lda, ldw, ldc;
  int M, N, K;
  int bias_f32;
  int n_dp;        // tiles run data-parallel
  int split;       // 1: the remaining tiles are split in K (workspace ws)
  float* ws;
};

template <int n>
GP_DEV void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}

__shared__ __attribute__((aligned(16))) float g_bias[3072];        // the bias row (N <= 3072), fp32
#ifndef GP_GEMM8_SCHED
#define GP_GEMM8_SCHED 1       // 1: both W halves of K-tile v+2 staged in Q3 of v (weights 4 phases ahead);
                               // 2: and both A halves of v+1 in Q0 of v (3 phases ahead)
#endif
#ifndef GP_GEMM8_SPLIT
#define GP_GEMM8_SPLIT 1       // split the last partial round of tiles in K (a second, small reduce kernel)
#endif

// NK = K / 64 as a template constant: the K loop is unrolled completely, so no loop header merges the
// LDS-DMA state of two paths (hipcc's wait insertion then put a vmcnt(0) before every iteration's first
// fragment read although the pending DMA targets the other buffer).
//
// Work: persistent, one workgroup per CU (G = grid).  Tiles [0, n_dp) run data-parallel: workgroup sid
// takes sid, sid + G, ... and the K-tile sequence runs on across its tiles (the next tile's first K-tiles
// stream in during the current tile's last phases).  Tiles [n_dp, ntiles) -- the last, partial round --
// are split S ways in K when the host asks for it (n_dp a multiple of G, (ntiles - n_dp) * S <= G):
// unit u = sid takes tile n_dp + u / S, K-tiles [(u % S) NK/S, +NK/S), and writes its fp32 partial
// tile to the workspace; gemm8_reduce sums the S partials, adds the bias and stores bf16.
template <int NK, int S>
__global__ __launch_bounds__(kThreads, 1) void gemm8_kernel(const GemmArgs g) {
  static_assert(NK % 2 == 0 && NK >= 2 && (S == 1 || (NK % (2 * S) == 0)), "");
  const int tiles_n = g.N / kBN;
  const int ntiles = ((g.M + kBM - 1) / kBM) * tiles_n;
  const int G = (int)gridDim.x;
  const int sid = xcd_remap((int)blockIdx.x, G);
  const int n_dp = g.n_dp;
  const int n_my = sid < n_dp ? (n_dp - 1 - sid) / G + 1 : 0;
  const bool tail = S > 1 && g.split && sid < (ntiles - n_dp) * S;
  if (n_my == 0 && !tail) return;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;

  if (g.bias != nullptr) {
    for (int c = threadIdx.x; c < g.N; c += kThreads)
      g_bias[c] = g.bias_f32 ? static_cast<const float*>(g.bias)[c] : bf2f(static_cast<const uint16_t*>(g.bias)[c]);
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
  bf16x8 as[4][2], ws[2][2][2];     // one A m-half (8 frags), both W n-halves
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
  auto quadrant = [&](auto mqc, auto nqc) {
    constexpr int MQ = decltype(mqc)::value, NQ = decltype(nqc)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[MQ * 4 + f][NQ * 2 + e] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws[NQ][e][ks], as[f][ks], acc[MQ * 4 + f][NQ * 2 + e], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // bf16 epilogue of tile T: 16-byte stores (T21 with v_permlane16_swap): for each n-frag pair (2p, 2p+1)
  // one swap per dword gives lane groups q = 0 / 2 the 8 columns 8(q>>1) .. +7 of n-frag 2p and q = 1 / 3
  // those of n-frag 2p+1; stored through a per-wave buffer descriptor whose record count ends at row M
  // (rows past it are dropped by the hardware), row group in the scalar offset
  auto store_tile = [&](int T) {
    const int mw = (T / tiles_n) * kBM + wm * 128, nw = (T % tiles_n) * kBN + wn * 64;
    const int64_t c_rows = g.M - mw < 128 ? (g.M - mw > 0 ? g.M - mw : 0) : 128;
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(g.C + (int64_t)mw * g.ldc + nw), (short)0, (int)(c_rows * g.ldc * 2), 0x00020000);
    const int c_lane = (int)((r16 * g.ldc + 16 * (q & 1) + 8 * (q >> 1)) * 2);
    const int c_mi = (int)(16 * g.ldc * 2);
    float4 bq[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      bq[ni] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (g.bias != nullptr) bq[ni] = *reinterpret_cast<const float4*>(g_bias + nw + ni * 16 + 4 * q);
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        uint32_t pk[2][2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int ni = 2 * pr + e;
          pk[e][0] = (uint32_t)f2bf(acc[mi][ni][0] + bq[ni].x) | ((uint32_t)f2bf(acc[mi][ni][1] + bq[ni].y) << 16);
          pk[e][1] = (uint32_t)f2bf(acc[mi][ni][2] + bq[ni].z) | ((uint32_t)f2bf(acc[mi][ni][3] + bq[ni].w) << 16);
        }
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto r = __builtin_amdgcn_permlane16_swap(pk[0][d], pk[1][d], false, false);
          pk[0][d] = r[0];
          pk[1][d] = r[1];
        }
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        const i32x4 v4 = {(int)pk[0][0], (int)pk[0][1], (int)pk[1][0], (int)pk[1][1]};
        __builtin_amdgcn_raw_buffer_store_b128(v4, rc, c_lane + pr * 64, mi * c_mi, 0);
      }
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
  auto run_seq = [&](auto nkc, int count, int kt0, auto&& tile_of, auto&& epilogue) {
    constexpr int nk = decltype(nkc)::value;
    __amdgpu_buffer_rsrc_t ra = rsrc_a(tile_of(0)), rw = rsrc_w(tile_of(0));
    bool has_next = false;
    int i_cur = 0;
    // stage half H of operand OP of the tile-local K-tile vv (vv >= nk: the next tile's K-tile vv - nk)
    auto stage = [&](auto opc, auto hc, auto bc, int vv) {
      constexpr int OP = decltype(opc)::value;
      if (vv < nk || has_next) issue(opc, hc, bc, OP == 0 ? ra : rw, kt0 + (vv < nk ? vv : vv - nk));
    };
    // one K-tile v of the current output tile, in buffer B (v even: B = 0).  Phases (quadrant; fragments
    // read; DMA issued): Q0 (m0, n0; A m-half 0 + W n-half 0; A half 0 of K-tile v+1), Q1 (m0, n1; W
    // n-half 1; A half 1 of v+1), Q2 (m1, n1; A m-half 1; W half 1 of v+1), Q3 (m1, n0; none; W half 0 of
    // v+2).  A halves are last read in Q2, W halves in Q1, so every restage comes >= 2 phases after the
    // last read of its buffer half; one counted vmcnt(2) in Q3 retires all of K-tile v+1, which is read one
    // phase later
    auto ktile = [&](auto bc, int v) {
      constexpr int B = decltype(bc)::value;
      using BN_ = std::integral_constant<int, 1 - B>;
      read_a(bc, I0());
      read_w(bc, I0());
      stage(I0(), I0(), BN_(), v + 1);
      if constexpr (GP_GEMM8_SCHED == 2) stage(I0(), I1(), BN_(), v + 1);   // both A halves in Q0
      sync();
      quadrant(I0(), I0());
      sync();
      read_w(bc, I1());
      if constexpr (GP_GEMM8_SCHED != 2) stage(I0(), I1(), BN_(), v + 1);
      sync();
      quadrant(I0(), I1());
      sync();
      read_a(bc, I1());
      if constexpr (GP_GEMM8_SCHED == 0) stage(I1(), I1(), BN_(), v + 1);
      sync();
      quadrant(I1(), I1());
      sync();
      if (v + 2 == nk && has_next) {   // every DMA of this tile is issued: switch to the next tile's
        ra = rsrc_a(tile_of(i_cur + 1));
        rw = rsrc_w(tile_of(i_cur + 1));
      }
      if (v + 2 < nk || has_next) {
        stage(I1(), I0(), bc, v + 2);
        if constexpr (GP_GEMM8_SCHED >= 1) {   // both W halves of v+2 here (4 phases of lead)
          stage(I1(), I1(), bc, v + 2);
          wait_vmcnt<4>();
        } else {
          wait_vmcnt<2>();
        }
      } else {
        wait_vmcnt<0>();
      }
      sync();
      quadrant(I1(), I0());
      sync();
    };
    // prologue: K-tile 0 whole, K-tile 1's W half 0 (its other halves come in K-tile 0's Q0-Q2)
    issue(I0(), I0(), I0(), ra, kt0);
    issue(I0(), I1(), I0(), ra, kt0);
    issue(I1(), I0(), I0(), rw, kt0);
    issue(I1(), I1(), I0(), rw, kt0);
    issue(I1(), I0(), I1(), rw, kt0 + 1);
    if constexpr (GP_GEMM8_SCHED >= 1) {
      issue(I1(), I1(), I1(), rw, kt0 + 1);
      wait_vmcnt<4>();
    } else {
      wait_vmcnt<2>();
    }
    sync();                         // (also publishes g_bias)
    for (int i = 0; i < count; ++i) {
      has_next = i + 1 < count;
      i_cur = i;
      // opaque per tile: the DMA scalar offsets derived from these are then computed where they are used
      // instead of being hoisted out of the tile loop (~100 loop-invariant SGPRs for K = 3072 -> spills)
      asm volatile("" : "+s"(hoff[0]), "+s"(hoff[1]));
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4v{0.f, 0.f, 0.f, 0.f};
      if (wm == 1) sync();          // waves 4-7 one barrier behind
#pragma unroll
      for (int v = 0; v < nk; v += 2) {
        ktile(I0(), v);
        ktile(I1(), v + 1);
      }
      if (wm == 0) sync();          // realign
      epilogue(i);
    }
    wait_vmcnt<0>();   // no LDS-DMA in flight past the sequence (LDS reuse, hand-off)
  };

  if (n_my > 0)
    run_seq(std::integral_constant<int, NK>(), n_my, 0, [&](int i) { return sid + i * G; },
            [&](int i) { store_tile(sid + i * G); });
  if constexpr (S > 1) {
    if (tail) {
      constexpr int NKS = NK / S;
      if (n_my > 0) sync();         // every wave done reading the last data-parallel tile's buffers
      const int T = n_dp + sid / S, part = sid % S;
      run_seq(std::integral_constant<int, NKS>(), 1, part * NKS, [&](int) { return T; },
              [&](int) { store_partial(sid); });
    }
  }
}

// sum of the S fp32 partials of each split tail tile + bias -> bf16 C; one thread per 8 columns of a row
__global__ __launch_bounds__(256) void gemm8_reduce(const GemmArgs g, int S) {
  const int tiles_n = g.N / kBN;
  const int unit = blockIdx.x / (kBM * kBN / 8 / 256);          // tail tile ordinal
  const int idx = (blockIdx.x % (kBM * kBN / 8 / 256)) * 256 + threadIdx.x;
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
  if (g.bias != nullptr) {
    for (int e = 0; e < 8; ++e)
      v[e] += g.bias_f32 ? static_cast<const float*>(g.bias)[n + e] : bf2f(static_cast<const uint16_t*>(g.bias)[n + e]);
  }
  store_bf16<8>(g.C + (int64_t)m * g.ldc + n, v);
}

}  // namespace

extern "C" int gp_gemm_bf16_tn(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, const void* bias,
                               int bias_is_f32, uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                               void* stream) {
  GP_REQUIRE(A && W && C, "gp_gemm_bf16_tn: null pointer");
  GP_REQUIRE(M > 0 && M < (int64_t)0x7fffffff && N > 0 && K > 0, "gp_gemm_bf16_tn: bad sizes");
  GP_REQUIRE(N <= 3072, "gp_gemm_bf16_tn: N=%lld > 3072 (the bias row is staged in LDS)", (long long)N);
  GP_REQUIRE(N % kBN == 0 && K % (2 * kBK) == 0,
             "gp_gemm_bf16_tn: N must be a multiple of %d and K of %d (N=%lld K=%lld)", kBN, 2 * kBK,
             (long long)N, (long long)K);
  GP_REQUIRE(lda >= K && ldw >= K && ldc >= N && lda % 8 == 0 && ldw % 8 == 0 && ldc % 4 == 0,
             "gp_gemm_bf16_tn: bad leading dimensions");
  GP_REQUIRE(gp_aligned(A, 16) && gp_aligned(W, 16) && gp_aligned(C, 8) && (!bias || gp_aligned(bias, 16)),
             "gp_gemm_bf16_tn: misaligned operand");
  GP_REQUIRE((int64_t)kBM * lda * 2 < 0x7fffffff && (int64_t)kBN * ldw * 2 < 0x7fffffff,
             "gp_gemm_bf16_tn: leading dimension too large for 32-bit tile offsets");
  GemmArgs g;
  g.A = A; g.W = W; g.bias = bias; g.C = C;
  g.lda = lda; g.ldw = ldw; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.bias_f32 = bias_is_f32 ? 1 : 0;
  const int64_t tiles = ((M + kBM - 1) / kBM) * (N / kBN);
  int cus = 256;
  {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      cus = n;
  }
  const int G = (int)(tiles < cus ? tiles : cus);
  // the last partial round split in K when it is at most half full (S = 4, or 2 for K = 768)
  const int S = K == 768 ? 2 : 4;
  const int64_t rem = tiles % G;
  g.n_dp = (int)tiles;
  g.split = 0;
  g.ws = nullptr;
  static float* lab_ws = nullptr;            // LAB: a workspace of its own (the product passes one in)
  if (GP_GEMM8_SPLIT && tiles > G && rem > 0 && rem * S <= G && rem * 2 <= G) {
    const size_t need = (size_t)rem * S * kBM * kBN * sizeof(float);
    static size_t lab_ws_bytes = 0;
    if (lab_ws_bytes < need) {
      if (lab_ws) (void)hipFree(lab_ws);
      GP_REQUIRE(hipMalloc(&lab_ws, need) == hipSuccess, "gp_gemm_bf16_tn: workspace");
      lab_ws_bytes = need;
    }
    g.n_dp = (int)(tiles - rem);
    g.split = 1;
    g.ws = lab_ws;
  }
  const dim3 grid((unsigned)G), block(kThreads);
  switch (K) {
    case 768: gemm8_kernel<12, 2><<<grid, block, 0, gp_stream(stream)>>>(g); break;
    case 1536: gemm8_kernel<24, 4><<<grid, block, 0, gp_stream(stream)>>>(g); break;
    case 3072: gemm8_kernel<48, 4><<<grid, block, 0, gp_stream(stream)>>>(g); break;
    default: GP_REQUIRE(false, "gp_gemm_bf16_tn: K=%lld not instantiated (768 / 1536 / 3072)", (long long)K);
  }
  if (g.split)
    gemm8_reduce<<<(unsigned)(rem * (kBM * kBN / 8 / 256)), 256, 0, gp_stream(stream)>>>(g, S);
  return gp_check_launch("gp_gemm_bf16_tn");
}
