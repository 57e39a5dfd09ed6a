// LAB BUILD (not the product): bf16 GEMM v4 for the slide encoder's projections on gfx950 -- the
// LDS-bandwidth fix of v2 (gp_gemm_lab.hip) plus a persistent tile loop.  Measured against hipBLASLt with
// tools/gemm_bench.py --lib tools/attn_lab/liblab_gemm4.so.
// C[M, N] = A[M, K] . W[N, K]^T (+ bias[N]), fp32 accumulation, bf16 output -- the nn.Linear of the
// QKV / out-proj / fc1 / fc2 / patch layers (torchscale/component/multihead_attention.py:43-48,
// feedforward_network.py:131-142, gigapath/slide_encoder.py:47-51), A and W both K-contiguous.
//
// Why v2 stalled: a 64 x 64 wave tile reads (64 + 64) rows x BK from LDS per 64 x 64 x BK MACs = 1/16 B per
// MAC; at 4 SIMDs x 512 bf16 MAC/clk that is 128 B/clk per CU -- exactly the LDS bandwidth, so the MFMA pipe
// could never be fed.  v4:
//   * 256 x 256 output tile per 256-thread workgroup, 4 waves as 2 x 2, 128 x 128 per wave (the fp32
//     accumulators, 256 per lane, live in AGPRs; one wave per SIMD): 1/32 B of LDS per MAC, 50 % of LDS peak;
//   * BK = 32 (64-byte LDS rows, one v_mfma_f32_16x16x32_bf16 k-step per stage), a ring of four 32 KiB stages
//     filled by LDS-DMA (buffer_load_dwordx4 ... lds, lane-linear 1 KiB per instruction) three stages ahead;
//     the 16-byte chunks of row r sit at chunk ^ (2 * bit 3 of r), set through the per-lane SOURCE address, so
//     the 16-row fragment reads are conflict free;
//   * per stage: wait for the next stage's DMA, one barrier, refill the stage just consumed, issue the next
//     stage's fragment reads into the second register set, then 64 MFMAs on the current set;
//   * persistent: one workgroup per CU walks its tiles (XCD-grouped order: the tiles of consecutive ids share A
//     rows and run on one XCD) with one global stage counter, so the next tile's first stages stream in while
//     the current tile's epilogue stores run;
//   * rows past M read as zero through the buffer descriptor's record count (ragged M = L tokens).
#include "gp_api.h"
#include "gp_common.h"

namespace {

constexpr int kBM = 256, kBN = 256, kBK = 32;
constexpr int kThreads = 256;
constexpr int kRowB = kBK * 2;                // 64-byte LDS rows
constexpr int kATile = kBM * kRowB;           // 16 KiB
constexpr int kWTile = kBN * kRowB;           // 16 KiB
constexpr int kStage = kATile + kWTile;       // 32 KiB
constexpr int kStages = 4;                    // 128 KiB ring
constexpr int kGldsA = kATile / 1024 / 4;     // LDS-DMA instructions per wave per stage: 4 (A) + 4 (W)
constexpr int kGldsW = kWTile / 1024 / 4;
constexpr int kGlds = kGldsA + kGldsW;

typedef float f32x4v __attribute__((ext_vector_type(4)));

// chunk c of row r at c ^ (2 * bit 3 of r): conflict-free for the 16-row x 4-chunk fragment reads under the
// ds_read_b128 lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md, LDS table)
GP_DEV int swz_x(int r) { return ((r >> 3) & 1) << 1; }
GP_DEV int swz(int r, int c) { return r * kRowB + ((c ^ swz_x(r)) << 4); }

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
};

template <int n>
GP_DEV void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}
GP_DEV void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xc07f); }   // lgkmcnt(0), vmcnt 63, expcnt 7

// one LDS object per ring slot: the compiler's wait insertion then knows a slot's fragment reads depend on
// that slot's LDS-DMA only (one array: it waited on every in-flight DMA before each read)
__shared__ __attribute__((aligned(1024))) char g_slot0[kStage];
__shared__ __attribute__((aligned(1024))) char g_slot1[kStage];
__shared__ __attribute__((aligned(1024))) char g_slot2[kStage];
__shared__ __attribute__((aligned(1024))) char g_slot3[kStage];
__shared__ __attribute__((aligned(16))) float g_bias[4096];   // the whole bias row (N <= 4096), fp32
template <int S>
GP_DEV char* slot_base() {
  if constexpr (S == 0) return g_slot0;
  else if constexpr (S == 1) return g_slot1;
  else if constexpr (S == 2) return g_slot2;
  else return g_slot3;
}

#ifndef GP_GEMM_SGB
#define GP_GEMM_SGB 1     // interleave the next stage's fragment reads with the MFMAs (sched_group_barrier)
#endif

__global__ __launch_bounds__(kThreads, 1) void gemm4_kernel(const GemmArgs g) {
  const int tiles_n = g.N / kBN;
  const int tiles_m = (g.M + kBM - 1) / kBM;
  const int ntiles = tiles_m * tiles_n;
  const int G = (int)gridDim.x;
  const int sid = xcd_remap((int)blockIdx.x, G);
  if (sid >= ntiles) return;
  const int n_my = (ntiles - 1 - sid) / G + 1;
  const int nk = g.K / kBK;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;

  // LDS-DMA: instruction i covers rows 16i .. 16i + 15 of a tile; lane l writes row 16i + l / 4, physical chunk
  // l % 4, which holds the logical chunk (l % 4) ^ ((row >> 2) & 3)
  int voff_a[kGldsA], voff_w[kGldsW];
#pragma unroll
  for (int j = 0; j < kGldsA; ++j) {
    const int r = 16 * (w + 4 * j) + (lane >> 2), c = (lane & 3) ^ swz_x(r);
    voff_a[j] = (int)((int64_t)r * g.lda * 2) + c * 16;
  }
#pragma unroll
  for (int j = 0; j < kGldsW; ++j) {
    const int r = 16 * (w + 4 * j) + (lane >> 2), c = (lane & 3) ^ swz_x(r);
    voff_w[j] = (int)((int64_t)r * g.ldw * 2) + c * 16;
  }

  // DMA side: the stage being fetched is (d_i = my tile ordinal, d_kt)
  int d_i = 0, d_kt = 0;
  __amdgpu_buffer_rsrc_t ra, rw;
  auto set_rsrc = [&](int i) {
    const int T = sid + i * G;
    const int tm = T / tiles_n, tn = T - tm * tiles_n;
    const int m0 = tm * kBM, n0 = tn * kBN;
    const int64_t a_bytes = (int64_t)(g.M - m0) * g.lda * 2;
    ra = __builtin_amdgcn_make_buffer_rsrc((void*)(g.A + (int64_t)m0 * g.lda), (short)0,
                                           (int)(a_bytes < 0x7fffffff ? a_bytes : 0x7fffffff), 0x00020000);
    rw = __builtin_amdgcn_make_buffer_rsrc((void*)(g.W + (int64_t)n0 * g.ldw), (short)0,
                                           (int)((int64_t)kBN * g.ldw * 2), 0x00020000);
  };
  set_rsrc(0);
  auto issue = [&](auto slotc) {
    constexpr int S = decltype(slotc)::value;
    char* base = slot_base<S>();
#pragma unroll
    for (int j = 0; j < kGldsA; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(base + (w + 4 * j) * 1024),
                                               16, voff_a[j] + d_kt * kRowB, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < kGldsW; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(base + kATile + (w + 4 * j) * 1024),
                                               16, voff_w[j] + d_kt * kRowB, 0, 0, 0);
    if (++d_kt == nk) {
      d_kt = 0;
      if (d_i + 1 < n_my) set_rsrc(++d_i);
    }
  };

  f32x4v acc[8][8];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = f32x4v{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][8], wf[2][8];
  const int lr = lane & 15, lq = lane >> 4;
  auto read_frags = [&](auto slotc, auto setc) {
    constexpr int S = decltype(slotc)::value, P = decltype(setc)::value;
    const char* As = slot_base<S>();
    const char* Ws = As + kATile;
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) wf[P][ni] = *reinterpret_cast<const bf16x8*>(Ws + swz(wn * 128 + ni * 16 + lr, lq));
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) af[P][mi] = *reinterpret_cast<const bf16x8*>(As + swz(wm * 128 + mi * 16 + lr, lq));
  };
  auto mfmas = [&](auto setc) {
    constexpr int P = decltype(setc)::value;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 8; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[P][ni], af[P][mi], acc[mi][ni], 0, 0, 0);
  };

  auto epilogue = [&](int i) {
    const int T = sid + i * G;
    const int tm = T / tiles_n, tn = T - tm * tiles_n;
    const int m0 = tm * kBM + wm * 128, n0 = tn * kBN + wn * 128;
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const int n = n0 + ni * 16 + 4 * lq;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (g.bias != nullptr) {   // from LDS: a global load here would wait on the whole DMA ring (vmcnt is in order)
        const float4 b4 = *reinterpret_cast<const float4*>(g_bias + n);
        bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w;
      }
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const int m = m0 + mi * 16 + lr;
        if (m < g.M) {
          float v[4] = {acc[mi][ni][0] + bv[0], acc[mi][ni][1] + bv[1], acc[mi][ni][2] + bv[2], acc[mi][ni][3] + bv[3]};
          store_bf16<4>(g.C + (int64_t)m * g.ldc + n, v);
        }
        acc[mi][ni] = f32x4v{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  if (g.bias != nullptr) {
    for (int c = threadIdx.x; c < g.N; c += kThreads)
      g_bias[c] = g.bias_f32 ? static_cast<const float*>(g.bias)[c] : bf2f(static_cast<const uint16_t*>(g.bias)[c]);
  }
  // prologue: stages 0..3 in flight (total = n_my * nk >= 4), stage 0's fragments in set 0
  issue(std::integral_constant<int, 0>());
  issue(std::integral_constant<int, 1>());
  issue(std::integral_constant<int, 2>());
  issue(std::integral_constant<int, 3>());
  wait_vmcnt<3 * kGlds>();
  __builtin_amdgcn_s_barrier();
  read_frags(std::integral_constant<int, 0>(), std::integral_constant<int, 0>());

  // step s (slot S = s % 4, register set P = s % 2; nk % 4 == 0, so S = kt % 4 in every tile): wait for stage
  // s + 1's DMA (stages s + 2, s + 3 stay in flight), barrier (every wave holds stage s in registers, so slot
  // S is free), refill slot S with stage s + 4, read stage s + 1's fragments, 64 MFMAs on stage s.  In the
  // first three stages of a tile the previous epilogue's stores sit behind the DMAs being waited on.
  auto step = [&](bool after_epi, auto slotc) {
    constexpr int S = decltype(slotc)::value, P = S & 1;
    constexpr int S1 = (S + 1) % kStages;
    wait_lgkm0();                                   // this wave's reads of slot S are complete
    if (after_epi) wait_vmcnt<63>();
    else wait_vmcnt<2 * kGlds>();
    __builtin_amdgcn_s_barrier();
    issue(slotc);                                   // past the last stage: re-reads the last tile (harmless)
    read_frags(std::integral_constant<int, S1>(), std::integral_constant<int, 1 - P>());
    mfmas(std::integral_constant<int, P>());
    if constexpr (GP_GEMM_SGB) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);   // one ds_read
        __builtin_amdgcn_sched_group_barrier(0x0008, 4, 0);   // four MFMAs
      }
    }
  };
  for (int i = 0; i < n_my; ++i) {
    for (int kt = 0; kt < nk; kt += kStages) {
      const bool ae = i > 0 && kt == 0;
      step(ae, std::integral_constant<int, 0>());
      step(ae, std::integral_constant<int, 1>());
      step(ae, std::integral_constant<int, 2>());
      step(false, std::integral_constant<int, 3>());
    }
    epilogue(i);
  }
  wait_vmcnt<0>();   // no LDS-DMA may land after the workgroup's LDS is handed to another one
}

}  // namespace

extern "C" int gp_gemm_bf16_tn(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, const void* bias,
                               int bias_is_f32, uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                               void* stream) {
  GP_REQUIRE(A && W && C, "gp_gemm_bf16_tn: null pointer");
  GP_REQUIRE(M > 0 && M < (int64_t)0x7fffffff && N > 0 && K > 0, "gp_gemm_bf16_tn: bad sizes");
  GP_REQUIRE(N <= 4096, "gp_gemm_bf16_tn: N=%lld > 4096 (the bias row is staged in LDS)", (long long)N);
  GP_REQUIRE(N % kBN == 0 && K % (kBK * kStages) == 0,
             "gp_gemm_bf16_tn: N must be a multiple of %d and K of %d (N=%lld K=%lld)", kBN, kBK * kStages,
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
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) cus = n;
  }
  const int64_t tiles = ((M + kBM - 1) / kBM) * (N / kBN);
  const unsigned grid = (unsigned)(tiles < cus ? tiles : cus);
  gemm4_kernel<<<grid, kThreads, 0, gp_stream(stream)>>>(g);
  return gp_check_launch("gp_gemm_bf16_tn");
}
