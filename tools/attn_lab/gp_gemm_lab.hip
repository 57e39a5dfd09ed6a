// LAB BUILD (not the product): a hand-written bf16 GEMM for the slide encoder's projections on gfx950,
// measured against hipBLASLt (tools/gemm_bench.py, profiles/r02_gemm_*.json) and NOT used by the
// forward: it reaches 0.66-0.95 PF/s where hipBLASLt's tuned solutions reach 0.88-1.31 PF/s on the same
// shapes.  Kept as the starting point of the 8-phase rewrite.
// C[M, N] = A[M, K] . W[N, K]^T (+ bias[N]),
// fp32 accumulation, bf16 output -- the nn.Linear of the QKV / out-proj / fc1 / fc2 / patch layers
// (torchscale/component/multihead_attention.py:43-48, feedforward_network.py:131-142,
// gigapath/slide_encoder.py:47-51), A and W both K-contiguous (torch's addmm(b, A, W.t())).
//
// Design (MI355X-first):
//   * 256 x 128 output tile per 512-thread workgroup (8 waves as 4 (M) x 2 (N), 64 x 64 per wave),
//     BK = 64, v_mfma_f32_16x16x32_bf16; the wave computes C^T tiles (W fragments as the MFMA A operand,
//     A fragments as B), so each lane ends with 4 consecutive output columns of one row (8-byte stores);
//   * both operand tiles are staged global -> LDS by LDS-DMA (buffer_load ... lds, 1 KiB per
//     wave-instruction, 8 rows of 128 B) into a ring of three 48 KiB stages: tile kt + 2 is in flight
//     while tile kt is computed (counted vmcnt, raw s_barrier); the 16-B chunks of each LDS row
//     are XOR-swizzled by row bits (chunk c of row r at c ^ ((r >> 1) & 7)) through the per-lane SOURCE
//     address (the DMA writes lane-linearly), so the ds_read_b128 fragment reads are bank-conflict free;
//   * rows past M read as zero through the buffer descriptor's record count (ragged M = L tokens);
//   * XCD-aware tile order: the tiles of consecutive ids share A rows and run on one XCD.
#include "gp_api.h"
#include "gp_common.h"

namespace {

constexpr int kBM = 256, kBN = 128, kBK = 64;
constexpr int kThreads = 512;
constexpr int kATile = kBM * kBK * 2;         // 32 KiB: 256 rows x 128 B
constexpr int kWTile = kBN * kBK * 2;         // 16 KiB: 128 rows x 128 B
constexpr int kStage = kATile + kWTile;       // 48 KiB
constexpr int kStages = 3;                    // ring: tile kt + 2 in flight while tile kt is computed
constexpr int kGldsA = kATile / 1024 / 8;     // LDS-DMA instructions per wave per tile: 4 (A) + 2 (W)
constexpr int kGldsW = kWTile / 1024 / 8;
constexpr int kGlds = kGldsA + kGldsW;

typedef float f32x4v __attribute__((ext_vector_type(4)));

GP_DEV int swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// bijective XCD remap: ids that share an XCD (b, b + 8, ...) become consecutive tile ids
GP_DEV int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

struct GemmArgs {
  const uint16_t* A;
  const uint16_t* W;
  const void* bias;     // [N] bf16 (bias_f32 == 0) or fp32, or null
  uint16_t* C;
  int64_t lda, ldw, ldc;
  int M, N, K;
  int bias_f32;
};

// s_waitcnt with vmcnt = n (expcnt, lgkmcnt untouched): gfx9 encoding vmcnt[3:0] | vmcnt[5:4] << 14
template <int n>
GP_DEV void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}

__global__ __launch_bounds__(kThreads, 1) void gemm_bf16_tn_kernel(const GemmArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[kStages * kStage];
  const int tiles_n = g.N / kBN;
  const int tiles_m = (g.M + kBM - 1) / kBM;
  const int tid = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int tm = tid / tiles_n, tn = tid % tiles_n;
  if (tm >= tiles_m) return;
  const int m0 = tm * kBM, n0 = tn * kBN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;          // wave tile: rows wm*64 .., cols wn*64 ..

  // ---- LDS-DMA staging: instruction i covers tile rows 8i .. 8i+7; lane l writes row 8i + l/8, chunk
  // position l % 8, which holds the logical chunk (l % 8) ^ ((row >> 1) & 7)
  const int64_t a_bytes = (int64_t)(g.M - m0) * g.lda * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.A + (int64_t)m0 * g.lda), (short)0, (int)(a_bytes < 0x7fffffff ? a_bytes : 0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.W + (int64_t)n0 * g.ldw), (short)0, (int)((int64_t)kBN * g.ldw * 2), 0x00020000);
  int voff_a[kGldsA], voff_w[kGldsW];
#pragma unroll
  for (int j = 0; j < kGldsA; ++j) {
    const int r = 8 * (w + 8 * j) + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
    voff_a[j] = (int)((int64_t)r * g.lda * 2) + c * 16;
  }
#pragma unroll
  for (int j = 0; j < kGldsW; ++j) {
    const int r = 8 * (w + 8 * j) + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
    voff_w[j] = (int)((int64_t)r * g.ldw * 2) + c * 16;
  }
  auto stage = [&](int kt, int slot) {
    char* base = smem + slot * kStage;
#pragma unroll
    for (int j = 0; j < kGldsA; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(base + (w + 8 * j) * 1024),
                                               16, voff_a[j] + kt * kBK * 2, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < kGldsW; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(base + kATile + (w + 8 * j) * 1024),
                                               16, voff_w[j] + kt * kBK * 2, 0, 0, 0);
  };

  f32x4v acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lq = lane >> 4;
  auto compute = [&](int slot) {
    const char* As = smem + slot * kStage;
    const char* Ws = As + kATile;
    bf16x8 af[2][4], wf[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        wf[ks][ni] = *reinterpret_cast<const bf16x8*>(Ws + swz(wn * 64 + ni * 16 + lr, 4 * ks + lq));
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
        af[ks][mi] = *reinterpret_cast<const bf16x8*>(As + swz(wm * 64 + mi * 16 + lr, 4 * ks + lq));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][ni], af[ks][mi], acc[mi][ni], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // ring of three stages; at tile kt: wait for tile kt's DMA (tile kt + 1's may stay in flight), barrier
  // (every wave has also finished reading tile kt - 1), refill tile kt - 1's slot with tile kt + 2,
  // compute tile kt.  The loop is unrolled by three so each slot index is a compile-time constant.
  // (Measured and dropped: SIMD partners staggered by half a tile -- 2 barriers per tile -- 7-12 % slower.)
  const int nk = g.K / kBK;
  stage(0, 0);
  if (nk > 1) stage(1, 1);
  auto step = [&](int kt, auto slotc) {
    constexpr int S = decltype(slotc)::value;
    if (kt + 1 < nk) wait_vmcnt<kGlds>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) stage(kt + 2, (S + 2) % kStages);
    compute(S);
  };
  for (int kt = 0; kt < nk; kt += 3) {
    step(kt, std::integral_constant<int, 0>());
    if (kt + 1 < nk) step(kt + 1, std::integral_constant<int, 1>());
    if (kt + 2 < nk) step(kt + 2, std::integral_constant<int, 2>());
  }

  // ---- epilogue: lane holds C[m][n .. n+3] for m = row base + lr, n = col base + 4 * lq
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + 4 * lq;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (g.bias != nullptr) {
      if (g.bias_f32) {
        const float4 b4 = *reinterpret_cast<const float4*>(static_cast<const float*>(g.bias) + n);
        bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w;
      } else {
        load_bf16<4>(static_cast<const uint16_t*>(g.bias) + n, bv);
      }
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int m = m0 + wm * 64 + mi * 16 + lr;
      if (m < g.M) {
        float v[4] = {acc[mi][ni][0] + bv[0], acc[mi][ni][1] + bv[1], acc[mi][ni][2] + bv[2], acc[mi][ni][3] + bv[3]};
        store_bf16<4>(g.C + (int64_t)m * g.ldc + n, v);
      }
    }
  }
}

}  // namespace

extern "C" int gp_gemm_bf16_tn(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, const void* bias,
                               int bias_is_f32, uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                               void* stream) {
  GP_REQUIRE(A && W && C, "gp_gemm_bf16_tn: null pointer");
  GP_REQUIRE(M > 0 && M < (int64_t)0x7fffffff && N > 0 && K > 0, "gp_gemm_bf16_tn: bad sizes");
  GP_REQUIRE(N % kBN == 0 && K % kBK == 0, "gp_gemm_bf16_tn: N must be a multiple of %d and K of %d (N=%lld K=%lld)",
             kBN, kBK, (long long)N, (long long)K);
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
  gemm_bf16_tn_kernel<<<(unsigned)tiles, kThreads, 0, gp_stream(stream)>>>(g);
  return gp_check_launch("gp_gemm_bf16_tn");
}
