// Wide bf16 GEMM tile for the large TinyGPT step shapes (included by gemm.hip).
//
// 256x128x64 block tile, 8 waves (4 along M x 2 along N) of 64x64, v_mfma_f32_16x16x32_bf16.
// Operands go global -> LDS with LDS-DMA (buffer_load_dwordx4 ... lds: no VGPR round trip, no
// ds_write pass) into a 3-stage ring; two stages stay in flight across each raw s_barrier
// (counted vmcnt, never drained to 0 inside the k-loop).  The DMA destination is lane-linear
// (1 KiB per wave-instruction), so the XOR swizzle of the images is applied on the per-lane
// SOURCE address and undone by the fragment reads (the same kc_off / mc_off images as the
// 128x128 kernel).  Out-of-range rows/columns of partial tiles read as zero (buffer range
// check) or as in-buffer values that only reach output rows/columns that are not stored.
// Requires K-chunk % 64 == 0.  Blocks are remapped so that the tiles one XCD runs are
// contiguous in (m-tile, n-tile) order: the A rows a block streams stay in that XCD's L2.
#include <type_traits>
namespace bfw {
constexpr int BM = 256, BN = 128, BKT = 64, WAVES = 8, THREADS = 512, STAGES = 3;
constexpr int A_BYTES = BM * BKT * 2;             // 32 KiB
constexpr int B_BYTES = BN * BKT * 2;             // 16 KiB
constexpr int STAGE_BYTES = A_BYTES + B_BYTES;    // 48 KiB
constexpr int A_CHUNKS = A_BYTES / 1024 / WAVES;  // 4 DMA wave-instructions per stage
constexpr int B_CHUNKS = B_BYTES / 1024 / WAVES;  // 2
constexpr int EPI_LD = 68;
constexpr int EPI_BYTES = WAVES * 64 * EPI_LD * 4;
constexpr int SMEM = STAGES * STAGE_BYTES > EPI_BYTES ? STAGES * STAGE_BYTES : EPI_BYTES;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
#ifndef SGB_DMA
#define SGB_DMA 0x020
#endif

// byte offset (into the operand, relative to the tile origin at k = 0) that the lane whose
// DMA destination is image byte `pos` must load.
//   K-contiguous image [rows][64]          : row = pos/128, physical chunk -> logical chunk
//   MN-contiguous image, 128-col sub-images: sub = pos/16K, k-row = (pos%16K)/256
template <bool KC>
__device__ __forceinline__ uint32_t src_off(int pos, long long ld) {
  if (KC) {
    const int row = pos >> 7, phys = (pos >> 4) & 7;
    const int ch = phys ^ ((row >> 1) & 7);
    return (uint32_t)(((long long)row * ld + 8 * ch) * 2);
  } else {
    const int sub = pos >> 14, q = pos & 16383;
    const int krow = q >> 8, phys = (q >> 4) & 15;
    const int ch = phys ^ (((krow & 3) << 2) | ((krow >> 2) & 3));
    return (uint32_t)(((long long)krow * ld + 128 * sub + 8 * ch) * 2);
  }
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, char* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)lds, 16, voff, 0, 0, 0);
}

}  // namespace bfw

template <bool AK, bool BKC, int EPI, int CT>
__global__ __launch_bounds__(512, 1) void gemm_bf16_wide_kernel(GemmParams p) {
  using namespace bfw;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m * p.split;
  const int wg = cg_xcd_remap(blockIdx.x, nwg);
  const int zt = wg / (tiles_n * tiles_m), rem = wg % (tiles_n * tiles_m);
  const int m0 = (rem / tiles_n) * BM, n0 = (rem % tiles_n) * BN;
  const int kbeg = zt * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nt = (kend - kbeg) / BKT;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  // buffer resources: the whole operand (range-checked), origin at this tile's (row, kbeg)
  const bf16_t* A = (const bf16_t*)p.A;
  const bf16_t* B = (const bf16_t*)p.B;
  const long long a_extent = AK ? (long long)(p.M - 1) * p.lda + p.K : (long long)(p.K - 1) * p.lda + p.M;
  const long long b_extent = BKC ? (long long)(p.N - 1) * p.ldb + p.K : (long long)(p.K - 1) * p.ldb + p.N;
  const long long a_org = AK ? (long long)m0 * p.lda + kbeg : (long long)kbeg * p.lda + m0;
  const long long b_org = BKC ? (long long)n0 * p.ldb + kbeg : (long long)kbeg * p.ldb + n0;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)(A + a_org), (short)0, (int)((a_extent - a_org) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(B + b_org), (short)0, (int)((b_extent - b_org) * 2), 0x00020000);
  uint32_t va[A_CHUNKS], vb[B_CHUNKS];
#pragma unroll
  for (int i = 0; i < A_CHUNKS; ++i) va[i] = src_off<AK>((wave + WAVES * i) * 1024 + 16 * lane, p.lda);
#pragma unroll
  for (int i = 0; i < B_CHUNKS; ++i) vb[i] = src_off<BKC>((wave + WAVES * i) * 1024 + 16 * lane, p.ldb);
  const uint32_t a_step = AK ? BKT * 2 : (uint32_t)(BKT * p.lda * 2);
  const uint32_t b_step = BKC ? BKT * 2 : (uint32_t)(BKT * p.ldb * 2);

  auto issue = [&](int t) {
    char* st = smem + (t % STAGES) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) dma16(ra, st + (wave + WAVES * i) * 1024, va[i] + t * a_step);
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) dma16(rb, st + A_BYTES + (wave + WAVES * i) * 1024, vb[i] + t * b_step);
  };

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  // one k-step: barrier (stage t visible, stage t-1 free), both k-halves' fragments read
  // up front, the DMAs of stage t+2 and the second half's fragment reads interleaved with
  // the first half's MFMAs (pinned with sched_group_barrier so no wave stalls on a burst of
  // DMA issue while its SIMD partner idles)
  auto step = [&](int t, auto dma_tag, auto wait_tag) {
    constexpr bool DMA = decltype(dma_tag)::value;
    if constexpr (decltype(wait_tag)::value) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const char* st = smem + (t % STAGES) * STAGE_BYTES;
    const char* as = st + (AK ? 0 : (wm >> 7) * 16384);
    const int ar = AK ? wm : (wm & 127);
    const char* bs = st + A_BYTES;
    v8bf af[2][4], bfr[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[0][i] = bfg::frag<AK>(as, ar + 16 * i, 0, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[0][j] = bfg::frag<BKC>(bs, wn + 16 * j, 0, lane);
    // half 0: per pair of MFMAs one half-1 fragment read and (first 6 pairs) one DMA of
    // stage t+2.  An LDS-DMA is a scheduling boundary, so this source order is the issue order.
    char* nx = smem + ((t + 2) % STAGES) * STAGE_BYTES;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const int i = g >> 1, j0 = 2 * (g & 1);
      acc[i][j0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[0][j0], acc[i][j0], 0, 0, 0);
      acc[i][j0 + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[0][j0 + 1], acc[i][j0 + 1], 0, 0, 0);
      if (g < 4) af[1][g] = bfg::frag<AK>(as, ar + 16 * g, 1, lane);
      else bfr[1][g - 4] = bfg::frag<BKC>(bs, wn + 16 * (g - 4), 1, lane);
      if constexpr (DMA) {
        if (g < A_CHUNKS) dma16(ra, nx + (wave + WAVES * g) * 1024, va[g] + (t + 2) * a_step);
        else if (g < A_CHUNKS + B_CHUNKS)
          dma16(rb, nx + A_BYTES + (wave + WAVES * (g - A_CHUNKS)) * 1024, vb[g - A_CHUNKS] + (t + 2) * b_step);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bfr[1][j], acc[i][j], 0, 0, 0);
    // (a K-contiguous fragment is one ds_read_b128, an MN-contiguous one two ds_read_b64_tr_b16)
    constexpr int RA = AK ? 1 : 2, RB = BKC ? 1 : 2;
    __builtin_amdgcn_sched_group_barrier(0x100, 4 * (RA + RB), 0);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      if (g < 4) __builtin_amdgcn_sched_group_barrier(0x100, RA, 0);
      else __builtin_amdgcn_sched_group_barrier(0x100, RB, 0);
      if constexpr (DMA)
        if (g < A_CHUNKS + B_CHUNKS) __builtin_amdgcn_sched_group_barrier(SGB_DMA, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (nt > 0) issue(0);
  if (nt > 1) issue(1);
  int t = 0;
  for (; t + 2 < nt; ++t) step(t, T_{}, T_{});
  if (t + 1 < nt) step(t++, F_{}, T_{});
  if (t < nt) step(t, F_{}, F_{});
  __syncthreads();  // ring no longer read: reuse it for the epilogue staging
  float* stg = (float*)smem + wave * 64 * EPI_LD;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) stg[(16 * i + 4 * (lane >> 4) + v) * EPI_LD + 16 * j + (lane & 15)] = acc[i][j][v];
  __syncthreads();
#pragma unroll 2
  for (int it = 0; it < 8; ++it) {
    const int c = lane + 64 * it, r = c >> 3, ch = c & 7;
    const int row = m0 + wm + r, col = n0 + wn + ch * 8;
    if (row >= p.M || col >= p.N) continue;
    float v[8];
    ld8f(stg + r * EPI_LD + ch * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= p.alpha;
    if (p.split > 1) {
      st8f(p.ws + ((long long)zt * p.M + row) * p.N + col, v);
      continue;
    }
    epi_apply8<EPI, CT>(p, row, col, v);
  }
}
