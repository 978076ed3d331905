// Persistent bf16 GEMM for the TinyGPT forward and dX products (included by gemm.hip).
//
// Both operands K-contiguous, no split-K, K % 64 == 0 and K >= 128.  One 512-thread
// workgroup per CU walks its tiles (256x128, 8 waves of 64x64, v_mfma_f32_16x16x32_bf16)
// with ONE LDS-DMA ring (3 stages of 48 KiB) that never drains between tiles: the DMAs of a
// tile's first two k-steps are issued during the previous tile's last two k-steps, so the
// pipeline fill and the epilogue of tile i overlap the operand stream of tile i+1.
//
// The epilogue needs no LDS.  The MFMA operands are swapped (D = B_frag x A_frag, i.e. the
// tile is computed transposed) and the B rows are fed in a permuted order, so that after
// the k-loop every lane owns 16 consecutive output columns of 4 rows (two 8-column chunks):
// bias / GELU / dGELU / dropout / residual are applied in registers and every global access
// is a 16-byte buffer load/store.  All epilogue accesses are buffer ops with out-of-range
// offsets for rows/columns outside the matrix, so every wave issues the same compile-time
// number of VMEM ops (E) and the counted vmcnt waits of the next tile's first two k-steps
// can leave the epilogue's stores in flight (vmcnt counts loads, stores and LDS-DMA in
// issue order).
namespace bfp {
using bfw::A_BYTES;
using bfw::A_CHUNKS;
using bfw::B_CHUNKS;
using bfw::BKT;
using bfw::BM;
using bfw::BN;
using bfw::STAGE_BYTES;
using bfw::STAGES;
using bfw::THREADS;
using bfw::WAVES;
constexpr int SMEM = STAGES * STAGE_BYTES;  // 144 KiB
constexpr int DMA_PER_STAGE = A_CHUNKS + B_CHUNKS;
constexpr uint32_t OOR = 0x80000000u;  // voffset past every range used here (host: extents < 2^31 - 2^24)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// B image [128 rows][64 bf16], 16-B chunk `ch` of row r stored at chunk ch ^ fb(r): with the
// permuted fragment rows below every ds_read_b128 lane group hits 16 distinct bank slots.
__device__ __forceinline__ int fb(int row) { return (row & 2) | ((row >> 1) & 4); }
__device__ __forceinline__ uint32_t b_src_off(int pos, long long ld) {
  const int row = pos >> 7, phys = (pos >> 4) & 7;
  return (uint32_t)(((long long)row * ld + 8 * (phys ^ fb(row))) * 2);
}
// fragment of B for output-column block j (it sits in the MFMA's A slot): lane l supplies the
// row that makes D[4g+v][l&15] land on column wn + 32(j>>1) + 8g + 4(j&1) + v
__device__ __forceinline__ v8bf bfrag(const char* img, int wn, int j, int ks, int lane) {
  const int nl = lane & 15;
  const int row = wn + 32 * (j >> 1) + 8 * (nl >> 2) + 4 * (j & 1) + (nl & 3);
  const int ch = ks * 4 + (lane >> 4);
  return *(const v8bf*)(img + row * 128 + 16 * (ch ^ fb(row)));
}

template <int EPI, int CT>
struct Epi {
  static constexpr int W = CT == CG_BF16 ? 1 : 2;  // 16-B accesses per 8 values of C dtype
  static constexpr bool SWG = EPI == CG_EPI_SWIGLU, DSW = EPI == CG_EPI_DSWIGLU;
  // epilogue operand LOADS (bias, residual, dGELU pre-activation, accumulate source, SwiGLU
  // gate|up), issued at the top of the tile's last k-step, before that step's DMAs
  static constexpr int L = DSW ? 16
                               : 8 * (((EPI & CG_EPI_RESID) ? 2 : 0) + ((EPI & CG_EPI_DGELU) ? W : 0) +
                                      ((EPI & CG_EPI_ACCUM) ? 2 : 0)) + ((EPI & CG_EPI_BIAS) ? 4 : 0);
  // epilogue STORES (C, GELU pre-activation, column-sum partials; SwiGLU: g, u, s per row chunk /
  // d(g), d(u) per chunk), issued after the last k-step
  static constexpr int S = SWG ? 12 : DSW ? 16 : 8 * (W + ((EPI & CG_EPI_GELU) ? W : 0)) + ((EPI & CG_EPI_COLSUM) ? 4 : 0);
};
// SwiGLU B image: tile row r holds B row ((r >> 5) & 1) * N + 32 (r >> 6) + (r & 31) of [gate; up]
// (N rows each), so a wave's column chunk c = 0 is gate j and c = 1 is up j for the same j
__device__ __forceinline__ uint32_t b_src_off_swg(int pos, long long ld, int N) {
  const int row = pos >> 7, phys = (pos >> 4) & 7;
  const int brow = ((row >> 5) & 1) * N + 32 * (row >> 6) + (row & 31);
  return (uint32_t)(((long long)brow * ld + 8 * (phys ^ fb(row))) * 2);
}

__device__ __forceinline__ u32x4 bld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
// epilogue stores with the default cache policy (sc1 and nt measured no faster / slower: the
// outputs are re-read by the next product)
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}
// the GELU-derivative / pre-activation store: read again only by the backward, after the rest of
// the forward has streamed through L2 and the Infinity Cache, so it is written nontemporal
// (cache-policy bit nt = 2 on gfx950).  Round 5, same-box A/B of the C4 step: default policy
// 15.13 ms, nt 14.92 ms, sc0 sc1 15.23 ms (profiles/round5/nt_stores_ab.txt).
__device__ __forceinline__ void bst_aux(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 2);
}
__device__ __forceinline__ void unpack_f32(u32x4 a, u32x4 b, float v[8]) {
  v[0] = __uint_as_float(a.x); v[1] = __uint_as_float(a.y); v[2] = __uint_as_float(a.z); v[3] = __uint_as_float(a.w);
  v[4] = __uint_as_float(b.x); v[5] = __uint_as_float(b.y); v[6] = __uint_as_float(b.z); v[7] = __uint_as_float(b.w);
}
__device__ __forceinline__ void unpack_bf16(u32x4 a, float v[8]) {
  const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
  }
}
typedef float v2f_t __attribute__((ext_vector_type(2)));
typedef __bf16 v2bf_t __attribute__((ext_vector_type(2)));
// one v_cvt_pk_bf16_f32 per pair (RNE, NaN kept)
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((v2f_t){a, b}, v2bf_t));
}
__device__ __forceinline__ u32x4 pack_bf16(const float v[8]) {
  return (u32x4){pk2(v[0], v[1]), pk2(v[2], v[3]), pk2(v[4], v[5]), pk2(v[6], v[7])};
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
// sum over each 16-lane row by DPP moves (VALU, no LDS): quad xor 1, quad xor 2, row_half_mirror,
// row_mirror -- every lane of the row ends with the row's total
__device__ __forceinline__ float dpp_sum16(float t) {
  t += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0xB1, 0xF, 0xF, false));
  t += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0x4E, 0xF, 0xF, false));
  t += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0x141, 0xF, 0xF, false));
  t += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0x140, 0xF, 0xF, false));
  return t;
}
#define PMFMA(b, a, c, x, y, z) __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c, x, y, z)
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
}  // namespace bfp

template <int EPI, int CT>
__global__ __launch_bounds__(512, 1) void gemm_bf16_pers_kernel(GemmParams p) {
  using namespace bfp;
  constexpr int NL = Epi<EPI, CT>::L, NS = Epi<EPI, CT>::S;
  constexpr bool SWG = Epi<EPI, CT>::SWG, DSW = Epi<EPI, CT>::DSW;
  constexpr int BNO = SWG ? BN / 2 : BN;  // output columns per tile (SwiGLU: 64 s-columns from 128 B rows)
  constexpr int ES = CT == CG_BF16 ? 2 : 4;
  static_assert(NL + NS + DMA_PER_STAGE <= 63, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tiles_n = (p.N + BNO - 1) / BNO, tiles_m = (p.M + BM - 1) / BM;
  const int ntiles = tiles_n * tiles_m;
  const int nblk = gridDim.x;
  const int lb = cg_xcd_remap(blockIdx.x, nblk);  // an XCD's blocks walk contiguous tile ranges
  const int my_tiles = lb < ntiles ? (ntiles - 1 - lb) / nblk + 1 : 0;
  const int nt = p.K / BKT;
  const int S = my_tiles * nt;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  const __amdgpu_buffer_rsrc_t ra = rsrc(p.A, ((long long)(p.M - 1) * p.lda + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = rsrc(p.B, ((long long)((SWG ? 2 : 1) * p.N - 1) * p.ldb + p.K) * 2);
  uint32_t va[A_CHUNKS], vb[B_CHUNKS];
#pragma unroll
  for (int i = 0; i < A_CHUNKS; ++i) va[i] = bfw::src_off<true>((wave + WAVES * i) * 1024 + 16 * lane, p.lda);
#pragma unroll
  for (int i = 0; i < B_CHUNKS; ++i) {
    const int pos = (wave + WAVES * i) * 1024 + 16 * lane;
    vb[i] = SWG ? b_src_off_swg(pos, p.ldb, p.N) : b_src_off(pos, p.ldb);
  }

  auto tile_org = [&](int k, int& m0, int& n0) __attribute__((always_inline)) {
    const int tile = lb + k * nblk;
    m0 = (tile / tiles_n) * BM;
    n0 = (tile % tiles_n) * BNO;
  };
  // DMA source origins of global k-step g (OOR past the end: the DMA then fills a free slot with zeros)
  auto stage_org = [&](int g, uint32_t& ao, uint32_t& bo) __attribute__((always_inline)) {
    if (g >= S) {
      ao = bo = OOR;
      return;
    }
    const int k = g / nt, t = g - k * nt;
    int m0, n0;
    tile_org(k, m0, n0);
    ao = (uint32_t)(((long long)m0 * p.lda + t * BKT) * 2);
    bo = (uint32_t)(((long long)n0 * p.ldb + t * BKT) * 2);
  };
  auto issue = [&](int g) __attribute__((always_inline)) {
    uint32_t ao, bo;
    stage_org(g, ao, bo);
    char* st = smem + (g % STAGES) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) bfw::dma16(ra, st + (wave + WAVES * i) * 1024, ao + va[i]);
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) bfw::dma16(rb, st + A_BYTES + (wave + WAVES * i) * 1024, bo + vb[i]);
  };

  // epilogue of local tile k straight from the accumulators: lane owns rows
  // m0+wm+16i+(l&15) (i = 0..3) x columns n0+wn+32c+8(l>>4)+[0,8) (c = 0..1)
  const __amdgpu_buffer_rsrc_t rc = rsrc(p.C, ((long long)(p.M - 1) * p.ldc + (DSW ? 2 : 1) * p.N) * ES);
  const int g4 = lane >> 4, r16 = lane & 15;
  u32x4 xa[4][2], xb[4][2], bq[2][2];
  uint32_t off_c[4][2];
  int col[2];
  // operand loads of tile k (issued in its last k-step so that the compiler's wait for them in
  // the epilogue does not also wait for the next tile's stage DMAs)
  auto epi_loads_rows = [&](int k, auto lo_t, auto hi_t, auto bias_t) __attribute__((always_inline)) {
    constexpr int LO = decltype(lo_t)::value, HI = decltype(hi_t)::value;
    int m0, n0;
    tile_org(k, m0, n0);
    bool cok[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      col[c] = SWG ? n0 + (wn >> 1) + 8 * g4 : n0 + wn + 32 * c + 8 * g4;
      cok[c] = col[c] < p.N;
    }
    if constexpr (decltype(bias_t)::value && (EPI & CG_EPI_BIAS) != 0) {
      const __amdgpu_buffer_rsrc_t rbias = rsrc(p.bias, (long long)p.N * 4);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const uint32_t o = cok[c] ? (uint32_t)col[c] * 4u : OOR;
        bq[c][0] = bld(rbias, o);
        bq[c][1] = bld(rbias, o + 16);
      }
    }
#pragma unroll
    for (int i = LO; i < HI; ++i) {
      const int row = m0 + wm + 16 * i + r16;
      const bool rok = row < p.M;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bool ok = rok && cok[c];
        off_c[i][c] = ok ? (uint32_t)(((long long)row * p.ldc + col[c]) * ES) : OOR;
        if constexpr ((EPI & CG_EPI_RESID) != 0) {
          const __amdgpu_buffer_rsrc_t rr = rsrc(p.resid, ((long long)(p.M - 1) * p.ldr + p.N) * 4);
          const uint32_t o = ok ? (uint32_t)(((long long)row * p.ldr + col[c]) * 4) : OOR;
          xa[i][c] = bld(rr, o);
          xb[i][c] = bld(rr, o + 16);
        }
        if constexpr ((EPI & CG_EPI_DGELU) != 0) {
          const __amdgpu_buffer_rsrc_t rx = rsrc(p.aux, ((long long)(p.M - 1) * p.ld_aux + p.N) * ES);
          const uint32_t o = ok ? (uint32_t)(((long long)row * p.ld_aux + col[c]) * ES) : OOR;
          xa[i][c] = bld(rx, o);
          if constexpr (CT != CG_BF16) xb[i][c] = bld(rx, o + 16);
        }
        if constexpr ((EPI & CG_EPI_ACCUM) != 0) {
          xa[i][c] = bld(rc, off_c[i][c]);
          xb[i][c] = bld(rc, off_c[i][c] + 16);
        }
        if constexpr (DSW) {  // gate at column col, up at N + col of aux
          const __amdgpu_buffer_rsrc_t rx = rsrc(p.aux, ((long long)(p.M - 1) * p.ld_aux + 2 * p.N) * 2);
          const uint32_t o = ok ? (uint32_t)(((long long)row * p.ld_aux + col[c]) * 2) : OOR;
          xa[i][c] = bld(rx, o);
          xb[i][c] = bld(rx, ok ? o + (uint32_t)p.N * 2u : OOR);
        }
      }
    }
  };
  auto epi_loads = [&](int k) __attribute__((always_inline)) {
    epi_loads_rows(k, std::integral_constant<int, 0>{}, std::integral_constant<int, 4>{}, std::true_type{});
  };
  v4f acc[4][4];
  // one k-step of global index g (the DMAs of stage g+2 interleaved with the MFMAs, as in the
  // non-persistent 256x128 kernel; they are always issued, so every step carries 6)
  // VMEM ops issued after stage g's DMAs, by position of step g in its tile (k = tile, t = step):
  // stage g+1's DMAs always; the previous tile's epilogue stores when t < 2; its operand loads
  // (issued in its last step, before that step's DMAs) when t == 0
  auto step = [&](int g, auto&& wait_fn, auto&& after_fn, auto last_tag) __attribute__((always_inline)) {
    wait_fn();
    __builtin_amdgcn_s_barrier();
    if constexpr (decltype(last_tag)::value) epi_loads(g / nt);
    const char* st = smem + (g % STAGES) * STAGE_BYTES;
    const char* as = st;
    const char* bs = st + A_BYTES;
    v8bf af[2][4], bfr[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[0][i] = bfg::frag<true>(as, wm + 16 * i, 0, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[0][j] = bfrag(bs, wn, j, 0, lane);
    uint32_t ao, bo;
    stage_org(g + 2, ao, bo);
    char* nx = smem + ((g + 2) % STAGES) * STAGE_BYTES;
#pragma unroll
    for (int gr = 0; gr < 8; ++gr) {
      const int i = gr >> 1, j0 = 2 * (gr & 1);
      acc[i][j0] = PMFMA(bfr[0][j0], af[0][i], acc[i][j0], 0, 0, 0);
      acc[i][j0 + 1] = PMFMA(bfr[0][j0 + 1], af[0][i], acc[i][j0 + 1], 0, 0, 0);
      if (gr < 4) af[1][gr] = bfg::frag<true>(as, wm + 16 * gr, 1, lane);
      else bfr[1][gr - 4] = bfrag(bs, wn, gr - 4, 1, lane);
      if (gr < A_CHUNKS) bfw::dma16(ra, nx + (wave + WAVES * gr) * 1024, ao + va[gr]);
      else if (gr < A_CHUNKS + B_CHUNKS)
        bfw::dma16(rb, nx + A_BYTES + (wave + WAVES * (gr - A_CHUNKS)) * 1024, bo + vb[gr - A_CHUNKS]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = PMFMA(bfr[1][j], af[1][i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int gr = 0; gr < 8; ++gr) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if (gr < A_CHUNKS + B_CHUNKS) __builtin_amdgcn_sched_group_barrier(SGB_DMA, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
    after_fn();
  };

  // Prefetching step (default): the half-0 fragments of step g are read at the END of step g-1 --
  // after its first eight half-1 MFMAs it waits for stage g's DMAs (its own `vmcnt`, then
  // lgkmcnt(0) so no wave still reads the slot the next DMAs overwrite), meets the other waves at
  // the barrier and issues the eight reads under its last eight MFMAs -- so a step starts with
  // MFMAs instead of LDS latency.  Only a tile's first step syncs at its top (the tile's last
  // step is followed by the epilogue, which must not hold 32 more registers).  Waits: the top one
  // as in `step`; the mid one (stage g+1 of step g) counts the ops issued after DMA(g+1): the
  // pieces / epilogue stores after step g-1 and this step's 6 DMAs.
  // not for the fp32-residual and SwiGLU-backward epilogues: their piece registers plus the
  // prefetched fragments exceed 256 VGPRs (spills)
  constexpr bool PREF = !DSW && (EPI & CG_EPI_RESID) == 0;
  v8bf f0a[4], f0b[4];
  auto read_half0 = [&](int g) __attribute__((always_inline)) {
    const char* st = smem + (g % STAGES) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) f0a[i] = bfg::frag<true>(st, wm + 16 * i, 0, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) f0b[j] = bfrag(st + A_BYTES, wn, j, 0, lane);
  };
  auto pstep = [&](int g, bool top, auto&& wait_top, auto mid_tag, auto&& wait_mid, auto&& after_fn,
                   auto last_tag) __attribute__((always_inline)) {
    constexpr bool MID = decltype(mid_tag)::value;
    if (top) {
      wait_top();
      __builtin_amdgcn_s_barrier();
      read_half0(g);
    }
    if constexpr (decltype(last_tag)::value) epi_loads(g / nt);
    const char* st = smem + (g % STAGES) * STAGE_BYTES;
    const char* as = st;
    const char* bs = st + A_BYTES;
    v8bf af1[4], bf1[4];
    uint32_t ao, bo;
    stage_org(g + 2, ao, bo);
    char* nx = smem + ((g + 2) % STAGES) * STAGE_BYTES;
#pragma unroll
    for (int gr = 0; gr < 8; ++gr) {
      const int i = gr >> 1, j0 = 2 * (gr & 1);
      acc[i][j0] = PMFMA(f0b[j0], f0a[i], acc[i][j0], 0, 0, 0);
      acc[i][j0 + 1] = PMFMA(f0b[j0 + 1], f0a[i], acc[i][j0 + 1], 0, 0, 0);
      if (gr < 4) af1[gr] = bfg::frag<true>(as, wm + 16 * gr, 1, lane);
      else bf1[gr - 4] = bfrag(bs, wn, gr - 4, 1, lane);
      if (gr < A_CHUNKS) bfw::dma16(ra, nx + (wave + WAVES * gr) * 1024, ao + va[gr]);
      else if (gr < A_CHUNKS + B_CHUNKS)
        bfw::dma16(rb, nx + A_BYTES + (wave + WAVES * (gr - A_CHUNKS)) * 1024, bo + vb[gr - A_CHUNKS]);
    }
    if constexpr (MID) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = PMFMA(bf1[j], af1[i], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int gr = 0; gr < 8; ++gr) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if (gr < A_CHUNKS + B_CHUNKS) __builtin_amdgcn_sched_group_barrier(SGB_DMA, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_barrier(0);
      wait_mid();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      read_half0(g + 1);
#pragma unroll
      for (int i = 2; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = PMFMA(bf1[j], af1[i], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int gr = 0; gr < 8; ++gr) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = PMFMA(bf1[j], af1[i], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int gr = 0; gr < 8; ++gr) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if (gr < A_CHUNKS + B_CHUNKS) __builtin_amdgcn_sched_group_barrier(SGB_DMA, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
    }
    after_fn();
  };

  const bool scaled = p.alpha != 1.0f;
  auto epilogue = [&](int k) __attribute__((always_inline)) {
    int m0, n0;
    tile_org(k, m0, n0);
    // alpha != 1 (the tied head's scaled gradient) is rare: a real branch (the empty volatile asm
    // keeps hipcc from if-converting it into 64 selects per tile on every epilogue)
    if (__builtin_expect(scaled, 0)) {
      asm volatile("");
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] *= p.alpha;
    }
    float bia[2][8];
    if constexpr ((EPI & CG_EPI_BIAS) != 0) {
#pragma unroll
      for (int c = 0; c < 2; ++c) unpack_f32(bq[c][0], bq[c][1], bia[c]);
    }
    float csum[2][8];
    if constexpr ((EPI & CG_EPI_COLSUM) != 0) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) csum[c][j] = 0.f;
    }
    if constexpr (SWG) {
      // chunk 0 = gate, chunk 1 = up of the same 8 columns j: pre-activations to aux_out (g at j,
      // u at N + j), s = silu(g) * u to C (0 past n_valid)
      const __amdgpu_buffer_rsrc_t rx = rsrc(p.aux_out, ((long long)(p.M - 1) * p.ld_aux + 2 * p.N) * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wm + 16 * i + r16;
        float g[8], u[8], sv[8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            g[4 * h + q] = acc[i][h][q];
            u[4 * h + q] = acc[i][2 + h][q];
          }
        const bool ok = off_c[i][0] != OOR;
        const uint32_t o = ok ? (uint32_t)(((long long)row * p.ld_aux + col[0]) * 2) : OOR;
        bst_aux(rx, o, pack_bf16(g));  // (read again only by the backward: nontemporal)
        bst_aux(rx, ok ? o + (uint32_t)p.N * 2u : OOR, pack_bf16(u));
#pragma unroll
        for (int j = 0; j < 8; ++j) sv[j] = col[0] + j < p.n_valid ? silu_f(g[j]) * u[j] : 0.f;
        bst(rc, off_c[i][0], pack_bf16(sv));
      }
      return;
    } else if constexpr (DSW) {
      // v = dL/ds for columns j: d(g) to C at j, d(u) to C at N + j (0 past n_valid)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          float v[8], g[8], u[8], dg[8], du[8];
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int q = 0; q < 4; ++q) v[4 * h + q] = acc[i][2 * c + h][q];
          unpack_bf16(xa[i][c], g);
          unpack_bf16(xb[i][c], u);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            dg[j] = du[j] = 0.f;
            if (col[c] + j < p.n_valid) {
              const float sg = 1.0f / (1.0f + __expf(-g[j]));
              du[j] = v[j] * (g[j] * sg);
              dg[j] = v[j] * u[j] * sg * (1.0f + g[j] * (1.0f - sg));
            }
          }
          bst(rc, off_c[i][c], pack_bf16(dg));
          bst(rc, off_c[i][c] == OOR ? OOR : off_c[i][c] + (uint32_t)p.N * 2u, pack_bf16(du));
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + wm + 16 * i + r16;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float v[8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int u = 0; u < 4; ++u) v[4 * h + u] = acc[i][2 * c + h][u];
        if constexpr ((EPI & CG_EPI_BIAS) != 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += bia[c][j];
        }
        if constexpr ((EPI & CG_EPI_GELU) != 0) {
          const __amdgpu_buffer_rsrc_t rx = rsrc(p.aux_out, ((long long)(p.M - 1) * p.ld_aux + p.N) * ES);
          const uint32_t o = off_c[i][c] == OOR ? OOR : (uint32_t)(((long long)row * p.ld_aux + col[c]) * ES);
          float s[8];  // what aux_out receives: the pre-activation, or gelu' of it
          if constexpr ((EPI & CG_EPI_GELU_DERIV) != 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = gelu_fast_d(v[j], s[j]);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] = v[j];
          }
          if constexpr (CT == CG_BF16) {
            bst_aux(rx, o, pack_bf16(s));
          } else {
            bst(rx, o, (u32x4){__float_as_uint(s[0]), __float_as_uint(s[1]), __float_as_uint(s[2]), __float_as_uint(s[3])});
            bst(rx, o + 16, (u32x4){__float_as_uint(s[4]), __float_as_uint(s[5]), __float_as_uint(s[6]), __float_as_uint(s[7])});
          }
          if constexpr ((EPI & CG_EPI_GELU_DERIV) == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = gelu_fast(v[j]);
          }
        }
        if constexpr ((EPI & CG_EPI_DGELU) != 0) {
          float a[8];
          if constexpr (CT == CG_BF16) unpack_bf16(xa[i][c], a);
          else unpack_f32(xa[i][c], xb[i][c], a);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= (EPI & CG_EPI_GELU_DERIV) ? a[j] : dgelu_fast(a[j]);
        }
        if constexpr ((EPI & CG_EPI_DROPOUT) != 0) {
          const uint32_t rh = cg_row_hash(p.drop_seed, (uint32_t)row);
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const uint32_t hsh = cg_pair_mix(rh + ((uint32_t)(col[c] + j) >> 1) * CG_COLK);
            v[j] = (hsh & 0xFFFFu) >= p.drop_thr ? v[j] * p.drop_scale : 0.f;
            v[j + 1] = (hsh >> 16) >= p.drop_thr ? v[j + 1] * p.drop_scale : 0.f;
          }
        }
        if constexpr ((EPI & (CG_EPI_RESID | CG_EPI_ACCUM)) != 0) {
          float r[8];
          unpack_f32(xa[i][c], xb[i][c], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += r[j];
        }
        if constexpr ((EPI & CG_EPI_COLSUM) != 0) {
          const float keep = row < p.M ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) csum[c][j] = fmaf(keep, v[j], csum[c][j]);
        }
        if constexpr (CT == CG_BF16) {
          bst(rc, off_c[i][c], pack_bf16(v));
        } else {
          bst(rc, off_c[i][c], (u32x4){__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])});
          bst(rc, off_c[i][c] + 16, (u32x4){__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7])});
        }
      }
    }
    if constexpr ((EPI & CG_EPI_COLSUM) != 0) {
      // sum over the 16 row lanes sharing these columns, then lane r16 == 0 writes the wave's
      // 64-row partial (every lane issues the stores; the others at an out-of-range offset)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) csum[c][j] = dpp_sum16(csum[c][j]);
      const int prow = (m0 + wm) >> 6;
      const __amdgpu_buffer_rsrc_t rw = rsrc(p.ws, (long long)((p.M + 63) >> 6) * p.N * 4);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const uint32_t o = (r16 == 0 && col[c] < p.N) ? (uint32_t)(((long long)prow * p.N + col[c]) * 4) : OOR;
        bst(rw, o, (u32x4){__float_as_uint(csum[c][0]), __float_as_uint(csum[c][1]), __float_as_uint(csum[c][2]),
                           __float_as_uint(csum[c][3])});
        bst(rw, o + 16, (u32x4){__float_as_uint(csum[c][4]), __float_as_uint(csum[c][5]), __float_as_uint(csum[c][6]),
                                __float_as_uint(csum[c][7])});
      }
    }
  };

  // Epilogue operand loads (NL > 0).  NP == 0: all of them at the top of the tile's last k-step,
  // before its DMAs.  NP > 0 (nt >= 4): in NP pieces -- piece q loads the lane's row groups
  // i in [4q/NP, 4(q+1)/NP) (+ the bias with piece 0) -- issued after ALL of step nt-1-NP+q's DMAs
  // and MFMAs.  A piece then has until the wait of the step three later (which needs the DMAs
  // issued after it) to land, instead of one k-step, and the loads of all CUs do not arrive as one
  // burst at the tile's end (C4 dX of fc2 with dGELU: +25 us over the plain product).  Every wait
  // counts exactly the VMEM ops issued after the stage it needs: the stage after it (6 DMAs) plus
  // the pieces / epilogue stores issued after each of the two steps before.
  const auto nopf = [] {};
  auto tiles = [&](auto np_t) __attribute__((always_inline)) {
    constexpr int NP = decltype(np_t)::value;
    constexpr int PI = NP ? (NL - ((EPI & CG_EPI_BIAS) ? 4 : 0)) / 4 : 0;  // ops per row group
    constexpr int NB = (EPI & CG_EPI_BIAS) ? 4 : 0;
    // ops of piece x (0 outside [0, NP))
    constexpr auto pc = [](int x) constexpr {
      return (x < 0 || x >= NP) ? 0 : PI * (4 * (x + 1) / (NP ? NP : 1) - 4 * x / (NP ? NP : 1)) + (x == 0 ? NB : 0);
    };
    constexpr int WL = NP ? pc(NP - 1) : NL;  // ops issued after the last stage of the previous tile
    issue(0);
    issue(1);
    int g = 0;
    for (int k = 0; k < my_tiles; ++k) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
      const int tl = NP ? nt - 1 - NP : nt - 1;  // steps of the runtime loop (NP > 0: >= 2)
      if constexpr (PREF) {
      for (int t = 0; t < tl; ++t, ++g) {
        const bool top = t == 0;
        const int sel = k > 0 ? 2 : 0;
        const bool msel = t == 0 && k > 0;
        pstep(
            g, top,
            [&] {
              if (sel == 0) wait_vm<DMA_PER_STAGE>();
              else wait_vm<DMA_PER_STAGE + NS + WL>();
            },
            std::true_type{},
            [&] {
              if (msel) wait_vm<DMA_PER_STAGE + NS>();
              else wait_vm<DMA_PER_STAGE>();
            },
            nopf, std::false_type{});
      }
      if constexpr (NP == 0) {
        pstep(g, false, nopf, std::false_type{}, nopf, nopf, std::true_type{});
        ++g;
      } else {
        auto tail = [&](auto q_t) __attribute__((always_inline)) {
          constexpr int Q = decltype(q_t)::value;
          constexpr int WM = DMA_PER_STAGE + pc(Q - 1);
          pstep(
              g, false, nopf, std::bool_constant<(Q < NP)>{}, [] { wait_vm<WM>(); },
              [&] {
                if constexpr (Q < NP) {
                  __builtin_amdgcn_sched_barrier(0);  // after this step's DMAs, in program order
                  epi_loads_rows(k, std::integral_constant<int, 4 * Q / NP>{},
                                 std::integral_constant<int, 4 * (Q + 1) / NP>{}, std::bool_constant<Q == 0>{});
                }
              },
              std::false_type{});
          ++g;
        };
        tail(std::integral_constant<int, 0>{});
        tail(std::integral_constant<int, 1>{});
        if constexpr (NP >= 2) tail(std::integral_constant<int, 2>{});
        if constexpr (NP >= 4) {
          tail(std::integral_constant<int, 3>{});
          tail(std::integral_constant<int, 4>{});
        }
      }
      epilogue(k);
      continue;
      }
      for (int t = 0; t < tl; ++t, ++g) {
        const int sel = k > 0 && t < 2 ? (t == 0 ? 2 : 1) : 0;
        step(
            g,
            [&] {
              if (sel == 0) wait_vm<DMA_PER_STAGE>();
              else if (sel == 1) wait_vm<DMA_PER_STAGE + NS>();
              else wait_vm<DMA_PER_STAGE + NS + WL>();
            },
            nopf, std::false_type{});
      }
      if constexpr (NP == 0) {
        const int sel = k > 0 && nt - 1 < 2 ? 1 : 0;  // nt >= 2: the last step is never t == 0
        step(
            g,
            [&] {
              if (sel == 0) wait_vm<DMA_PER_STAGE>();
              else wait_vm<DMA_PER_STAGE + NS>();
            },
            nopf, std::true_type{});
        ++g;
      } else {
        auto tail = [&](auto q_t) __attribute__((always_inline)) {
          constexpr int Q = decltype(q_t)::value;
          constexpr int WN = DMA_PER_STAGE + pc(Q - 2) + pc(Q - 1);
          step(
              g, [] { wait_vm<WN>(); },
              [&] {
                if constexpr (Q < NP) {
                  __builtin_amdgcn_sched_barrier(0);  // after this step's DMAs, in program order
                  epi_loads_rows(k, std::integral_constant<int, 4 * Q / NP>{},
                                 std::integral_constant<int, 4 * (Q + 1) / NP>{}, std::bool_constant<Q == 0>{});
                }
              },
              std::false_type{});
          ++g;
        };
        tail(std::integral_constant<int, 0>{});
        tail(std::integral_constant<int, 1>{});
        if constexpr (NP >= 2) tail(std::integral_constant<int, 2>{});
        if constexpr (NP >= 4) {
          tail(std::integral_constant<int, 3>{});
          tail(std::integral_constant<int, 4>{});
        }
      }
      epilogue(k);
    }
  };
  const int np = NL == 0 ? 0 : nt >= 7 ? 4 : nt >= 5 ? 2 : nt >= 4 ? 1 : 0;
  // DSW: its operands in earlier pieces spill (52 more VGPRs held over 5 steps: 204 -> 256 +
  // scratch; measured slower, round 4), so they load at the top of the tile's last k-step
  if constexpr (NL == 0 || DSW) {
    tiles(std::integral_constant<int, 0>{});
  } else {
    if (np == 4) tiles(std::integral_constant<int, 4>{});
    else if (np == 2) tiles(std::integral_constant<int, 2>{});
    else if (np == 1) tiles(std::integral_constant<int, 1>{});
    else tiles(std::integral_constant<int, 0>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
}
