// 256x256 ping-pong persistent bf16 GEMM for the wide (N >= 2048) TinyGPT forward / dX products
// (included by gemm.hip after gemm_pp.h): fc1 forward (bias + GELU, gelu' stored) and fc2 dX
// (dGELU + bias-gradient column sums) at C4 -- K-contiguous operands, bf16 output.
//
// Why: measured on the C4 products (tools/pp_diag.sh, diagnostic builds of gemm_pp.h), the
// 256x128x64 k-step is bound by the CU's vector-memory path, not by its MFMAs: with the MFMAs
// removed the k-loop runs at ~1700 cycles per k-step (48 KiB of LDS-DMA), against 1024 MFMA
// cycles per SIMD.  A 256x256 tile moves 1.5x fewer operand bytes per MFMA (and reads 0.75x the
// LDS bytes: 128x64 per wave instead of 64x64), so the operand stream and the MFMAs balance.
//
// Structure: 8 waves, G0 = waves 0-3 (tile rows 0-127), G1 = waves 4-7 (rows 128-255), each wave
// 128 rows x 64 columns (acc[8][4] of 16x16 blocks, v_mfma_f32_16x16x32_bf16, transposed as in
// gemm_pers.h so a lane owns 16 consecutive output columns of 8 rows).  G1 runs one workgroup
// barrier behind G0 (the ping-pong of gemm_pp.h): between two barriers one wave of every SIMD
// runs its 32 MFMAs of a 32-deep k-step while its partner reads its next 12 fragments and issues
// its 4 DMA pieces of the operand stream.  k-step g (BK = 32):
//   L(g): 12 fragment reads from stage g; the 4 DMA pieces of stage g + 3 into the slot of
//         stage g - 1; vmcnt: stage g + 1 landed (own pieces); lgkmcnt(0); barrier
//   M(g): 32 MFMAs (+ the tile's epilogue after its last k-step); barrier
// Interval I0(g) = G0 L(g) | G1 M(g-1), I1(g) = G0 M(g) | G1 L(g).  RAW: every wave waits for its
// stage-(g+1) pieces before the barrier that ends its L(g); G1's is the barrier that opens G0's
// L(g+1).  WAR: stage g - 1's slot is written from L(g); G1 read it last in L(g-1) and retired
// those reads (lgkmcnt(0)) before the barrier that ends I1(g-1), which precedes I0(g).
//
// LDS: a 4-stage ring of 32 KiB stages ([256][32] A image + [256][32] B image, 64-B rows).  The
// 16-B chunk c of row r sits at chunk c ^ f(r) with f linear over two row bits --
// A images f(r) = F((r >> 2) & 3), B images (permuted fragment rows, bfrag) F((r >> 3) & 3),
// F(1) = 2, F(2) = 3 -- so each ds_read_b128 lane group of a fragment read hits 16 distinct 16-B
// bank slots.  The DMA destination is lane-linear, so the swizzle is applied on the source.
namespace bp2 {
constexpr int BM = 256, BN = 256, BK = 32, WAVES = 8, THREADS = 512, STAGES = 4;
constexpr int IMG = 256 * BK * 2;           // 16 KiB per operand image
constexpr int STAGE_BYTES = 2 * IMG;        // 32 KiB
constexpr int SMEM = STAGES * STAGE_BYTES;  // 128 KiB
constexpr int PIECES = STAGE_BYTES / 1024 / WAVES;  // 4 DMA pieces per wave per stage
__device__ __forceinline__ int F2(int x) { return ((x & 1) << 1) ^ ((x & 2) ? 3 : 0); }
__device__ __forceinline__ int fa(int row) { return F2((row >> 2) & 3); }
__device__ __forceinline__ int fb(int row) { return F2((row >> 3) & 3); }
// source byte offset (relative to the image's origin row at k = 0) of the 16 B that the lane whose
// DMA destination is image byte `pos` loads
template <bool B_IMG>
__device__ __forceinline__ uint32_t src_off(int pos, long long ld) {
  const int row = pos >> 6, phys = (pos >> 4) & 3;
  const int ch = phys ^ (B_IMG ? fb(row) : fa(row));
  return (uint32_t)(((long long)row * ld + 8 * ch) * 2);
}
__device__ __forceinline__ v8bf afrag(const char* img, int rr0, int lane) {
  const int row = rr0 + (lane & 15), ch = lane >> 4;
  return *(const v8bf*)(img + row * 64 + 16 * (ch ^ fa(row)));
}
// B fragment for the wave's output-column block j (0..3 over its 64 columns; in the MFMA's A
// slot): lane l supplies the row that puts D[4g+v][l&15] on column wn + 32(j>>1) + 8g + 4(j&1) + v
__device__ __forceinline__ v8bf bfragk(const char* img, int wn, int j, int lane) {
  const int nl = lane & 15;
  const int row = wn + 32 * (j >> 1) + 8 * (nl >> 2) + 4 * (j & 1) + (nl & 3);
  const int ch = lane >> 4;
  return *(const v8bf*)(img + row * 64 + 16 * (ch ^ fb(row)));
}
template <int EPI>
struct Epi2 {
  // stores per wave per tile: 8 row groups x 2 chunks of C (+ gelu' / pre-activation), + the
  // column-sum partial rows
  static constexpr int S = 16 * (1 + ((EPI & CG_EPI_GELU) ? 1 : 0)) + ((EPI & CG_EPI_COLSUM) ? 4 : 0);
};
}  // namespace bp2

template <int EPI>
__global__ __launch_bounds__(bp2::THREADS, 1) void gemm_bf16_pp2_kernel(GemmParams p) {
  using namespace bp2;
  using bfp::u32x4;
  constexpr int NS = Epi2<EPI>::S;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int ntiles = tiles_n * tiles_m;
  const int nblk = gridDim.x;
  const int lb = cg_xcd_remap(blockIdx.x, nblk);
  const int my_tiles = lb < ntiles ? (ntiles - 1 - lb) / nblk + 1 : 0;
  const int nt = p.K / BK;
  const int S = my_tiles * nt;
  const int wm = grp * 128, wn = (wave & 3) * 64;
  auto tile_org = [&](int k, int& m0, int& n0) __attribute__((always_inline)) {
    const int tile = lb + k * nblk;
    m0 = (tile / tiles_n) * BM;
    n0 = (tile % tiles_n) * BN;
  };
  auto barrier = [] __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---------------------------------------------------------------- operand DMA (4 per stage)
  // wave w loads A pieces w, w + 8 and B pieces w, w + 8 of every stage; past the CU's last stage
  // the pieces read through a zero-size descriptor (zero fill into a slot nobody reads), so every
  // wave issues the same count every k-step
  const __amdgpu_buffer_rsrc_t ra = bfp::rsrc(p.A, ((long long)(p.M - 1) * p.lda + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = bfp::rsrc(p.B, ((long long)(p.N - 1) * p.ldb + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rz = bfp::rsrc(p.A, 0);
  uint32_t va[2], vb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    va[i] = src_off<false>((wave + WAVES * i) * 1024 + 16 * lane, p.lda);
    vb[i] = src_off<true>((wave + WAVES * i) * 1024 + 16 * lane, p.ldb);
  }
  int ik = 0, it = 0;  // (tile, k-step) of the next stage to be issued
  uint32_t ta = 0, tb = 0;
  auto tile_base = [&]() __attribute__((always_inline)) {
    int m0, n0;
    tile_org(ik, m0, n0);
    ta = (uint32_t)((long long)m0 * p.lda * 2);
    tb = (uint32_t)((long long)n0 * p.ldb * 2);
  };
  tile_base();
  int gi = 0;  // next stage index
  auto issue = [&]() __attribute__((always_inline)) {
    const bool ok = ik < my_tiles;
    const uint32_t ko = (uint32_t)(it * BK * 2);
    char* st = smem + (gi & (STAGES - 1)) * STAGE_BYTES;
    // (the whole offset in voffset: the buffer range check that zero-fills rows past M / N
    // does not cover soffset)
    const uint32_t ao = ok ? ta + ko : 0u, bo = ok ? tb + ko : 0u;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bfw::dma16(ok ? ra : rz, st + (wave + WAVES * i) * 1024, ao + va[i]);
      bfw::dma16(ok ? rb : rz, st + IMG + (wave + WAVES * i) * 1024, bo + vb[i]);
    }
    ++gi;
    if (ok && ++it == nt) {
      it = 0;
      ++ik;
      if (ik < my_tiles) tile_base();
    }
  };

  // ---------------------------------------------------------------- epilogue
  v4f acc[8][4];
  const int g4 = lane >> 4, r16 = lane & 15;
  const __amdgpu_buffer_rsrc_t rc = bfp::rsrc(p.C, ((long long)(p.M - 1) * p.ldc + p.N) * 2);
  auto epilogue = [&](int k) __attribute__((always_inline)) {
    int m0, n0;
    tile_org(k, m0, n0);
    if (__builtin_expect(p.alpha != 1.0f, 0)) {
      asm volatile("");
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] *= p.alpha;
    }
    int col[2];
    bool cok[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      col[c] = n0 + wn + 32 * c + 8 * g4;
      cok[c] = col[c] < p.N;
    }
    float bia[2][8];
    if constexpr ((EPI & CG_EPI_BIAS) != 0) {
      const __amdgpu_buffer_rsrc_t rbias = bfp::rsrc(p.bias, (long long)p.N * 4);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const uint32_t o = cok[c] ? (uint32_t)col[c] * 4u : bfp::OOR;
        bfp::unpack_f32(bfp::bld(rbias, o), bfp::bld(rbias, o + 16), bia[c]);
      }
    }
    u32x4 xa[8][2];  // dGELU operand (bf16), issued for all row groups before any is used
    if constexpr ((EPI & CG_EPI_DGELU) != 0) {
      const __amdgpu_buffer_rsrc_t rx = bfp::rsrc(p.aux, ((long long)(p.M - 1) * p.ld_aux + p.N) * 2);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = m0 + wm + 16 * i + r16;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const bool ok = row < p.M && cok[c];
          xa[i][c] = bfp::bld(rx, ok ? (uint32_t)(((long long)row * p.ld_aux + col[c]) * 2) : bfp::OOR);
        }
      }
    }
    float csum[2][2][8];  // [64-row half][chunk][column]
    if constexpr ((EPI & CG_EPI_COLSUM) != 0) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int j = 0; j < 8; ++j) csum[hh][c][j] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = m0 + wm + 16 * i + r16;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bool ok = row < p.M && cok[c];
        const uint32_t oc = ok ? (uint32_t)(((long long)row * p.ldc + col[c]) * 2) : bfp::OOR;
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
          const __amdgpu_buffer_rsrc_t rx = bfp::rsrc(p.aux_out, ((long long)(p.M - 1) * p.ld_aux + p.N) * 2);
          const uint32_t o = ok ? (uint32_t)(((long long)row * p.ld_aux + col[c]) * 2) : bfp::OOR;
          float s[8];
          if constexpr ((EPI & CG_EPI_GELU_DERIV) != 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = gelu_fast_d(v[j], s[j]);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] = v[j];
          }
          bfp::bst(rx, o, bfp::pack_bf16(s));
          if constexpr ((EPI & CG_EPI_GELU_DERIV) == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = gelu_fast(v[j]);
          }
        }
        if constexpr ((EPI & CG_EPI_DGELU) != 0) {
          float a[8];
          bfp::unpack_bf16(xa[i][c], a);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= (EPI & CG_EPI_GELU_DERIV) ? a[j] : dgelu_fast(a[j]);
        }
        if constexpr ((EPI & CG_EPI_COLSUM) != 0) {
          const float keep = row < p.M ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) csum[i >> 2][c][j] = fmaf(keep, v[j], csum[i >> 2][c][j]);
        }
        bfp::bst(rc, oc, bfp::pack_bf16(v));
      }
    }
    if constexpr ((EPI & CG_EPI_COLSUM) != 0) {
      // the wave's 128 rows are two of the 64-row partial rows the column-sum reduction reads
      const __amdgpu_buffer_rsrc_t rw = bfp::rsrc(p.ws, (long long)((p.M + 63) >> 6) * p.N * 4);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int prow = (m0 + wm + 64 * hh) >> 6;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
#pragma unroll
          for (int j = 0; j < 8; ++j) csum[hh][c][j] = bfp::dpp_sum16(csum[hh][c][j]);
          const uint32_t o =
              (r16 == 0 && cok[c] && 64 * prow < p.M) ? (uint32_t)(((long long)prow * p.N + col[c]) * 4) : bfp::OOR;
          bfp::bst(rw, o, (u32x4){__float_as_uint(csum[hh][c][0]), __float_as_uint(csum[hh][c][1]),
                                  __float_as_uint(csum[hh][c][2]), __float_as_uint(csum[hh][c][3])});
          bfp::bst(rw, o + 16, (u32x4){__float_as_uint(csum[hh][c][4]), __float_as_uint(csum[hh][c][5]),
                                       __float_as_uint(csum[hh][c][6]), __float_as_uint(csum[hh][c][7])});
        }
      }
    }
  };

  // ---------------------------------------------------------------- the ping-pong k-loop
  issue();
  issue();
  issue();
  bfp::wait_vm<2 * PIECES>();  // stage 0 landed (own pieces)
  barrier();
  if (grp == 1) barrier();  // the stagger: G1 one barrier behind G0
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  v8bf af[8], bf[4];
  int t = 0, k = 0;
  bool after_epi = false;
  for (int g = 0; g < S; ++g) {
    // L(g)
    const char* st = smem + (g & (STAGES - 1)) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = afrag(st, wm + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = bfragk(st + IMG, wn, j, lane);
    issue();  // stage g + 3, into the slot of stage g - 1
    // stage g + 1 landed: all but the pieces of stages g + 2, g + 3 (and, right after an
    // epilogue, its stores -- younger than stage g + 2, older than g + 3)
    if (after_epi) bfp::wait_vm<2 * PIECES + NS>();
    else bfp::wait_vm<2 * PIECES>();
    after_epi = false;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this segment's reads retired (WAR)
    barrier();
    // M(g)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    if (t == nt - 1) {
      epilogue(k);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
      t = 0;
      ++k;
      after_epi = true;
    } else {
      ++t;
    }
    barrier();
  }
  if (grp == 0) barrier();  // the same barrier count in both groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
}
