// Grouped weight-gradient GEMM for the TinyGPT backward (included by gemm.hip).
//
//   dW_p[n][k] (+)= alpha_p * sum_m dY_p[m][n] X_p[m][k]      (every nn.Linear weight of a
//   block: qkv, proj, fc1/fc2 or gate|up / down -- the autograd of model_tiny_gpt.py:85-93,
//   132, 143-148, 50-57)
//
// Both operands are token-major ([M][cols], the reduction index m is the strided one), so the
// tiles are DMA'd into LDS as [64 m-rows][128 cols] images (lane-linear LDS-DMA destination,
// XOR swizzle applied on the per-lane source address) and the MFMA fragments are read with
// ds_read_b64_tr_b16 (bfg::frag<false>).
//
// Every output tile is reduced over the WHOLE token range inside one workgroup: no split-K
// slabs, no reduction pass -- the fp32 result is written once (HBM traffic = the operands
// once + dW once).  The tiles of several products (one or more blocks' weights) form one
// persistent launch so that there are enough of them to fill the CUs; each workgroup walks
// its tiles with one LDS-DMA ring that runs across tile seams (stages are addressed by a
// global step index; steps past the end DMA from an out-of-range offset, which the buffer
// range check turns into zero fills, so every wave issues the same number of VMEM ops and
// the counted vmcnt waits stay exact).  The token count K need not be a multiple of the 64-row
// k-step: the rows m >= K of the last step lie past the buffer's range end ((K-1)*ld + cols
// elements), so they load as zeros and add nothing -- the dynamic-length loader's B*T
// (data_loading.py:380-393 pads each batch only to its own longest sequence) runs as is.
//
// The MFMA operands are swapped (D^T = X_frag x dY_frag), so each lane ends with 4
// consecutive output columns of each 16x16 block: the epilogue is 16-byte stores straight
// from the accumulators.
namespace bfd {
constexpr int BN = 128, BKT = 64;

// LDS-DMA hidden from the compiler: with the builtin, hipcc cannot prove that the
// ds_read_b64_tr_b16 fragment reads of the current stage do not alias the DMA writes into the
// next slot and drains vmcnt(0) before every fragment read (the whole ring serialises).  The
// kernel counts these DMAs itself (explicit vmcnt + barrier before a stage is read).  M0 (the
// LDS destination base) is saved and restored around the load.
__device__ __forceinline__ void dma16_asm(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds), "s"(r)
      : "memory");
}

// BNT: output-tile columns (128: waves of 64x64; 256: waves of 64x128, 8 B fragments per k-half)
template <int BM, int NSTAGE, int BNT = BN>
struct Geo {
  static constexpr int WAVES = BM / 32;                   // (BM/64) x 2 waves of 64 x BNT/2
  static constexpr int JN = BNT / 32;                     // 16-column blocks per wave
  static constexpr int THREADS = WAVES * 64;
  static constexpr int STAGES = NSTAGE;
  static constexpr int A_BYTES = BM * BKT * 2;
  static constexpr int B_BYTES = BNT * BKT * 2;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int A_CHUNKS = A_BYTES / 1024 / WAVES;  // 4
  static constexpr int B_CHUNKS = B_BYTES / 1024 / WAVES;  // 4 (BM 128), 2 (BM 256) or 4 (256 x 256)
  static constexpr int DPS = A_CHUNKS + B_CHUNKS;          // DMA wave-instructions per stage
  static constexpr int SMEM = STAGES * STAGE_BYTES;
};

struct Prod {
  const bf16_t* A;  // dY [K][lda], columns 0..N_out-1
  const bf16_t* B;  // X  [K][ldb], columns 0..K_out-1
  float* C;         // dW [N_out][ldc]
  long long lda, ldb, ldc;
  int N_out, K_out, tiles_n, tile0;
  float alpha;
  int accum;
  float* colsum;  // [N_out] (+)= alpha * sum_m A[m][n], or null (kernel CS variant only)
};
struct Params {
  Prod p[CG_DW_MAX];
  int nprod, K, ntiles;  // ntiles: work items = output tiles x ksplit
  // split of the token range (round 4): item = tile * ksplit + s covers rows [s kc, (s+1) kc) of K
  // (kc = kc_steps k-steps); slice 0 writes C as before, slices s >= 1 write fp32 slab s-1
  // ([N_out][K_out] at slab + (s-1) slab_stride + the product's slab_off), added into C by
  // dw_slab_reduce_kernel in slice order
  int ksplit, kc_steps;
  int max_wg;  // grid cap (0: one workgroup per CU)
  float* slab;
  long long slab_stride;
  long long slab_off[CG_DW_MAX];
};
}  // namespace bfd

// CS: the launch has a product with a column-sum output (Prod::colsum).  Every wave then also sums
// the dY fragments it feeds to the MFMAs (v_dot2 against (1, 1): 4 VALU per 8-token fragment, in
// the MFMAs' shadow); the even waves (wn = 0: every dY column of the tile once) of a product's first
// column tile write the sums -- the bias gradient for free where a separate pass or a GEMM-epilogue
// column sum would re-read or hold the whole dY.
template <int BM, int NSTAGE, int BNT, bool CS>
__global__ __launch_bounds__((bfd::Geo<BM, NSTAGE, BNT>::THREADS), 1) void gemm_dw_kernel(const bfd::Params P) {
  using namespace bfd;
  using G = Geo<BM, NSTAGE, BNT>;
  constexpr int JN = G::JN;
  constexpr int S = G::STAGES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const int nblk = gridDim.x;
  const int lb = cg_xcd_remap(blockIdx.x, nblk);  // an XCD's workgroups take consecutive tiles
  const int my_tiles = lb < P.ntiles ? (P.ntiles - 1 - lb) / nblk + 1 : 0;
  // k-steps per work item (a ragged last step -- and a last slice past K -- reads rows >= K out of
  // range: zero fill)
  const int nt = P.ksplit > 1 ? P.kc_steps : (P.K + BKT - 1) / BKT;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * (BNT / 2);
  if (my_tiles == 0) return;

  auto find = [&](int tile, int& pi) {
    pi = 0;
    while (pi + 1 < P.nprod && tile >= P.p[pi + 1].tile0) ++pi;
  };
  // DMA cursor: the stage (local tile dk, k-step dt) the next issue() loads, with its
  // product's buffer resources, tile origin and per-lane source offsets (rebuilt per tile)
  uint32_t va[G::A_CHUNKS], vb[G::B_CHUNKS];
  __amdgpu_buffer_rsrc_t ra, rb;
  uint32_t a_org = 0, b_org = 0, a_step = 0, b_step = 0;
  int dk = 0, dt = 0;
  auto load_tile = [&]() {
    if (dk >= my_tiles) {  // past the end: every DMA reads out of range (zero fill)
      a_org = b_org = 0x80000000u;
      a_step = b_step = 0;
      return;
    }
    int pi;
    const int item = lb + dk * nblk;
    const int tile = item / P.ksplit, sl = item - tile * P.ksplit;
    find(tile, pi);
    const Prod& pr = P.p[pi];
    const int lt = tile - pr.tile0;
    const int m0 = (lt / pr.tiles_n) * BM, n0 = (lt % pr.tiles_n) * BNT;
    ra = __builtin_amdgcn_make_buffer_rsrc((void*)pr.A, (short)0,
                                           (int)(((long long)(P.K - 1) * pr.lda + pr.N_out) * 2), 0x00020000);
    rb = __builtin_amdgcn_make_buffer_rsrc((void*)pr.B, (short)0,
                                           (int)(((long long)(P.K - 1) * pr.ldb + pr.K_out) * 2), 0x00020000);
    const long long r0 = (long long)sl * nt * BKT;  // first token row of the slice
    a_org = (uint32_t)((long long)m0 * 2 + r0 * pr.lda * 2);
    b_org = (uint32_t)((long long)n0 * 2 + r0 * pr.ldb * 2);
    a_step = (uint32_t)(BKT * pr.lda * 2);
    b_step = (uint32_t)(BKT * pr.ldb * 2);
#pragma unroll
    for (int i = 0; i < G::A_CHUNKS; ++i) va[i] = bfw::src_off<false>((wave + G::WAVES * i) * 1024 + 16 * lane, pr.lda);
#pragma unroll
    for (int i = 0; i < G::B_CHUNKS; ++i) vb[i] = bfw::src_off<false>((wave + G::WAVES * i) * 1024 + 16 * lane, pr.ldb);
  };
  auto advance = [&]() {
    if (++dt == nt) {
      dt = 0;
      ++dk;
      load_tile();
    }
  };
  auto issue = [&](int g) {
    // (readfirstlane: the M0 operand of the LDS-DMA must stay scalar whatever the optimiser does with g)
    const uint32_t st = __builtin_amdgcn_readfirstlane(lds0 + (g % S) * G::STAGE_BYTES + wave * 1024);
    const uint32_t ao = a_org + dt * a_step, bo = b_org + dt * b_step;
#pragma unroll
    for (int i = 0; i < G::A_CHUNKS; ++i) dma16_asm(ra, st + G::WAVES * i * 1024, ao + va[i]);
#pragma unroll
    for (int i = 0; i < G::B_CHUNKS; ++i) dma16_asm(rb, st + G::A_BYTES + G::WAVES * i * 1024, bo + vb[i]);
    advance();
  };

  v4f acc[4][JN];
  float cs[4];
  auto step = [&](int g, auto cs_c) __attribute__((always_inline)) {
    constexpr bool TCS = decltype(cs_c)::value;  // this tile sums its dY fragments
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 2) * G::DPS) : "memory");
    __builtin_amdgcn_s_barrier();
    const char* st = smem + (g % S) * G::STAGE_BYTES;
    const char* as = st + (wm >> 7) * 16384;
    const int ar = wm & 127;
    const char* bs = st + G::A_BYTES + (wn >> 7) * 16384;  // the wave's 128-column sub-image
    const int bc = wn & 127;
    v8bf af[2][4], bfr[2][JN];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[0][i] = bfg::frag<false>(as, ar + 16 * i, 0, lane);
#pragma unroll
    for (int j = 0; j < JN; ++j) bfr[0][j] = bfg::frag<false>(bs, bc + 16 * j, 0, lane);
    // the DMAs of stage g + S - 1 go into the slot step g - 1 read (every wave is past it)
    const uint32_t nx = __builtin_amdgcn_readfirstlane(lds0 + ((g + S - 1) % S) * G::STAGE_BYTES + wave * 1024);
    const uint32_t ao = a_org + dt * a_step, bo = b_org + dt * b_step;
    if constexpr (JN == 4) {
#pragma unroll
      for (int gr = 0; gr < 8; ++gr) {
        const int i = gr >> 1, j0 = 2 * (gr & 1);
        acc[i][j0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[0][j0], af[0][i], acc[i][j0], 0, 0, 0);
        acc[i][j0 + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[0][j0 + 1], af[0][i], acc[i][j0 + 1], 0, 0, 0);
        if (gr < 4) af[1][gr] = bfg::frag<false>(as, ar + 16 * gr, 1, lane);
        else bfr[1][gr - 4] = bfg::frag<false>(bs, bc + 16 * (gr - 4), 1, lane);
        if (gr < G::A_CHUNKS) dma16_asm(ra, nx + G::WAVES * gr * 1024, ao + va[gr]);
        else if (gr < G::DPS) dma16_asm(rb, nx + G::A_BYTES + G::WAVES * (gr - G::A_CHUNKS) * 1024, bo + vb[gr - G::A_CHUNKS]);
      }
    } else {
      // 64 x 128 per wave: column block j's four MFMAs, then its half-1 fragment into the
      // registers half 0's fragment j just released (and one of A's half-1 fragments, and a DMA)
#pragma unroll
      for (int j = 0; j < JN; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[0][j], af[0][i], acc[i][j], 0, 0, 0);
        bfr[1][j] = bfg::frag<false>(bs, bc + 16 * j, 1, lane);
        if (j < 4) af[1][j] = bfg::frag<false>(as, ar + 16 * j, 1, lane);
        if (j < G::A_CHUNKS) dma16_asm(ra, nx + G::WAVES * j * 1024, ao + va[j]);
        else if (j < G::DPS) dma16_asm(rb, nx + G::A_BYTES + G::WAVES * (j - G::A_CHUNKS) * 1024, bo + vb[j - G::A_CHUNKS]);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[1][j], af[1][i], acc[i][j], 0, 0, 0);
    if constexpr (JN == 4) {
      __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);  // half 0's fragment reads (2 tr-reads each)
#pragma unroll
      for (int gr = 0; gr < 8; ++gr) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        if (gr < G::DPS) __builtin_amdgcn_sched_group_barrier(SGB_DMA, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
    } else {
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * (4 + JN), 0);
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        if (j < 4) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // B and A half-1 fragments
        else __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        if (j < G::DPS) __builtin_amdgcn_sched_group_barrier(SGB_DMA, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * JN, 0);
    }
    if constexpr (TCS) {
      // lane l: dY column wm + 16 i + (l & 15), tokens 8 (l >> 4) .. + 7 of each 32-token half
      typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
      const bf2_t one2 = __builtin_bit_cast(bf2_t, 0x3F803F80u);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint4 u = __builtin_bit_cast(uint4, af[h][i]);
          cs[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.x), one2, cs[i], false);
          cs[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.y), one2, cs[i], false);
          cs[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.z), one2, cs[i], false);
          cs[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.w), one2, cs[i], false);
        }
    }
    advance();
  };

  auto epilogue = [&](int k) {
    const int item = lb + k * nblk;
    const int tile = item / P.ksplit, sl = item - tile * P.ksplit;
    int pi;
    find(tile, pi);
    const Prod& pr = P.p[pi];
    const int lt = tile - pr.tile0;
    const int m0 = (lt / pr.tiles_n) * BM, n0 = (lt % pr.tiles_n) * BNT;
    const int g4 = lane >> 4, r16 = lane & 15;
    if (sl > 0) {  // a later token slice: its partial to the slab (dense [N_out][K_out])
      float* slab = P.slab + (long long)(sl - 1) * P.slab_stride + P.slab_off[pi];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm + 16 * i + r16;
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int n = n0 + wn + 16 * j + 4 * g4;
          if (m < pr.N_out && n < pr.K_out)
            *(float4*)(slab + (long long)m * pr.K_out + n) =
                make_float4(acc[i][j][0] * pr.alpha, acc[i][j][1] * pr.alpha, acc[i][j][2] * pr.alpha,
                            acc[i][j][3] * pr.alpha);
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm + 16 * i + r16;
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int n = n0 + wn + 16 * j + 4 * g4;
        if (m < pr.N_out && n < pr.K_out) {
          float4* c = (float4*)(pr.C + (long long)m * pr.ldc + n);
          float4 v = make_float4(acc[i][j][0] * pr.alpha, acc[i][j][1] * pr.alpha, acc[i][j][2] * pr.alpha,
                                 acc[i][j][3] * pr.alpha);
          if (pr.accum) {
            const float4 o = *c;
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *c = v;  // (a nontemporal store measured no different, round 5)
        }
      }
    }
  };

  load_tile();
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s);
  int g = 0;
  for (int k = 0; k < my_tiles; ++k) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
    // only the first column tile of a product with a column-sum output pays the sums' VALU (the
    // branch is per tile, outside the k-loop, so the loop bodies keep their MFMA schedule, and the
    // sums are live only in that branch)
    int cpi = -1;
    if constexpr (CS) {
      const int tile = (lb + k * nblk) / P.ksplit;
      int pi;
      find(tile, pi);
      if (P.p[pi].colsum && (tile - P.p[pi].tile0) % P.p[pi].tiles_n == 0) cpi = pi;
    }
    if (cpi >= 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) cs[i] = 0.f;
      for (int t = 0; t < nt; ++t, ++g) step(g, std::true_type{});
      // the even waves (wn = 0) hold every dY column of the tile once; the four lane groups hold
      // the column's four token subsets (ksplit is 1 with a column sum)
      const Prod& pr = P.p[cpi];
      if (wn == 0) {
        const int m0 = ((lb + k * nblk) - pr.tile0) / pr.tiles_n * BM;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = cs[i];
          v += __shfl_xor(v, 16);
          v += __shfl_xor(v, 32);
          const int m = m0 + wm + 16 * i + (lane & 15);
          if ((lane >> 4) == 0 && m < pr.N_out) pr.colsum[m] = v * pr.alpha + (pr.accum ? pr.colsum[m] : 0.f);
        }
      }
    } else {
      for (int t = 0; t < nt; ++t, ++g) step(g, std::false_type{});
    }
    epilogue(k);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
}

// C_p += sum over slabs 1 .. ksplit-1 (slice order, after slice 0's C update): one workgroup row
// per product (blockIdx.y), 4 consecutive columns per thread
__global__ __launch_bounds__(256) void dw_slab_reduce_kernel(const bfd::Params P) {
  const bfd::Prod& pr = P.p[blockIdx.y];
  const float* slab = P.slab + P.slab_off[blockIdx.y];
  const long long n4 = (long long)pr.N_out * pr.K_out / 4;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n4; e += (long long)gridDim.x * 256) {
    const long long idx = 4 * e;
    const int m = (int)(idx / pr.K_out), n = (int)(idx - (long long)m * pr.K_out);
    float4* c = (float4*)(pr.C + (long long)m * pr.ldc + n);
    float4 v = *c;
    for (int s = 1; s < P.ksplit; ++s) {
      const float4 w = *(const float4*)(slab + (long long)(s - 1) * P.slab_stride + idx);
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    *c = v;
  }
}

