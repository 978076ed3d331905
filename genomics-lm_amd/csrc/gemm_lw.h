// Persistent bf16 GEMM with dedicated LDS-DMA loader waves (included by gemm.hip after
// gemm_pers.h; same operands, tile, LDS images and epilogues as gemm_bf16_pers_kernel).
//
// Why: in gemm_bf16_pers_kernel every one of the 8 waves issues its share of the operand
// LDS-DMA between its MFMAs.  Measured on the C4 products (tools/gemm_diag.py, same box), the
// k-loop with the DMAs removed takes 27 us (fc1 dX), the DMA stream with the MFMAs removed 24 us,
// the two together 37-40 us: a DMA wave-instruction stalls its wave's issue for 100+ cycles under
// load, so the MFMA pipe idles while both waves of a SIMD issue DMAs (neither a stagger of the
// two waves nor issue priority moved it; L2-hot operands did not either, so it is not the data
// latency).  Here the 256x128 tile is computed by 8 compute waves (4 along M x 2 along N of
// 64x64, v_mfma_f32_16x16x32_bf16, as before) that never issue a DMA, and 4 loader waves (one
// per SIMD: waves w, w+4 and w+8 share a SIMD) stream the operand stages into the 3-stage
// ring.  One raw s_barrier per k-step: before barrier g the loaders have waited (counted
// vmcnt) for stage g, and the compute waves have retired their reads of stage g-1; after it the
// loaders issue stage g+2 into the slot of stage g-1 and the compute waves read stage g.  Two
// stages stay in flight across every barrier and the ring runs across tile seams, so the
// next tile's stages stream in while the compute waves run an epilogue.
//
// The compute waves' vector-memory queue then holds only their own epilogue loads and stores:
// the epilogue operands (bias, residual, dGELU operand, SwiGLU pre-activations, accumulate
// source) are loaded two k-steps before the tile's end (or partly after its MFMAs where the
// registers do not allow it) and waited for with vmcnt(0) -- no counted interleaving with the
// DMA stream.
// (Measured and removed, round 4: an L2 prefetch of the A rows a few stages ahead by the loaders,
// 10-18 % slower; an L2 prefetch of the fp32-residual block during a tile's first k-steps, slower --
// DESIGN.md section 10.)
namespace bfl {
constexpr int CWAVES = 8, LWAVES = 4, THREADS = 64 * (CWAVES + LWAVES);
constexpr int A_PIECES = bfw::A_BYTES / 1024, B_PIECES = bfw::B_BYTES / 1024;  // 32, 16 per stage
constexpr int LA = A_PIECES / LWAVES, LB = B_PIECES / LWAVES;                  // 8, 4 per loader
constexpr int PER_STAGE = LA + LB;                                             // DMAs per loader per stage
constexpr int SMEM = bfp::SMEM;
}  // namespace bfl

template <int EPI, int CT>
__global__ __launch_bounds__(bfl::THREADS, 1) void gemm_bf16_lw_kernel(GemmParams p) {
  using namespace bfp;
  constexpr bool SWG = Epi<EPI, CT>::SWG, DSW = Epi<EPI, CT>::DSW;
  constexpr bool RP = (EPI & CG_EPI_ROPE) != 0;
  constexpr int BNO = SWG ? BN / 2 : BN;
  constexpr int ES = CT == CG_BF16 ? 2 : 4;
  // RoPE column order: logical column n = 64 w + 32 c + 8 g + e (the lane's chunk c of group g in
  // 64-column block w) is pair unit U = 4 w + g, half c -- U < rope_uqk: head U / G, dims
  // 8 (U % G) + e (c = 0) and their rotation partners + half (c = 1); past the q / k heads:
  // column 16 U + 8 c + e.  Both halves of a rotation pair then sit in one lane's two chunks.
  auto rope_col = [&](int n) __attribute__((always_inline)) {
    const int U = ((n >> 6) << 2) | ((n >> 3) & 3), c = (n >> 5) & 1, e = n & 7;
    if (U < p.rope_uqk) {
      const int h = (U * p.rope_mul) >> 16;
      return h * 2 * p.rope_half + 8 * (U - h * p.rope_G) + c * p.rope_half + e;
    }
    return 16 * U + 8 * c + e;
  };
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_n = (p.N + BNO - 1) / BNO, tiles_m = (p.M + BM - 1) / BM;
  const int ntiles = tiles_n * tiles_m;
  const int nblk = gridDim.x;
  const int lb = cg_xcd_remap(blockIdx.x, nblk);
  const int my_tiles = lb < ntiles ? (ntiles - 1 - lb) / nblk + 1 : 0;
  const int nt = p.K / BKT;
  const int S = my_tiles * nt;
  auto tile_org = [&](int k, int& m0, int& n0) __attribute__((always_inline)) {
    const int tile = lb + k * nblk;
    m0 = (tile / tiles_n) * BM;
    n0 = (tile % tiles_n) * BNO;
  };

  if (wave >= bfl::CWAVES) {
    // ------------------------------------------------------------------ loader wave
    const int L = wave - bfl::CWAVES;
    const __amdgpu_buffer_rsrc_t ra = rsrc(p.A, ((long long)(p.M - 1) * p.lda + p.K) * 2);
    const __amdgpu_buffer_rsrc_t rb = rsrc(p.B, ((long long)((SWG ? 2 : 1) * p.N - 1) * p.ldb + p.K) * 2);
    uint32_t va[bfl::LA], vb[bfl::LB];
#pragma unroll
    for (int j = 0; j < bfl::LA; ++j) va[j] = bfw::src_off<true>((L + bfl::LWAVES * j) * 1024 + 16 * lane, p.lda);
#pragma unroll
    for (int j = 0; j < bfl::LB; ++j) {
      const int pos = (L + bfl::LWAVES * j) * 1024 + 16 * lane;
      vb[j] = SWG ? b_src_off_swg(pos, p.ldb, p.N) : b_src_off(pos, p.ldb);
    }
    // RoPE: the B rows of a tile are not an affine image of n0 (rotation-pair order), so the
    // loader keeps the piece offsets of the tile it is streaming (vcur) and forms the next tile's
    // (vnext) right after issuing the last stage of the current one -- off the path between a
    // barrier and the DMAs behind it
    uint32_t vcur[bfl::LB], vnext[bfl::LB];
    auto rope_offsets = [&](int k) __attribute__((always_inline)) {
      int m0, n0;
      tile_org(k < my_tiles ? k : 0, m0, n0);
#pragma unroll
      for (int j = 0; j < bfl::LB; ++j) {
        const int pos = (L + bfl::LWAVES * j) * 1024 + 16 * lane;
        const int row = pos >> 7, phys = (pos >> 4) & 7;
        vnext[j] = ((uint32_t)rope_col(n0 + row) * (uint32_t)p.ldb + 8u * (uint32_t)(phys ^ fb(row))) * 2u;
      }
    };
    // stage g: the DMA origins of its (tile, k-step); past the CU's last stage every piece reads
    // out of range (zero fill into a slot nobody reads), so every step issues the same count
    auto issue = [&](int g) __attribute__((always_inline)) {
      uint32_t ao = OOR, bo = OOR;
      if (g < S) {
        const int k = g / nt, t = g - k * nt;
        int m0, n0;
        tile_org(k, m0, n0);
        ao = (uint32_t)(((long long)m0 * p.lda + t * BKT) * 2);
        if constexpr (RP) {
          bo = (uint32_t)(t * BKT * 2);
          if (t == 0) {
#pragma unroll
            for (int j = 0; j < bfl::LB; ++j) vcur[j] = vnext[j];
          }
        } else {
          bo = (uint32_t)(((long long)n0 * p.ldb + t * BKT) * 2);
        }
      }
      char* st = smem + (g % STAGES) * STAGE_BYTES;
#pragma unroll
      for (int j = 0; j < bfl::LA; ++j) bfw::dma16(ra, st + (L + bfl::LWAVES * j) * 1024, ao + va[j]);
#pragma unroll
      for (int j = 0; j < bfl::LB; ++j)
        bfw::dma16(rb, st + A_BYTES + (L + bfl::LWAVES * j) * 1024, RP ? (bo == OOR ? OOR : bo + vcur[j]) : bo + vb[j]);
      if constexpr (RP) {
        if ((g + 1) % nt == 0) rope_offsets((g + 1) / nt);
      }
    };
    if constexpr (RP) rope_offsets(0);
    issue(0);
    issue(1);
    for (int g = 0; g < S; ++g) {
      wait_vm<bfl::PER_STAGE>();  // stage g landed; stage g+1 may still be in flight
      __builtin_amdgcn_s_barrier();
      issue(g + 2);  // into the slot of stage g-1, whose reads retired before this barrier
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
    return;
  }

  // -------------------------------------------------------------------- compute wave
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const __amdgpu_buffer_rsrc_t rc = rsrc(p.C, ((long long)(p.M - 1) * p.ldc + (DSW ? 2 : 1) * p.N) * ES);
  const int g4 = lane >> 4, r16 = lane & 15;
  u32x4 xa[4][2], xb[4][2], bq[2][2];
  // the lane's columns of tile k (chunks c = 0, 1) and its C offsets (OOR outside the matrix)
  auto cols_of = [&](int n0, int c) __attribute__((always_inline)) {
    if constexpr (RP) return rope_col(n0 + wn + 32 * c + 8 * g4);
    return SWG ? n0 + (wn >> 1) + 8 * g4 : n0 + wn + 32 * c + 8 * g4;
  };
  // epilogue operand loads of tile k for the lane's row groups [LO, HI) (+ the bias with BIAS_);
  // only the loaded registers stay live until the epilogue (addresses are recomputed there)
  auto epi_loads = [&](int k, auto lo_t, auto hi_t, auto bias_t) __attribute__((always_inline)) {
    constexpr int LO = decltype(lo_t)::value, HI = decltype(hi_t)::value;
    int m0, n0;
    tile_org(k, m0, n0);
    if constexpr (decltype(bias_t)::value && (EPI & CG_EPI_BIAS) != 0) {
      const __amdgpu_buffer_rsrc_t rbias = rsrc(p.bias, (long long)p.N * 4);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int cc = cols_of(n0, c);
        const uint32_t o = cc < p.N ? (uint32_t)cc * 4u : OOR;
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
        const int cc = cols_of(n0, c);
        const bool ok = rok && cc < p.N;
        if constexpr ((EPI & CG_EPI_RESID) != 0) {
          const __amdgpu_buffer_rsrc_t rr = rsrc(p.resid, ((long long)(p.M - 1) * p.ldr + p.N) * 4);
          const uint32_t o = ok ? (uint32_t)(((long long)row * p.ldr + cc) * 4) : OOR;
          xa[i][c] = bld(rr, o);
          xb[i][c] = bld(rr, o + 16);
        }
        if constexpr ((EPI & CG_EPI_DGELU) != 0) {
          const __amdgpu_buffer_rsrc_t rx = rsrc(p.aux, ((long long)(p.M - 1) * p.ld_aux + p.N) * ES);
          const uint32_t o = ok ? (uint32_t)(((long long)row * p.ld_aux + cc) * ES) : OOR;
          xa[i][c] = bld(rx, o);
          if constexpr (CT != CG_BF16) xb[i][c] = bld(rx, o + 16);
        }
        if constexpr ((EPI & CG_EPI_ACCUM) != 0) {
          const uint32_t o = ok ? (uint32_t)(((long long)row * p.ldc + cc) * ES) : OOR;
          xa[i][c] = bld(rc, o);
          xb[i][c] = bld(rc, o + 16);
        }
        if constexpr (DSW) {
          const __amdgpu_buffer_rsrc_t rx = rsrc(p.aux, ((long long)(p.M - 1) * p.ld_aux + 2 * p.N) * 2);
          const uint32_t o = ok ? (uint32_t)(((long long)row * p.ld_aux + cc) * 2) : OOR;
          xa[i][c] = bld(rx, o);
          xb[i][c] = bld(rx, ok ? o + (uint32_t)p.N * 2u : OOR);
        }
      }
    }
  };

  v4f acc[4][4];
  // one k-step on stage g (the `step` body of gemm_bf16_pers_kernel without its DMAs)
  auto cstep = [&](int g) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of stage g-1 retired
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const char* st = smem + (g % STAGES) * STAGE_BYTES;
    const char* as = st;
    const char* bs = st + A_BYTES;
    v8bf af[2][4], bfr[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[0][i] = bfg::frag<true>(as, wm + 16 * i, 0, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[0][j] = bfrag(bs, wn, j, 0, lane);
#pragma unroll
    for (int gr = 0; gr < 8; ++gr) {
      const int i = gr >> 1, j0 = 2 * (gr & 1);
      acc[i][j0] = PMFMA(bfr[0][j0], af[0][i], acc[i][j0], 0, 0, 0);
      acc[i][j0 + 1] = PMFMA(bfr[0][j0 + 1], af[0][i], acc[i][j0 + 1], 0, 0, 0);
      if (gr < 4) af[1][gr] = bfg::frag<true>(as, wm + 16 * gr, 1, lane);
      else bfr[1][gr - 4] = bfrag(bs, wn, gr - 4, 1, lane);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = PMFMA(bfr[1][j], af[1][i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int gr = 0; gr < 8; ++gr) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
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
    int col[2];
    uint32_t off_c[4][2];
#pragma unroll
    for (int c = 0; c < 2; ++c) col[c] = cols_of(n0, c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + wm + 16 * i + r16;
#pragma unroll
      for (int c = 0; c < 2; ++c)
        off_c[i][c] = (row < p.M && col[c] < p.N)
                          ? (uint32_t)(((long long)row * p.ldc + col[c]) * ES)
                          : OOR;
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
    } else if constexpr (RP) {
      // chunk 0 = dims i, chunk 1 = dims i + half of one q / k head (a V pair unit: cos 1, sin 0
      // from out-of-range table loads): y_i = x_i cos - x_{i+h} sin, y_{i+h} = x_{i+h} cos + x_i sin
      // at the row's position m % rope_T (model_tiny_gpt.py:35-45)
      const int U = (((n0 + wn) >> 6) << 2) | g4;
      const bool rot = U < p.rope_uqk;
      const int dim0 = rot ? 8 * (U - ((U * p.rope_mul) >> 16) * p.rope_G) : 0;
      const long long tab_bytes = (long long)p.rope_T * p.rope_half * 4;
      const __amdgpu_buffer_rsrc_t rcs = rsrc(p.rope_cos, tab_bytes), rsn = rsrc(p.rope_sin, tab_bytes);
      u32x4 cq[4][2], sq[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wm + 16 * i + r16;
        const uint32_t t = (uint32_t)row % (uint32_t)p.rope_T;
        const uint32_t o = rot ? (t * (uint32_t)p.rope_half + (uint32_t)dim0) * 4u : OOR;
        cq[i][0] = bld(rcs, o);
        cq[i][1] = bld(rcs, o + 16);
        sq[i][0] = bld(rsn, o);
        sq[i][1] = bld(rsn, o + 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v0[8], v1[8], cs[8], sn[8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            v0[4 * h + u] = acc[i][h][u];
            v1[4 * h + u] = acc[i][2 + h][u];
          }
        if constexpr ((EPI & CG_EPI_BIAS) != 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            v0[j] += bia[0][j];
            v1[j] += bia[1][j];
          }
        }
        unpack_f32(cq[i][0], cq[i][1], cs);
        unpack_f32(sq[i][0], sq[i][1], sn);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float c = rot ? cs[j] : 1.0f;
          const float y0 = fmaf(v0[j], c, -v1[j] * sn[j]);
          const float y1 = fmaf(v1[j], c, v0[j] * sn[j]);
          v0[j] = y0;
          v1[j] = y1;
        }
        bst(rc, off_c[i][0], pack_bf16(v0));
        bst(rc, off_c[i][1], pack_bf16(v1));
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
          float s[8];
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

  // The epilogue operands are loaded two k-steps before the tile's end (they are then younger
  // than the previous tile's epilogue stores, which have long completed when the epilogue's
  // vmcnt(0) waits for them) -- all of them when they fit the register budget (bias, bf16 dGELU
  // operand: <= 32 VGPRs), else the first two row groups early and the rest after the MFMAs.
  constexpr int XW = ((EPI & CG_EPI_RESID) ? 2 : 0) + ((EPI & CG_EPI_DGELU) ? (CT == CG_BF16 ? 1 : 2) : 0) +
                     ((EPI & CG_EPI_ACCUM) ? 2 : 0) + (DSW ? 2 : 0);  // u32x4 per (row group, chunk)
  // row groups loaded early: at most 32 registers held through the last k-steps (the bias takes
  // 16); the SwiGLU backward's epilogue is too register-hungry to hold any
  constexpr int HA0 = XW == 0 ? 4 : (32 - ((EPI & CG_EPI_BIAS) ? 16 : 0)) / (8 * XW);
  constexpr int HA = DSW ? 0 : (HA0 > 4 ? 4 : HA0);
  const int ta = nt >= 3 ? nt - 3 : 0;
  int g = 0;
  for (int k = 0; k < my_tiles; ++k) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < nt; ++t, ++g) {
      cstep(g);
      if (t == ta) {
        __builtin_amdgcn_sched_barrier(0);
        epi_loads(k, std::integral_constant<int, 0>{}, std::integral_constant<int, HA>{}, std::true_type{});
      }
    }
    if constexpr (HA < 4)
      epi_loads(k, std::integral_constant<int, HA>{}, std::integral_constant<int, 4>{}, std::false_type{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the epilogue operands (older stores long done)
    __builtin_amdgcn_sched_barrier(0);
    epilogue(k);
  }
}
