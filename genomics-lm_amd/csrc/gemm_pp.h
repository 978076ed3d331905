// Ping-pong persistent bf16 GEMM for the TinyGPT forward and dX products (included by gemm.hip
// after gemm_lw.h; same operands, 256x128 tile, LDS images, DMA sources and epilogues as
// gemm_bf16_pers_kernel / gemm_bf16_lw_kernel).
//
// Why: in the eight-wave kernels both compute waves of a SIMD run the same k-step in lock step --
// they read their fragments together (the MFMA pipe idles on LDS latency at every step start) and
// issue their MFMAs together (the pipe takes one wave's at a time).  Here the compute waves of
// each SIMD (w and w + 4: a workgroup's waves are dealt to SIMDs cyclically) alternate roles: G0 =
// waves 0-3 (tile rows 0-127) and G1 = waves 4-7 (rows 128-255) run the same program with G1 one
// workgroup barrier behind, so between two barriers one compute wave of every SIMD is in an MFMA
// segment while its partner reads the fragments of its next segment (MI355X_MICROARCH.md, "Two
// waves per SIMD"; cdna_hip_programming.md, the 8-phase template's `if (wr == 1) s_barrier`
// stagger).  As in gemm_lw.h, the operand DMAs come from four loader waves (8-11, one per SIMD),
// so no compute wave ever stalls on a DMA issue.
//
// A 64-deep k-step g is two segments with a workgroup barrier after each:
//   L(g): the 16 fragments of the k-step (4 A m-blocks, 4 B n-blocks, 2 k-halves) from stage g
//   M(g): 32 x v_mfma_f32_16x16x32_bf16 over the wave's 64x64 accumulators (+ a tile's epilogue)
// (a k-step split in two 16-MFMA phases, i.e. four barriers per k-step, measured slower: each
// barrier interval costs ~280 cycles beyond its MFMAs).  Interval I_k(g) between barriers 2g + k
// and 2g + k + 1:  I0 = G0 L(g) | G1 M(g-1);  I1 = G0 M(g) | G1 L(g).
// Loader waves, 3-stage ring: stage g + 2 goes into the slot of stage g - 1, whose last reads
// (G1's L(g-1) in I1(g-1)) the compiler's lgkmcnt before G1's M(g-1) retired inside I0(g): its
// first half in I1(g), its second in I0(g + 1); at the end of I1(g) they wait (counted vmcnt) for
// stage g + 1, which G0 reads in I0(g + 1).
// timing-only diagnostic builds (results invalid): CG_PP_DIAG=1 compute waves issue no MFMAs
// (fragments kept live), 2 no fragment reads (MFMAs on the previous fragments), 3 loaders issue
// no DMAs after the prologue
#ifndef CG_PP_DIAG
#define CG_PP_DIAG 0
#endif
namespace bpp {
constexpr int CWAVES = 8, LWAVES = 4, THREADS = 64 * (CWAVES + LWAVES), STAGES = 3;
constexpr int SMEM = STAGES * bfw::STAGE_BYTES;  // 144 KiB
}  // namespace bpp

template <int EPI, int CT>
__global__ __launch_bounds__(bpp::THREADS, 1) void gemm_bf16_pp_kernel(GemmParams p) {
  using namespace bfp;
  constexpr bool SWG = Epi<EPI, CT>::SWG, DSW = Epi<EPI, CT>::DSW;
  constexpr int BNO = SWG ? BN / 2 : BN;
  constexpr int ES = CT == CG_BF16 ? 2 : 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;
  const int tiles_n = (p.N + BNO - 1) / BNO, tiles_m = (p.M + BM - 1) / BM;
  const int ntiles = tiles_n * tiles_m;
  const int nblk = gridDim.x;
  const int lb = cg_xcd_remap(blockIdx.x, nblk);
  const int my_tiles = lb < ntiles ? (ntiles - 1 - lb) / nblk + 1 : 0;
  const int nt = p.K / BKT;
  const int S = my_tiles * nt;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  auto tile_org = [&](int k, int& m0, int& n0) __attribute__((always_inline)) {
    const int tile = lb + k * nblk;
    m0 = (tile / tiles_n) * BM;
    n0 = (tile % tiles_n) * BNO;
  };

  auto barrier = [] __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  if (wave >= bpp::CWAVES) {
    // ---------------------------------------------------------------- loader wave
    const int L = wave - bpp::CWAVES;
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
    // stage g: the DMA origins of its (tile, k-step), advanced incrementally (no divisions in the
    // loop); past the CU's last stage every piece reads out of range (zero fill into a slot nobody
    // reads), so every step issues the same count.  A stage's 12 pieces go out in halves of 6 (A
    // pieces 0-7, then B 0-3), one half per interval: a DMA wave-instruction holds its wave for
    // many cycles, and every loader wave must reach each barrier within the interval.
    int ik = 0, it = 0;  // (tile, k-step) of the next stage to be originated
    uint32_t ta = 0, tb = 0;
    auto tile_base = [&]() __attribute__((always_inline)) {
      int m0, n0;
      tile_org(ik, m0, n0);
      ta = (uint32_t)((long long)m0 * p.lda * 2);
      tb = (uint32_t)((long long)n0 * p.ldb * 2);
    };
    tile_base();
    auto next_org = [&](uint32_t& ao, uint32_t& bo) __attribute__((always_inline)) {
      ao = bo = OOR;
      if (ik < my_tiles) {
        ao = ta + (uint32_t)(it * BKT * 2);
        bo = tb + (uint32_t)(it * BKT * 2);
        if (++it == nt) {
          it = 0;
          ++ik;
          if (ik < my_tiles) tile_base();
        }
      }
      if (CG_PP_DIAG == 3 && ao != OOR) ao = bo = 1u << 30;  // diagnostic: no DMA traffic (zero fill)
    };
    auto piece = [&](char* st, int j, uint32_t ao, uint32_t bo) __attribute__((always_inline)) {
      if (j < bfl::LA) bfw::dma16(ra, st + (L + bfl::LWAVES * j) * 1024, ao + va[j]);
      else bfw::dma16(rb, st + A_BYTES + (L + bfl::LWAVES * (j - bfl::LA)) * 1024, bo + vb[j - bfl::LA]);
    };
    uint32_t ao = 0, bo = 0;
    auto half = [&](int g, auto h_t) __attribute__((always_inline)) {
      constexpr int H = decltype(h_t)::value;
      if (H == 0) next_org(ao, bo);  // stage g's origins (stages are originated in order)
      char* st = smem + (g % bpp::STAGES) * STAGE_BYTES;
#pragma unroll
      for (int j = 6 * H; j < 6 * H + 6; ++j) piece(st, j, ao, bo);
    };
    using h0 = std::integral_constant<int, 0>;
    using h1 = std::integral_constant<int, 1>;
    half(0, h0{});
    half(0, h1{});
    half(1, h0{});
    half(1, h1{});
    wait_vm<bfl::PER_STAGE>();  // stage 0 landed
    barrier();
    // stage g + 2 goes into the slot of stage g - 1, free from I1(g): its first half in I1(g),
    // its second in I0(g + 1); stage g + 1 is complete at the end of I1(g) once all but the 6
    // youngest pieces (stage g + 2's first half) have landed
    for (int g = 0; g < S; ++g) {
      if (g > 0) half(g + 1, h1{});
      barrier();  // end of I0(g)
      half(g + 2, h0{});
      wait_vm<6>();  // stage g + 1 landed
      barrier();  // end of I1(g)
    }
    barrier();  // the stagger's barrier (G1's first, G0's last)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
    return;
  }

  // ---------------------------------------------------------------- epilogue operands / epilogue
  const __amdgpu_buffer_rsrc_t rc = rsrc(p.C, ((long long)(p.M - 1) * p.ldc + (DSW ? 2 : 1) * p.N) * ES);
  const int g4 = lane >> 4, r16 = lane & 15;
  u32x4 xa[4][2], xb[4][2], bq[2][2];
  auto cols_of = [&](int n0, int c) __attribute__((always_inline)) {
    return SWG ? n0 + (wn >> 1) + 8 * g4 : n0 + wn + 32 * c + 8 * g4;
  };
  auto epi_loads = [&](int k) __attribute__((always_inline)) {
    int m0, n0;
    tile_org(k, m0, n0);
    if constexpr ((EPI & CG_EPI_BIAS) != 0) {
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
    for (int i = 0; i < 4; ++i) {
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
  const bool scaled = p.alpha != 1.0f;
  auto epilogue = [&](int k) __attribute__((always_inline)) {
    int m0, n0;
    tile_org(k, m0, n0);
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
        off_c[i][c] = (row < p.M && col[c] < p.N) ? (uint32_t)(((long long)row * p.ldc + col[c]) * ES) : OOR;
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
        bst(rx, o, pack_bf16(g));
        bst(rx, ok ? o + (uint32_t)p.N * 2u : OOR, pack_bf16(u));
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
            bst(rx, o, pack_bf16(s));
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

  // ---------------------------------------------------------------- the ping-pong k-loop
  v8bf af[2][4], bf[2][4];
  barrier();                // stage 0 landed
  if (grp == 1) barrier();  // the stagger: G1 one barrier behind G0
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  int t = 0, k = 0;
  for (int g = 0; g < S; ++g) {
    const char* st = smem + (g % bpp::STAGES) * STAGE_BYTES;
    const bool last = t == nt - 1;
    // L(g): all 16 fragments of the k-step
    if (last) epi_loads(k);
    if (CG_PP_DIAG != 2 || g == 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 4; ++i) af[h][i] = bfg::frag<true>(st, wm + 16 * i, h, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[h][j] = bfrag(st + A_BYTES, wn, j, h, lane);
      }
    }
    barrier();
    // M(g)
    if (CG_PP_DIAG == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[0][i]), "v"(bf[0][i]), "v"(af[1][i]), "v"(bf[1][i]));
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = PMFMA(bf[h][j], af[h][i], acc[i][j], 0, 0, 0);
    }
    if (last) {
      epilogue(k);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
      t = 0;
      ++k;
    } else {
      ++t;
    }
    barrier();
  }
  if (grp == 0) barrier();  // the same barrier count in both groups (and the loaders)
}
