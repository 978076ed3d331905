// fp32 MFMA flash attention forward for the parity mode (included by attention.hip).
//
// The fp32 engine (extract_embeddings / query_model default, fp32 training parity) computes
// attention with exact fp32 products: v_mfma_f32_32x32x2_f32 is an fp32 FMA chain (no input
// rounding), at the f32 MFMA rate (64 FLOP/clk/SIMD = 157 TF/s on the chip, the same as the packed
// f32 VALU peak, but without spending the VALU on it).  Same contract as attn_fwd_vec / the bf16
// attn_fwd_mfma (causal + SEP-segment + window mask, GQA, hashed attention-prob dropout; the
// reference path is model_tiny_gpt.py:102-131 with build_attention_mask :273-295).
//
// Layout (32x32x2 f32 MFMA: A lane l = A[l&31][k = l>>5], B lane l = B[k = l>>5][l&31],
// C/D lane l register r = C[(r&3) + 8(r>>2) + 4(l>>5)][l&31]):
//   * S^T = K Q^T ("swapped": the query on the lane, so softmax statistics are per-lane): A = K rows
//     from LDS, B = Q in registers.  The head-dim contraction runs in the order d = 8g + 4h + t for
//     k-step 4g + t of half-wave h, so one ds_read_b128 of a K row feeds four MFMAs;
//   * O^T = V^T P^T: the B operand is the S accumulator register itself (k-step r pairs key
//     acc_row(r, 0) of lanes 0-31 with key acc_row(r, 1) of lanes 32-63), the A operand the V rows of
//     those keys, read as (V[key][c], V[key][c + 32]) pairs for the two 32-wide output blocks.
// K image rows are 256 B with 16-B chunks XOR-swizzled by (row & 15) (conflict-free row reads); V
// image rows hold the (c, c + 32) pairs interleaved.  Tiles of 64 keys, register-staged and double
// buffered (64 KiB of LDS per workgroup, 2 workgroups per CU); WG = 4 waves x 32 queries.
#pragma once

namespace fa32 {
constexpr int KT = 64;                // keys per tile
constexpr int ROWB = 256;             // bytes per image row (64 fp32)
constexpr int IMG = KT * ROWB;        // 16 KiB per K or V image
constexpr int LDS = 4 * IMG;          // two buffers x (K, V)

__device__ __forceinline__ int k_off(int row, int ch) { return row * ROWB + 16 * (ch ^ (row & 15)); }
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

struct Stage {
  float4 k[4];     // K chunks (row c >> 4, chunk c & 15), c = tid + 256 i
  float4 v[2][2];  // V chunk pairs (row u >> 3, chunks u & 7 and (u & 7) + 8), u = tid + 256 i
};

__device__ __forceinline__ float4 ld4(const float* p, bool ok) {
  return ok ? *(const float4*)p : make_float4(0.f, 0.f, 0.f, 0.f);
}
__device__ __forceinline__ void stage_load(Stage& s, const float* base, long long ld, int k0, int T, int hd,
                                           long long kcol, long long vcol, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, row = c >> 4, ch = c & 15;
    const int key = k0 + row;
    s.k[i] = ld4(base + (long long)key * ld + kcol + 4 * ch, key < T && 4 * ch < hd);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int u = tid + 256 * i, row = u >> 3, ch = u & 7;
    const int key = k0 + row;
    const float* vr = base + (long long)key * ld + vcol;
    s.v[i][0] = ld4(vr + 4 * ch, key < T && 4 * ch < hd);
    s.v[i][1] = ld4(vr + 32 + 4 * ch, key < T && 32 + 4 * ch < hd);
  }
}
__device__ __forceinline__ void stage_store(const Stage& s, char* kimg, char* vimg, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    *(float4*)(kimg + k_off(c >> 4, c & 15)) = s.k[i];
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int u = tid + 256 * i, row = u >> 3, ch = u & 7;
    const float4 a = s.v[i][0], b = s.v[i][1];  // d = 4ch + e and 32 + 4ch + e
    float4* dst = (float4*)(vimg + row * ROWB + 32 * ch);
    dst[0] = make_float4(a.x, b.x, a.y, b.y);
    dst[1] = make_float4(a.z, b.z, a.w, b.w);
  }
}
}  // namespace fa32

// NG: head dim / 8 (compile time, so the k-steps and the second output block unroll).
// DROP: attention-prob dropout with the in-kernel hash (cg_keep); the normaliser uses the
// undropped probabilities, the 1/(1-p) scale is folded into the kept ones
template <int DROP, int NG>
__global__ __launch_bounds__(256, 2) void attn_fwd_f32mfma(const float* __restrict__ qkv, long long ld,
                                                           const int32_t* __restrict__ seg, float* __restrict__ y,
                                                           long long ldy, float* __restrict__ lse, int T, int H, int KV,
                                                           int hd, int window, uint32_t seed, uint32_t thr,
                                                           float dscale, float scale) {
  using namespace fa32;
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5;
  const int bh = blockIdx.x, b = bh / H, hh = bh % H, kvh = hh / (H / KV);
  const int qtile = gridDim.y - 1 - blockIdx.y;  // heaviest (latest) query tiles first
  const int q0 = qtile * 128, q0w = q0 + wave * 32;
  const int myq = q0w + (lane & 31);
  const bool qok = myq < T;
  const long long rowbase = (long long)b * T;
  const float* base = qkv + rowbase * ld;
  constexpr int ng = NG;  // 8-wide head-dim groups (hd = 8 NG)
  constexpr bool WIDE = NG > 4;  // a second 32-wide output block

  // Q in registers: q[g][t] = Q[myq][8g + 4hl + t]
  float qf[8][4];
  {
    const float* qr = base + (long long)(qok ? myq : 0) * ld + (long long)hh * hd + 4 * hl;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const float4 v = ld4(qr + 8 * g, qok && g < ng);
      qf[g][0] = v.x; qf[g][1] = v.y; qf[g][2] = v.z; qf[g][3] = v.w;
    }
  }
  const int lo = qok ? fa::lo_of(seg, rowbase, myq, T, window) : 0x7fffffff;
  const int kmin = fa::lo_of(seg, rowbase, q0, T, window);
  const int kmax = min(T - 1, q0 + 127);
  const int w_lo_min = fa::lo_of(seg, rowbase, q0w, T, window);
  const int w_lo_max = fa::lo_of(seg, rowbase, min(q0w + 31, T - 1), T, window);
  const int w_qmax = min(T - 1, q0w + 31);
  const long long kcol = (long long)(H + kvh) * hd, vcol = (long long)(H + KV + kvh) * hd;
  const float c = scale * 1.4426950408889634f;
  const uint32_t hrow = DROP ? cg_row_hash(seed, (uint32_t)(((long long)b * H + hh) * T + myq)) : 0u;

  // per-lane LDS offsets: K row (l & 31) chunk (2g + hl) ^ (l & 15); V pair c = l & 31 of key row 4hl
  uint32_t koff[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) koff[g] = (uint32_t)k_off(lane & 31, 2 * g + hl);
  const uint32_t voff = (uint32_t)(4 * hl * ROWB + 8 * (lane & 31));

  float m = -INFINITY, lsum = 0.f;
  v16f o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) o0[r] = o1[r] = 0.f;

  const int t0 = kmin / KT, t1 = kmax / KT;
  Stage st;
  stage_load(st, base, ld, t0 * KT, T, hd, kcol, vcol, tid);
  stage_store(st, smem + (t0 & 1) * 2 * IMG, smem + (t0 & 1) * 2 * IMG + IMG, tid);  // tile t reads buffer t & 1
  __syncthreads();

  auto body = [&](const char* Ki, const char* Vi, int k0, auto full_c) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(full_c)::value;
    v16f s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if (g < ng) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const float4 kf = *(const float4*)(Ki + kb * 32 * ROWB + koff[g]);
          s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.x, qf[g][0], s[kb], 0, 0, 0);
          s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.y, qf[g][1], s[kb], 0, 0, 0);
          s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.z, qf[g][2], s[kb], 0, 0, 0);
          s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf.w, qf[g][3], s[kb], 0, 0, 0);
        }
      }
    }
    if constexpr (!FULL) {
      const int kq = myq - k0, kl = lo - k0;  // visible iff kl <= key - k0 <= kq
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = 32 * kb + acc_row(r, lane);
          s[kb][r] = (j > kq || j < kl) ? -INFINITY : s[kb][r];
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(mx, fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])));
    }
    // lazy rescale (exact: the same m serves P, the row sum and the LSE); NaN-safe for -inf
    const bool grow = (mx - m) * c > 8.0f;
    if (__any(grow)) {
      const float mn = grow ? mx : m;
      const float alpha = grow ? exp2f((m - mn) * c) : 1.0f;
      lsum *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        o0[r] *= alpha;
        o1[r] *= alpha;
      }
      m = mn;
    }
    const float mc = (m == -INFINITY ? 0.f : m) * c;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = exp2f(fmaf(s[kb][r], c, -mc));
        lsum += p;
        s[kb][r] = p;
      }
      if constexpr (DROP) {
        // elements r, r + 1 (r even) are keys 2j, 2j + 1: one hash per pair
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const uint32_t key = (uint32_t)(k0 + 32 * kb + acc_row(r, lane));
          const uint32_t h = cg_pair_mix(hrow + (key >> 1) * CG_COLK);
          s[kb][r] = (h & 0xFFFFu) >= thr ? s[kb][r] * dscale : 0.f;
          s[kb][r + 1] = (h >> 16) >= thr ? s[kb][r + 1] * dscale : 0.f;
        }
      }
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float2 vv = *(const float2*)(Vi + voff + (32 * kb + (r & 3) + 8 * (r >> 2)) * ROWB);
        o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(vv.x, s[kb][r], o0, 0, 0, 0);
        if constexpr (WIDE) o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(vv.y, s[kb][r], o1, 0, 0, 0);
      }
  };

  for (int t = t0; t <= t1; ++t) {
    char* Ki = smem + (t & 1) * 2 * IMG;
    const bool more = t < t1;
    if (more) stage_load(st, base, ld, (t + 1) * KT, T, hd, kcol, vcol, tid);
    const int k0 = t * KT;
    if (k0 <= w_qmax && k0 + KT - 1 >= w_lo_min) {
      if ((k0 + KT - 1 <= q0w) && (k0 >= w_lo_max)) body(Ki, Ki + IMG, k0, std::true_type{});
      else body(Ki, Ki + IMG, k0, std::false_type{});
    }
    if (more) {
      char* Kn = smem + ((t + 1) & 1) * 2 * IMG;  // last read before the previous barrier
      stage_store(st, Kn, Kn + IMG, tid);
    }
    __syncthreads();
  }
  // the two half-waves hold the same queries over different keys: add their partial sums
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(lsum), __float_as_uint(lsum), false, false);
  const float ltot = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  if (qok) {
    const float inv = 1.0f / ltot;
    float* yr = y + (rowbase + myq) * ldy + (long long)hh * hd;
#pragma unroll
    for (int r = 0; r < 16; r += 4) {
      const int d0 = acc_row(r, lane);  // 8 (r >> 2) + 4 hl
      if (d0 < hd) *(float4*)(yr + d0) = make_float4(o0[r] * inv, o0[r + 1] * inv, o0[r + 2] * inv, o0[r + 3] * inv);
      if (WIDE && d0 + 32 < hd)
        *(float4*)(yr + d0 + 32) = make_float4(o1[r] * inv, o1[r + 1] * inv, o1[r + 2] * inv, o1[r + 3] * inv);
    }
    if (hl == 0) lse[((long long)b * H + hh) * T + myq] = m * scale + __logf(ltot);
  }
}

static inline bool attn_f32mfma_supported(int hd, const void* qkv, long long ld, const void* y, long long ldy) {
  return hd > 0 && hd <= 64 && hd % 8 == 0 && ld % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)qkv & 15) == 0 &&
         ((uintptr_t)y & 15) == 0;
}

static inline int attn_fwd_f32mfma_launch(const float* qkv, long long ld, const int32_t* seg, float* y, long long ldy,
                                          float* lse, int B, int T, int H, int KV, int hd, int window, uint32_t seed,
                                          uint32_t thr, float dscale, float scale, hipStream_t s) {
  const dim3 g(B * H, cg_cdiv(T, 128));
#define CG_F32A(D, NG)                                                                                          \
  hipLaunchKernelGGL((attn_fwd_f32mfma<D, NG>), g, dim3(256), 0, s, qkv, ld, seg, y, ldy, lse, T, H, KV, hd, \
                     window, seed, thr, dscale, scale)
#define CG_F32A_NG(D)          \
  switch (hd >> 3) {           \
    case 1: CG_F32A(D, 1); break; \
    case 2: CG_F32A(D, 2); break; \
    case 3: CG_F32A(D, 3); break; \
    case 4: CG_F32A(D, 4); break; \
    case 5: CG_F32A(D, 5); break; \
    case 6: CG_F32A(D, 6); break; \
    case 7: CG_F32A(D, 7); break; \
    default: CG_F32A(D, 8); break; \
  }
  if (thr) {
    CG_F32A_NG(1)
  } else {
    CG_F32A_NG(0)
  }
#undef CG_F32A_NG
#undef CG_F32A
  CG_LAUNCH_CHECK();
  return CG_OK;
}

// ============================================================================
// fp32 MFMA flash attention BACKWARD for the parity mode (the reference trains in fp32 on
// CUDA/ROCm: autocast only on MPS, loop.py:498).  Same contract and arithmetic as
// attn_bwd_dq_vec / attn_bwd_dkdv_vec (P recomputed from the forward's LSE, dS = P (dP' - delta),
// keep bits from the same hash), with the products on v_mfma_f32_32x32x2_f32 (exact fp32 FMA
// chains).  Two kernels, as the bf16 path: dQ per (batch, head, 128 queries), dK / dV per (batch,
// kv head, 128 keys) summed over the kv group's query heads -- no atomics, deterministic.
//
//   dQ kernel: query on the lane (the forward's swapped layout): S^T = K Q^T and dP^T = V dO^T
//     (A = K / V rows of the row images, B = Q / dO in registers), dS^T in the accumulator, then
//     dQ^T += K^T dS^T with the accumulator register as the B operand (k-step r pairs key
//     acc_row(r, 0) of lanes 0-31 with acc_row(r, 1) of lanes 32-63) and K[key][d = lane] as A
//     (one ds_read_b32 per 32-wide output block);
//   dK/dV kernel: key on the lane: S = Q K^T and dP = dO V^T (A = Q / dO rows of the images, B = the
//     lane key's K / V in registers), per-query constants (-lse log2 e, delta, segment start) from
//     LDS by row, then dV^T += dO^T P' and dK^T += Q^T dS with the accumulators as B operands.
// Row images as the forward's K image (256-B rows, 16-B chunks XOR-swizzled by row & 15), double
// buffered, register-staged (64 KiB + 1.5 KiB per workgroup, 2 workgroups per CU).
// ============================================================================
// workgroups per CU the backward kernels are compiled for (1: up to 512 registers per lane, no
// spills; 2: 256, which spills the staged rows)
#ifndef ATTN_F32B_WPS
#define ATTN_F32B_WPS 1
#endif
namespace fa32 {
constexpr int QC_BYTES = 2 * 3 * KT * 4;
struct Rows {
  float4 a[4], b[4];  // chunks c = tid + 256 i of two 64-row tiles (row c >> 4, chunk c & 15)
};
__device__ __forceinline__ void rows_load(Rows& s, const float* pa, long long lda, const float* pb, long long ldb,
                                          int r0, int T, int hd, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, row = c >> 4, ch = c & 15;
    const bool ok = r0 + row < T && 4 * ch < hd;
    s.a[i] = ld4(pa + (long long)(r0 + row) * lda + 4 * ch, ok);
    s.b[i] = ld4(pb + (long long)(r0 + row) * ldb + 4 * ch, ok);
  }
}
__device__ __forceinline__ void rows_store(const Rows& s, char* ia, char* ib, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    *(float4*)(ia + k_off(c >> 4, c & 15)) = s.a[i];
    *(float4*)(ib + k_off(c >> 4, c & 15)) = s.b[i];
  }
}
// element d (< 64) of image row `row` (the A operand of the transposed products)
__device__ __forceinline__ float img_at(const char* img, int row, int d) {
  return *(const float*)(img + k_off(row, d >> 2) + 4 * (d & 3));
}
// 32 x 32 block of a row-image tile times a register operand: acc += Img[row0 + l&31][d] X[d][l&31]
// over d = 8g + 4hl + t (the forward's QK^T contraction order)
template <int NG>
__device__ __forceinline__ void rows_x_reg(v16f& acc, const char* img, const uint32_t* off, const float (&x)[8][4],
                                           int row0) {
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    if (g < NG) {
      const float4 f = *(const float4*)(img + row0 * ROWB + off[g]);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.x, x[g][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.y, x[g][1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.z, x[g][2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.w, x[g][3], acc, 0, 0, 0);
    }
  }
}
// out^T[d][lane] += sum_j Img[row0 + j][d] Y[j][lane] for the 32 rows j of one accumulator block Y
// (register r of lane l = Y[acc_row(r, l)][l & 31]); d = l & 31 (o0) and 32 + (l & 31) (o1)
template <bool WIDE>
__device__ __forceinline__ void imgT_x_acc(v16f& o0, v16f& o1, const char* img, const v16f& y, int row0, int lane) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = row0 + acc_row(r, lane);
    o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(img_at(img, row, lane & 31), y[r], o0, 0, 0, 0);
    if constexpr (WIDE) o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(img_at(img, row, 32 + (lane & 31)), y[r], o1, 0, 0, 0);
  }
}
// a row of d values held as o0 / o1 (register r of lane l: d = acc_row(r, l) (+ 32)) to memory, scaled
__device__ __forceinline__ void store_row_f32(float* dst, const v16f& o0, const v16f& o1, float sc, int hd, int lane) {
#pragma unroll
  for (int r = 0; r < 16; r += 4) {
    const int d0 = acc_row(r, lane);
    if (d0 < hd) *(float4*)(dst + d0) = make_float4(o0[r] * sc, o0[r + 1] * sc, o0[r + 2] * sc, o0[r + 3] * sc);
    if (d0 + 32 < hd)
      *(float4*)(dst + d0 + 32) = make_float4(o1[r] * sc, o1[r + 1] * sc, o1[r + 2] * sc, o1[r + 3] * sc);
  }
}
__device__ __forceinline__ void reg_rows(float (&x)[8][4], const float* rowp, bool ok, int ng, int hl) {
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const float4 v = ld4(rowp + 8 * g + 4 * hl, ok && g < ng);
    x[g][0] = v.x; x[g][1] = v.y; x[g][2] = v.z; x[g][3] = v.w;
  }
}
}  // namespace fa32

template <int DROP, int NG>
__global__ __launch_bounds__(256, ATTN_F32B_WPS) void attn_bwd_dq_f32mfma(const float* __restrict__ qkv, long long ld,
                                                              const int32_t* __restrict__ seg,
                                                              const float* __restrict__ dy, long long lddy,
                                                              const float* __restrict__ yo, long long ldy,
                                                              const float* __restrict__ lse,
                                                              float* __restrict__ delta, float* __restrict__ dqkv,
                                                              long long lddq, int T, int H, int KV, int hd, int window,
                                                              uint32_t seed, uint32_t thr, float dscale, float scale) {
  using namespace fa32;
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  constexpr bool WIDE = NG > 4;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5;
  const int bh = blockIdx.x, b = bh / H, hh = bh % H, kvh = hh / (H / KV);
  const int qtile = gridDim.y - 1 - blockIdx.y;
  const int q0 = qtile * 128, q0w = q0 + wave * 32;
  const int myq = q0w + (lane & 31);
  const bool qok = myq < T;
  const long long rowbase = (long long)b * T;
  const float* base = qkv + rowbase * ld;
  float qf[8][4], df[8][4];
  reg_rows(qf, base + (long long)(qok ? myq : 0) * ld + (long long)hh * hd, qok, NG, hl);
  reg_rows(df, dy + (rowbase + (qok ? myq : 0)) * lddy + (long long)hh * hd, qok, NG, hl);
  const long long bhq = ((long long)b * H + hh) * T + (qok ? myq : 0);
  const float nl2 = qok ? -lse[bhq] * 1.4426950408889634f : 0.f;
  // delta = rowsum(dO o O) of the lane's query (the two half-waves hold complementary d), written
  // for the dK / dV kernel
  float dl;
  {
    float yv[8][4];
    reg_rows(yv, yo + (rowbase + (qok ? myq : 0)) * ldy + (long long)hh * hd, qok, NG, hl);
    float part = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g)
#pragma unroll
      for (int t = 0; t < 4; ++t) part = fmaf(df[g][t], yv[g][t], part);
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(part), __float_as_uint(part), false, false);
    dl = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    if (qok && hl == 0) delta[bhq] = dl;
  }
  const int lo = qok ? fa::lo_of(seg, rowbase, myq, T, window) : 0x7fffffff;
  const int kmin = fa::lo_of(seg, rowbase, q0, T, window);
  const int kmax = min(T - 1, q0 + 127);
  const int w_lo_min = fa::lo_of(seg, rowbase, q0w, T, window);
  const int w_lo_max = fa::lo_of(seg, rowbase, min(q0w + 31, T - 1), T, window);
  const int w_qmax = min(T - 1, q0w + 31);
  const float* kb_ = base + (long long)(H + kvh) * hd;
  const float* vb_ = base + (long long)(H + KV + kvh) * hd;
  const float c = scale * 1.4426950408889634f;
  const uint32_t hrow = DROP ? cg_row_hash(seed, (uint32_t)(((long long)b * H + hh) * T + myq)) : 0u;
  uint32_t off[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) off[g] = (uint32_t)k_off(lane & 31, 2 * g + hl);
  v16f o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) o0[r] = o1[r] = 0.f;

  const int t0 = kmin / KT, t1 = kmax / KT;
  Rows st;
  rows_load(st, kb_, ld, vb_, ld, t0 * KT, T, hd, tid);
  rows_store(st, smem + (t0 & 1) * 2 * IMG, smem + (t0 & 1) * 2 * IMG + IMG, tid);
  __syncthreads();
  auto body = [&](const char* Ki, const char* Vi, int k0, auto full_c) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(full_c)::value;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      v16f s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
      rows_x_reg<NG>(s, Ki, off, qf, 32 * kb);
      rows_x_reg<NG>(dp, Vi, off, df, 32 * kb);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = 32 * kb + acc_row(r, lane);
        float p = exp2f(fmaf(s[r], c, nl2));
        if constexpr (!FULL) p = (k0 + j > myq || k0 + j < lo) ? 0.f : p;
        s[r] = p;
      }
      if constexpr (DROP) {
        // keys 2i, 2i + 1 of a pair sit in registers r, r + 1 (r even): one hash per pair
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const uint32_t key = (uint32_t)(k0 + 32 * kb + acc_row(r, lane));
          const uint32_t h = cg_pair_mix(hrow + (key >> 1) * CG_COLK);
          dp[r] = (h & 0xFFFFu) >= thr ? dp[r] * dscale : 0.f;
          dp[r + 1] = (h >> 16) >= thr ? dp[r + 1] * dscale : 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = s[r] * (dp[r] - dl);  // dS^T
      imgT_x_acc<WIDE>(o0, o1, Ki, s, 32 * kb, lane);
    }
  };
  for (int t = t0; t <= t1; ++t) {
    char* Ki = smem + (t & 1) * 2 * IMG;
    const bool more = t < t1;
    if (more) rows_load(st, kb_, ld, vb_, ld, (t + 1) * KT, T, hd, tid);
    const int k0 = t * KT;
    if (k0 <= w_qmax && k0 + KT - 1 >= w_lo_min) {
      if ((k0 + KT - 1 <= q0w) && (k0 >= w_lo_max)) body(Ki, Ki + IMG, k0, std::true_type{});
      else body(Ki, Ki + IMG, k0, std::false_type{});
    }
    if (more) {
      char* Kn = smem + ((t + 1) & 1) * 2 * IMG;
      rows_store(st, Kn, Kn + IMG, tid);
    }
    __syncthreads();
  }
  if (qok) store_row_f32(dqkv + (rowbase + myq) * lddq + (long long)hh * hd, o0, o1, scale, hd, lane);
}

// dK / dV: WG = 4 waves x 32 keys (128 keys of one (batch, kv head)); query tiles of 64 from the
// workgroup's first key on (causal), for every query head of the kv group
template <int DROP, int NG>
__global__ __launch_bounds__(256, ATTN_F32B_WPS) void attn_bwd_dkdv_f32mfma(const float* __restrict__ qkv, long long ld,
                                                                const int32_t* __restrict__ seg,
                                                                const float* __restrict__ dy, long long lddy,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ delta,
                                                                float* __restrict__ dqkv, long long lddq, int T, int H,
                                                                int KV, int hd, int window, uint32_t seed, uint32_t thr,
                                                                float dscale, float scale) {
  using namespace fa32;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // LDS + QC_BYTES (dynamic: > 64 KiB)
  // per query of the tile: -lse log2 e, delta, segment start (int bits)
  float(*qc)[3][KT] = (float(*)[3][KT])(smem + LDS);
  constexpr bool WIDE = NG > 4;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5;
  const int bk = blockIdx.x, b = bk / KV, kvh = bk % KV, rep = H / KV;
  const int ktile = gridDim.y - 1 - blockIdx.y;  // the keys with the most queries first
  const int k0 = ktile * 128, kw0 = k0 + wave * 32;
  const int mykey = kw0 + (lane & 31);
  const bool kok = mykey < T;
  const long long rowbase = (long long)b * T;
  const float* base = qkv + rowbase * ld;
  const long long koff = (long long)(H + kvh) * hd, voff = (long long)(H + KV + kvh) * hd;
  float kf[8][4], vf[8][4];
  reg_rows(kf, base + (long long)(kok ? mykey : 0) * ld + koff, kok, NG, hl);
  reg_rows(vf, base + (long long)(kok ? mykey : 0) * ld + voff, kok, NG, hl);
  const float c = scale * 1.4426950408889634f;
  uint32_t off[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) off[g] = (uint32_t)k_off(lane & 31, 2 * g + hl);
  v16f dk0, dk1, dv0, dv1;
#pragma unroll
  for (int r = 0; r < 16; ++r) dk0[r] = dk1[r] = dv0[r] = dv1[r] = 0.f;
  if (k0 >= T) return;  // (uniform per workgroup)
  // queries that can see one of the workgroup's keys: [k0, qend] (window: q < key + window)
  const int qend = window > 0 ? min(T - 1, k0 + 127 + window - 1) : T - 1;
  const int tq0 = k0 / KT, tq1 = qend / KT, ntq = tq1 - tq0 + 1;
  const int total = rep * ntq;  // (query head, query tile) steps

  Rows st;
  float cst[3] = {0.f, 0.f, 0.f};
  auto load_step = [&](int i) __attribute__((always_inline)) {
    const int h = kvh * rep + i / ntq, qt = tq0 + i % ntq;
    rows_load(st, base + (long long)h * hd, ld, dy + rowbase * lddy + (long long)h * hd, lddy, qt * KT, T, hd, tid);
    if (tid < KT) {
      const int q = qt * KT + tid;
      const bool ok = q < T;
      const long long bhq = ((long long)b * H + h) * T + (ok ? q : 0);
      cst[0] = ok ? -lse[bhq] * 1.4426950408889634f : 0.f;
      cst[1] = ok ? delta[bhq] : 0.f;
      cst[2] = __int_as_float(ok ? fa::lo_of(seg, rowbase, q, T, window) : 0x7fffffff);
    }
  };
  auto store_step = [&](int i) __attribute__((always_inline)) {
    char* im = smem + (i & 1) * 2 * IMG;
    rows_store(st, im, im + IMG, tid);
    if (tid < KT) {
      qc[i & 1][0][tid] = cst[0];
      qc[i & 1][1][tid] = cst[1];
      qc[i & 1][2][tid] = cst[2];
    }
  };
  load_step(0);
  store_step(0);
  __syncthreads();
  for (int i = 0; i < total; ++i) {
    const bool more = i + 1 < total;
    if (more) load_step(i + 1);
    const int h = kvh * rep + i / ntq, q0 = (tq0 + i % ntq) * KT;
    const char* Qi = smem + (i & 1) * 2 * IMG;
    const char* Di = Qi + IMG;
    const float* nl2 = qc[i & 1][0];
    const float* dlt = qc[i & 1][1];
    const int* los = (const int*)qc[i & 1][2];
    // the wave's 32 keys against the tile's 64 queries: any pair visible / all pairs visible
    const int qlast = min(T - 1, q0 + KT - 1);
    const bool any = q0 < T && q0 + KT - 1 >= kw0 && los[0] <= kw0 + 31;
    const bool full = any && q0 >= kw0 + 31 && q0 + KT - 1 < T && los[qlast - q0] <= kw0;
    const uint32_t hbase = (uint32_t)(((long long)b * H + h) * T);
    if (any) {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        v16f s, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
        rows_x_reg<NG>(s, Qi, off, kf, 32 * qb);   // S[q][key]
        rows_x_reg<NG>(dp, Di, off, vf, 32 * qb);  // dP[q][key]
        v16f pd;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = 32 * qb + acc_row(r, lane), q = q0 + j;
          float p = exp2f(fmaf(s[r], c, nl2[j]));
          if (!full) p = (mykey > q || mykey < los[j] || q >= T) ? 0.f : p;
          float d = dp[r];
          float pv = p;
          if constexpr (DROP) {
            // the pair (2i, 2i + 1) of this lane's key: one hash per (query, pair), half by key parity
            const uint32_t hsh = cg_pair_mix(cg_row_hash(seed, hbase + (uint32_t)q) + ((uint32_t)mykey >> 1) * CG_COLK);
            const bool keep = ((mykey & 1) ? (hsh >> 16) : (hsh & 0xFFFFu)) >= thr;
            d = keep ? d * dscale : 0.f;
            pv = keep ? p * dscale : 0.f;
          }
          s[r] = p * (d - dlt[j]);  // dS
          pd[r] = pv;
        }
        imgT_x_acc<WIDE>(dv0, dv1, Di, pd, 32 * qb, lane);  // dV^T += dO^T P'
        imgT_x_acc<WIDE>(dk0, dk1, Qi, s, 32 * qb, lane);   // dK^T += Q^T dS
      }
    }
    if (more) store_step(i + 1);  // the other buffer was last read before the previous barrier
    __syncthreads();
  }
  if (kok) {
    float* r = dqkv + (rowbase + mykey) * lddq;
    store_row_f32(r + koff, dk0, dk1, scale, hd, lane);
    store_row_f32(r + voff, dv0, dv1, 1.0f, hd, lane);
  }
}

static inline int attn_bwd_f32mfma_launch(const float* qkv, long long ld, const int32_t* seg, const float* dy,
                                          long long lddy, const float* y, long long ldy, const float* lse,
                                          float* delta, float* dqkv,
                                          long long lddq, int B, int T, int H, int KV, int hd, int window,
                                          uint32_t seed, uint32_t thr, float dscale, float scale, hipStream_t s) {
  const dim3 gq(B * H, cg_cdiv(T, 128)), gk(B * KV, cg_cdiv(T, 128));
#define CG_F32B(D, NG)                                                                                               \
  do {                                                                                                               \
    hipLaunchKernelGGL((attn_bwd_dq_f32mfma<D, NG>), gq, dim3(256), 0, s, qkv, ld, seg, dy, lddy, y, ldy, lse,    \
                       delta, dqkv, lddq, T, H, KV, hd, window, seed, thr, dscale, scale);                           \
    cg_func_lds((const void*)attn_bwd_dkdv_f32mfma<D, NG>, fa32::LDS + fa32::QC_BYTES);                            \
    hipLaunchKernelGGL((attn_bwd_dkdv_f32mfma<D, NG>), gk, dim3(256), fa32::LDS + fa32::QC_BYTES, s, qkv, ld, seg, \
                       dy, lddy, lse, delta, dqkv, lddq, T, H, KV, hd, window, seed, thr, dscale, scale);            \
  } while (0)
#define CG_F32B_NG(D)             \
  switch (hd >> 3) {              \
    case 1: CG_F32B(D, 1); break; \
    case 2: CG_F32B(D, 2); break; \
    case 3: CG_F32B(D, 3); break; \
    case 4: CG_F32B(D, 4); break; \
    case 5: CG_F32B(D, 5); break; \
    case 6: CG_F32B(D, 6); break; \
    case 7: CG_F32B(D, 7); break; \
    default: CG_F32B(D, 8); break; \
  }
  if (thr) {
    CG_F32B_NG(1)
  } else {
    CG_F32B_NG(0)
  }
#undef CG_F32B_NG
#undef CG_F32B
  CG_LAUNCH_CHECK();
  return CG_OK;
}
