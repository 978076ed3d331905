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
