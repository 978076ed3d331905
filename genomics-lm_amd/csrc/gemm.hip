// MFMA GEMMs with fused epilogues for every nn.Linear call site of TinyGPT
// (model_tiny_gpt.py:85-93 qkv, :132 proj, :143-148 MLP, :50-57 SwiGLU, :327 head)
// and their autograd products (dX = dY.W, dW = dY^T.X).
//
//   C[m,n] = epi( alpha * sum_k A(m,k) B(n,k) )
//   A(m,k) = AK ? A[m*lda+k] : A[k*lda+m]      B(n,k) = BK ? B[n*ldb+k] : B[k*ldb+n]
//
// bf16 path : 128x128x64 block tile, 4 waves (2x2) of 64x64, v_mfma_f32_16x16x32_bf16,
//             register-staged double-buffered LDS (loads for tile t+1 issued before the
//             MFMAs of tile t, written after them), XOR-swizzled images:
//               K-contiguous operand  -> [row][64] image, ds_read_b128 fragments
//               MN-contiguous operand -> [k][128] image, ds_read_b64_tr_b16 fragments
// fp32 path : 64x64x16 tile, v_mfma_f32_16x16x4_f32 (exact fp32 fma chain) -- parity mode.
#include "common.h"
#include <algorithm>

struct GemmParams {
  int M, N, K, kchunk;
  const void* A; long long lda;
  const void* B; long long ldb;
  void* C; long long ldc; int c_dtype;
  int epi; float alpha;
  const float* bias;
  const float* resid; long long ldr;
  const void* aux; void* aux_out; long long ld_aux;
  uint32_t drop_seed, drop_thr; float drop_scale;
  float* ws; int split;
  int n_valid;  // SWIGLU / DSWIGLU live columns
  // CG_EPI_ROPE: tables, sequence length, half head dim, 16-column pair units per head (G) and
  // its reciprocal (U / G = (U * rope_mul) >> 16), pair units of the rotated q / k columns
  const float* rope_cos; const float* rope_sin;
  int rope_T, rope_half, rope_G, rope_mul, rope_uqk;
};

// ---------------------------------------------------------------------------
// epilogue (shared by both kernels and the split-K reducer)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void epi_apply(const GemmParams& p, int row, int col, float v) {
  const int e = p.epi;
  if (e & CG_EPI_BIAS) v += p.bias[col];
  const long long ai = (long long)row * p.ld_aux + col;
  if (e & CG_EPI_GELU) {
    const float s = (e & CG_EPI_GELU_DERIV) ? dgelu_f(v) : v;
    if (p.c_dtype == CG_BF16) ((bf16_t*)p.aux_out)[ai] = f2bf(s);
    else ((float*)p.aux_out)[ai] = s;
    v = gelu_f(v);
  }
  if (e & CG_EPI_DGELU) {
    float a = (p.c_dtype == CG_BF16) ? bf2f(((const bf16_t*)p.aux)[ai]) : ((const float*)p.aux)[ai];
    v *= (e & CG_EPI_GELU_DERIV) ? a : dgelu_f(a);
  }
  if (e & CG_EPI_DROPOUT) v = cg_keep(p.drop_seed, (uint32_t)row, (uint32_t)col, p.drop_thr) ? v * p.drop_scale : 0.0f;
  if (e & CG_EPI_RESID) v += p.resid[(long long)row * p.ldr + col];
  const long long ci = (long long)row * p.ldc + col;
  if (p.c_dtype == CG_BF16) {
    ((bf16_t*)p.C)[ci] = f2bf(v);
  } else {
    float* c = (float*)p.C;
    if (e & CG_EPI_ACCUM) v += c[ci];
    c[ci] = v;
  }
}

__device__ __forceinline__ void epi_store(const GemmParams& p, int row, int col, float v, int z) {
  if (row >= p.M || col >= p.N) return;
  v *= p.alpha;
  if (p.split > 1) {
    p.ws[((long long)z * p.M + row) * p.N + col] = v;
    return;
  }
  epi_apply(p, row, col, v);
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmParams p) {
  const long long total = (long long)p.M * p.N;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    float s = 0.f;
    for (int z = 0; z < p.split; ++z) s += p.ws[z * total + i];
    const int row = (int)(i / p.N), col = (int)(i % p.N);
    epi_apply(p, row, col, s);
  }
}

// ---------------------------------------------------------------------------
// fp32 kernel (parity mode): 64x64x16, f32 MFMA 16x16x4
// ---------------------------------------------------------------------------
template <bool AK, bool BKC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmParams p) {
  constexpr int BM = 64, BN = 64, BKT = 16, PAD = 4;
  __shared__ float As[BKT][BM + PAD];
  __shared__ float Bs[BKT][BN + PAD];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = blockIdx.z * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const float* A = (const float*)p.A;
  const float* B = (const float*)p.B;
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  for (int k0 = kbeg; k0 < kend; k0 += BKT) {
    // ---- stage A (64 m x 16 k) and B (64 n x 16 k) as [k][mn] images
    if (AK) {
      const int r = tid >> 2, kq = (tid & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + r, k = k0 + kq + e;
        As[kq + e][r] = (m < p.M && k < kend) ? A[(long long)m * p.lda + k] : 0.f;
      }
    } else {
      const int kr = tid >> 4, mq = (tid & 15) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + mq + e, k = k0 + kr;
        As[kr][mq + e] = (m < p.M && k < kend) ? A[(long long)k * p.lda + m] : 0.f;
      }
    }
    if (BKC) {
      const int r = tid >> 2, kq = (tid & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + r, k = k0 + kq + e;
        Bs[kq + e][r] = (n < p.N && k < kend) ? B[(long long)n * p.ldb + k] : 0.f;
      }
    } else {
      const int kr = tid >> 4, nq = (tid & 15) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + nq + e, k = k0 + kr;
        Bs[kr][nq + e] = (n < p.N && k < kend) ? B[(long long)k * p.ldb + n] : 0.f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BKT; kk += 4) {
      const int kr = kk + (lane >> 4);
      float a0 = As[kr][wm + (lane & 15)], a1 = As[kr][wm + 16 + (lane & 15)];
      float b0 = Bs[kr][wn + (lane & 15)], b1 = Bs[kr][wn + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + v;
        const int col = n0 + wn + 16 * j + (lane & 15);
        epi_store(p, row, col, acc[i][j][v], blockIdx.z);
      }
}

// ---------------------------------------------------------------------------
// fp32 kernel (parity mode: the forward, dX and dW products of the fp32 engine): 128x128x16 tile,
// 4 waves of 64x64, v_mfma_f32_32x32x2_f32 (an exact fp32 fma chain at 64 FLOP/clk/SIMD).
// Operands are register-staged 16-B chunks into double-buffered images, one per operand layout:
//   K-contiguous (AK / BKC): [128 rows][16 k], 16-B chunks XOR-swizzled by (row >> 2) & 3, read as
//     one ds_read_b128 per 4 MFMA k-steps (half-wave h takes k = 8g + 4h + t at k-step 4g + t);
//   MN-contiguous: [16 k][128 rows] (the global rows as they are), read as one ds_read_b32 per
//     k-step (32 consecutive rows per half-wave: conflict-free) in the same k order.
// The contraction order differs from the 64x64 kernel's (fp32 rounding differences only).
// ---------------------------------------------------------------------------
#ifndef CG_F32_BK
#define CG_F32_BK 16
#endif
namespace f32b {
constexpr int BM = 128, BN = 128, BKT = CG_F32_BK;  // k per stage: 16 or 32
constexpr int RB = BKT * 4;                        // bytes per K-contiguous image row
constexpr int CPR = BKT / 4;                       // 16-B chunks per such row
constexpr int NCH = BM * BKT / 4 / 256;            // chunks per thread per operand
constexpr int IMG = BM * BKT * 4;                  // bytes per operand image
// chunk swizzle: conflict-free ds_read_b128 of 32 consecutive rows (16-lane groups hit 64 banks)
__device__ __forceinline__ int swz(int row) { return CPR == 4 ? ((row >> 2) & 3) : ((row >> 1) & 7); }
__device__ __forceinline__ int off(int row, int ch) { return row * RB + 16 * (ch ^ swz(row)); }
// stage one operand's BKT k x 128 rows: chunk c = tid + 256 i
template <bool KC>
__device__ __forceinline__ void load_op(float4 (&st)[NCH], const float* X, long long ld, int r0, int rlim, int k0,
                                        int kend, int tid) {
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = tid + 256 * i;
    if (KC) {
      const int row = c / CPR, k = k0 + 4 * (c % CPR), r = r0 + row;
      st[i] = (r < rlim && k < kend) ? *(const float4*)(X + (long long)r * ld + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      const int kr = c >> 5, r = r0 + 4 * (c & 31), k = k0 + kr;  // rlim % 4 == 0 on this path
      st[i] = (r < rlim && k < kend) ? *(const float4*)(X + (long long)k * ld + r) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}
template <bool KC>
__device__ __forceinline__ void store_op(const float4 (&st)[NCH], char* img, int tid) {
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = tid + 256 * i;
    if (KC) *(float4*)(img + off(c / CPR, c % CPR)) = st[i];
    else *(float4*)(img + (c >> 5) * 512 + 16 * (c & 31)) = st[i];
  }
}
// the 4 k-steps t = 0..3 of group g for the 32-row block at r0 (lane row r0 + (l & 31))
template <bool KC>
__device__ __forceinline__ float4 frag4(const char* img, int r0, int g, int lane) {
  if (KC) return *(const float4*)(img + r0 * RB + off(lane & 31, 2 * g + (lane >> 5)));  // r0 % 16 == 0
  const float* col = (const float*)img + (8 * g + 4 * (lane >> 5)) * 128 + r0 + (lane & 31);
  return make_float4(col[0], col[128], col[256], col[384]);
}
}  // namespace f32b

template <bool AK, bool BKC>
__global__ __launch_bounds__(256) void gemm_f32_big_kernel(GemmParams p) {
  using namespace f32b;
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = blockIdx.z * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const float* A = (const float*)p.A;
  const float* B = (const float*)p.B;
  v16f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float4 sa[NCH], sb[NCH];
  auto load = [&](int k0) __attribute__((always_inline)) {
    load_op<AK>(sa, A, p.lda, m0, p.M, k0, kend, tid);
    load_op<BKC>(sb, B, p.ldb, n0, p.N, k0, kend, tid);
  };
  auto store = [&](char* img) __attribute__((always_inline)) {
    store_op<AK>(sa, img, tid);
    store_op<BKC>(sb, img + IMG, tid);
  };
  load(kbeg);
  store(smem);
  __syncthreads();
  int cur = 0;
  for (int k0 = kbeg; k0 < kend; k0 += BKT) {
    const bool more = k0 + BKT < kend;
    if (more) load(k0 + BKT);
    const char* img = smem + cur * 2 * IMG;
#pragma unroll
    for (int g = 0; g < BKT / 8; ++g) {
      float4 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = frag4<AK>(img, wm + 32 * i, g, lane);
        b[i] = frag4<BKC>(img + IMG, wn + 32 * i, g, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
        }
    }
    if (more) store(smem + (cur ^ 1) * 2 * IMG);  // last read before the previous barrier
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const int col = n0 + wn + 32 * j + (lane & 31);
        epi_store(p, row, col, acc[i][j][r], blockIdx.z);
      }
}

// ---------------------------------------------------------------------------
// bf16 kernel: 128x128x64, 16x16x32 bf16 MFMA
// ---------------------------------------------------------------------------
namespace bfg {
constexpr int BM = 128, BN = 128, BKT = 64;
constexpr int TILE_BYTES = 128 * 64 * 2;  // 16 KiB per operand image

// byte offset of 16-B chunk `ch` (0..7) of row `row` in a [128][64] K-contiguous image
__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }
// byte offset of 16-B chunk `ch` (0..15) of k-row `row` in a [64][128] MN-contiguous image
__device__ __forceinline__ int mc_off(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

struct Stage { uint4 v[4]; };

template <bool KC>
__device__ __forceinline__ void stage_load(Stage& s, const bf16_t* X, long long ld, int r0, int rlim,
                                           int k0, int kend, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    if (KC) {
      const int row = c >> 3, ch = c & 7;
      const int r = r0 + row, k = k0 + ch * 8;
      if (r < rlim && k < kend) s.v[i] = *(const uint4*)(X + (long long)r * ld + k);
      else s.v[i] = make_uint4(0, 0, 0, 0);
    } else {
      const int row = c >> 4, ch = c & 15;
      const int k = k0 + row, r = r0 + ch * 8;
      if (k < kend && r < rlim) s.v[i] = *(const uint4*)(X + (long long)k * ld + r);
      else s.v[i] = make_uint4(0, 0, 0, 0);
    }
  }
}

template <bool KC>
__device__ __forceinline__ void stage_store(const Stage& s, char* img, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    int off;
    if (KC) off = kc_off(c >> 3, c & 7);
    else off = mc_off(c >> 4, c & 15);
    *(uint4*)(img + off) = s.v[i];
  }
}

// 16x16x32 operand fragment: rows rr0..rr0+15 of the tile, k = ks*32 + 8*(lane>>4) + j
template <bool KC>
__device__ __forceinline__ v8bf frag(const char* img, int rr0, int ks, int lane) {
  if (KC) {
    const int row = rr0 + (lane & 15), ch = ks * 4 + (lane >> 4);
    return *(const v8bf*)(img + kc_off(row, ch));
  } else {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
    const int krow = ks * 32 + 8 * g + q;
    const int ch = (rr0 >> 3) + (pp >> 1);
    const int b0 = mc_off(krow, ch) + 8 * (pp & 1);
    const int b1 = mc_off(krow + 4, ch) + 8 * (pp & 1);
    typedef v4s __attribute__((address_space(3))) * lp4;
    v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp4)(img + b0));
    v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp4)(img + b1));
    v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(v8bf, r);
  }
}
}  // namespace bfg

// ---------------------------------------------------------------------------
// Vectorised epilogue: 8 consecutive columns of one row (N % 8 == 0 on this path).
// EPI >= 0: compile-time epilogue flags / C dtype; EPI == -1: read them from p.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ld8f(const float* p, float v[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8f(float* p, const float v[8]) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void ld8b(const bf16_t* p, float v[8]) {
  const uint4 u = *(const uint4*)p;
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
  }
}
__device__ __forceinline__ void st8b(bf16_t* p, const float v[8]) {
  uint4 u;
  u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  u.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
  u.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  *(uint4*)p = u;
}

template <int EPI, int CT>
__device__ __forceinline__ void epi_apply8(const GemmParams& p, int row, int col, float v[8]) {
  const int e = EPI >= 0 ? EPI : p.epi;
  const int ct = EPI >= 0 ? CT : p.c_dtype;
  if (e & CG_EPI_BIAS) {
    float bb[8];
    ld8f(p.bias + col, bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += bb[j];
  }
  const long long ai = (long long)row * p.ld_aux + col;
  if (e & CG_EPI_GELU) {
    if (e & CG_EPI_GELU_DERIV) {
      float dg[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = gelu_fast_d(v[j], dg[j]);
      if (ct == CG_BF16) st8b((bf16_t*)p.aux_out + ai, dg);
      else st8f((float*)p.aux_out + ai, dg);
    } else {
      if (ct == CG_BF16) st8b((bf16_t*)p.aux_out + ai, v);
      else st8f((float*)p.aux_out + ai, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = gelu_fast(v[j]);
    }
  }
  if (e & CG_EPI_DGELU) {
    float a[8];
    if (ct == CG_BF16) ld8b((const bf16_t*)p.aux + ai, a);
    else ld8f((const float*)p.aux + ai, a);
    if (e & CG_EPI_GELU_DERIV) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= a[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= dgelu_fast(a[j]);
    }
  }
  if (e & CG_EPI_DROPOUT) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const uint32_t h = cg_hash_pair(p.drop_seed, (uint32_t)row, (uint32_t)(col + j) >> 1);
      v[j] = (h & 0xFFFFu) >= p.drop_thr ? v[j] * p.drop_scale : 0.f;
      v[j + 1] = (h >> 16) >= p.drop_thr ? v[j + 1] * p.drop_scale : 0.f;
    }
  }
  if (e & CG_EPI_RESID) {
    float r[8];
    ld8f(p.resid + (long long)row * p.ldr + col, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += r[j];
  }
  const long long ci = (long long)row * p.ldc + col;
  if (ct == CG_BF16) {
    st8b((bf16_t*)p.C + ci, v);
  } else {
    float* c = (float*)p.C + ci;
    if (e & CG_EPI_ACCUM) {
      float o[8];
      ld8f(c, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += o[j];
    }
    st8f(c, v);
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_vec_kernel(GemmParams p) {
  const long long total8 = (long long)p.M * p.N / 8;
  const long long slab = (long long)p.M * p.N;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total8; i += (long long)gridDim.x * 256) {
    float s[8], t[8];
    ld8f(p.ws + i * 8, s);
    for (int z = 1; z < p.split; ++z) {
      ld8f(p.ws + z * slab + i * 8, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += t[j];
    }
    const long long e = i * 8;
    epi_apply8<-1, 0>(p, (int)(e / p.N), (int)(e % p.N), s);
  }
}

// ---------------------------------------------------------------------------
// bf16 main loop + epilogue
// ---------------------------------------------------------------------------
namespace bfg {
constexpr int EPI_LD = 68;                     // fp32 staging row stride (conflict-free writes)
constexpr int EPI_BYTES = 4 * 64 * EPI_LD * 4;  // 4 waves x [64][68] fp32
constexpr int SMEM = EPI_BYTES > 4 * TILE_BYTES ? EPI_BYTES : 4 * TILE_BYTES;
}  // namespace bfg

template <bool AK, bool BKC, int EPI, int CT, bool VEC>
__device__ __forceinline__ void gemm_bf16_body(const GemmParams& p, char* smem) {
  using namespace bfg;
#define AS(i) (smem + (i) * TILE_BYTES)
#define BS(i) (smem + (2 + (i)) * TILE_BYTES)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  // XCD-grouped tile order (n fastest, then m, then the split-K slab)
  const int nwg = gridDim.x * gridDim.y * gridDim.z;
  const int wg = cg_xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), nwg);
  const int bz = wg / (gridDim.x * gridDim.y), bxy = wg % (gridDim.x * gridDim.y);
  const int m0 = (bxy / gridDim.x) * BM, n0 = (bxy % gridDim.x) * BN;
  const int kbeg = bz * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const bf16_t* A = (const bf16_t*)p.A;
  const bf16_t* B = (const bf16_t*)p.B;

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  const int nt = (kend - kbeg + BKT - 1) / BKT;
  Stage sa, sb;
  if (nt > 0) {
    stage_load<AK>(sa, A, p.lda, m0, p.M, kbeg, kend, tid);
    stage_load<BKC>(sb, B, p.ldb, n0, p.N, kbeg, kend, tid);
    stage_store<AK>(sa, AS(0), tid);
    stage_store<BKC>(sb, BS(0), tid);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const bool more = (t + 1) < nt;
    if (more) {
      const int kn = kbeg + (t + 1) * BKT;
      stage_load<AK>(sa, A, p.lda, m0, p.M, kn, kend, tid);
      stage_load<BKC>(sb, B, p.ldb, n0, p.N, kn, kend, tid);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8bf af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<AK>(AS(cur), wm + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BKC>(BS(cur), wn + 16 * j, ks, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (more) {
      stage_store<AK>(sa, AS(cur ^ 1), tid);
      stage_store<BKC>(sb, BS(cur ^ 1), tid);
    }
    __syncthreads();
  }
#undef AS
#undef BS
  if (!VEC) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + v;
          const int col = n0 + wn + 16 * j + (lane & 15);
          epi_store(p, row, col, acc[i][j][v], bz);
        }
    return;
  }
  // ---- stage the wave's 64x64 fp32 tile through LDS, then 8-column vector epilogue
  float* st = (float*)smem + wave * 64 * EPI_LD;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) st[(16 * i + 4 * (lane >> 4) + v) * EPI_LD + 16 * j + (lane & 15)] = acc[i][j][v];
  __syncthreads();
#pragma unroll 2
  for (int it = 0; it < 8; ++it) {
    const int c = lane + 64 * it, r = c >> 3, ch = c & 7;
    const int row = m0 + wm + r, col = n0 + wn + ch * 8;
    if (row >= p.M || col >= p.N) continue;
    float v[8];
    ld8f(st + r * EPI_LD + ch * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= p.alpha;
    if (p.split > 1) {
      st8f(p.ws + ((long long)bz * p.M + row) * p.N + col, v);
      continue;
    }
    epi_apply8<EPI, CT>(p, row, col, v);
  }
}

template <bool AK, bool BKC>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  gemm_bf16_body<AK, BKC, -1, 0, false>(p, smem);
}

template <bool AK, bool BKC, int EPI, int CT>
__global__ __launch_bounds__(256, 2) void gemm_bf16_vec_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  gemm_bf16_body<AK, BKC, EPI, CT, true>(p, smem);
}

#include "gemm_wide.h"
#include "gemm_pers.h"
#include "gemm_lw.h"
#include "gemm_dw.h"

// CG_EPI_COLSUM fallback: part[r/64][n] = sum of C rows [64r, 64r+64) (column n)
__global__ __launch_bounds__(256) void colsum64_kernel(const void* C, long long ldc, int ct, int M, int N,
                                                       float* __restrict__ part) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int r0 = blockIdx.y * 64, r1 = min(M, r0 + 64);
  float acc = 0.f;
  for (int r = r0; r < r1; ++r)
    acc += ct == CG_BF16 ? bf2f(((const bf16_t*)C)[(long long)r * ldc + n]) : ((const float*)C)[(long long)r * ldc + n];
  part[(long long)blockIdx.y * N + n] = acc;
}

// ---------------------------------------------------------------------------
// host launcher
// ---------------------------------------------------------------------------
typedef void (*gemm_kernel_t)(GemmParams);

template <typename K>
static void launch4(K k00, K k01, K k10, K k11, bool ak, bool bk, dim3 g, dim3 b, size_t sh,
                    hipStream_t s, const GemmParams& p) {
  K k = ak ? (bk ? k11 : k10) : (bk ? k01 : k00);
  hipLaunchKernelGGL(k, g, b, sh, s, p);
}

// compile-time-specialised epilogues for the combinations the TinyGPT step issues
template <template <bool, bool, int, int> class KS>
static gemm_kernel_t pick_spec(bool ak, bool bk, int e, int ct) {
#define SPEC(AK_, BK_, E, T) \
  if (ak == AK_ && bk == BK_ && e == (E) && ct == (T)) return KS<AK_, BK_, (E), (T)>::fn;
  SPEC(true, true, 0, CG_BF16)
  SPEC(true, true, 0, CG_F32)
  SPEC(true, true, CG_EPI_BIAS, CG_BF16)
  SPEC(true, true, CG_EPI_BIAS | CG_EPI_RESID, CG_F32)
  SPEC(true, true, CG_EPI_BIAS | CG_EPI_GELU, CG_BF16)
  SPEC(true, true, CG_EPI_BIAS | CG_EPI_DROPOUT | CG_EPI_RESID, CG_F32)
  SPEC(true, true, CG_EPI_RESID, CG_F32)
  SPEC(true, true, CG_EPI_DROPOUT | CG_EPI_RESID, CG_F32)
  SPEC(true, true, CG_EPI_DGELU, CG_BF16)
  SPEC(true, true, CG_EPI_BIAS | CG_EPI_GELU | CG_EPI_GELU_DERIV, CG_BF16)
  SPEC(true, true, CG_EPI_DGELU | CG_EPI_GELU_DERIV, CG_BF16)
  SPEC(true, false, 0, CG_BF16)
  SPEC(true, false, 0, CG_F32)
  SPEC(true, false, CG_EPI_DGELU, CG_BF16)
  SPEC(false, false, 0, CG_F32)
  SPEC(false, false, CG_EPI_ACCUM, CG_F32)
#undef SPEC
  if (ak) return bk ? KS<true, true, -1, 0>::fn : KS<true, false, -1, 0>::fn;
  return bk ? KS<false, true, -1, 0>::fn : KS<false, false, -1, 0>::fn;
}
template <bool AK, bool BKC, int E, int T>
struct VecK { static constexpr gemm_kernel_t fn = gemm_bf16_vec_kernel<AK, BKC, E, T>; };
template <bool AK, bool BKC, int E, int T>
struct WideK { static constexpr gemm_kernel_t fn = gemm_bf16_wide_kernel<AK, BKC, E, T>; };

// Tile choice per call (cg_gemm_desc.tile; the library keeps no mutable process-wide settings).
// CG_TILE_AUTO: the persistent 256x128 tile whenever it is legal (K-contiguous operands, no split,
// an epilogue it implements), on its loader-wave variant (gemm_lw.h) for the epilogues measured
// faster there (round 3-4, tools/gemm_c4.py same box: qkv dX 28.3 -> 26.9 us, fc1 dX 35.0 -> 32.7,
// fc1 forward GELU' 54.7 -> 52.0, proj forward bias + fp32 residual 23.5 -> 22.0, C3 SwiGLU forward
// 90.2 -> 87.4; the dGELU, dropout-residual and column-sum epilogues stay on the 8-wave kernel:
// fc2 dX 52.1 vs 53.5, fc2 forward 49.8 vs 51.5 on the loader-wave one); else the 256x128 LDS-DMA
// tile for K-contiguous products with >= 192 tiles; else the 128x128 register-staged tile.
// The other codes force one kernel for tests and A/B runs (CG_EUNSUPPORTED where it cannot run
// the product).  fp32 products always take the 128x128 f32-MFMA tile where its 16-B operand
// chunks are legal, else the 64x64 one.
static bool lw_auto_for(int e) {
  return e == 0 || e == CG_EPI_BIAS || e == (CG_EPI_BIAS | CG_EPI_GELU) ||
         e == (CG_EPI_BIAS | CG_EPI_GELU | CG_EPI_GELU_DERIV) || e == (CG_EPI_BIAS | CG_EPI_RESID) ||
         e == CG_EPI_RESID || e == CG_EPI_SWIGLU || (e & CG_EPI_ROPE);
}
// the persistent kernel for epilogue e, output type ct under tile code `tile` (nullptr: none)
static gemm_kernel_t pick_pers(int e, int ct, int tile, bool* lw_out) {
  bool lw = tile == CG_TILE_PERS_LW || (tile == CG_TILE_AUTO && lw_auto_for(e));
  // the SwiGLU backward's epilogue does not fit the loader-wave kernel's 168-register budget;
  // the RoPE epilogue exists only there
  if (e == CG_EPI_DSWIGLU) lw = false;
  if (e & CG_EPI_ROPE) {
    if (ct != CG_BF16 || !lw) return nullptr;
    *lw_out = true;
    if (e == (CG_EPI_BIAS | CG_EPI_ROPE)) return gemm_bf16_lw_kernel<CG_EPI_BIAS | CG_EPI_ROPE, CG_BF16>;
    if (e == CG_EPI_ROPE) return gemm_bf16_lw_kernel<CG_EPI_ROPE, CG_BF16>;
    return nullptr;
  }
  *lw_out = lw;
#define PSPEC(E, T) \
  if (e == (E) && ct == (T)) return lw ? gemm_bf16_lw_kernel<(E), (T)> : gemm_bf16_pers_kernel<(E), (T)>;
  PSPEC(0, CG_BF16)
  PSPEC(0, CG_F32)
  PSPEC(CG_EPI_BIAS, CG_BF16)
  PSPEC(CG_EPI_BIAS | CG_EPI_RESID, CG_F32)
  PSPEC(CG_EPI_BIAS | CG_EPI_GELU, CG_BF16)
  PSPEC(CG_EPI_BIAS | CG_EPI_DROPOUT | CG_EPI_RESID, CG_F32)
  PSPEC(CG_EPI_RESID, CG_F32)
  PSPEC(CG_EPI_DROPOUT | CG_EPI_RESID, CG_F32)
  PSPEC(CG_EPI_DGELU, CG_BF16)
  PSPEC(CG_EPI_ACCUM, CG_F32)
  PSPEC(CG_EPI_DGELU | CG_EPI_COLSUM, CG_BF16)
  PSPEC(CG_EPI_BIAS | CG_EPI_GELU | CG_EPI_GELU_DERIV, CG_BF16)
  PSPEC(CG_EPI_DGELU | CG_EPI_GELU_DERIV, CG_BF16)
  PSPEC(CG_EPI_DGELU | CG_EPI_GELU_DERIV | CG_EPI_COLSUM, CG_BF16)
  PSPEC(CG_EPI_COLSUM, CG_BF16)
  PSPEC(CG_EPI_SWIGLU, CG_BF16)
  PSPEC(CG_EPI_DSWIGLU, CG_BF16)
#undef PSPEC
  return nullptr;
}
static int cu_count() {
  static int n[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (!n[dev]) {  // a benign race: every thread stores the same value
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    n[dev] = v;
  }
  return n[dev];
}
// CUs the persistent launches (forward / dX tiles, grouped dW) spread over.  (A reserve of CUs
// left free for an RCCL all-reduce beside the backward was measured and removed in round 5: a
// one-tile-per-CU launch becomes two rounds either way)
extern "C" int cg_pers_cus(void) { return cu_count(); }
static bool use_pers(const cg_gemm_desc* d, int split) {
  if (split != 1) return false;
  if (d->tile != CG_TILE_AUTO && d->tile != CG_TILE_PERS && d->tile != CG_TILE_PERS_LW) return false;
  if (!d->a_kcontig || !d->b_kcontig) return false;
  if (d->K % bfp::BKT || d->K < 2 * bfp::BKT) return false;
  bool lw = false;
  if (!pick_pers(d->epilogue, d->c_dtype, d->tile, &lw)) return false;
  // every buffer extent must stay below the out-of-range voffset used for masked lanes
  const long long lim = (long long)bfp::OOR - (1ll << 24);
  const long long es = d->c_dtype == CG_BF16 ? 2 : 4;
  if (((long long)(d->M - 1) * d->lda + d->K) * 2 >= lim) return false;
  if (((long long)(d->N - 1) * d->ldb + d->K) * 2 >= lim) return false;
  if (((long long)(d->M - 1) * d->ldc + d->N) * es >= lim) return false;
  if ((d->epilogue & CG_EPI_RESID) && ((long long)(d->M - 1) * d->ldr + d->N) * 4 >= lim) return false;
  if ((d->epilogue & (CG_EPI_GELU | CG_EPI_DGELU)) && ((long long)(d->M - 1) * d->ld_aux + d->N) * es >= lim)
    return false;
  // SwiGLU: B has 2N rows; aux / aux_out (and C for DSWIGLU) are 2N columns wide
  if ((d->epilogue & (CG_EPI_SWIGLU | CG_EPI_DSWIGLU)) &&
      (((long long)(2 * d->N - 1) * d->ldb + d->K) * 2 >= lim ||
       ((long long)(d->M - 1) * d->ld_aux + 2 * d->N) * 2 >= lim ||
       ((long long)(d->M - 1) * d->ldc + 2 * d->N) * 2 >= lim))
    return false;
  return true;
}

// 256x128 LDS-DMA tile: large, 64-aligned K chunks and enough tiles to fill the chip
static bool use_wide(const cg_gemm_desc* d, int kchunk, int split) {
  if (d->tile != CG_TILE_AUTO && d->tile != CG_TILE_WIDE) return false;
  if (d->K % bfw::BKT || kchunk % bfw::BKT || d->M < bfw::BM || d->N < bfw::BN) return false;
  if (d->tile == CG_TILE_WIDE) return true;
  // auto: the LDS-DMA tile wins on K-contiguous operands (forward products); with an
  // MN-contiguous operand (dX, dW) the 128x128 register-staged tile is still faster
  if (!d->a_kcontig || !d->b_kcontig) return false;
  const long long tiles = (long long)cg_cdiv(d->M, bfw::BM) * cg_cdiv(d->N, bfw::BN) * split;
  return tiles >= 192;
}

static bool vec_ok(const cg_gemm_desc* d, int split) {
  const int e = d->epilogue;
  if (d->N % 8 || d->ldc % 8 || ((uintptr_t)d->C & 15)) return false;
  if ((e & CG_EPI_BIAS) && ((uintptr_t)d->bias & 15)) return false;
  if ((e & CG_EPI_RESID) && (d->ldr % 8 || ((uintptr_t)d->resid & 15))) return false;
  if ((e & (CG_EPI_GELU | CG_EPI_DGELU)) &&
      (d->ld_aux % 8 || ((uintptr_t)((e & CG_EPI_GELU) ? d->aux_out : d->aux) & 15)))
    return false;
  if (split > 1 && ((uintptr_t)d->workspace & 15)) return false;
  return true;
}

extern "C" int cg_gemm(const cg_gemm_desc* d, void* stream) {
  if (!d || d->M < 0 || d->N < 0 || d->K < 0) return CG_EINVAL;
  if (d->M == 0 || d->N == 0) return CG_OK;
  hipStream_t s = (hipStream_t)stream;
  GemmParams p{};
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.A = d->A; p.lda = d->lda; p.B = d->B; p.ldb = d->ldb;
  p.C = d->C; p.ldc = d->ldc; p.c_dtype = d->c_dtype;
  p.epi = d->epilogue; p.alpha = d->alpha;
  p.bias = d->bias; p.resid = d->resid; p.ldr = d->ldr;
  p.aux = d->aux; p.aux_out = d->aux_out; p.ld_aux = d->ld_aux;
  p.drop_seed = d->drop_seed;
  p.drop_thr = cg_drop_threshold(d->drop_p);
  p.drop_scale = d->drop_p < 1.f ? 1.0f / (1.0f - d->drop_p) : 0.f;
  if ((p.epi & CG_EPI_ACCUM) && p.c_dtype != CG_F32) return CG_EINVAL;
  if ((p.epi & CG_EPI_BIAS) && !p.bias) return CG_EINVAL;
  if ((p.epi & CG_EPI_RESID) && !p.resid) return CG_EINVAL;
  if ((p.epi & CG_EPI_GELU) && !p.aux_out) return CG_EINVAL;
  if ((p.epi & CG_EPI_DGELU) && !p.aux) return CG_EINVAL;
  if ((p.epi & CG_EPI_GELU_DERIV) && !(p.epi & (CG_EPI_GELU | CG_EPI_DGELU))) return CG_EINVAL;
  if ((p.epi & CG_EPI_COLSUM) && (!d->workspace || d->split_k > 1)) return CG_EINVAL;
  if ((p.epi & CG_EPI_COLSUM) && d->ws_bytes < (size_t)cg_cdiv(p.M, 64) * (size_t)p.N * sizeof(float)) return CG_EINVAL;
  // SwiGLU epilogues: only the persistent bf16 tile implements them (the caller keeps the
  // separate cg_swiglu_* passes on CG_EUNSUPPORTED)
  const bool swg = (p.epi & (CG_EPI_SWIGLU | CG_EPI_DSWIGLU)) != 0;
  if (swg) {
    if (p.epi != CG_EPI_SWIGLU && p.epi != CG_EPI_DSWIGLU) return CG_EUNSUPPORTED;
    if (d->in_dtype != CG_BF16 || p.c_dtype != CG_BF16 || d->split_k > 1 || !d->a_kcontig || !d->b_kcontig ||
        p.alpha != 1.0f || (p.N & 63) || (p.ldc & 7) || (p.ld_aux & 7) || ((uintptr_t)p.C & 15) ||
        ((uintptr_t)(p.epi == CG_EPI_SWIGLU ? p.aux_out : p.aux) & 15))
      return CG_EUNSUPPORTED;
    if (p.epi == CG_EPI_SWIGLU ? !p.aux_out : !p.aux) return CG_EINVAL;
    p.n_valid = d->n_valid > 0 ? std::min(d->n_valid, p.N) : p.N;
  }
  // RoPE epilogue: only the loader-wave persistent tile implements it (the caller keeps the
  // separate cg_rope_tab pass on CG_EUNSUPPORTED)
  const bool rope = (p.epi & CG_EPI_ROPE) != 0;
  if (rope) {
    if ((p.epi & ~(CG_EPI_ROPE | CG_EPI_BIAS)) || !d->rope_cos || !d->rope_sin || d->rope_T <= 0) return CG_EINVAL;
    const int hd = d->rope_hd;
    if (d->in_dtype != CG_BF16 || p.c_dtype != CG_BF16 || d->split_k > 1 || hd <= 0 || hd % 16 ||
        d->rope_heads <= 0 || (long long)d->rope_heads * hd > p.N || p.N % 16 || p.N >= 65536 ||
        (((uintptr_t)d->rope_cos | (uintptr_t)d->rope_sin) & 15))
      return CG_EUNSUPPORTED;
    p.rope_cos = d->rope_cos;
    p.rope_sin = d->rope_sin;
    p.rope_T = d->rope_T;
    p.rope_half = hd / 2;
    p.rope_G = hd / 16;
    p.rope_mul = (65536 + p.rope_G - 1) / p.rope_G;
    p.rope_uqk = d->rope_heads * hd / 16;
  }
  // a forced tile names a bf16 kernel: out of range is a caller error, and an fp32-operand product
  // (which only the f32-MFMA kernels run) cannot honour it
  if (d->tile < CG_TILE_AUTO || d->tile > CG_TILE_PERS_LW) return CG_EINVAL;
  if (d->tile != CG_TILE_AUTO && d->in_dtype != CG_BF16) return CG_EUNSUPPORTED;
  int split = d->split_k > 1 ? d->split_k : 1;
  const int bkt = d->in_dtype == CG_BF16 ? bfg::BKT : 16;
  if (d->K == 0) split = 1;
  int kchunk = cg_cdiv(cg_cdiv(d->K > 0 ? d->K : 1, split), bkt) * bkt;
  split = cg_cdiv(d->K > 0 ? d->K : 1, kchunk);
  if (split > 1 && (!d->workspace || d->ws_bytes < (size_t)split * (size_t)p.M * (size_t)p.N * sizeof(float)))
    return CG_EINVAL;
  p.kchunk = kchunk; p.split = split; p.ws = d->workspace;
  bool vec = false;
  const bool colsum = (p.epi & CG_EPI_COLSUM) != 0;
  bool colsum_fused = false;

  if (d->in_dtype == CG_F32) {
    p.epi &= ~CG_EPI_COLSUM;
    // the 128x128 f32-MFMA tile: 16-B operand chunks (leading dims and the contiguous extent of
    // each operand -- K for a K-contiguous one, M / N for an MN-contiguous one -- multiples of 4)
    const bool big = !(d->lda & 3) && !(d->ldb & 3) && !((uintptr_t)d->A & 15) &&
                     !((uintptr_t)d->B & 15) && ((d->a_kcontig || d->b_kcontig) ? !(d->K & 3) : true) &&
                     (d->a_kcontig || !(d->M & 3)) && (d->b_kcontig || !(d->N & 3));
    if (big) {
      launch4(gemm_f32_big_kernel<false, false>, gemm_f32_big_kernel<false, true>, gemm_f32_big_kernel<true, false>,
              gemm_f32_big_kernel<true, true>, d->a_kcontig, d->b_kcontig,
              dim3(cg_cdiv(p.N, f32b::BN), cg_cdiv(p.M, f32b::BM), split), dim3(256), 0, s, p);
    } else {
      dim3 g(cg_cdiv(p.N, 64), cg_cdiv(p.M, 64), split);
      launch4(gemm_f32_kernel<false, false>, gemm_f32_kernel<false, true>, gemm_f32_kernel<true, false>,
              gemm_f32_kernel<true, true>, d->a_kcontig, d->b_kcontig, g, dim3(256), 0, s, p);
    }
  } else if (d->in_dtype == CG_BF16) {
    if ((d->lda & 7) || (d->ldb & 7)) return CG_EUNSUPPORTED;
    if (((uintptr_t)d->A & 15) || ((uintptr_t)d->B & 15)) return CG_EUNSUPPORTED;
    if (d->a_kcontig ? (d->K & 7) : (d->M & 7)) return CG_EUNSUPPORTED;
    if (d->b_kcontig ? (d->K & 7) : (d->N & 7)) return CG_EUNSUPPORTED;
    dim3 g(cg_cdiv(p.N, bfg::BN), cg_cdiv(p.M, bfg::BM), split);
    dim3 blk(256);
    size_t sh = bfg::SMEM;
    vec = vec_ok(d, split);
    gemm_kernel_t k;
    const bool pers = vec && use_pers(d, split);
    if ((swg || rope) && !pers) return CG_EUNSUPPORTED;
    if (!pers) p.epi &= ~CG_EPI_COLSUM;  // only the persistent tile fuses the column sums
    const int ke = split > 1 ? 0 : p.epi, kt = split > 1 ? CG_F32 : p.c_dtype;
    if (pers) {
      bool lw = false;
      k = pick_pers(p.epi, p.c_dtype, d->tile, &lw);
      colsum_fused = colsum;
      const int tiles = cg_cdiv(p.N, (p.epi & CG_EPI_SWIGLU) ? bfp::BN / 2 : bfp::BN) * cg_cdiv(p.M, bfp::BM);
      g = dim3(std::min(tiles, d->max_wg > 0 ? d->max_wg : cg_pers_cus()));
      blk = dim3(lw ? bfl::THREADS : bfp::THREADS);
      sh = lw ? bfl::SMEM : bfp::SMEM;
    } else if (vec && use_wide(d, kchunk, split)) {
      k = pick_spec<WideK>(d->a_kcontig, d->b_kcontig, ke, kt);
      g = dim3(cg_cdiv(p.N, bfw::BN) * cg_cdiv(p.M, bfw::BM) * split);
      blk = dim3(bfw::THREADS);
      sh = bfw::SMEM;
    } else if (vec && (d->tile == CG_TILE_AUTO || d->tile == CG_TILE_VEC)) {
      k = pick_spec<VecK>(d->a_kcontig, d->b_kcontig, ke, kt);
    } else if (d->tile != CG_TILE_AUTO && d->tile != CG_TILE_VEC) {
      return CG_EUNSUPPORTED;  // the forced tile cannot run this product
    } else {
      k = d->a_kcontig ? (d->b_kcontig ? gemm_bf16_kernel<true, true> : gemm_bf16_kernel<true, false>)
                       : (d->b_kcontig ? gemm_bf16_kernel<false, true> : gemm_bf16_kernel<false, false>);
    }
    cg_func_lds((const void*)k, (int)sh);
    // the persistent tile is one probe class (every forward and dX product of the step, all its
    // epilogue specialisations); the other tiles are classed by operand layout
    const int pk = pers ? CG_PROBE_GEMM_PERS
                        : d->a_kcontig ? (d->b_kcontig ? CG_PROBE_GEMM_FWD : CG_PROBE_GEMM_DX)
                                       : (d->b_kcontig ? CG_PROBE_NONE : CG_PROBE_GEMM_DW);
    cg_probe_begin(pk, s);
    hipLaunchKernelGGL(k, g, blk, sh, s, p);
    if (cg_probe_kind() == pk) {
      // algorithmic work of the launch: the SwiGLU forward multiplies against both the gate and
      // the up rows (2N weight rows); bytes = operands once + outputs once (+ epilogue operands)
      const double M = p.M, N = p.N, K = p.K, ce = p.c_dtype == CG_F32 ? 4.0 : 2.0;
      const bool sw = (p.epi & CG_EPI_SWIGLU) != 0, dsw = (p.epi & CG_EPI_DSWIGLU) != 0;
      const double nb = sw ? 2.0 * N : N;  // weight rows read
      double bytes = 2.0 * (M * K + nb * K) + M * N * ce;
      if (p.epi & CG_EPI_BIAS) bytes += 4.0 * N;
      if (p.epi & CG_EPI_RESID) bytes += 4.0 * M * N;
      if (p.epi & (CG_EPI_GELU | CG_EPI_DGELU)) bytes += M * N * ce;
      if (p.epi & CG_EPI_ACCUM) bytes += 4.0 * M * N;
      if (sw) bytes += 2.0 * M * 2.0 * N;                   // pre-activations g|u
      if (dsw) bytes += 2.0 * M * 2.0 * N + M * N * ce;     // g|u read, d(g|u) is 2N wide
      if (p.epi & CG_EPI_COLSUM) bytes += 4.0 * cg_cdiv(p.M, 64) * N;
      cg_probe_end(pk, s, 2.0 * M * nb * K, bytes);
    }
  } else {
    return CG_EUNSUPPORTED;
  }
  CG_LAUNCH_CHECK();
  if (split > 1) {
    const long long total = (long long)p.M * p.N;
    if (vec) {
      int blocks = (int)((total / 8 + 255) / 256);
      if (blocks > 4096) blocks = 4096;
      hipLaunchKernelGGL(splitk_reduce_vec_kernel, dim3(blocks), dim3(256), 0, s, p);
    } else {
      int blocks = (int)((total + 255) / 256);
      if (blocks > 4096) blocks = 4096;
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, p);
    }
    CG_LAUNCH_CHECK();
  }
  if (colsum && !colsum_fused) {  // unfused fallback: the same 64-row partials, read back from C
    hipLaunchKernelGGL(colsum64_kernel, dim3(cg_cdiv(p.N, 256), cg_cdiv(p.M, 64)), dim3(256), 0, s, p.C, p.ldc,
                       p.c_dtype, p.M, p.N, p.ws);
    CG_LAUNCH_CHECK();
  }
  return CG_OK;
}

// ---------------------------------------------------------------------------
// grouped weight-gradient GEMM (gemm_dw.h)
// ---------------------------------------------------------------------------
static bool dw_tile_code(int bm) { return bm == 128 || bm == 129 || bm == 256 || bm == 512; }
// tile codes: 128 / 129 = 128 x 128 (4 / 5 ring stages), 256 = 256 x 128 (3 stages),
// 512 = 256 x 256 (2 stages of 64 KiB)
extern "C" int cg_gemm_dw_tiles(int bm, int N_out, int K_out) {
  if (!dw_tile_code(bm)) bm = 128;
  return cg_cdiv(N_out, bm >= 256 ? 256 : 128) * cg_cdiv(K_out, bm == 512 ? 256 : 128);
}
template <int BM, int NS, int BNT = bfd::BN>
static int launch_dw(bfd::Params& P, hipStream_t s) {
  using G = bfd::Geo<BM, NS, BNT>;
  bool cs = false;
  for (int i = 0; i < P.nprod; ++i) cs |= P.p[i].colsum != nullptr;
  auto kern = cs ? gemm_dw_kernel<BM, NS, BNT, true> : gemm_dw_kernel<BM, NS, BNT, false>;
  int ntiles = 0;
  for (int i = 0; i < P.nprod; ++i) {
    bfd::Prod& pr = P.p[i];
    pr.tiles_n = cg_cdiv(pr.K_out, BNT);
    pr.tile0 = ntiles;
    ntiles += cg_cdiv(pr.N_out, BM) * pr.tiles_n;
  }
  P.ntiles = ntiles * P.ksplit;
  if (!ntiles) return CG_OK;
  if (P.ksplit > 1) P.kc_steps = cg_cdiv(cg_cdiv(P.K, P.ksplit), bfd::BKT);
  const int grid = std::min(P.ntiles, P.max_wg > 0 ? P.max_wg : cg_pers_cus());
  cg_func_lds((const void*)kern, G::SMEM);
  double flops = 0, bytes = 0;
  for (int i = 0; i < P.nprod; ++i) {
    const bfd::Prod& q = P.p[i];
    flops += 2.0 * q.N_out * (double)q.K_out * P.K;
    bytes += 2.0 * P.K * ((double)q.N_out + q.K_out) + (q.accum ? 8.0 : 4.0) * q.N_out * (double)q.K_out;
  }
  cg_probe_begin(CG_PROBE_GEMM_DW_GROUPED, s);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(G::THREADS), G::SMEM, s, P);
  // the probe window is the grouped kernel alone; the k-split slab reduce is its own HBM-bound
  // probe class (CG_PROBE_DW_SLAB), so a plan that splits the tokens carries its slab pass in the
  // kernel tables instead of looking cheaper than it is
  cg_probe_end(CG_PROBE_GEMM_DW_GROUPED, s, flops, bytes);
  if (P.ksplit > 1) {
    long long most = 0;
    double elems = 0;
    for (int i = 0; i < P.nprod; ++i) {
      most = std::max<long long>(most, (long long)P.p[i].N_out * P.p[i].K_out / 4);
      elems += (double)P.p[i].N_out * P.p[i].K_out;
    }
    cg_probe_begin(CG_PROBE_DW_SLAB, s);
    hipLaunchKernelGGL(dw_slab_reduce_kernel, dim3((unsigned)std::min<long long>(cg_cdiv(most, 256), 512), P.nprod),
                       dim3(256), 0, s, P);
    cg_probe_end(CG_PROBE_DW_SLAB, s, (P.ksplit - 1) * elems, (4.0 * (P.ksplit - 1) + 8.0) * elems);
  }
  CG_LAUNCH_CHECK();
  return CG_OK;
}
// slab bytes cg_gemm_dw_grouped needs for grp->ksplit > 1
extern "C" size_t cg_gemm_dw_grouped_workspace(const cg_dw_group* grp) {
  if (!grp || grp->ksplit <= 1) return 0;
  size_t e = 0;
  for (int i = 0; i < grp->n && i < CG_DW_MAX; ++i)
    if (grp->p[i].N_out > 0 && grp->p[i].K_out > 0) e += (size_t)grp->p[i].N_out * (size_t)grp->p[i].K_out;
  return (size_t)(grp->ksplit - 1) * e * sizeof(float);
}
extern "C" size_t cg_gemm_dw_grouped_workspace(const cg_dw_group* grp);
extern "C" int cg_gemm_dw_grouped(const cg_dw_group* grp, void* stream) {
  if (!grp || grp->n < 0 || grp->n > CG_DW_MAX || grp->K <= 0) return CG_EINVAL;
  bfd::Params P{};
  P.nprod = 0;
  P.K = grp->K;
  const long long lim = (1ll << 31) - (1ll << 24);
  for (int i = 0; i < grp->n; ++i) {
    const cg_dw_product& q = grp->p[i];
    if (q.N_out <= 0 || q.K_out <= 0) continue;
    if (!q.A || !q.B || !q.C) return CG_EINVAL;
    if (q.N_out % 8 || q.K_out % 8 || q.lda % 8 || q.ldb % 8 || q.ldc % 4 || q.lda < q.N_out || q.ldb < q.K_out ||
        q.ldc < q.K_out)
      return CG_EUNSUPPORTED;
    if (((uintptr_t)q.A & 15) || ((uintptr_t)q.B & 15) || ((uintptr_t)q.C & 15)) return CG_EUNSUPPORTED;
    if (((long long)(grp->K - 1) * q.lda + q.N_out) * 2 >= lim || ((long long)(grp->K - 1) * q.ldb + q.K_out) * 2 >= lim)
      return CG_EUNSUPPORTED;
    bfd::Prod& pr = P.p[P.nprod++];
    pr.A = (const bf16_t*)q.A; pr.lda = q.lda;
    pr.B = (const bf16_t*)q.B; pr.ldb = q.ldb;
    pr.C = q.C; pr.ldc = q.ldc;
    pr.N_out = q.N_out; pr.K_out = q.K_out;
    pr.alpha = q.alpha; pr.accum = q.accumulate;
    pr.colsum = q.col_sum;
    if (q.col_sum && grp->ksplit > 1) return CG_EUNSUPPORTED;
  }
  if (!P.nprod) return CG_OK;
  P.ksplit = grp->ksplit > 1 ? grp->ksplit : 1;
  if (P.ksplit > 8) return CG_EUNSUPPORTED;
  if (P.ksplit > 1) {
    if (!grp->workspace || ((uintptr_t)grp->workspace & 15) || grp->ws_bytes < cg_gemm_dw_grouped_workspace(grp))
      return CG_EINVAL;
    P.slab = grp->workspace;
    long long off = 0;
    for (int i = 0; i < P.nprod; ++i) {
      P.slab_off[i] = off;
      off += (long long)P.p[i].N_out * P.p[i].K_out;
    }
    P.slab_stride = off;
  }
  hipStream_t s = (hipStream_t)stream;
  const int bm = grp->tile_m > 0 ? grp->tile_m : 128;
  P.max_wg = grp->max_wg;
  // tile_m codes: 128 / 256 = rows of the C tile (ring of 4 / 3 stages); 129 / 257 = the same
  // tile with one more ring stage (5 / 4... 160 KB LDS for 128)
  if (bm == 512) return launch_dw<256, 2, 256>(P, s);
  if (bm == 256) return launch_dw<256, 3>(P, s);
  if (bm == 129) return launch_dw<128, 5>(P, s);
  return launch_dw<128, 4>(P, s);
}
