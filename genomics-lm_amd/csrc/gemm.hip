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
};

// ---------------------------------------------------------------------------
// epilogue (shared by both kernels and the split-K reducer)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void epi_apply(const GemmParams& p, int row, int col, float v) {
  const int e = p.epi;
  if (e & CG_EPI_BIAS) v += p.bias[col];
  const long long ai = (long long)row * p.ld_aux + col;
  if (e & CG_EPI_GELU) {
    if (p.c_dtype == CG_BF16) ((bf16_t*)p.aux_out)[ai] = f2bf(v);
    else ((float*)p.aux_out)[ai] = v;
    v = gelu_f(v);
  }
  if (e & CG_EPI_DGELU) {
    float a = (p.c_dtype == CG_BF16) ? bf2f(((const bf16_t*)p.aux)[ai]) : ((const float*)p.aux)[ai];
    v *= dgelu_f(a);
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

__device__ __forceinline__ void epi_store(const GemmParams& p, int row, int col, float v) {
  if (row >= p.M || col >= p.N) return;
  v *= p.alpha;
  if (p.split > 1) {
    p.ws[((long long)blockIdx.z * p.M + row) * p.N + col] = v;
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
        epi_store(p, row, col, acc[i][j][v]);
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

template <bool AK, bool BKC>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmParams p) {
  using namespace bfg;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // images: A0 | A1 | B0 | B1
#define AS(i) (smem + (i) * TILE_BYTES)
#define BS(i) (smem + (2 + (i)) * TILE_BYTES)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = blockIdx.z * p.kchunk;
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
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      stage_store<AK>(sa, AS(cur ^ 1), tid);
      stage_store<BKC>(sb, BS(cur ^ 1), tid);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + v;
        const int col = n0 + wn + 16 * j + (lane & 15);
        epi_store(p, row, col, acc[i][j][v]);
      }
#undef AS
#undef BS
}

// ---------------------------------------------------------------------------
// host launcher
// ---------------------------------------------------------------------------
template <typename K>
static void launch4(K k00, K k01, K k10, K k11, bool ak, bool bk, dim3 g, dim3 b, size_t sh,
                    hipStream_t s, const GemmParams& p) {
  K k = ak ? (bk ? k11 : k10) : (bk ? k01 : k00);
  hipLaunchKernelGGL(k, g, b, sh, s, p);
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
  int split = d->split_k > 1 ? d->split_k : 1;
  const int bkt = d->in_dtype == CG_BF16 ? bfg::BKT : 16;
  if (d->K == 0) split = 1;
  int kchunk = cg_cdiv(cg_cdiv(d->K > 0 ? d->K : 1, split), bkt) * bkt;
  split = cg_cdiv(d->K > 0 ? d->K : 1, kchunk);
  if (split > 1 && !d->workspace) return CG_EINVAL;
  p.kchunk = kchunk; p.split = split; p.ws = d->workspace;

  if (d->in_dtype == CG_F32) {
    dim3 g(cg_cdiv(p.N, 64), cg_cdiv(p.M, 64), split);
    launch4(gemm_f32_kernel<false, false>, gemm_f32_kernel<false, true>, gemm_f32_kernel<true, false>,
            gemm_f32_kernel<true, true>, d->a_kcontig, d->b_kcontig, g, dim3(256), 0, s, p);
  } else if (d->in_dtype == CG_BF16) {
    if ((d->lda & 7) || (d->ldb & 7)) return CG_EUNSUPPORTED;
    if (((uintptr_t)d->A & 15) || ((uintptr_t)d->B & 15)) return CG_EUNSUPPORTED;
    if (d->a_kcontig ? (d->K & 7) : (d->M & 7)) return CG_EUNSUPPORTED;
    if (d->b_kcontig ? (d->K & 7) : (d->N & 7)) return CG_EUNSUPPORTED;
    dim3 g(cg_cdiv(p.N, bfg::BN), cg_cdiv(p.M, bfg::BM), split);
    const size_t sh = 4 * bfg::TILE_BYTES;
    static bool attr_done = false;
    if (!attr_done) {
      (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, sh);
      (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, sh);
      (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, sh);
      (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, sh);
      attr_done = true;
    }
    launch4(gemm_bf16_kernel<false, false>, gemm_bf16_kernel<false, true>, gemm_bf16_kernel<true, false>,
            gemm_bf16_kernel<true, true>, d->a_kcontig, d->b_kcontig, g, dim3(256), sh, s, p);
  } else {
    return CG_EUNSUPPORTED;
  }
  CG_LAUNCH_CHECK();
  if (split > 1) {
    const long long total = (long long)p.M * p.N;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, p);
    CG_LAUNCH_CHECK();
  }
  return CG_OK;
}
