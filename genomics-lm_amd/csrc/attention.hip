// Causal + SEP-segment (+local window) attention with GQA and attention-prob dropout,
// flash-style (online softmax, no T x T matrix) -- replaces the SDPA / manual path of
// model_tiny_gpt.py:102-131 with the mask of build_attention_mask (:273-295).
//
// Mask for query q, key j (same batch row):  j <= q  &&  j >= segstart[q]
//                                             && (window <= 0 || q - j < window)
// (segstart[q] = last SEP position <= q; equal cumsum(idx==SEP) <=> no SEP in (j, q].)
// Dropout (training): P_ij * keep(seed, (b*H+h)*T+q, j) / (1-p) feeds P.V only; the
// softmax normaliser uses the undropped P, exactly like att=softmax; att=dropout(att).
//
// Two implementations share this contract:
//   * attn_*_vec   : one query (or key) row per lane, fp32 VALU math.  Any T, hd <= 64,
//                    fp32 or bf16 storage.  Used for the fp32 parity mode and as the
//                    bf16 fallback for head dims the MFMA kernel does not cover.
//   * attn_*_mfma  : bf16 MFMA 32x32x16 kernels (hd in {32, 48, 64}) -- attention_mfma.h
//   * attn_fwd_f32mfma : the fp32 forward on f32 MFMA (hd % 8 == 0, hd <= 64) -- attention_f32.h
#include "common.h"

constexpr int AV_HD = 64;   // max head dim of the vector kernels
constexpr int AV_TQ = 64;   // queries (or keys) per block
constexpr int AV_SUB = 16;  // keys per online-softmax update in the forward

__device__ __forceinline__ bool attn_visible(int q, int j, int lo) { return j <= q && j >= lo; }

template <typename T>
__global__ __launch_bounds__(64) void attn_fwd_vec(const T* __restrict__ qkv, long long ld,
                                                   const int32_t* __restrict__ segstart, T* __restrict__ y,
                                                   long long ldy, float* __restrict__ lse, int Tn, int H, int KV,
                                                   int hd, int window, uint32_t seed, uint32_t thr, float dscale,
                                                   float scale) {
  // every lane reads the same K/V row (broadcast): rows unpadded and 16-B aligned so the reads
  // are ds_read_b128 (4 FMAs per LDS read instead of 1)
  __shared__ __attribute__((aligned(16))) float Ks[AV_TQ][AV_HD];
  __shared__ __attribute__((aligned(16))) float Vs[AV_TQ][AV_HD];
  const int lane = threadIdx.x;
  const int bh = blockIdx.y, b = bh / H, h = bh % H, kvh = h / (H / KV);
  const int q = blockIdx.x * AV_TQ + lane;
  const bool qok = q < Tn;
  const long long qrow = (long long)b * Tn + (qok ? q : 0);
  float qv[AV_HD], o[AV_HD];
#pragma unroll
  for (int d = 0; d < AV_HD; ++d) {
    qv[d] = (qok && d < hd) ? ld_act<T>(qkv + qrow * ld + (long long)h * hd + d) : 0.f;
    o[d] = 0.f;
  }
  int lo = (qok && segstart) ? segstart[qrow] : 0;
  if (window > 0) lo = max(lo, q - window + 1);
  int lo_min = qok ? lo : 0x7fffffff;
#pragma unroll
  for (int o2 = 32; o2 > 0; o2 >>= 1) lo_min = min(lo_min, __shfl_xor(lo_min, o2, 64));
  const int qmax = min(Tn - 1, (int)blockIdx.x * AV_TQ + AV_TQ - 1);
  const long long koff = (long long)H * hd + (long long)kvh * hd;
  const long long voff = (long long)(H + KV) * hd + (long long)kvh * hd;
  const uint32_t drow = (uint32_t)(((long long)b * H + h) * Tn + q);
  float m = -INFINITY, l = 0.f;
  for (int k0 = (lo_min / AV_TQ) * AV_TQ; k0 <= qmax; k0 += AV_TQ) {
    __syncthreads();
    for (int e = lane; e < AV_TQ * AV_HD; e += 64) {
      const int j = e / AV_HD, d = e % AV_HD;
      const int key = k0 + j;
      const bool ok = key < Tn && d < hd;
      const long long kr = ((long long)b * Tn + key) * ld;
      Ks[j][d] = ok ? ld_act<T>(qkv + kr + koff + d) : 0.f;
      Vs[j][d] = ok ? ld_act<T>(qkv + kr + voff + d) : 0.f;
    }
    __syncthreads();
    // keys in sub-tiles of AV_SUB with an online-softmax update each: the score row stays in
    // registers (a whole 64-key row unrolled makes hipcc hoist every K read and spill)
#pragma unroll 1
    for (int jb = 0; jb < AV_TQ; jb += AV_SUB) {
      float s[AV_SUB];
      float mt = -INFINITY;
#pragma unroll
      for (int jj = 0; jj < AV_SUB; ++jj) {
        const int j = jb + jj, key = k0 + j;
        float acc = 0.f;
#pragma unroll
        for (int d = 0; d < AV_HD; d += 4) {
          const float4 k4 = *(const float4*)&Ks[j][d];
          acc = fmaf(qv[d], k4.x, acc);
          acc = fmaf(qv[d + 1], k4.y, acc);
          acc = fmaf(qv[d + 2], k4.z, acc);
          acc = fmaf(qv[d + 3], k4.w, acc);
        }
        const bool vis = qok && key < Tn && attn_visible(q, key, lo);
        s[jj] = vis ? acc * scale : -INFINITY;
        mt = fmaxf(mt, s[jj]);
      }
      const float mn = fmaxf(m, mt);
      if (mn == -INFINITY) continue;
      const float alpha = __expf(m - mn);
      l *= alpha;
#pragma unroll
      for (int d = 0; d < AV_HD; ++d) o[d] *= alpha;
#pragma unroll
      for (int jj = 0; jj < AV_SUB; ++jj) {
        const int j = jb + jj;
        float p = __expf(s[jj] - mn);
        l += p;
        if (thr) p = cg_keep(seed, drow, (uint32_t)(k0 + j), thr) ? p * dscale : 0.f;
#pragma unroll
        for (int d = 0; d < AV_HD; d += 4) {
          const float4 v4 = *(const float4*)&Vs[j][d];
          o[d] = fmaf(p, v4.x, o[d]);
          o[d + 1] = fmaf(p, v4.y, o[d + 1]);
          o[d + 2] = fmaf(p, v4.z, o[d + 2]);
          o[d + 3] = fmaf(p, v4.w, o[d + 3]);
        }
      }
      m = mn;
    }
  }
  if (qok) {
    const float il = 1.0f / l;
    for (int d = 0; d < hd; ++d) st_act<T>(y + qrow * ldy + (long long)h * hd + d, o[d] * il);
    lse[((long long)b * H + h) * Tn + q] = m + __logf(l);
  }
}

// delta[bh,q] = sum_d dy * y   (rowsum(dO o O), valid with dropout)
template <typename T>
__global__ void attn_delta_kernel(const T* __restrict__ y, long long ldy, const T* __restrict__ dy, long long lddy,
                                  float* __restrict__ delta, int B, int Tn, int H, int hd) {
  const long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (e >= (long long)B * H * Tn) return;
  const int q = (int)(e % Tn);
  const long long bh = e / Tn;
  const int b = (int)(bh / H), h = (int)(bh % H);
  const long long r = (long long)b * Tn + q;
  float s = 0.f;
  for (int d = 0; d < hd; ++d)
    s += ld_act<T>(dy + r * lddy + (long long)h * hd + d) * ld_act<T>(y + r * ldy + (long long)h * hd + d);
  delta[e] = s;
}

template <typename T>
__global__ __launch_bounds__(64) void attn_bwd_dq_vec(const T* __restrict__ qkv, long long ld,
                                                      const int32_t* __restrict__ segstart, const T* __restrict__ dy,
                                                      long long lddy, const float* __restrict__ lse,
                                                      const float* __restrict__ delta, T* __restrict__ dqkv,
                                                      long long lddq, int Tn, int H, int KV, int hd, int window,
                                                      uint32_t seed, uint32_t thr, float dscale, float scale) {
  __shared__ float Ks[AV_TQ][AV_HD + 1];
  __shared__ float Vs[AV_TQ][AV_HD + 1];
  const int lane = threadIdx.x;
  const int bh = blockIdx.y, b = bh / H, h = bh % H, kvh = h / (H / KV);
  const int q = blockIdx.x * AV_TQ + lane;
  const bool qok = q < Tn;
  const long long qrow = (long long)b * Tn + (qok ? q : 0);
  float qv[AV_HD], dov[AV_HD], dq[AV_HD];
#pragma unroll
  for (int d = 0; d < AV_HD; ++d) {
    const bool ok = qok && d < hd;
    qv[d] = ok ? ld_act<T>(qkv + qrow * ld + (long long)h * hd + d) : 0.f;
    dov[d] = ok ? ld_act<T>(dy + qrow * lddy + (long long)h * hd + d) : 0.f;
    dq[d] = 0.f;
  }
  int lo = (qok && segstart) ? segstart[qrow] : 0;
  if (window > 0) lo = max(lo, q - window + 1);
  int lo_min = qok ? lo : 0x7fffffff;
#pragma unroll
  for (int o2 = 32; o2 > 0; o2 >>= 1) lo_min = min(lo_min, __shfl_xor(lo_min, o2, 64));
  const long long bhq = ((long long)b * H + h) * Tn + (qok ? q : 0);
  const float L = qok ? lse[bhq] : 0.f;
  const float dl = qok ? delta[bhq] : 0.f;
  const int qmax = min(Tn - 1, (int)blockIdx.x * AV_TQ + AV_TQ - 1);
  const long long koff = (long long)H * hd + (long long)kvh * hd;
  const long long voff = (long long)(H + KV) * hd + (long long)kvh * hd;
  const uint32_t drow = (uint32_t)bhq;
  for (int k0 = (lo_min / AV_TQ) * AV_TQ; k0 <= qmax; k0 += AV_TQ) {
    __syncthreads();
    for (int e = lane; e < AV_TQ * AV_HD; e += 64) {
      const int j = e / AV_HD, d = e % AV_HD;
      const int key = k0 + j;
      const bool ok = key < Tn && d < hd;
      const long long kr = ((long long)b * Tn + key) * ld;
      Ks[j][d] = ok ? ld_act<T>(qkv + kr + koff + d) : 0.f;
      Vs[j][d] = ok ? ld_act<T>(qkv + kr + voff + d) : 0.f;
    }
    __syncthreads();
    for (int j = 0; j < AV_TQ; ++j) {
      const int key = k0 + j;
      if (!(qok && key < Tn && attn_visible(q, key, lo))) continue;
      float sacc = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < AV_HD; ++d) { sacc += qv[d] * Ks[j][d]; dp += dov[d] * Vs[j][d]; }
      const float p = __expf(sacc * scale - L);
      if (thr) dp = cg_keep(seed, drow, (uint32_t)key, thr) ? dp * dscale : 0.f;
      const float ds = p * (dp - dl);
#pragma unroll
      for (int d = 0; d < AV_HD; ++d) dq[d] += ds * Ks[j][d];
    }
  }
  if (qok)
    for (int d = 0; d < hd; ++d) st_act<T>(dqkv + qrow * lddq + (long long)h * hd + d, dq[d] * scale);
}

template <typename T>
__global__ __launch_bounds__(64) void attn_bwd_dkdv_vec(const T* __restrict__ qkv, long long ld,
                                                        const int32_t* __restrict__ segstart, const T* __restrict__ dy,
                                                        long long lddy, const float* __restrict__ lse,
                                                        const float* __restrict__ delta, T* __restrict__ dqkv,
                                                        long long lddq, int Tn, int H, int KV, int hd, int window,
                                                        uint32_t seed, uint32_t thr, float dscale, float scale) {
  __shared__ float Ks[AV_TQ][AV_HD + 1];
  __shared__ float Vs[AV_TQ][AV_HD + 1];
  __shared__ float Qs[AV_TQ][AV_HD];
  __shared__ float Ds[AV_TQ][AV_HD];
  __shared__ float Ls[AV_TQ], Dl[AV_TQ];
  __shared__ int Lo[AV_TQ];
  const int lane = threadIdx.x;
  const int bk = blockIdx.y, b = bk / KV, kvh = bk % KV;
  const int rep = H / KV;
  const int k0 = blockIdx.x * AV_TQ;
  const int key = k0 + lane;
  const bool kok = key < Tn;
  const long long koff = (long long)H * hd + (long long)kvh * hd;
  const long long voff = (long long)(H + KV) * hd + (long long)kvh * hd;
  for (int e = lane; e < AV_TQ * AV_HD; e += 64) {
    const int j = e / AV_HD, d = e % AV_HD;
    const bool ok = (k0 + j) < Tn && d < hd;
    const long long kr = ((long long)b * Tn + k0 + j) * ld;
    Ks[j][d] = ok ? ld_act<T>(qkv + kr + koff + d) : 0.f;
    Vs[j][d] = ok ? ld_act<T>(qkv + kr + voff + d) : 0.f;
  }
  float dk[AV_HD], dv[AV_HD];
#pragma unroll
  for (int d = 0; d < AV_HD; ++d) { dk[d] = 0.f; dv[d] = 0.f; }
  int qend = Tn;
  if (window > 0) qend = min(Tn, k0 + AV_TQ - 1 + window);
  for (int hh = 0; hh < rep; ++hh) {
    const int h = kvh * rep + hh;
    const long long bh = (long long)b * H + h;
    for (int q0 = k0; q0 < qend; q0 += AV_TQ) {
      __syncthreads();
      for (int e = lane; e < AV_TQ * AV_HD; e += 64) {
        const int i = e / AV_HD, d = e % AV_HD;
        const bool ok = (q0 + i) < Tn && d < hd;
        const long long r = (long long)b * Tn + q0 + i;
        Qs[i][d] = ok ? ld_act<T>(qkv + r * ld + (long long)h * hd + d) : 0.f;
        Ds[i][d] = ok ? ld_act<T>(dy + r * lddy + (long long)h * hd + d) : 0.f;
      }
      {
        const int qi = q0 + lane;
        const bool ok = qi < Tn;
        Ls[lane] = ok ? lse[bh * Tn + qi] : 0.f;
        Dl[lane] = ok ? delta[bh * Tn + qi] : 0.f;
        int lo = (ok && segstart) ? segstart[(long long)b * Tn + qi] : 0;
        if (window > 0) lo = max(lo, qi - window + 1);
        Lo[lane] = ok ? lo : 0x7fffffff;
      }
      __syncthreads();
      if (!kok) continue;
      for (int i = 0; i < AV_TQ; ++i) {
        const int qi = q0 + i;
        if (qi >= Tn || !attn_visible(qi, key, Lo[i])) continue;
        float sacc = 0.f, dp = 0.f;
#pragma unroll
        for (int d = 0; d < AV_HD; ++d) { sacc += Qs[i][d] * Ks[lane][d]; dp += Ds[i][d] * Vs[lane][d]; }
        const float p = __expf(sacc * scale - Ls[i]);
        float pd = p;
        if (thr) {
          const bool kp = cg_keep(seed, (uint32_t)(bh * Tn + qi), (uint32_t)key, thr);
          pd = kp ? p * dscale : 0.f;
          dp = kp ? dp * dscale : 0.f;
        }
        const float ds = p * (dp - Dl[i]);
#pragma unroll
        for (int d = 0; d < AV_HD; ++d) {
          dv[d] += pd * Ds[i][d];
          dk[d] += ds * Qs[i][d];
        }
      }
    }
  }
  if (kok) {
    const long long r = (long long)b * Tn + key;
    for (int d = 0; d < hd; ++d) {
      st_act<T>(dqkv + r * lddq + koff + d, dk[d] * scale);
      st_act<T>(dqkv + r * lddq + voff + d, dv[d]);
    }
  }
}

#include "attention_mfma.h"
#include "attention_f32.h"

// ---------------------------------------------------------------------------
// Attention probabilities of one layer, materialised (the manual path's `last_attn`,
// model_tiny_gpt.py:117-128: softmax(QK^T/sqrt(hd) masked), before dropout) from the forward's
// qkv rows and LSE: p = exp(S*scale - lse) on visible (query, key), 0 elsewhere.  Inspection
// path (B*H*T^2 outputs): one workgroup per (b, h, query) row, the query row in LDS.
// ---------------------------------------------------------------------------
template <typename T_>
__global__ __launch_bounds__(256) void attn_probs_kernel(const T_* __restrict__ qkv, long long ld,
                                                         const int32_t* __restrict__ seg, const float* __restrict__ lse,
                                                         float* __restrict__ out, int T, int H, int KV, int hd,
                                                         int window, float scale) {
  __shared__ float qs[AV_HD];
  const long long row = blockIdx.x;  // (b*H + h)*T + q
  const int q = (int)(row % T);
  const long long bh = row / T;
  const int b = (int)(bh / H), h = (int)(bh % H), kvh = h / (H / KV);
  const long long rb = (long long)b * T;
  for (int dd = threadIdx.x; dd < hd; dd += blockDim.x) qs[dd] = ld_act<T_>(qkv + (rb + q) * ld + (long long)h * hd + dd);
  __syncthreads();
  int lo = seg ? seg[rb + q] : 0;
  if (window > 0) lo = max(lo, q - window + 1);
  const float l = lse[row];
  for (int k = threadIdx.x; k < T; k += blockDim.x) {
    float p = 0.f;
    if (k <= q && k >= lo) {
      const T_* kr = qkv + (rb + k) * ld + (long long)(H + kvh) * hd;
      float sdot = 0.f;
      for (int dd = 0; dd < hd; ++dd) sdot = fmaf(qs[dd], ld_act<T_>(kr + dd), sdot);
      p = __expf(sdot * scale - l);
    }
    out[row * T + k] = p;
  }
}

extern "C" int cg_attn_probs(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart, const float* lse,
                             float* out, int B, int T, int H, int KV, int hd, int window, void* stream) {
  if (KV <= 0 || H % KV || !qkv || !lse || !out) return CG_EINVAL;
  if (hd <= 0 || hd > AV_HD) return CG_EUNSUPPORTED;
  if (B == 0 || T == 0) return CG_OK;
  const float scale = 1.0f / sqrtf((float)hd);
  const dim3 g((unsigned)((long long)B * H * T));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CG_BF16)
    hipLaunchKernelGGL(attn_probs_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)qkv, ldqkv, segstart, lse, out, T,
                       H, KV, hd, window, scale);
  else
    hipLaunchKernelGGL(attn_probs_kernel<float>, g, dim3(256), 0, s, (const float*)qkv, ldqkv, segstart, lse, out, T,
                       H, KV, hd, window, scale);
  CG_LAUNCH_CHECK();
  return CG_OK;
}

// ---------------------------------------------------------------------------
// host entry points
// ---------------------------------------------------------------------------
extern "C" size_t cg_attn_drop_mask_bytes(int B, int T, int H) {
  return B <= 0 || T <= 0 || H <= 0 ? 0 : attn_drop_mask_words(B, T, H) * sizeof(uint32_t);
}

extern "C" int cg_attn_drop_mask(int B, int T, int H, uint32_t drop_seed, float drop_p, void* mask, void* stream) {
  if (!(drop_p > 0.f) || drop_p >= 1.f) return CG_EINVAL;
  if (!mask) return CG_EINVAL;
  if (B == 0 || T == 0) return CG_OK;
  return attn_drop_mask_launch((uint32_t*)mask, B, T, H, drop_seed, cg_drop_threshold(drop_p), (hipStream_t)stream);
}

extern "C" int cg_attn_fwd(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart, void* y,
                           long long ldy, float* lse, int B, int T, int H, int KV, int hd, int window,
                           uint32_t drop_seed, float drop_p, const void* drop_mask, void* stream) {
  if (KV <= 0 || H % KV) return CG_EINVAL;
  if (hd <= 0 || hd > AV_HD) return CG_EUNSUPPORTED;
  if (B == 0 || T == 0) return CG_OK;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t thr = drop_p > 0.f ? cg_drop_threshold(drop_p) : 0u;
  const float dscale = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const float scale = 1.0f / sqrtf((float)hd);
  if (dtype == CG_BF16 && attn_mfma_supported(hd, ldqkv, ldy)) {
    return attn_fwd_mfma_launch((const bf16_t*)qkv, ldqkv, segstart, (bf16_t*)y, ldy, lse, B, T, H, KV, hd, window,
                                drop_seed, thr, dscale, scale, (const uint32_t*)drop_mask, s);
  }
  if (dtype != CG_BF16 && attn_f32mfma_supported(hd, qkv, ldqkv, y, ldy))
    return attn_fwd_f32mfma_launch((const float*)qkv, ldqkv, segstart, (float*)y, ldy, lse, B, T, H, KV, hd, window,
                                   drop_seed, thr, dscale, scale, s);
  dim3 g(cg_cdiv(T, AV_TQ), B * H);
  if (dtype == CG_BF16)
    hipLaunchKernelGGL(attn_fwd_vec<bf16_t>, g, dim3(64), 0, s, (const bf16_t*)qkv, ldqkv, segstart, (bf16_t*)y,
                       ldy, lse, T, H, KV, hd, window, drop_seed, thr, dscale, scale);
  else
    hipLaunchKernelGGL(attn_fwd_vec<float>, g, dim3(64), 0, s, (const float*)qkv, ldqkv, segstart, (float*)y, ldy,
                       lse, T, H, KV, hd, window, drop_seed, thr, dscale, scale);
  CG_LAUNCH_CHECK();
  return CG_OK;
}

extern "C" int cg_attn_fwd_keep(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart, void* y,
                                long long ldy, float* lse, int B, int T, int H, int KV, int hd, int window,
                                uint32_t drop_seed, float drop_p, void* mask_out, void* stream) {
  if (!(drop_p > 0.f) || drop_p >= 1.f || !mask_out) return CG_EINVAL;
  if (KV <= 0 || H % KV) return CG_EINVAL;
  if (hd <= 0 || hd > AV_HD) return CG_EUNSUPPORTED;
  if (B == 0 || T == 0) return CG_OK;
  if (dtype == CG_BF16 && attn_mfma_supported(hd, ldqkv, ldy))
    return attn_fwd_mfma_launch((const bf16_t*)qkv, ldqkv, segstart, (bf16_t*)y, ldy, lse, B, T, H, KV, hd, window,
                                drop_seed, cg_drop_threshold(drop_p), 1.f / (1.f - drop_p), 1.0f / sqrtf((float)hd),
                                nullptr, (hipStream_t)stream, (uint32_t*)mask_out);
  // other kernels: the words by the mask kernel, then the forward that reads them
  const int rc = cg_attn_drop_mask(B, T, H, drop_seed, drop_p, mask_out, stream);
  if (rc != CG_OK) return rc;
  return cg_attn_fwd(dtype, qkv, ldqkv, segstart, y, ldy, lse, B, T, H, KV, hd, window, drop_seed, drop_p, mask_out,
                     stream);
}

// nd (the vector path's delta = rowsum(dO o O); the MFMA paths' -delta/dscale) | -lse2 (MFMA paths)
// | dq_acc (the fused pass's fp32 dQ^T sums, attention_mfma.h fa::dqa_off)
extern "C" size_t cg_attn_bwd_workspace(int B, int T, int H) {
  return (2 * (size_t)B * H * T + attn_dq_acc_floats(B, T, H)) * sizeof(float);
}

extern "C" int cg_attn_bwd(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart, const void* y,
                           long long ldy, const void* dy, long long lddy, const float* lse, void* dqkv,
                           long long lddqkv, int B, int T, int H, int KV, int hd, int window, uint32_t drop_seed,
                           float drop_p, const void* drop_mask, float* bias_part, long long ld_part, void* ws,
                           size_t ws_bytes, void* stream) {
  return cg_attn_bwd_algo(CG_ATTN_BWD_AUTO, dtype, qkv, ldqkv, segstart, y, ldy, dy, lddy, lse, dqkv, lddqkv, B, T,
                          H, KV, hd, window, drop_seed, drop_p, drop_mask, bias_part, ld_part, nullptr, nullptr, ws,
                          ws_bytes, stream);
}
extern "C" int cg_attn_bwd_rope(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart,
                                const void* y, long long ldy, const void* dy, long long lddy, const float* lse,
                                void* dqkv, long long lddqkv, int B, int T, int H, int KV, int hd, int window,
                                uint32_t drop_seed, float drop_p, const void* drop_mask, float* bias_part,
                                long long ld_part, const float* rope_cos, const float* rope_sin, void* ws,
                                size_t ws_bytes, void* stream) {
  return cg_attn_bwd_algo(CG_ATTN_BWD_AUTO, dtype, qkv, ldqkv, segstart, y, ldy, dy, lddy, lse, dqkv, lddqkv, B, T,
                          H, KV, hd, window, drop_seed, drop_p, drop_mask, bias_part, ld_part, rope_cos, rope_sin, ws,
                          ws_bytes, stream);
}
// cg_attn_bwd with the gradients of RoPE-rotated q / k rotated back (rope_cos / rope_sin: the
// [>= T][hd/2] tables of cg_rope_tab; both NULL = no RoPE): the dQ and dK outputs -- and their
// bias partials -- are w.r.t. the un-rotated q / k projections (the MFMA kernels only; the vector
// path returns CG_EUNSUPPORTED with tables)
extern "C" int cg_attn_bwd_algo(int algo, int dtype, const void* qkv, long long ldqkv, const int32_t* segstart,
                                const void* y, long long ldy, const void* dy, long long lddy, const float* lse,
                                void* dqkv, long long lddqkv, int B, int T, int H, int KV, int hd, int window,
                                uint32_t drop_seed, float drop_p, const void* drop_mask, float* bias_part,
                                long long ld_part, const float* rope_cos, const float* rope_sin, void* ws,
                                size_t ws_bytes, void* stream) {
  if (algo < CG_ATTN_BWD_AUTO || algo > CG_ATTN_BWD_FUSED) return CG_EINVAL;
  if (KV <= 0 || H % KV) return CG_EINVAL;
  if ((rope_cos == nullptr) != (rope_sin == nullptr)) return CG_EINVAL;
  if (B > 0 && T > 0 && (!ws || ws_bytes < cg_attn_bwd_workspace(B, T, H))) return CG_EINVAL;
  if (hd <= 0 || hd > AV_HD) return CG_EUNSUPPORTED;
  if (B == 0 || T == 0) return CG_OK;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t thr = drop_p > 0.f ? cg_drop_threshold(drop_p) : 0u;
  const float dscale = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const float scale = 1.0f / sqrtf((float)hd);
  float* delta = (float*)ws;
  const long long nbt = (long long)B * H * T;
  const bool mfma = dtype == CG_BF16 && attn_mfma_supported(hd, ldqkv, lddy) && (lddqkv & 7) == 0 && (ldy & 7) == 0;
  if (bias_part && (!mfma || ld_part < (long long)(H + 2 * KV) * hd)) return CG_EUNSUPPORTED;
  if (rope_cos && (!mfma || hd % 16 || ((uintptr_t)rope_cos & 15) || ((uintptr_t)rope_sin & 15)))
    return CG_EUNSUPPORTED;
  if (mfma) {
    if (algo == CG_ATTN_BWD_FUSED && thr && !drop_mask) return CG_EUNSUPPORTED;  // keep words needed
    // delta = rowsum(dO o O): inside the split pass's dQ kernel, or the fused pass's pre-pass
    return attn_bwd_mfma_launch((const bf16_t*)qkv, ldqkv, segstart, (const bf16_t*)y, ldy, (const bf16_t*)dy,
                                lddy, lse, delta, (bf16_t*)dqkv, lddqkv, B, T, H, KV, hd, window, drop_seed, thr,
                                dscale, scale, (const uint32_t*)drop_mask, bias_part, ld_part, s, rope_cos,
                                rope_sin, algo);
  }
  if (algo == CG_ATTN_BWD_FUSED) return CG_EUNSUPPORTED;
  // fp32: the f32-MFMA kernels (exact fp32 products; delta formed inside the dQ kernel) where the
  // layout allows
  if (dtype != CG_BF16 && attn_f32mfma_supported(hd, qkv, ldqkv, dy, lddy) && (lddqkv & 3) == 0 &&
      ((uintptr_t)dqkv & 15) == 0 && (ldy & 3) == 0 && ((uintptr_t)y & 15) == 0)
    return attn_bwd_f32mfma_launch((const float*)qkv, ldqkv, segstart, (const float*)dy, lddy, (const float*)y, ldy,
                                   lse, delta, (float*)dqkv, lddqkv, B, T, H, KV, hd, window, drop_seed, thr, dscale,
                                   scale, s);
  if (dtype == CG_BF16) {
    hipLaunchKernelGGL(attn_delta_kernel<bf16_t>, dim3(cg_cdiv(nbt, 256)), dim3(256), 0, s, (const bf16_t*)y, ldy,
                       (const bf16_t*)dy, lddy, delta, B, T, H, hd);
  } else {
    hipLaunchKernelGGL(attn_delta_kernel<float>, dim3(cg_cdiv(nbt, 256)), dim3(256), 0, s, (const float*)y, ldy,
                       (const float*)dy, lddy, delta, B, T, H, hd);
  }
  CG_LAUNCH_CHECK();
  dim3 gq(cg_cdiv(T, AV_TQ), B * H), gk(cg_cdiv(T, AV_TQ), B * KV);
  if (dtype == CG_BF16) {
    hipLaunchKernelGGL(attn_bwd_dq_vec<bf16_t>, gq, dim3(64), 0, s, (const bf16_t*)qkv, ldqkv, segstart,
                       (const bf16_t*)dy, lddy, lse, delta, (bf16_t*)dqkv, lddqkv, T, H, KV, hd, window, drop_seed,
                       thr, dscale, scale);
    hipLaunchKernelGGL(attn_bwd_dkdv_vec<bf16_t>, gk, dim3(64), 0, s, (const bf16_t*)qkv, ldqkv, segstart,
                       (const bf16_t*)dy, lddy, lse, delta, (bf16_t*)dqkv, lddqkv, T, H, KV, hd, window, drop_seed,
                       thr, dscale, scale);
  } else {
    hipLaunchKernelGGL(attn_bwd_dq_vec<float>, gq, dim3(64), 0, s, (const float*)qkv, ldqkv, segstart,
                       (const float*)dy, lddy, lse, delta, (float*)dqkv, lddqkv, T, H, KV, hd, window, drop_seed,
                       thr, dscale, scale);
    hipLaunchKernelGGL(attn_bwd_dkdv_vec<float>, gk, dim3(64), 0, s, (const float*)qkv, ldqkv, segstart,
                       (const float*)dy, lddy, lse, delta, (float*)dqkv, lddqkv, T, H, KV, hd, window, drop_seed,
                       thr, dscale, scale);
  }
  CG_LAUNCH_CHECK();
  return CG_OK;
}

// ===========================================================================
// Single-token attention over a KV cache (incremental decoding): the query of position
// `pos` attends to keys lo..pos of its sequence, lo = its segment start (SEP mask,
// model_tiny_gpt.py:289-294) raised to pos-window+1 with a local window -- the same keys
// the full forward's mask row for `pos` admits.  One workgroup per (head, sequence); the
// scores live in LDS (pos < CG_DECODE_MAX_T).
// ===========================================================================
constexpr int DEC_MAXT = 4096;
template <typename T_>
__global__ __launch_bounds__(256) void attn_decode_kernel(const T_* __restrict__ q, long long ldq,
                                                          const T_* __restrict__ cache, long long ldc, int Tmax,
                                                          int pos, const int32_t* __restrict__ seg, int window, int H,
                                                          int KV, int hd, float scale, T_* __restrict__ y,
                                                          long long ldy) {
  __shared__ float sc[DEC_MAXT];
  __shared__ float qs[64];
  __shared__ float red[256];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int kvh = h / (H / KV);
  int lo = seg ? seg[b] : 0;
  if (window > 0) lo = max(lo, pos - window + 1);
  const int n = pos - lo + 1;
  if (tid < hd) qs[tid] = ld_act<T_>(q + (long long)b * ldq + (long long)h * hd + tid);
  __syncthreads();
  const T_* kb = cache + (long long)b * Tmax * ldc + (long long)kvh * hd;
  const T_* vb = kb + (long long)KV * hd;
  float mx = -INFINITY;
  for (int j = tid; j < n; j += 256) {
    const T_* kr = kb + (long long)(lo + j) * ldc;
    float s = 0.f;
    for (int e = 0; e < hd; ++e) s = fmaf(qs[e], ld_act<T_>(kr + e), s);
    s *= scale;
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  red[tid] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmaxf(red[tid], red[tid + o]);
    __syncthreads();
  }
  const float m = red[0];
  __syncthreads();
  float sum = 0.f;
  for (int j = tid; j < n; j += 256) {
    const float e = __expf(sc[j] - m);
    sc[j] = e;
    sum += e;
  }
  red[tid] = sum;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  const float l = red[0];
  __syncthreads();
  const int G = 256 / hd;  // key groups per output dim
  float acc = 0.f;
  if (tid < G * hd) {
    const int e = tid % hd, g = tid / hd;
    for (int j = g; j < n; j += G) acc = fmaf(sc[j], ld_act<T_>(vb + (long long)(lo + j) * ldc + e), acc);
  }
  red[tid] = acc;
  __syncthreads();
  if (tid < hd) {
    float o = 0.f;
    for (int g = 0; g < G; ++g) o += red[g * hd + tid];
    st_act<T_>(y + (long long)b * ldy + (long long)h * hd + tid, o / l);
  }
}

extern "C" int cg_attn_decode(int dtype, const void* q, long long ldq, const void* cache, long long ldc, int Tmax,
                              int pos, const int32_t* segstate, int window, int B, int H, int KV, int hd, void* y,
                              long long ldy, void* stream) {
  if (B <= 0 || H <= 0 || KV <= 0 || H % KV || hd <= 0 || hd > 64 || pos < 0 || pos >= Tmax || pos >= DEC_MAXT)
    return CG_EINVAL;
  if (!q || !cache || !y || ldc < 2 * KV * hd) return CG_EINVAL;
  const float scale = 1.0f / sqrtf((float)hd);
  const dim3 g(H, B);
  if (dtype == CG_BF16)
    hipLaunchKernelGGL(attn_decode_kernel<bf16_t>, g, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)q, ldq,
                       (const bf16_t*)cache, ldc, Tmax, pos, segstate, window, H, KV, hd, scale, (bf16_t*)y, ldy);
  else if (dtype == CG_F32)
    hipLaunchKernelGGL(attn_decode_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, (const float*)q, ldq,
                       (const float*)cache, ldc, Tmax, pos, segstate, window, H, KV, hd, scale, (float*)y, ldy);
  else
    return CG_EUNSUPPORTED;
  CG_LAUNCH_CHECK();
  return CG_OK;
}

// decoding segment state: seg[b] = pos when the token written at `pos` is the SEP id
__global__ void segstate_step_kernel(const int64_t* __restrict__ tok, int B, int sep, int pos, int32_t* __restrict__ seg) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b < B && tok[b] == sep) seg[b] = pos;
}
extern "C" int cg_segstate_step(const int64_t* tok, int B, int sep_id, int pos, int32_t* segstate, void* stream) {
  if (B <= 0 || sep_id < 0) return CG_OK;
  if (!tok || !segstate) return CG_EINVAL;
  hipLaunchKernelGGL(segstate_step_kernel, dim3(cg_cdiv(B, 64)), dim3(64), 0, (hipStream_t)stream, tok, B, sep_id, pos,
                     segstate);
  CG_LAUNCH_CHECK();
  return CG_OK;
}
