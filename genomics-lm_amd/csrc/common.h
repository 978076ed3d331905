// Shared device helpers for the codon-LM MI355X (gfx950) kernels.
// Wave = 64 lanes everywhere; all reductions are written for 64-wide waves.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <mutex>
#include "../../include/codonlm_hip.h"
#include "probe.h"

#define CG_WAVE 64

typedef uint16_t bf16_t;  // raw bf16 storage
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));

// ---------------------------------------------------------------------------
// bf16 <-> f32 (round-to-nearest-even, NaN preserved)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf2f(bf16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
// hardware v_cvt_pk_bf16_f32 (RNE, NaN stays NaN): no per-element NaN branch
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// Typed load/store of one activation element (T = float or bf16_t).
template <typename T> __device__ __forceinline__ float ld_act(const T* p);
template <> __device__ __forceinline__ float ld_act<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld_act<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T> __device__ __forceinline__ void st_act(T* p, float v);
template <> __device__ __forceinline__ void st_act<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st_act<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// ---------------------------------------------------------------------------
// wave / block reductions (64 lanes)
// ---------------------------------------------------------------------------
// All in VALU (no LDS round trip per step, as __shfl_xor's ds_bpermute would take): DPP within
// each 16-lane row (quad xor 1, quad xor 2, row_half_mirror, row_mirror), then
// v_permlane16_swap and v_permlane32_swap, whose two results called with (v, v) are the two
// partners' values in every lane.  Every lane ends with the total, in a fixed order.
template <typename F>
__device__ __forceinline__ float wave_reduce(float v, F op) {
  v = op(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false)));
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = op(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return op(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float wave_sum(float v) {
  return wave_reduce(v, [](float a, float b) { return a + b; });
}
__device__ __forceinline__ float wave_max(float v) {
  return wave_reduce(v, [](float a, float b) { return fmaxf(a, b); });
}

// ---------------------------------------------------------------------------
// Counter-based dropout hash.  keep(seed,row,col) is a pure function so the
// backward pass regenerates the forward mask.  Restated bit-for-bit in
// oracle/tinygpt_oracle.py dropout_keep (the parity tests compare them).
// One 32-bit hash covers the column pair (2c, 2c+1): low half -> even column.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t cg_fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}
// two-stage hash: a full mix per row (hoisted out of inner loops), then one multiply
// per column pair: pair_mix(row_hash + colpair * K)
__device__ __forceinline__ uint32_t cg_row_hash(uint32_t seed, uint32_t row) {
  return cg_fmix32(seed ^ (row * 0x9E3779B1u));
}
// (24-bit multiply: v_mul_u32_u24 issues at full rate, v_mul_lo_u32 at quarter rate; the
// shift-xor before it folds the high bits into the multiplied low 24)
__device__ __forceinline__ uint32_t cg_pair_mix(uint32_t x) {
  x ^= x >> 15; x = __umul24(x, 0x2C1B3Du); x ^= x >> 12;
  return x;
}
constexpr uint32_t CG_COLK = 0x85EBCA77u;
__device__ __forceinline__ uint32_t cg_hash_pair(uint32_t seed, uint32_t row, uint32_t colpair) {
  return cg_pair_mix(cg_row_hash(seed, row) + colpair * CG_COLK);
}
__device__ __forceinline__ bool cg_keep(uint32_t seed, uint32_t row, uint32_t col, uint32_t thr) {
  uint32_t h = cg_hash_pair(seed, row, col >> 1);
  uint32_t bits = (col & 1u) ? (h >> 16) : (h & 0xFFFFu);
  return bits >= thr;
}
// ---- the attention-dropout keep words of one 64x64 block of the causal lower triangle (query
// block qb, key block kb of triangle index i) for row bh = b*H + h: keep = cg_keep(seed,
// bh*T + q, key, thr), one wave, lane = query; per key pair one hash, two compares, two shift-ins
// (10 VALU ops).  Words in "pair-split" order (bit c = key 2c, bit 16 + c = key 2c + 1) at
// qmask[((bh*(wpr/2) + kb)*T + q)*2 + w] (attention_mfma.h attn_drop_mask_kernel, and beside the
// LayerNorm rows in ops.hip ln_fwd_mask_kernel).
// acc = 2 acc + (half SEL of h >= thr): v_cmp (SDWA word select) into VCC, v_addc shifts it in
template <int SEL>
__device__ __forceinline__ uint32_t cg_shift_in_keep(uint32_t acc, uint32_t h, uint32_t thr) {
  uint32_t r;
  if constexpr (SEL == 0)
    asm("v_cmp_ge_u32_sdwa vcc, %1, %2 src0_sel:WORD_0 src1_sel:DWORD\n\tv_addc_co_u32_e32 %0, vcc, %3, %3, vcc"
        : "=v"(r) : "v"(h), "s"(thr), "v"(acc) : "vcc");
  else
    asm("v_cmp_ge_u32_sdwa vcc, %1, %2 src0_sel:WORD_1 src1_sel:DWORD\n\tv_addc_co_u32_e32 %0, vcc, %3, %3, vcc"
        : "=v"(r) : "v"(h), "s"(thr), "v"(acc) : "vcc");
  return r;
}
__device__ __forceinline__ void cg_drop_mask_block(uint32_t* __restrict__ qmask, int T, int wpr, uint32_t seed,
                                                   uint32_t thr, int i, long long bh, int lane) {
  int qb = (int)((sqrtf(8.f * (float)i + 1.f) - 1.f) * 0.5f);
  while ((qb + 1) * (qb + 2) / 2 <= i) ++qb;
  while (qb * (qb + 1) / 2 > i) --qb;
  const int kb = i - qb * (qb + 1) / 2;
  const int q = qb * 64 + lane;
  if (q >= T) return;
  const uint32_t hrow = cg_row_hash(seed, (uint32_t)(bh * T + q));
  uint32_t wq[2];
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    uint32_t ev = 0, od = 0;
#pragma unroll
    for (int c = 15; c >= 0; --c) {  // high pairs first: pair c lands on bits c / 16 + c
      const uint32_t h = cg_pair_mix(hrow + (uint32_t)(kb * 32 + w * 16 + c) * CG_COLK);
      ev = cg_shift_in_keep<0>(ev, h, thr);
      od = cg_shift_in_keep<1>(od, h, thr);
    }
    wq[w] = ev | (od << 16);
  }
  *(uint2*)(qmask + ((bh * (wpr >> 1) + kb) * T + q) * 2) = make_uint2(wq[0], wq[1]);
}
__host__ __device__ inline uint32_t cg_drop_threshold(float p) {
  float t = p * 65536.0f + 0.5f;
  uint32_t u = (uint32_t)t;
  return u > 65536u ? 65536u : u;
}
__host__ __device__ inline uint32_t cg_site_seed(uint32_t seed, int layer, int site) {
  uint32_t x = seed * 0x01000193u + (uint32_t)layer * 0x9E37u + (uint32_t)site * 0x7F4A7C15u + 0x3C6EF372u;
  x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
  return x;
}
enum { CG_SITE_EMB = 0, CG_SITE_ATTN = 1, CG_SITE_MLP = 2 };

// GELU (erf form, nn.GELU default) and its derivative
__device__ __forceinline__ float gelu_f(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float dgelu_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + __expf(-x)); }

// bf16-mode GELU: Phi(x) from Abramowitz-Stegun 7.1.26 (|erf error| <= 1.5e-7, far below the
// bf16 rounding of the output), one exp2 + one rcp instead of the ocml erff call.  The
// Gaussian factor e^{-x^2/2} is shared by Phi and the pdf, so dGELU costs one exp as well.
// (fp32 parity mode keeps gelu_f / dgelu_f above.)
__device__ __forceinline__ float gelu_phi_q(float x, float& e) {
  e = __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x);  // e^{-x^2/2}
  const float t = __builtin_amdgcn_rcpf(fmaf(0.23164189992f, fabsf(x), 1.0f));  // p/sqrt(2) = 0.3275911/1.41421
  // the A&S polynomial with its coefficients times -1/2: h = 0.5 - 0.5 erfc(|x|/sqrt2) in one fma
  float poly = fmaf(t, -0.5307027145f, 0.7265760135f);
  poly = fmaf(t, poly, -0.7107068705f);
  poly = fmaf(t, poly, 0.142248368f);
  poly = fmaf(t, poly, -0.127414796f);
  const float h = fmaf(t * poly, e, 0.5f);  // = 1/2 - q, q = 0.5 * erfc(|x|/sqrt2)
  // Phi(x) = 1/2 + sign(x) h (h >= 0): the sign bit of x copied onto h, one v_bfi
  return 0.5f + __uint_as_float((__float_as_uint(h) & 0x7FFFFFFFu) | (__float_as_uint(x) & 0x80000000u));
}
__device__ __forceinline__ float gelu_fast(float x) {
  float e;
  return x * gelu_phi_q(x, e);
}
// gelu(x) and gelu'(x) from one evaluation of Phi and the Gaussian factor
__device__ __forceinline__ float gelu_fast_d(float x, float& dg) {
  float e;
  const float phi = gelu_phi_q(x, e);
  dg = fmaf(x * 0.39894228040143268f, e, phi);
  return x * phi;
}
__device__ __forceinline__ float dgelu_fast(float x) {
  float e;
  const float phi = gelu_phi_q(x, e);
  return fmaf(x * 0.39894228040143268f, e, phi);
}

// host-side launch check
// bijective remap of a linear workgroup id so that the ids one XCD receives (round-robin
// dispatch: XCD = id mod 8) become one contiguous logical range (MI355X_MICROARCH guide)
__device__ __forceinline__ int cg_xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): the attribute belongs to
// the kernel on the CURRENT device, so a process that drives several GPUs sets it on each of them
static inline void cg_func_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static const void* fns[512];
  static int devs[512], lds[512], n = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  for (int i = 0; i < n; ++i)
    if (fns[i] == fn && devs[i] == dev && lds[i] >= bytes) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (n < 512) {
    fns[n] = fn;
    devs[n] = dev;
    lds[n] = bytes;
    ++n;
  }
}

#define CG_LAUNCH_CHECK()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return CG_ELAUNCH;                \
  } while (0)

static inline int cg_cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
