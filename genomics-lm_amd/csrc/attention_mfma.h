// bf16 MFMA flash attention for gfx950 (included by attention.hip).
//
// All products use v_mfma_f32_32x32x16_bf16.  Layout conventions (cdna_hip_programming §3):
//   A frag: lane l holds A[row l&31][k = 8*(l>>5) + j], j = 0..7
//   B frag: lane l holds B[k = 8*(l>>5) + j][col l&31]
//   C/D   : lane l holds C[row (r&3) + 8*(r>>2) + 4*(l>>5)][col l&31], r = 0..15
// "Swapped" products keep the query (or key) on the lane, so softmax statistics are
// per-lane scalars; an accumulator whose rows are the reduction index of the next
// product is fed to it as the B operand with no data movement (rows 8s..8s+7 of the
// accumulator = k-step s, in the permuted k order k(j,h) = 16s + 8(j>>2) + 4h + (j&3)),
// and the other operand is read from LDS with ds_read_b64_tr_b16 in that same order.
//
// Every K/V/Q/dO tile lives in LDS as a [64 rows][64 bf16] "dual" image whose 16-byte
// chunks are XOR-swizzled so that both the row reads (ds_read_b128, 32 rows x 16 B) and
// the transposed reads (ds_read_b64_tr_b16, 4 rows x 32 cols per half-wave) are
// bank-conflict free (see dual_off).  Head dims < 64 are zero-padded in the image.
#pragma once
#include <type_traits>

#ifndef ATTN_FWD_WPS
#define ATTN_FWD_WPS 2
#endif
#ifndef ATTN_DQ_WPS
#define ATTN_DQ_WPS 3  // waves per SIMD the dQ kernel is register-limited to (<= 168 VGPRs)
#endif

namespace fa {
constexpr int HDP = 64;        // padded head dim held in LDS / registers
constexpr int KT = 64;         // rows per staged tile
constexpr int IMG = KT * 128;  // bytes of one [64][64] bf16 image

__device__ __forceinline__ int dual_off(int row, int ch) {
  const int j = row >> 1;
  const int g = (j & 7) ^ ((j & 1) << 2);
  return row * 128 + 16 * (ch ^ g);
}

// ---- LDS-DMA staging (buffer_load ... lds): no staging registers, no ds_write.  A 64-row image
// is written by the 4 waves as 8 lane-linear 1-KiB pieces (wave w: rows 16w .. 16w+15); the
// dual_off XOR swizzle is applied on the per-lane SOURCE chunk.  The source is a buffer
// descriptor over one batch's T rows of a row-major bf16 matrix (rows >= T read as zero; columns
// >= hd get an offset past the records).  The DMA is inline asm: with the builtin, hipcc cannot
// prove that the image reads of the current buffer do not alias the DMA into the other one and
// drains vmcnt before every LDS read.  The kernels wait for it themselves (dma_drain + barrier
// before a buffer is read).  M0 (the LDS destination) is saved and restored around the load.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds), "s"(r)
      : "memory");
}
__device__ __forceinline__ void dma_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct TileDma {
  __amdgpu_buffer_rsrc_t r;
  uint32_t off[2];  // byte offsets of the lane's source chunk in its two pieces, from (row 0, column 0)
};
__device__ __forceinline__ TileDma tile_dma_src(const bf16_t* batch_rows, long long ld, int T, int hd, int wave,
                                                int lane) {
  TileDma t;
  t.r = __builtin_amdgcn_make_buffer_rsrc((void*)batch_rows, (short)0, (int)((long long)T * ld * 2), 0x00020000);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * wave + 8 * i + (lane >> 3), j = row >> 1;
    const int ch = (lane & 7) ^ ((j & 7) ^ ((j & 1) << 2));  // LDS slot lane&7 holds chunk ch
    t.off[i] = ch * 8 < hd ? (uint32_t)(((long long)row * ld + ch * 8) * 2) : 0x80000000u;
  }
  return t;
}
// img: LDS byte address of the image; ubase: byte offset of (tile row 0, head column 0); both
// wave-uniform
__device__ __forceinline__ void tile_dma(uint32_t img, const TileDma& t, uint32_t ubase, int wave) {
#pragma unroll
  for (int i = 0; i < 2; ++i) dma16(t.r, img + (uint32_t)((16 * wave + 8 * i) * 128), t.off[i] + ubase);
}
// A operand, rows rb..rb+31 of the image on the lane, k-step ks (16 columns)
__device__ __forceinline__ v8bf frag_row(const char* img, int rb, int ks, int lane) {
  return *(const v8bf*)(img + dual_off(rb + (lane & 31), 2 * ks + (lane >> 5)));
}

typedef v4s __attribute__((address_space(3))) * lds_v4s_p;

// A operand = transpose of the image: A[m = column cb*32 + (l&31)][k = image rows in the
// accumulator-permuted order of k-step s within the 32-row block rb]
__device__ __forceinline__ v8bf frag_tr(const char* img, int rb, int s, int cb, int lane) {
  const int h = lane >> 5, g16 = (lane >> 4) & 1, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int ch = ((cb * 32 + g16 * 16) >> 3) + (p >> 1);
  const int ra = rb + 16 * s + 4 * h + q;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_p)(img + dual_off(ra, ch) + 8 * (p & 1)));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_p)(img + dual_off(ra + 8, ch) + 8 * (p & 1)));
  const v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(v8bf, r);
}

typedef float v2f_a __attribute__((ext_vector_type(2)));
typedef __bf16 v2bf_a __attribute__((ext_vector_type(2)));
typedef uint32_t v4u_a __attribute__((ext_vector_type(4)));
// one v_cvt_pk_bf16_f32 per pair (RNE)
__device__ __forceinline__ uint32_t pk2bf(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((v2f_a){a, b}, v2bf_a));
}
// B operand from an accumulator: rows 8s..8s+7 as bf16
__device__ __forceinline__ v8bf pack_b(const v16f& x, int s) {
  const v4u_a w = {pk2bf(x[8 * s], x[8 * s + 1]), pk2bf(x[8 * s + 2], x[8 * s + 3]),
                   pk2bf(x[8 * s + 4], x[8 * s + 5]), pk2bf(x[8 * s + 6], x[8 * s + 7])};
  return __builtin_bit_cast(v8bf, w);
}

// v_max3_f32 as one instruction (fmaxf on MFMA results makes hipcc insert canonicalising
// v_max x, x, x before every compare)
__device__ __forceinline__ float max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// max over lane l and lane l^32 with one v_permlane32_swap
__device__ __forceinline__ float max_xhalf(float x) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return max3(__uint_as_float(sw[0]), __uint_as_float(sw[1]), x);
}

// ---- dropout keep bits (attn_drop_mask_kernel's "pair-split" words: within a 32-wide word,
// bit c = index 2c, bit 16 + c = index 2c + 1).  Accumulator element r of a lane holds index
// (r&3) + 8(r>>2) + 4(lane>>5); with the word pre-shifted right by 2(lane>>5) its bit is kbit(r).
__host__ __device__ constexpr int kbit(int r) { return ((r & 3) >> 1) + 4 * (r >> 2) + 16 * (r & 1); }
// fp32 value kept or zeroed by one bit (v_bfe_i32 + v_and; hipcc would turn the bit test into
// v_and + v_cmp + v_cndmask)
__device__ __forceinline__ float keep_f(float v, uint32_t w, int bit) {
  int m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(w), "i"(bit));
  return __int_as_float(__float_as_int(v) & m);
}
// all-ones / zero from bit `pos` (a per-lane register) of w
__device__ __forceinline__ int keep_mask(uint32_t w, uint32_t pos) {
  int m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(w), "v"(pos));
  return m;
}
// packed bf16 pair (elements r, r+1, r even) kept or zeroed: bits kbit(r) and kbit(r)+16 moved
// to 15 and 31, each 16-bit half sign-filled, and-ed -- 3 VALU ops per pair
__device__ __forceinline__ uint32_t keep_pk(uint32_t pk, uint32_t w, int bit) {
  uint32_t t;
  // op_sel_hi:[0,1]: the high half's shift count is the constant's LOW half too (an inline
  // constant is not replicated into the high half of a packed operand)
  asm("v_lshlrev_b32 %0, %2, %1\n\tv_pk_ashrrev_i16 %0, 15, %0 op_sel_hi:[0,1]" : "=&v"(t) : "v"(w), "i"(15 - bit));
  return pk & t;
}
// B operand rows 8s..8s+7 as bf16 with the dropout keep bits applied in the packed domain
__device__ __forceinline__ v8bf pack_b_keep(const v16f& x, int s, uint32_t w) {
  const v4u_a v = {keep_pk(pk2bf(x[8 * s], x[8 * s + 1]), w, kbit(8 * s)),
                   keep_pk(pk2bf(x[8 * s + 2], x[8 * s + 3]), w, kbit(8 * s + 2)),
                   keep_pk(pk2bf(x[8 * s + 4], x[8 * s + 5]), w, kbit(8 * s + 4)),
                   keep_pk(pk2bf(x[8 * s + 6], x[8 * s + 7]), w, kbit(8 * s + 6))};
  return __builtin_bit_cast(v8bf, v);
}

// B operand straight from global: row `row` (the lane's column index), k-step ks
__device__ __forceinline__ v8bf frag_global(const bf16_t* rowp, bool ok, int ks, int hd, int lane) {
  const int c = ks * 16 + 8 * (lane >> 5);
  if (ok && c < hd) return *(const v8bf*)(rowp + c);
  v8bf z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
  return z;
}

__device__ __forceinline__ v16f zero16() {
  v16f z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// sum over the 32 lanes of a half-wave (lanes l and l^32 are summed separately)
__device__ __forceinline__ float half_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 16, 64);
  return v;
}
// The workgroup's 128 rows of two accumulator blocks x0 (columns 0..31) and x1 (32..63), one
// row per lane-half, summed per column into red[wave][c0 + column] (LDS, 4 waves x stride)
__device__ __forceinline__ void colsum_acc(const v16f& x0, const v16f& x1, float s, bool ok, float* red, int stride,
                                           int c0, int wave, int lane) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float v0 = half_sum(ok ? x0[r] * s : 0.f);
    const float v1 = half_sum(ok ? x1[r] * s : 0.f);
    if ((lane & 31) == 0) {
      red[wave * stride + c0 + acc_row(r, lane)] = v0;
      red[wave * stride + c0 + 32 + acc_row(r, lane)] = v1;
    }
  }
}

// visible-key lower bound for query q (monotone non-decreasing in q)
__device__ __forceinline__ int lo_of(const int32_t* seg, long long rowbase, int q, int T, int window) {
  if (q >= T) q = T - 1;
  int lo = seg ? seg[rowbase + q] : 0;
  if (window > 0) lo = max(lo, q - window + 1);
  return lo;
}
}  // namespace fa


// ============================================================================
// attention-dropout keep bits, precomputed once per layer: keep = cg_keep(seed, (b*H+h)*T + q,
// key, thr) exactly, so the attention kernels test one bit per (query, key) instead of hashing
//   qmask[(bh*T + q)*wpr + w]: keys 32w..32w+31 of query q
// in "pair-split" order (bit c = key 2c, bit 16 + c = key 2c + 1: fa::kbit), which lets the
// forward apply two bits to a packed bf16 pair at once.  wpr = 2*ceil(T/64) (every 64-key tile
// has both of its words in bounds).  One wave per 64x64 block of the causal lower triangle,
// lane = query; per key pair one hash, two compares, two shift-ins (10 VALU ops).  Words of
// blocks above the diagonal are never written and never consumed (those pairs are causally
// masked before the bit test).
// ============================================================================
// acc = 2 acc + (half SEL of h >= thr): v_cmp (SDWA word select) into VCC, v_addc shifts it in
template <int SEL>
__device__ __forceinline__ uint32_t shift_in_keep(uint32_t acc, uint32_t h, uint32_t thr) {
  uint32_t r;
  if constexpr (SEL == 0)
    asm("v_cmp_ge_u32_sdwa vcc, %1, %2 src0_sel:WORD_0 src1_sel:DWORD\n\tv_addc_co_u32_e32 %0, vcc, %3, %3, vcc"
        : "=v"(r) : "v"(h), "s"(thr), "v"(acc) : "vcc");
  else
    asm("v_cmp_ge_u32_sdwa vcc, %1, %2 src0_sel:WORD_1 src1_sel:DWORD\n\tv_addc_co_u32_e32 %0, vcc, %3, %3, vcc"
        : "=v"(r) : "v"(h), "s"(thr), "v"(acc) : "vcc");
  return r;
}

__global__ __launch_bounds__(64) void attn_drop_mask_kernel(uint32_t* __restrict__ qmask, int T, int wpr,
                                                            uint32_t seed, uint32_t thr) {
  const int i = blockIdx.x;
  int qb = (int)((sqrtf(8.f * (float)i + 1.f) - 1.f) * 0.5f);
  while ((qb + 1) * (qb + 2) / 2 <= i) ++qb;
  while (qb * (qb + 1) / 2 > i) --qb;
  const int kb = i - qb * (qb + 1) / 2;
  const long long bh = blockIdx.y;
  const int q = qb * 64 + (int)threadIdx.x;
  if (q >= T) return;
  const uint32_t hrow = cg_row_hash(seed, (uint32_t)(bh * T + q));
  uint32_t wq[2];
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    uint32_t ev = 0, od = 0;
#pragma unroll
    for (int c = 15; c >= 0; --c) {  // high pairs first: pair c lands on bits c / 16 + c
      const uint32_t h = cg_pair_mix(hrow + (uint32_t)(kb * 32 + w * 16 + c) * CG_COLK);
      ev = shift_in_keep<0>(ev, h, thr);
      od = shift_in_keep<1>(od, h, thr);
    }
    wq[w] = ev | (od << 16);
  }
  *(uint2*)(qmask + (bh * T + q) * wpr + 2 * kb) = make_uint2(wq[0], wq[1]);
}

// ============================================================================
// forward: WG = 4 waves x 32 queries (128), key tiles of 64, K/V double-buffered.
// Compile-time variants keep the per-tile VALU stream branch-free: DROP (dropout on),
// the two LDS buffers (addresses fold into immediate offsets) and fully-visible vs
// masked tiles.  The running max is rescaled lazily: only when some query's max grows
// by more than 2^8 in the exp2 domain (stale maxima are exact - the same m is used for
// P, the row sum and the LSE; P <= 256 stays in range).
// ============================================================================
// DROP: 0 none, 1 keep bits hashed in the kernel, 2 keep bits read from attn_drop_mask_kernel's
// query-major words
template <int DROP, int HD>
__global__ __launch_bounds__(256, ATTN_FWD_WPS) void attn_fwd_mfma(const bf16_t* __restrict__ qkv, long long ld,
                                                        const int32_t* __restrict__ seg, bf16_t* __restrict__ y,
                                                        long long ldy, float* __restrict__ lse, int T, int H, int KV,
                                                        int hd_rt, int window, uint32_t seed, uint32_t thr,
                                                        float dscale, float scale,
                                                        const uint32_t* __restrict__ qmask, int wpr) {
  using namespace fa;
  constexpr int hd = HD;  // head dim is a compile-time constant: k-steps and the second
  (void)hd_rt;            // output block unroll without branches
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5;
  // grid (B*H, q-tiles): consecutive workgroups are different heads of the same q-tile, so the
  // round-robin XCD dispatch keeps all q-tiles of one head (its K/V) on one XCD's L2
  const int bh = blockIdx.x, b = bh / H, hh = bh % H, kvh = hh / (H / KV);
  const int qtile = gridDim.y - 1 - blockIdx.y;  // heaviest (latest) query tiles first
  const int q0 = qtile * 128, q0w = q0 + wave * 32;
  const int myq = q0w + (lane & 31);
  const bool qok = myq < T;
  const long long rowbase = (long long)b * T;
  const bf16_t* qrow = qkv + (rowbase + (qok ? myq : 0)) * ld + (long long)hh * hd;
  v8bf qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) qf[ks] = frag_global(qrow, qok, ks, hd, lane);
  const int lo = qok ? lo_of(seg, rowbase, myq, T, window) : 0x7fffffff;
  const int kmin = lo_of(seg, rowbase, q0, T, window);
  const int kmax = min(T - 1, q0 + 127);
  const int w_lo_min = lo_of(seg, rowbase, q0w, T, window);
  const int w_lo_max = lo_of(seg, rowbase, min(q0w + 31, T - 1), T, window);
  const int w_qmax = min(T - 1, q0w + 31);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const TileDma kv = tile_dma_src(qkv + rowbase * ld, ld, T, hd, wave_u, lane);
  const uint32_t kcol = (uint32_t)((H + kvh) * hd * 2), vcol = (uint32_t)((H + KV + kvh) * hd * 2);
  const uint32_t tstride = (uint32_t)(KT * ld * 2);  // bytes per 64-row tile
  const float c = scale * 1.4426950408889634f;
  const uint32_t drow = (uint32_t)(((long long)b * H + hh) * T + myq);
  const uint32_t hrow = DROP == 1 ? cg_row_hash(seed, drow) : 0u;
  const uint32_t* qm = DROP == 2 ? qmask + ((long long)bh * T + (qok ? myq : 0)) * wpr : nullptr;
  constexpr int nks = (hd + 15) >> 4;

  float m = -INFINITY, lsum = 0.f;
  v16f o0 = zero16(), o1 = zero16();
  const int t0 = kmin / KT, t1 = kmax / KT;
  tile_dma(lds0, kv, t0 * tstride + kcol, wave_u);
  tile_dma(lds0 + IMG, kv, t0 * tstride + vcol, wave_u);
  dma_drain();
  __syncthreads();

  auto body = [&](const char* Ki, const char* Vi, int k0, uint2 wc, auto full_c) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(full_c)::value;
    v16f s0 = zero16(), s1 = zero16();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks < nks) {
        s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row(Ki, 0, ks, lane), qf[ks], s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row(Ki, 32, ks, lane), qf[ks], s1, 0, 0, 0);
      }
    }
    // S feeds inline asm (max3): hipcc pads the XDL-result -> VALU-read hazard only before its own
    // instructions, so the accumulators pass through a wait of 19 states here (>= the 16-pass
    // rule); without it v_max3 can read a stale accumulator and the row max varies run to run
    asm volatile("s_nop 15\n\ts_nop 2" : "+v"(s0), "+v"(s1));
    if constexpr (!FULL) {
      const int kq = myq - k0, kl = lo - k0;  // visible iff kl <= key-k0 <= kq
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j0 = acc_row(r, lane), j1 = j0 + 32;
        s0[r] = (j0 > kq || j0 < kl) ? -INFINITY : s0[r];
        s1[r] = (j1 > kq || j1 < kl) ? -INFINITY : s1[r];
      }
    }
    float ma = max3(s0[0], s0[1], s0[2]), mb = max3(s1[0], s1[1], s1[2]);
#pragma unroll
    for (int r = 3; r < 15; r += 2) {
      ma = max3(ma, s0[r], s0[r + 1]);
      mb = max3(mb, s1[r], s1[r + 1]);
    }
    const float mx = max_xhalf(max3(max3(ma, mb, s0[15]), s1[15], s1[15]));
    // NaN-safe: (-inf) - (-inf) compares false (a fully masked tile never grows m)
    const bool grow = (mx - m) * c > 8.0f;
    if (__any(grow)) {
      const float mn = grow ? mx : m;
      const float alpha = grow ? __builtin_amdgcn_exp2f((m - mn) * c) : 1.0f;
      lsum *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        o0[r] *= alpha;
        o1[r] *= alpha;
      }
      m = mn;
    }
    const float mc = (m == -INFINITY ? 0.f : m) * c;
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] = __builtin_amdgcn_exp2f(fmaf(s0[r], c, -mc));
      s1[r] = __builtin_amdgcn_exp2f(fmaf(s1[r], c, -mc));
      ps += s0[r] + s1[r];
    }
    lsum += ps;
    if constexpr (DROP == 1) {
      // colpair of (kb, r) = k0/2 + 2*hl + (r&3)/2 + 4*(r>>2) + 16*kb; the 1/(1-p) scale is
      // applied once to O at the end
      const uint32_t hb = hrow + ((uint32_t)(k0 >> 1) + 2u * (uint32_t)hl) * CG_COLK;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const uint32_t off = (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2));
        const uint32_t h0 = cg_pair_mix(hb + off * CG_COLK);
        const uint32_t h1 = cg_pair_mix(hb + (off + 16u) * CG_COLK);
        s0[r] = (h0 & 0xFFFFu) >= thr ? s0[r] : 0.f;
        s0[r + 1] = (h0 >> 16) >= thr ? s0[r + 1] : 0.f;
        s1[r] = (h1 & 0xFFFFu) >= thr ? s1[r] : 0.f;
        s1[r + 1] = (h1 >> 16) >= thr ? s1[r + 1] : 0.f;
      }
    }
    v8bf p00, p01, p10, p11;
    if constexpr (DROP == 2) {
      // keys k0 + acc_row(r) (s0) and k0 + 32 + acc_row(r) (s1): words wc.x / wc.y
      const uint32_t w0 = wc.x >> (2 * hl), w1 = wc.y >> (2 * hl);
      p00 = pack_b_keep(s0, 0, w0); p01 = pack_b_keep(s0, 1, w0);
      p10 = pack_b_keep(s1, 0, w1); p11 = pack_b_keep(s1, 1, w1);
    } else {
      p00 = pack_b(s0, 0); p01 = pack_b(s0, 1); p10 = pack_b(s1, 0); p11 = pack_b(s1, 1);
    }
    o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Vi, 0, 0, 0, lane), p00, o0, 0, 0, 0);
    o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Vi, 0, 1, 0, lane), p01, o0, 0, 0, 0);
    o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Vi, 32, 0, 0, lane), p10, o0, 0, 0, 0);
    o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Vi, 32, 1, 0, lane), p11, o0, 0, 0, 0);
    if constexpr (hd > 32) {
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Vi, 0, 0, 1, lane), p00, o1, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Vi, 0, 1, 1, lane), p01, o1, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Vi, 32, 0, 1, lane), p10, o1, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Vi, 32, 1, 1, lane), p11, o1, 0, 0, 0);
    }
  };
  // the keep words are fetched one tile ahead (tiles above the wave's diagonal read words that
  // were never written; their pairs are causally masked)
  uint2 wn = make_uint2(0, 0);
  if constexpr (DROP == 2) wn = *(const uint2*)(qm + 2 * t0);
  auto step = [&](auto cur_c, int t) __attribute__((always_inline)) {
    constexpr int CUR = decltype(cur_c)::value;
    const char* Ki = smem + CUR * 2 * IMG;
    const char* Vi = Ki + IMG;
    const bool more = t < t1;
    const uint2 wc = wn;
    if (more) {  // the other buffer was last read before the previous barrier
      tile_dma(lds0 + (CUR ^ 1) * 2 * IMG, kv, (t + 1) * tstride + kcol, wave_u);
      tile_dma(lds0 + (CUR ^ 1) * 2 * IMG + IMG, kv, (t + 1) * tstride + vcol, wave_u);
      if constexpr (DROP == 2) wn = *(const uint2*)(qm + 2 * (t + 1));
    }
    const int k0 = t * KT;
    if (k0 <= w_qmax && k0 + KT - 1 >= w_lo_min) {
      if ((k0 + KT - 1 <= q0w) && (k0 >= w_lo_max)) body(Ki, Vi, k0, wc, std::true_type{});
      else body(Ki, Vi, k0, wc, std::false_type{});
    }
    dma_drain();
    __syncthreads();
  };
  for (int t = t0; t <= t1; t += 2) {
    step(std::integral_constant<int, 0>{}, t);
    if (t + 1 <= t1) step(std::integral_constant<int, 1>{}, t + 1);
  }
  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  if (qok) {
    const float inv = (DROP ? dscale : 1.0f) / ltot;
    bf16_t* yr = y + (rowbase + myq) * ldy + (long long)hh * hd;
#pragma unroll
    for (int r = 0; r < 16; r += 4) {
      const int d0 = acc_row(r, lane);
      if (d0 < hd) {
        uint2 w;
        w.x = (uint32_t)f2bf(o0[r] * inv) | ((uint32_t)f2bf(o0[r + 1] * inv) << 16);
        w.y = (uint32_t)f2bf(o0[r + 2] * inv) | ((uint32_t)f2bf(o0[r + 3] * inv) << 16);
        *(uint2*)(yr + d0) = w;
      }
      if (d0 + 32 < hd) {
        uint2 w;
        w.x = (uint32_t)f2bf(o1[r] * inv) | ((uint32_t)f2bf(o1[r + 1] * inv) << 16);
        w.y = (uint32_t)f2bf(o1[r + 2] * inv) | ((uint32_t)f2bf(o1[r + 3] * inv) << 16);
        *(uint2*)(yr + d0 + 32) = w;
      }
    }
    if (hl == 0) lse[((long long)b * H + hh) * T + myq] = m * scale + __logf(ltot);
  }
}

// ============================================================================
// backward dQ: WG = 4 waves x 32 queries; key tiles of 64 (K, V images)
// dS^T = P^T o (dP^T - delta),  dQ^T[d][q] += K^T[d][key] dS^T[key][q]
// ============================================================================
template <int DROP, int HD>
__global__ __launch_bounds__(256, ATTN_DQ_WPS) void attn_bwd_dq_mfma(const bf16_t* __restrict__ qkv, long long ld,
                                                           const int32_t* __restrict__ seg,
                                                           const bf16_t* __restrict__ dy, long long lddy,
                                                           const bf16_t* __restrict__ yo, long long ldy,
                                                           const float* __restrict__ lse,
                                                           float* __restrict__ delta, bf16_t* __restrict__ dqkv,
                                                           long long lddq, int T, int H, int KV, int hd_rt, int window,
                                                           uint32_t seed, uint32_t thr, float dscale, float scale,
                                                           const uint32_t* __restrict__ qmask, int wpr,
                                                           float* __restrict__ bpart, long long ldp) {
  using namespace fa;
  constexpr int hd = HD;
  (void)hd_rt;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int bh = blockIdx.x, b = bh / H, hh = bh % H, kvh = hh / (H / KV);
  const int qtile = gridDim.y - 1 - blockIdx.y;
  const int q0 = qtile * 128, q0w = q0 + wave * 32;
  const int myq = q0w + (lane & 31);
  const bool qok = myq < T;
  const long long rowbase = (long long)b * T;
  const bf16_t* qrow = qkv + (rowbase + (qok ? myq : 0)) * ld + (long long)hh * hd;
  const bf16_t* dorow = dy + (rowbase + (qok ? myq : 0)) * lddy + (long long)hh * hd;
  const bf16_t* orow = yo + (rowbase + (qok ? myq : 0)) * ldy + (long long)hh * hd;
  v8bf qf[4], df[4];
  float dpart = 0.f;  // delta = rowsum(dO o O), the FA2 preprocessing, fused here
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = frag_global(qrow, qok, ks, hd, lane);
    df[ks] = frag_global(dorow, qok, ks, hd, lane);
    const v8bf of = frag_global(orow, qok, ks, hd, lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) dpart += (float)df[ks][j] * (float)of[j];
  }
  const long long bhq = ((long long)b * H + hh) * T + (qok ? myq : 0);
  const float c = scale * 1.4426950408889634f;
  const float lse2 = qok ? lse[bhq] * 1.4426950408889634f : 0.f;
  const float dl = dpart + __shfl_xor(dpart, 32, 64);
  if (qok && lane < 32) delta[bhq] = dl;
  const int lo = qok ? lo_of(seg, rowbase, myq, T, window) : 0x7fffffff;
  const int kmin = lo_of(seg, rowbase, q0, T, window);
  const int kmax = min(T - 1, q0 + 127);
  const int w_lo_min = lo_of(seg, rowbase, q0w, T, window);
  const int w_lo_max = lo_of(seg, rowbase, min(q0w + 31, T - 1), T, window);
  const int w_qmax = min(T - 1, q0w + 31);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const TileDma kv = tile_dma_src(qkv + rowbase * ld, ld, T, hd, wave_u, lane);
  const uint32_t kcol = (uint32_t)((H + kvh) * hd * 2), vcol = (uint32_t)((H + KV + kvh) * hd * 2);
  const uint32_t tstride = (uint32_t)(KT * ld * 2);
  const uint32_t drow = (uint32_t)bhq;
  const uint32_t hrow = DROP == 1 ? cg_row_hash(seed, drow) : 0u;
  const uint32_t* qm = DROP == 2 ? qmask + (long long)bhq * wpr : nullptr;
  constexpr int nks = (hd + 15) >> 4;
  v16f a0 = zero16(), a1 = zero16();
  const int t0 = kmin / KT, t1 = kmax / KT;
  tile_dma(lds0, kv, t0 * tstride + kcol, wave_u);
  tile_dma(lds0 + IMG, kv, t0 * tstride + vcol, wave_u);
  dma_drain();
  __syncthreads();
  uint2 wn = make_uint2(0, 0);
  if constexpr (DROP == 2) wn = *(const uint2*)(qm + 2 * t0);
  for (int t = t0; t <= t1; ++t) {
    const int cur = (t - t0) & 1;
    const char* Ki = smem + cur * 2 * IMG;
    const char* Vi = Ki + IMG;
    const bool more = t < t1;
    const uint2 wc = wn;
    if (more) {  // the other buffer was last read before the previous barrier
      tile_dma(lds0 + (cur ^ 1) * 2 * IMG, kv, (t + 1) * tstride + kcol, wave_u);
      tile_dma(lds0 + (cur ^ 1) * 2 * IMG + IMG, kv, (t + 1) * tstride + vcol, wave_u);
      if constexpr (DROP == 2) wn = *(const uint2*)(qm + 2 * (t + 1));
    }
    const int k0 = t * KT;
    // full: every (query, key) of the wave's tile visible.  Otherwise the invisible scores are
    // set to -inf before the exponent; the branch touches only s, so the dQ accumulators keep
    // their registers across it (a branch around the whole body made hipcc copy them back at
    // the join)
    auto body = [&](bool full) __attribute__((always_inline)) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        v16f s = zero16(), dp = zero16();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          if (ks < nks) {
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row(Ki, kb * 32, ks, lane), qf[ks], s, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row(Vi, kb * 32, ks, lane), df[ks], dp, 0, 0, 0);
          }
        }
        const int kq = myq - k0 - kb * 32, kl = lo - k0 - kb * 32;
        if (!full) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int j = acc_row(r, lane);
            s[r] = ((j > kq) | (j < kl)) ? -INFINITY : s[r];
          }
        }
        const uint32_t hb = hrow + ((uint32_t)((k0 + kb * 32) >> 1) + 2u * (uint32_t)(lane >> 5)) * CG_COLK;
        const uint32_t wb = (kb ? wc.y : wc.x) >> (2 * (lane >> 5));
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const float p0 = __builtin_amdgcn_exp2f(fmaf(s[r], c, -lse2));
          const float p1 = __builtin_amdgcn_exp2f(fmaf(s[r + 1], c, -lse2));
          float d0 = dp[r], d1 = dp[r + 1];
          if constexpr (DROP == 1) {
            const uint32_t off = (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2));
            const uint32_t hsh = cg_pair_mix(hb + off * CG_COLK);
            d0 = (hsh & 0xFFFFu) >= thr ? d0 * dscale : 0.f;
            d1 = (hsh >> 16) >= thr ? d1 * dscale : 0.f;
            s[r] = p0 * (d0 - dl);
            s[r + 1] = p1 * (d1 - dl);
          } else if constexpr (DROP == 2) {
            s[r] = p0 * fmaf(keep_f(d0, wb, kbit(r)), dscale, -dl);
            s[r + 1] = p1 * fmaf(keep_f(d1, wb, kbit(r + 1)), dscale, -dl);
          } else {
            s[r] = p0 * (d0 - dl);
            s[r + 1] = p1 * (d1 - dl);
          }
        }
        const v8bf b0 = pack_b(s, 0), b1 = pack_b(s, 1);
        a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Ki, kb * 32, 0, 0, lane), b0, a0, 0, 0, 0);
        a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Ki, kb * 32, 1, 0, lane), b1, a0, 0, 0, 0);
        if constexpr (hd > 32) {
          a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Ki, kb * 32, 0, 1, lane), b0, a1, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Ki, kb * 32, 1, 1, lane), b1, a1, 0, 0, 0);
        }
      }
    };
    if (k0 <= w_qmax && k0 + KT - 1 >= w_lo_min) body((k0 + KT - 1 <= q0w) && (k0 >= w_lo_max));
    dma_drain();
    __syncthreads();
  }
  if (qok) {
    bf16_t* dr = dqkv + (rowbase + myq) * lddq + (long long)hh * hd;
#pragma unroll
    for (int r = 0; r < 16; r += 4) {
      const int d0 = acc_row(r, lane);
      if (d0 < hd) {
        uint2 w;
        w.x = (uint32_t)f2bf(a0[r] * scale) | ((uint32_t)f2bf(a0[r + 1] * scale) << 16);
        w.y = (uint32_t)f2bf(a0[r + 2] * scale) | ((uint32_t)f2bf(a0[r + 3] * scale) << 16);
        *(uint2*)(dr + d0) = w;
      }
      if (d0 + 32 < hd) {
        uint2 w;
        w.x = (uint32_t)f2bf(a1[r] * scale) | ((uint32_t)f2bf(a1[r + 1] * scale) << 16);
        w.y = (uint32_t)f2bf(a1[r + 2] * scale) | ((uint32_t)f2bf(a1[r + 3] * scale) << 16);
        *(uint2*)(dr + d0 + 32) = w;
      }
    }
  }
  if (bpart) {  // q-bias gradient partial: column sums of this workgroup's dQ rows (fp32)
    float* red = (float*)smem;  // the ring is idle after the last barrier
    colsum_acc(a0, a1, scale, qok, red, 64, 0, wave, lane);
    __syncthreads();
    if (tid < hd)
      bpart[((long long)b * gridDim.y + qtile) * ldp + (long long)hh * hd + tid] =
          (red[tid] + red[64 + tid]) + (red[128 + tid] + red[192 + tid]);
  }
}

// ============================================================================
// backward dK/dV: WG = 4 waves x 32 keys (128 keys of one (b, kv head)); loops over
// the group's query heads and query tiles of 64 (Q, dO images + lse/delta/lo rows).
//   S = Q K^T, dP = dO V^T (query rows in registers, key on the lane)
//   dV^T[d][key] += dO^T[d][q] Pd[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
// ============================================================================
template <int DROP, int HD>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_mfma(const bf16_t* __restrict__ qkv, long long ld,
                                                             const int32_t* __restrict__ seg,
                                                             const bf16_t* __restrict__ dy, long long lddy,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ delta,
                                                             bf16_t* __restrict__ dqkv, long long lddq, int T, int H,
                                                             int KV, int hd_rt, int window, uint32_t seed, uint32_t thr,
                                                             float dscale, float scale,
                                                             const uint32_t* __restrict__ qmask, int wpr,
                                                             float* __restrict__ bpart, long long ldp) {
  using namespace fa;
  constexpr int hd = HD;
  (void)hd_rt;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // per buffer: Q image | dO image | lse2[64] | delta[64] | lo[64] | rowhash[64]
  //             (+ DROP 2: the keep words of the tile's 64 queries x 128 keys, [key word][query])
  constexpr int BUF = 2 * IMG + 4 * 64 * 4 + (DROP == 2 ? 4 * 64 * 4 : 0);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int bk = blockIdx.x, b = bk / KV, kvh = bk % KV;
  const int rep = H / KV;
  const int ktile = blockIdx.y;  // early keys see the most queries: dispatched first
  const int kt0 = ktile * 128, kw0 = kt0 + wave * 32;
  const int mykey = kw0 + (lane & 31);
  const bool kok = mykey < T;
  const long long rowbase = (long long)b * T;
  const long long koff = (long long)H * hd + (long long)kvh * hd;
  const long long voff = (long long)(H + KV) * hd + (long long)kvh * hd;
  const bf16_t* krow = qkv + (rowbase + (kok ? mykey : 0)) * ld + koff;
  const bf16_t* vrow = qkv + (rowbase + (kok ? mykey : 0)) * ld + voff;
  v8bf kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = frag_global(krow, kok, ks, hd, lane);
    vf[ks] = frag_global(vrow, kok, ks, hd, lane);
  }
  const float c = scale * 1.4426950408889634f;
  constexpr int nks = (hd + 15) >> 4;
  const uint32_t kcol = ((uint32_t)mykey >> 1) * CG_COLK;
  // the lane's key bit in a pair-split word: key 2c -> bit c, key 2c+1 -> bit 16 + c
  const uint32_t kpos = (uint32_t)(((mykey & 31) >> 1) + 16 * (mykey & 1));
  v16f dk0 = zero16(), dk1 = zero16(), dv0 = zero16(), dv1 = zero16();
  // query tile range: causal start; stop once every query's segment/window starts after the tile
  const int qt_begin = kt0 / KT;
  int qend = T;
  if (window > 0) qend = min(T, kt0 + 127 + window);
  const int qt_end = (qend - 1) / KT;  // inclusive
  const int nqt = qt_end - qt_begin + 1;
  const int total = nqt * rep;
  // the per-query rows (lse, delta, segment start) are prefetched with the tiles: loading
  // them at store time would expose a global-memory round trip every iteration
  float pl = 0.f, pdl = 0.f;
  int plo = 0x7fffffff;
  // keep words of (query head, query tile): thread tid fetches query tid&63's word for keys
  // kt0 + 32(tid>>6) .. +31 with the tiles
  uint32_t wn = 0;
  const int mw_idx = kt0 / 32 + (tid >> 6);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const TileDma qsrc = tile_dma_src(qkv + rowbase * ld, ld, T, hd, wave_u, lane);
  const TileDma dsrc = tile_dma_src(dy + rowbase * lddy, lddy, T, hd, wave_u, lane);
  const uint32_t qstride = (uint32_t)(KT * ld * 2), dstride = (uint32_t)(KT * lddy * 2);
  // iteration cursor: (query head, query tile), advanced without divisions
  struct Cur { int h2, qt; };
  auto next_of = [&](Cur c) { return c.qt < qt_end ? Cur{c.h2, c.qt + 1} : Cur{c.h2 + 1, qt_begin}; };
  // the images go straight to LDS buffer `nb`; the per-query rows through registers
  auto stage_load = [&](Cur cu, int nb) {
    const int h2 = cu.h2, qt = cu.qt;
    tile_dma(lds0 + nb * BUF, qsrc, qt * qstride + (uint32_t)(h2 * hd * 2), wave_u);
    tile_dma(lds0 + nb * BUF + IMG, dsrc, qt * dstride + (uint32_t)(h2 * hd * 2), wave_u);
    if constexpr (DROP == 2) {
      const int q = qt * KT + (tid & 63);
      wn = (q < T && mw_idx < wpr) ? qmask[(((long long)b * H + h2) * T + q) * wpr + mw_idx] : 0u;
    }
    if (tid < 64) {
      const int q = qt * KT + tid;
      const long long bhq = ((long long)b * H + h2) * T + (q < T ? q : 0);
      pl = q < T ? lse[bhq] : 0.f;
      pdl = q < T ? delta[bhq] : 0.f;
      plo = q < T ? lo_of(seg, rowbase, q, T, window) : 0x7fffffff;
    }
  };
  auto stage_store = [&](Cur cu, char* buf) {
    if (tid < 64) {
      const int h2 = cu.h2, qt = cu.qt;
      const int q = qt * KT + tid;
      float* fl = (float*)(buf + 2 * IMG);
      int* il = (int*)(buf + 2 * IMG + 2 * 64 * 4);
      fl[tid] = pl * 1.4426950408889634f;
      fl[64 + tid] = pdl;
      il[tid] = plo;
      il[64 + tid] = DROP == 1 ? (int)cg_row_hash(seed, (uint32_t)(((long long)b * H + h2) * T + q)) : 0;
    }
    if constexpr (DROP == 2) ((uint32_t*)(buf + 2 * IMG + 4 * 64 * 4))[tid] = wn;
  };
  Cur cur{kvh * rep, qt_begin};
  if (total > 0) {
    stage_load(cur, 0);
    stage_store(cur, smem);
    dma_drain();
  }
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    const char* buf = smem + (it & 1) * BUF;
    const char* Qi = buf;
    const char* Di = buf + IMG;
    const float* lse2s = (const float*)(buf + 2 * IMG);
    const float* dls = lse2s + 64;
    const int* los = (const int*)(buf + 2 * IMG + 2 * 64 * 4);
    const uint32_t* hrs = (const uint32_t*)(buf + 2 * IMG + 3 * 64 * 4);
    const bool more = it + 1 < total;
    // this wave's key word of the tile's keep bits, [query]
    const uint32_t* mws = (const uint32_t*)(buf + 2 * IMG + 4 * 64 * 4) + wave * 64;
    const Cur nx = next_of(cur);
    if (more) stage_load(nx, (it & 1) ^ 1);  // that buffer was last read before the previous barrier
    const int q0 = cur.qt * KT;
    // wave activity: some query q in [q0, q0+63] sees some key in [kw0, kw0+31]
    const int qlast = min(T - 1, q0 + KT - 1);
    const bool active = (qlast >= kw0) && (los[0] <= kw0 + 31);
    // full: every (query, key) of the wave's tile visible.  Otherwise the invisible scores are
    // set to -inf before the exponent (the branch touches only s: the dK/dV accumulators keep
    // their registers across it)
    auto body = [&](bool full) __attribute__((always_inline)) {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        v16f s = zero16(), dp = zero16();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          if (ks < nks) {
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row(Qi, qb * 32, ks, lane), kf[ks], s, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row(Di, qb * 32, ks, lane), vf[ks], dp, 0, 0, 0);
          }
        }
        if (!full) {
#pragma unroll
          for (int rg = 0; rg < 16; rg += 4) {
            const int qi = qb * 32 + acc_row(rg, lane);
            const int4 lo4 = *(const int4*)(los + qi);
            const int lov[4] = {lo4.x, lo4.y, lo4.z, lo4.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int q = q0 + qi + u;
              s[rg + u] = ((mykey > q) | (mykey < lov[u]) | (q >= T)) ? -INFINITY : s[rg + u];
            }
          }
        }
        v16f pd;
#pragma unroll
        for (int rg = 0; rg < 16; rg += 4) {
          const int qi = qb * 32 + acc_row(rg, lane);  // 4 consecutive queries qi..qi+3
          const float4 l4 = *(const float4*)(lse2s + qi);
          const float4 d4 = *(const float4*)(dls + qi);
          const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
          const float dv4[4] = {d4.x, d4.y, d4.z, d4.w};
          uint4 hr4 = make_uint4(0, 0, 0, 0);
          if constexpr (DROP == 1) hr4 = *(const uint4*)(hrs + qi);
          uint4 mw4 = make_uint4(0, 0, 0, 0);
          if constexpr (DROP == 2) mw4 = *(const uint4*)(mws + qi);
          const uint32_t mwv[4] = {mw4.x, mw4.y, mw4.z, mw4.w};
          const uint32_t hrv[4] = {hr4.x, hr4.y, hr4.z, hr4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = rg + u;
            const float p = __builtin_amdgcn_exp2f(fmaf(s[r], c, -lv[u]));
            float d = dp[r];
            float pdr = p;  // the 1/(1-p) of P~ is applied to dV once at the end
            if constexpr (DROP == 1) {
              const uint32_t hsh = cg_pair_mix(hrv[u] + kcol);
              const uint32_t bits = (mykey & 1) ? (hsh >> 16) : (hsh & 0xFFFFu);
              const bool keep = bits >= thr;
              d = keep ? d * dscale : 0.f;
              pdr = keep ? p : 0.f;
              s[r] = p * (d - dv4[u]);
            } else if constexpr (DROP == 2) {
              const int m = keep_mask(mwv[u], kpos);
              pdr = __int_as_float(__float_as_int(p) & m);
              s[r] = p * fmaf(__int_as_float(__float_as_int(d) & m), dscale, -dv4[u]);
            } else {
              s[r] = p * (d - dv4[u]);
            }
            pd[r] = pdr;
          }
        }
        const v8bf pb0 = pack_b(pd, 0), pb1 = pack_b(pd, 1);
        const v8bf sb0 = pack_b(s, 0), sb1 = pack_b(s, 1);
        dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Di, qb * 32, 0, 0, lane), pb0, dv0, 0, 0, 0);
        dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Di, qb * 32, 1, 0, lane), pb1, dv0, 0, 0, 0);
        dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Qi, qb * 32, 0, 0, lane), sb0, dk0, 0, 0, 0);
        dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Qi, qb * 32, 1, 0, lane), sb1, dk0, 0, 0, 0);
        if constexpr (hd > 32) {
          dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Di, qb * 32, 0, 1, lane), pb0, dv1, 0, 0, 0);
          dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Di, qb * 32, 1, 1, lane), pb1, dv1, 0, 0, 0);
          dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Qi, qb * 32, 0, 1, lane), sb0, dk1, 0, 0, 0);
          dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr(Qi, qb * 32, 1, 1, lane), sb1, dk1, 0, 0, 0);
        }
      }
    };
    if (active) body((q0 >= kw0 + 31) && (q0 + KT - 1 < T) && (los[qlast - q0] <= kw0));
    if (more) stage_store(nx, smem + ((it & 1) ^ 1) * BUF);
    cur = nx;
    dma_drain();
    __syncthreads();
  }
  if (kok) {
    bf16_t* kr = dqkv + (rowbase + mykey) * lddq + koff;
    bf16_t* vr = dqkv + (rowbase + mykey) * lddq + voff;
    const float vs = DROP ? dscale : 1.0f;
#pragma unroll
    for (int r = 0; r < 16; r += 4) {
      const int d0 = acc_row(r, lane);
      if (d0 < hd) {
        uint2 w;
        w.x = (uint32_t)f2bf(dk0[r] * scale) | ((uint32_t)f2bf(dk0[r + 1] * scale) << 16);
        w.y = (uint32_t)f2bf(dk0[r + 2] * scale) | ((uint32_t)f2bf(dk0[r + 3] * scale) << 16);
        *(uint2*)(kr + d0) = w;
        w.x = (uint32_t)f2bf(dv0[r] * vs) | ((uint32_t)f2bf(dv0[r + 1] * vs) << 16);
        w.y = (uint32_t)f2bf(dv0[r + 2] * vs) | ((uint32_t)f2bf(dv0[r + 3] * vs) << 16);
        *(uint2*)(vr + d0) = w;
      }
      if (d0 + 32 < hd) {
        uint2 w;
        w.x = (uint32_t)f2bf(dk1[r] * scale) | ((uint32_t)f2bf(dk1[r + 1] * scale) << 16);
        w.y = (uint32_t)f2bf(dk1[r + 2] * scale) | ((uint32_t)f2bf(dk1[r + 3] * scale) << 16);
        *(uint2*)(kr + d0 + 32) = w;
        w.x = (uint32_t)f2bf(dv1[r] * vs) | ((uint32_t)f2bf(dv1[r + 1] * vs) << 16);
        w.y = (uint32_t)f2bf(dv1[r + 2] * vs) | ((uint32_t)f2bf(dv1[r + 3] * vs) << 16);
        *(uint2*)(vr + d0 + 32) = w;
      }
    }
  }
  if (bpart) {  // k / v bias gradient partials: column sums of this workgroup's dK, dV rows
    const float vs = DROP ? dscale : 1.0f;
    float* red = (float*)smem;  // [wave][dK 64 | dV 64]; the ring is idle after the last barrier
    colsum_acc(dk0, dk1, scale, kok, red, 128, 0, wave, lane);
    colsum_acc(dv0, dv1, vs, kok, red, 128, 64, wave, lane);
    __syncthreads();
    if (tid < 128 && (tid & 63) < hd) {
      const float v = (red[tid] + red[128 + tid]) + (red[256 + tid] + red[384 + tid]);
      bpart[((long long)b * gridDim.y + ktile) * ldp + (tid < 64 ? koff + tid : voff + tid - 64)] = v;
    }
  }
}

// ----------------------------------------------------------------------------
static inline bool attn_mfma_supported(int hd, long long ld_in, long long ld_out) {
  if (getenv("CG_ATTN_VEC")) return false;  // diagnostic: force the vector kernels
  return (hd == 32 || hd == 48 || hd == 64) && (ld_in % 8 == 0) && (ld_out % 8 == 0);
}

// words per (bh, row) of the keep-bit array
static inline int attn_drop_wpr(int T) { return 2 * cg_cdiv(T, 64); }
static inline size_t attn_drop_mask_words(int B, int T, int H) { return (size_t)B * H * T * attn_drop_wpr(T); }

static inline int attn_drop_mask_launch(uint32_t* mask, int B, int T, int H, uint32_t seed, uint32_t thr,
                                        hipStream_t s) {
  const int nb = cg_cdiv(T, 64);
  hipLaunchKernelGGL(attn_drop_mask_kernel, dim3(nb * (nb + 1) / 2, B * H), dim3(64), 0, s, mask, T,
                     attn_drop_wpr(T), seed, thr);
  CG_LAUNCH_CHECK();
  return CG_OK;
}

static inline int attn_fwd_mfma_launch(const bf16_t* qkv, long long ld, const int32_t* seg, bf16_t* y, long long ldy,
                                       float* lse, int B, int T, int H, int KV, int hd, int window, uint32_t seed,
                                       uint32_t thr, float dscale, float scale, const uint32_t* dmask, hipStream_t s) {
  dim3 g(B * H, cg_cdiv(T, 128));
  const size_t sh = 4 * fa::IMG;
  const int wpr = attn_drop_wpr(T);
  // causal-exact products: QK^T and PV over the T(T+1)/2 visible (q, key) pairs
  const double tri = 2.0 * (double)B * H * hd * ((double)T * (T + 1) / 2.0);
  cg_probe_begin(CG_PROBE_ATTN_FWD, s);
#define FWD(D, HDv)                                                                                          \
  hipLaunchKernelGGL((attn_fwd_mfma<D, HDv>), g, dim3(256), sh, s, qkv, ld, seg, y, ldy, lse, T, H, KV, hd, window, \
                     seed, thr, dscale, scale, dmask, wpr)
  if (thr && dmask) {
    if (hd == 64) FWD(2, 64); else if (hd == 48) FWD(2, 48); else FWD(2, 32);
  } else if (thr) {
    if (hd == 64) FWD(1, 64); else if (hd == 48) FWD(1, 48); else FWD(1, 32);
  } else {
    if (hd == 64) FWD(0, 64); else if (hd == 48) FWD(0, 48); else FWD(0, 32);
  }
#undef FWD
  cg_probe_end(CG_PROBE_ATTN_FWD, s, 2.0 * tri);
  CG_LAUNCH_CHECK();
  return CG_OK;
}

static inline int attn_bwd_mfma_launch(const bf16_t* qkv, long long ld, const int32_t* seg, const bf16_t* y,
                                       long long ldy, const bf16_t* dy, long long lddy, const float* lse,
                                       float* delta, bf16_t* dqkv, long long lddq, int B, int T, int H, int KV,
                                       int hd, int window, uint32_t seed, uint32_t thr, float dscale, float scale,
                                       const uint32_t* dmask, float* bpart, long long ldp, hipStream_t s) {
  dim3 gq(B * H, cg_cdiv(T, 128));
  const int wpr = attn_drop_wpr(T);
  const int mode = thr ? (dmask ? 2 : 1) : 0;
  const double tri = 2.0 * (double)B * H * hd * ((double)T * (T + 1) / 2.0);
  cg_probe_begin(CG_PROBE_ATTN_DQ, s);
#define DQ(D, HDv)                                                                                             \
  hipLaunchKernelGGL((attn_bwd_dq_mfma<D, HDv>), gq, dim3(256), 4 * fa::IMG, s, qkv, ld, seg, dy, lddy, y, ldy, lse, \
                     delta, dqkv, lddq, T, H, KV, hd, window, seed, thr, dscale, scale, dmask, wpr, bpart, ldp)
#define DQH(D) if (hd == 64) DQ(D, 64); else if (hd == 48) DQ(D, 48); else DQ(D, 32)
  if (mode == 2) { DQH(2); } else if (mode == 1) { DQH(1); } else { DQH(0); }
#undef DQH
#undef DQ
  cg_probe_end(CG_PROBE_ATTN_DQ, s, 3.0 * tri);  // S, dP recomputed + dQ
  CG_LAUNCH_CHECK();
  dim3 gk(B * KV, cg_cdiv(T, 128));
  const size_t shk = 2 * (2 * fa::IMG + 4 * 64 * 4 + (mode == 2 ? 4 * 64 * 4 : 0));
  cg_probe_begin(CG_PROBE_ATTN_DKDV, s);
#define DKDV(D, HDv)                                                                                            \
  hipLaunchKernelGGL((attn_bwd_dkdv_mfma<D, HDv>), gk, dim3(256), shk, s, qkv, ld, seg, dy, lddy, lse, delta, dqkv,  \
                     lddq, T, H, KV, hd, window, seed, thr, dscale, scale, dmask, wpr, bpart, ldp)
#define DKH(D) if (hd == 64) DKDV(D, 64); else if (hd == 48) DKDV(D, 48); else DKDV(D, 32)
  if (mode == 2) { DKH(2); } else if (mode == 1) { DKH(1); } else { DKH(0); }
#undef DKH
#undef DKDV
  cg_probe_end(CG_PROBE_ATTN_DKDV, s, 4.0 * tri);  // S, dP recomputed + dV, dK
  CG_LAUNCH_CHECK();
  return CG_OK;
}
