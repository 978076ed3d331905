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

// waves per SIMD the forward and dQ kernels are register-limited to (dQ at 3, <= 168 VGPRs, spilled
// once S and dP were seeded by MFMAs; 2 measured 3-5 % faster on the C4 backward)
#define ATTN_FWD_WPS 2
#define ATTN_DQ_WPS 2
// Measured and removed (rounds 2-4): s_setprio around the MFMA chains; the dK/dV
// halves' S / dP issued before either half's softmax (with or without sched_group_barrier
// hints); a full / partial-tile split of the dK/dV body (the dQ body keeps it: 53 -> 50 us).

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
// one dword per lane into LDS at lds + 4 * lane (a 64-entry row of per-query values)
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds), "s"(r)
      : "memory");
}
template <int N>
__device__ __forceinline__ void dma_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

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

// Per-lane image offsets, computed once per kernel: the XOR swizzle of dual_off depends only on
// (row >> 1) & 7, so moving a read by 16 rows (or a multiple) moves it by a constant and every
// frag_row / frag_tr of the tile loops becomes (lane offset + immediate).  Without this hipcc
// re-derives the swizzled address of each of the ~24 reads per tile (one VALU op each).
struct RowOff {
  uint32_t o[4];  // frag_row(img, 0, ks, lane) for ks = 0..3
};
struct TrOff {
  uint32_t o[2][2];  // frag_tr(img, 0, 0, cb, lane): [cb][the lo / hi 8-row half]
};
__device__ __forceinline__ RowOff row_offsets(int lane) {
  RowOff r;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) r.o[ks] = (uint32_t)dual_off(lane & 31, 2 * ks + (lane >> 5));
  return r;
}
__device__ __forceinline__ TrOff tr_offsets(int lane) {
  const int h = lane >> 5, g16 = (lane >> 4) & 1, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  TrOff t;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int ch = ((cb * 32 + g16 * 16) >> 3) + (p >> 1);
    t.o[cb][0] = (uint32_t)(dual_off(4 * h + q, ch) + 8 * (p & 1));
    t.o[cb][1] = (uint32_t)(dual_off(4 * h + q + 8, ch) + 8 * (p & 1));
  }
  return t;
}
// rb: multiple of 16 rows
__device__ __forceinline__ v8bf frag_row_o(const char* img, const RowOff& ro, int rb, int ks) {
  return *(const v8bf*)(img + ro.o[ks] + rb * 128);
}
// frag_tr_o with the two half offsets passed explicitly (a runtime column block: indexing TrOff by
// a runtime cb would put it on the stack)
__device__ __forceinline__ v8bf frag_tr_p(const char* img, uint32_t o0, uint32_t o1, int rb, int s) {
  const int d = (rb + 16 * s) * 128;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_p)(img + o0 + d));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_p)(img + o1 + d));
  const v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(v8bf, r);
}
__device__ __forceinline__ v8bf frag_tr_o(const char* img, const TrOff& to, int rb, int s, int cb) {
  const int d = (rb + 16 * s) * 128;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_p)(img + to.o[cb][0] + d));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_p)(img + to.o[cb][1] + d));
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
// (m & a) | (~m & b) as one gfx950 v_bitop3_b32 (truth table 0xCA; hipcc lowers the plain select
// to and / xor chains here).  A builtin, not inline asm: `a` is an MFMA accumulator, and hipcc pads
// the XDL-write -> VALU-read hazard only before instructions it generates itself
__device__ __forceinline__ float bsel(uint32_t m, float a, float b) {
  return __uint_as_float(__builtin_amdgcn_bitop3_b32(m, __float_as_uint(a), __float_as_uint(b), 0xCA));
}
// all-ones / zero from constant bit `bit` of w
__device__ __forceinline__ int keep_mask_i(uint32_t w, int bit) {
  int m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(w), "i"(bit));
  return m;
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

// keep bits applied to an already packed B fragment (rows 8s..8s+7 of an accumulator)
__device__ __forceinline__ v8bf keep_b(v8bf u, int s, uint32_t w) {
  v4u_a v = __builtin_bit_cast(v4u_a, u);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = keep_pk(v[i], w, kbit(8 * s + 2 * i));
  return __builtin_bit_cast(v8bf, v);
}
// a register fragment times c, rounded to bf16 once (S = (cQ)K^T or Q(cK)^T lands in the exp2
// domain: the backward's p = exp2(S - lse2) then needs no multiply)
__device__ __forceinline__ v8bf scale_frag(v8bf f, float c) {
  v8bf r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)((float)f[j] * c);
  return r;
}
// A operand of all ones: ones x B sums B over its k rows into every row of the result
__device__ __forceinline__ v8bf ones_frag() {
  v8bf o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)1.0f;
  return o;
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

// One 32-row accumulator block x (lane: the query / key l&31; element r: head dim acc_row(r)),
// times sc, stored as bf16 from d = 0 of the block at row pointer rowp, nd valid dims (a multiple
// of 16).  Groups j = r/4 hold dims 8j + 4(l>>5) + 0..3; one v_permlane32_swap per dword of each
// group pair (j, j+1) leaves lanes 0-31 with dims 8j..8j+7 and lanes 32-63 with 8j+8..8j+15, so
// the block takes two 16-byte stores per lane instead of four 8-byte ones (T21).  Every lane
// takes part in the swaps; `ok` only predicates the stores.
__device__ __forceinline__ void store_blk16(bf16_t* rowp, const v16f& x, float sc, bool ok, int nd, int lane) {
  const int hl = lane >> 5;
#pragma unroll
  for (int jp = 0; jp < 4; jp += 2) {
    uint32_t a[2], b[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a[h] = pk2bf(x[4 * jp + 2 * h] * sc, x[4 * jp + 2 * h + 1] * sc);
      b[h] = pk2bf(x[4 * (jp + 1) + 2 * h] * sc, x[4 * (jp + 1) + 2 * h + 1] * sc);
      const auto r = __builtin_amdgcn_permlane32_swap(a[h], b[h], false, false);
      a[h] = r[0];
      b[h] = r[1];
    }
    const int d = 8 * jp + 8 * hl;
    if (ok && 8 * jp + 16 <= nd) *(uint4*)(rowp + d) = make_uint4(a[0], a[1], b[0], b[1]);
  }
}

// Inverse rotate-half RoPE (model_tiny_gpt.py:9-45 applied after the q / k projections; its
// gradient) on one row held in the two 32-dim accumulator blocks x0, x1 (element r of block b:
// dim 32 b + acc_row(r)), for position `cs` / `sn` rows of the [T][hd/2] tables:
//   dx_i = cos_i g_i + sin_i g_{i+h},  dx_{i+h} = cos_i g_{i+h} - sin_i g_i   (i < h = hd/2).
// h is a multiple of 8, so a dim and its partner sit in the same lane (acc_row keeps 4 (l >> 5)).
template <int HD>
__device__ __forceinline__ void rope_inv_blocks(v16f& x0, v16f& x1, const float* cs, const float* sn, int hl) {
  constexpr int h = HD / 2;
  static_assert(h % 8 == 0 && h <= 32, "rope: head dim 16, 32, 48 or 64");
#pragma unroll
  for (int j = 0; j < h / 8; ++j) {
    const float4 c4 = *(const float4*)(cs + 8 * j + 4 * hl);
    const float4 s4 = *(const float4*)(sn + 8 * j + 4 * hl);
    const float cc[4] = {c4.x, c4.y, c4.z, c4.w}, ss[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int r = t | (j << 2);                  // dim 8 j + t (+ 4 hl) of block 0
      const int dp = 8 * j + t + h;                // its partner
      const int rp = (dp & 3) | (((dp & 31) >> 3) << 2);
      const float g = x0[r];
      const float gp = dp < 32 ? x0[rp] : x1[rp];
      x0[r] = fmaf(cc[t], g, ss[t] * gp);
      const float np = fmaf(cc[t], gp, -ss[t] * g);
      if (dp < 32) x0[rp] = np;
      else x1[rp] = np;
    }
  }
}

// Column sums over the workgroup's 128 accumulator columns (4 waves x 32 lanes) of the 64 rows
// held in two accumulator blocks x0 (rows 0..31) and x1 (32..63), for the bias-gradient partials:
// the values go through LDS ([wave][row][33 lanes], conflict-free stores and reads), each thread
// sums one (wave, row) run of 32, and threads 0..63 add the 4 waves' sums -- fixed order, no
// cross-lane shuffle chains.  `red` needs COLSUM_LDS bytes; ends with a barrier (red reusable).
constexpr int COLSUM_LDS = (4 * 64 * 33 + 4 * 64) * 4;
__device__ __forceinline__ float colsum_wg(const v16f& x0, const v16f& x1, float s, bool ok, float* red, int wave,
                                           int lane, int tid) {
  float* t = red + wave * 64 * 33 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    t[acc_row(r, lane) * 33] = ok ? x0[r] * s : 0.f;
    t[(32 + acc_row(r, lane)) * 33] = ok ? x1[r] * s : 0.f;
  }
  __syncthreads();
  const float* run = red + (tid >> 6) * 64 * 33 + (tid & 63) * 33;
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int k = 0; k < 32; k += 2) {
    a += run[k];
    b += run[k + 1];
  }
  float* part = red + 4 * 64 * 33;
  part[tid] = a + b;
  __syncthreads();
  const float v = tid < 64 ? (part[tid] + part[64 + tid]) + (part[128 + tid] + part[192 + tid]) : 0.f;
  __syncthreads();
  return v;  // threads 0..63: the column sum of row tid
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
//   qmask[((bh*nt + t)*T + q)*2 + w]: keys 64t + 32w .. +31 of query q (nt = ceil(T/64) key tiles;
//   tile-major, so the 32 queries of a wave read / write 256 contiguous bytes per tile)
// in "pair-split" order (bit c = key 2c, bit 16 + c = key 2c + 1: fa::kbit), which lets the
// forward apply two bits to a packed bf16 pair at once.  wpr = 2*ceil(T/64) (every 64-key tile
// has both of its words in bounds).  One wave per 64x64 block of the causal lower triangle,
// lane = query; per key pair one hash, two compares, two shift-ins (10 VALU ops).  Words of
// blocks above the diagonal are never written and never consumed (those pairs are causally
// masked before the bit test).
// ============================================================================
__global__ __launch_bounds__(256) void attn_drop_mask_kernel(uint32_t* __restrict__ qmask, int T, int wpr,
                                                             uint32_t seed, uint32_t thr, int nbt) {
  // 4 waves per workgroup, one 64x64 block each (one-wave workgroups were dispatch-bound)
  const int i = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (i >= nbt) return;
  cg_drop_mask_block(qmask, T, wpr, seed, thr, i, (long long)blockIdx.y, (int)(threadIdx.x & 63));
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
// tile-major words, 3 keep bits hashed in the kernel AND written in those words for the
// backward (what attn_drop_mask_kernel would write for every (query, key) pair a query sees)
template <int DROP, int HD>
__global__ __launch_bounds__(256, ATTN_FWD_WPS) void attn_fwd_mfma(const bf16_t* __restrict__ qkv, long long ld,
                                                        const int32_t* __restrict__ seg, bf16_t* __restrict__ y,
                                                        long long ldy, float* __restrict__ lse, int T, int H, int KV,
                                                        int hd_rt, int window, uint32_t seed, uint32_t thr,
                                                        float dscale, float scale,
                                                        uint32_t* __restrict__ qmask, int wpr) {
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
  const uint32_t hrow = (DROP == 1 || DROP == 3) ? cg_row_hash(seed, drow) : 0u;
  // DROP == 3: thr - 1 in both 16-bit halves (1 <= thr <= 65536 on this path)
  const uint32_t thr2m1 = (thr - 1u) | ((thr - 1u) << 16);
  uint32_t* qm = (DROP == 2 || DROP == 3) ? qmask + ((long long)bh * (wpr >> 1) * T + (qok ? myq : 0)) * 2 : nullptr;
  const long long tstep = 2LL * T;  // words between a query's consecutive key tiles
  constexpr int nks = (hd + 15) >> 4;

  float m = -INFINITY;
  // row sums of P accumulate on the MFMA (ones x P, every row of ls = the lane's query sum; only
  // ls[0] is read or rescaled): 4 MFMAs per tile instead of 32 VALU adds
  v16f o0 = zero16(), o1 = zero16(), ls = zero16();
  const RowOff ro = row_offsets(lane);
  const TrOff to = tr_offsets(lane);
  const v8bf ones = ones_frag();
  const int t0 = kmin / KT, t1 = kmax / KT;
  tile_dma(lds0, kv, t0 * tstride + kcol, wave_u);
  tile_dma(lds0 + IMG, kv, t0 * tstride + vcol, wave_u);
  dma_drain();
  __syncthreads();

  // One 32-key half of a tile (keys k0 + 32 kb ..): mask, online-softmax update, exp, row sums
  // and the P.V product of that half.  The tile's two S halves are issued back to back, so the
  // second half's QK^T MFMAs run while the first half is exponentiated, and the first half's
  // PV MFMAs while the second is (MFMA/VALU overlap inside one wave).
  // DROP == 3: the half's keep word in memory order, this lane's pairs only (wout)
  auto half = [&](v16f& sx, const int kb, const char* Vi, int k0, uint32_t wword, uint32_t& wout, auto full_c)
                  __attribute__((always_inline)) {
    constexpr bool FULL = decltype(full_c)::value;
    if constexpr (!FULL) {
      const int kq = myq - k0 - 32 * kb, kl = lo - k0 - 32 * kb;  // visible iff kl <= key <= kq
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = acc_row(r, lane);
        sx[r] = (j > kq || j < kl) ? -INFINITY : sx[r];
      }
    }
    // row max as a depth-3 tree of v_max3 (a linear chain was 8 dependent instructions)
    const float ma = max3(max3(sx[0], sx[1], sx[2]), max3(sx[3], sx[4], sx[5]), max3(sx[6], sx[7], sx[8]));
    const float mb = max3(max3(sx[9], sx[10], sx[11]), max3(sx[12], sx[13], sx[14]), sx[15]);
    const float mx = max_xhalf(max3(ma, mb, mb));
    // NaN-safe: (-inf) - (-inf) compares false (a fully masked half never grows m)
    const bool grow = (mx - m) * c > 8.0f;
    if (__any(grow)) {
      const float mn = grow ? mx : m;
      const float alpha = grow ? __builtin_amdgcn_exp2f((m - mn) * c) : 1.0f;
      ls[0] *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        o0[r] *= alpha;
        o1[r] *= alpha;
      }
      m = mn;
    }
    const float mc = (m == -INFINITY ? 0.f : m) * c;
#pragma unroll
    for (int r = 0; r < 16; ++r) sx[r] = __builtin_amdgcn_exp2f(fmaf(sx[r], c, -mc));
    // the normaliser is the sum of the bf16-rounded P the PV product uses (before the keep bits;
    // the hash path sums before its fp32 keep test)
    if constexpr (DROP == 1) {
      ls = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pack_b(sx, 0), ls, 0, 0, 0);
      ls = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pack_b(sx, 1), ls, 0, 0, 0);
      // colpair of (kb, r) = k0/2 + 2*hl + (r&3)/2 + 4*(r>>2) + 16*kb; the 1/(1-p) scale is
      // applied once to O at the end
      const uint32_t hb = hrow + ((uint32_t)(k0 >> 1) + 2u * (uint32_t)hl + 16u * (uint32_t)kb) * CG_COLK;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const uint32_t off = (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2));
        const uint32_t h = cg_pair_mix(hb + off * CG_COLK);
        sx[r] = (h & 0xFFFFu) >= thr ? sx[r] : 0.f;
        sx[r + 1] = (h >> 16) >= thr ? sx[r + 1] : 0.f;
      }
    }
    v8bf pa = pack_b(sx, 0), pb = pack_b(sx, 1);
    if constexpr (DROP != 1) {
      ls = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pa, ls, 0, 0, 0);
      ls = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pb, ls, 0, 0, 0);
    }
    if constexpr (DROP == 2) {
      // keys k0 + 32 kb + acc_row(r): word wword
      const uint32_t w = wword >> (2 * hl);
      pa = keep_b(pa, 0, w);
      pb = keep_b(pb, 1, w);
    }
    if constexpr (DROP == 3) {
      // the lane's 8 key pairs (pair i = r/2 of r = 0, 2, .., 14: colpair k0/2 + 16 kb + 2 hl +
      // (r&3)/2 + 4 (r>>2)) hashed as attn_drop_mask_kernel does and shifted in, highest first, by
      // 1 or 3 places, so pair i lands directly on its memory ("pair-split") position kbit(2i) =
      // {0,1,4,5,8,9,12,13}[i] (even key) / 16 + kbit(2i) (odd key): no reshuffle afterwards
      const uint32_t hb = hrow + ((uint32_t)(k0 >> 1) + 2u * (uint32_t)hl + 16u * (uint32_t)kb) * CG_COLK;
      v4u_a va = __builtin_bit_cast(v4u_a, pa), vb = __builtin_bit_cast(v4u_a, pb);
      uint32_t wl = 0;
#pragma unroll
      for (int r = 14; r >= 0; r -= 2) {
        const uint32_t h = cg_pair_mix(hb + (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2)) * CG_COLK);
        // both halves at once: keep = 1 where half >= thr (clamped h - (thr - 1) > 0), shifted into
        // wl, and the packed bf16 pair's 16-bit lanes multiplied by keep (x 1 keeps the bits, x 0
        // is +0: one v_pk_mul_lo_u16 where a mask would take a negate and an and)
        uint32_t kp;
        asm("v_pk_sub_u16 %0, %1, %2 clamp\n\tv_pk_min_u16 %0, %0, 1 op_sel_hi:[1,0]"
            : "=&v"(kp) : "v"(h), "s"(thr2m1));
        // the shift applied when pair i goes in moves pairs i+1.. up: 1 for even i, 3 for odd i
        if ((r >> 1) & 1) asm("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(wl) : "v"(kp));
        else asm("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(wl) : "v"(kp));
        // (a compiler-visible packed multiply: the PV MFMA reads this register next, and hipcc
        // inserts the VALU-write -> MFMA-read wait states only after its own instructions)
        typedef unsigned short u16x2_k __attribute__((ext_vector_type(2)));
        const uint32_t pr = r < 8 ? va[r >> 1] : vb[(r - 8) >> 1];
        const uint32_t pm = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2_k, pr) * __builtin_bit_cast(u16x2_k, kp));
        if (r < 8) va[r >> 1] = pm;
        else vb[(r - 8) >> 1] = pm;
      }
      pa = __builtin_bit_cast(v8bf, va);
      pb = __builtin_bit_cast(v8bf, vb);
      wout = wl << (2 * hl);  // (+ 2 hl: the lane half's keys)
    }
    o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr_o(Vi, to, 32 * kb, 0, 0), pa, o0, 0, 0, 0);
    o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr_o(Vi, to, 32 * kb, 1, 0), pb, o0, 0, 0, 0);
    if constexpr (hd > 32) {
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr_o(Vi, to, 32 * kb, 0, 1), pa, o1, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_tr_o(Vi, to, 32 * kb, 1, 1), pb, o1, 0, 0, 0);
    }
  };
  auto body = [&](const char* Ki, const char* Vi, int k0, uint2 wc, auto full_c) __attribute__((always_inline)) {
    v16f s0 = zero16(), s1 = zero16();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      if (ks < nks) s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row_o(Ki, ro, 0, ks), qf[ks], s0, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);  // issue order: the s0 chain, then the s1 chain, then half 0
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      if (ks < nks) s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row_o(Ki, ro, 32, ks), qf[ks], s1, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    // S feeds inline asm (max3): hipcc pads the XDL-result -> VALU-read hazard only before its own
    // instructions, so each half's accumulator passes through a wait of 19 states first (>= the
    // 16-pass rule); without it v_max3 can read a stale accumulator and the row max varies run to run
    asm volatile("s_nop 15\n\ts_nop 2" : "+v"(s0));
    uint32_t w0 = 0, w1 = 0;
    half(s0, 0, Vi, k0, wc.x, w0, full_c);
    asm volatile("s_nop 15\n\ts_nop 2" : "+v"(s1));
    half(s1, 1, Vi, k0, wc.y, w1, full_c);
    if constexpr (DROP == 3) {
      // the two lane halves hold the query's other pairs: or them, lane half 0 stores both words
      const auto x0 = __builtin_amdgcn_permlane32_swap(w0, w0, false, false);
      const auto x1 = __builtin_amdgcn_permlane32_swap(w1, w1, false, false);
      // nontemporal: only the backward reads the bits, after every other layer's forward has
      // streamed through the caches (round 5, same-box A/B: C4 step 14.92 -> 14.85 ms)
      if (qok && hl == 0) {
        typedef uint32_t u32x2_nt __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store((u32x2_nt){w0 | x0[0] | x0[1], w1 | x1[0] | x1[1]}, (u32x2_nt*)(qm + tstep * (k0 / KT)));
      }
    }
  };
  // the keep words are fetched one tile ahead (tiles above the wave's diagonal read words that
  // were never written; their pairs are causally masked)
  uint2 wn = make_uint2(0, 0);
  if constexpr (DROP == 2) wn = *(const uint2*)(qm + tstep * t0);
  auto step = [&](auto cur_c, int t) __attribute__((always_inline)) {
    constexpr int CUR = decltype(cur_c)::value;
    const char* Ki = smem + CUR * 2 * IMG;
    const char* Vi = Ki + IMG;
    const bool more = t < t1;
    const uint2 wc = wn;
    if (more) {  // the other buffer was last read before the previous barrier
      tile_dma(lds0 + (CUR ^ 1) * 2 * IMG, kv, (t + 1) * tstride + kcol, wave_u);
      tile_dma(lds0 + (CUR ^ 1) * 2 * IMG + IMG, kv, (t + 1) * tstride + vcol, wave_u);
      if constexpr (DROP == 2) wn = *(const uint2*)(qm + tstep * (t + 1));
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
  const float ltot = ls[0];
  {
    const float inv = (DROP ? dscale : 1.0f) / ltot;
    bf16_t* yr = y + (rowbase + (qok ? myq : 0)) * ldy + (long long)hh * hd;
    store_blk16(yr, o0, inv, qok, hd < 32 ? hd : 32, lane);
    if (hd > 32) store_blk16(yr + 32, o1, inv, qok, hd - 32, lane);
  }
  if (qok) {
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
                                                           float* __restrict__ delta, float* __restrict__ nlse2,
                                                           bf16_t* __restrict__ dqkv,
                                                           long long lddq, int T, int H, int KV, int hd_rt, int window,
                                                           uint32_t seed, uint32_t thr, float dscale, float scale,
                                                           const uint32_t* __restrict__ qmask, int wpr,
                                                           float* __restrict__ bpart, long long ldp,
                                                           const float* __restrict__ rcos,
                                                           const float* __restrict__ rsin) {
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
  // for the dK/dV kernel's row DMAs, in the form its accumulators start from: nd = -delta/dscale
  // (the dP start) and -lse2 (the S start)
  if (qok && lane < 32) {
    delta[bhq] = -dl * (DROP ? 1.0f / dscale : 1.0f);
    nlse2[bhq] = -lse2;
  }
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
  const uint32_t* qm = DROP == 2 ? qmask + ((long long)bh * (wpr >> 1) * T + (qok ? myq : 0)) * 2 : nullptr;
  const long long tstep = 2LL * T;
  constexpr int nks = (hd + 15) >> 4;
  v16f a0 = zero16(), a1 = zero16();
  const int t0 = kmin / KT, t1 = kmax / KT;
  tile_dma(lds0, kv, t0 * tstride + kcol, wave_u);
  tile_dma(lds0 + IMG, kv, t0 * tstride + vcol, wave_u);
  dma_drain();
  __syncthreads();
  uint2 wn = make_uint2(0, 0);
  if constexpr (DROP == 2) wn = *(const uint2*)(qm + tstep * t0);
  const RowOff ro = row_offsets(lane);
  const TrOff to = tr_offsets(lane);
  // dP starts from nd = -delta/dscale, added by one MFMA (ones x [hi; lo] split-bf16 nd rows:
  // exact to ~2^-16): the accumulator is dP - delta/dscale and dS/dscale = p * (keep ? acc : nd)
  const float nd = -dl * (DROP ? 1.0f / dscale : 1.0f);
  // likewise S starts from -lse2 with Q pre-multiplied by c = scale*log2(e): the accumulator is
  // then the exp2 argument itself
  v8bf ndfrag, lsefrag, onesk;
  {
    const __bf16 hi = (__bf16)nd, lhi = (__bf16)(-lse2);
    const __bf16 lo = (__bf16)(nd - (float)hi), llo = (__bf16)(-lse2 - (float)lhi);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ndfrag[j] = (__bf16)0.f;
      lsefrag[j] = (__bf16)0.f;
      onesk[j] = (__bf16)0.f;
    }
    if (lane < 32) {
      ndfrag[0] = hi; ndfrag[1] = lo;
      lsefrag[0] = lhi; lsefrag[1] = llo;
      onesk[0] = (__bf16)1.f; onesk[1] = (__bf16)1.f;
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) qf[ks] = scale_frag(qf[ks], c);
  auto step = [&](auto cur_c, int t) __attribute__((always_inline)) {
    constexpr int CUR = decltype(cur_c)::value;
    const char* Ki = smem + CUR * 2 * IMG;
    const char* Vi = Ki + IMG;
    const bool more = t < t1;
    const uint2 wc = wn;
    if (more) {  // the other buffer was last read before the previous barrier
      tile_dma(lds0 + (CUR ^ 1) * 2 * IMG, kv, (t + 1) * tstride + kcol, wave_u);
      tile_dma(lds0 + (CUR ^ 1) * 2 * IMG + IMG, kv, (t + 1) * tstride + vcol, wave_u);
      if constexpr (DROP == 2) wn = *(const uint2*)(qm + tstep * (t + 1));
    }
    const int k0 = t * KT;
    // full: every (query, key) of the wave's tile visible.  Otherwise the invisible scores are
    // set to -inf before the exponent; the branch touches only s, so the dQ accumulators keep
    // their registers across it (a branch around the whole body made hipcc copy them back at
    // the join)
    auto body = [&](auto full_c) __attribute__((always_inline)) {
      bool full;
      if constexpr (std::is_same_v<decltype(full_c), bool>) full = full_c;
      else full = decltype(full_c)::value;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        v16f s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(onesk, lsefrag, zero16(), 0, 0, 0);
        v16f dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(onesk, ndfrag, zero16(), 0, 0, 0);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          if (ks < nks) {
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row_o(Ki, ro, kb * 32, ks), qf[ks], s, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row_o(Vi, ro, kb * 32, ks), df[ks], dp, 0, 0, 0);
          }
        }
        // the dQ product's K^T fragments (LDS only) issued before the softmax / keep VALU below
        v8bf kt[4];
#pragma unroll
        for (int i = 0; i < (hd > 32 ? 4 : 2); ++i) kt[i] = frag_tr_o(Ki, to, kb * 32, i & 1, i >> 1);
        __builtin_amdgcn_sched_barrier(0);
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
          const float p0 = __builtin_amdgcn_exp2f(s[r]);
          const float p1 = __builtin_amdgcn_exp2f(s[r + 1]);
          if constexpr (DROP == 1) {
            const uint32_t off = (uint32_t)(((r & 3) >> 1) + 4 * (r >> 2));
            const uint32_t hsh = cg_pair_mix(hb + off * CG_COLK);
            s[r] = p0 * ((hsh & 0xFFFFu) >= thr ? dp[r] : nd);
            s[r + 1] = p1 * ((hsh >> 16) >= thr ? dp[r + 1] : nd);
          } else if constexpr (DROP == 2) {
            const uint32_t m0 = (uint32_t)keep_mask_i(wb, kbit(r)), m1 = (uint32_t)keep_mask_i(wb, kbit(r + 1));
            s[r] = p0 * bsel(m0, dp[r], nd);
            s[r + 1] = p1 * bsel(m1, dp[r + 1], nd);
          } else {
            s[r] = p0 * dp[r];
            s[r + 1] = p1 * dp[r + 1];
          }
        }
        const v8bf b0 = pack_b(s, 0), b1 = pack_b(s, 1);
        a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kt[0], b0, a0, 0, 0, 0);
        a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kt[1], b1, a0, 0, 0, 0);
        if constexpr (hd > 32) {
          a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kt[2], b0, a1, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kt[3], b1, a1, 0, 0, 0);
        }
      }
    };
    if (k0 <= w_qmax && k0 + KT - 1 >= w_lo_min) {
      const bool full = (k0 + KT - 1 <= q0w) && (k0 >= w_lo_max);
      if (full) body(std::true_type{});
      else body(std::false_type{});
    }
    dma_drain();
    __syncthreads();
  };
  for (int t = t0; t <= t1; t += 2) {
    step(std::integral_constant<int, 0>{}, t);
    if (t + 1 <= t1) step(std::integral_constant<int, 1>{}, t + 1);
  }
  // dQ = qscale * (dS/dscale . K); with RoPE the gradient w.r.t. the rotated q, rotated back
  // (the inverse of the forward rotation at the query's position) before the store and the bias
  // partials
  const float qscale = DROP ? scale * dscale : scale;
  if (rcos) {
    const size_t ro = (size_t)(qok ? myq : 0) * (hd / 2);
    rope_inv_blocks<hd>(a0, a1, rcos + ro, rsin + ro, lane >> 5);
  }
  {
    bf16_t* dr = dqkv + (rowbase + (qok ? myq : 0)) * lddq + (long long)hh * hd;
    store_blk16(dr, a0, qscale, qok, hd < 32 ? hd : 32, lane);
    if (hd > 32) store_blk16(dr + 32, a1, qscale, qok, hd - 32, lane);
  }
  if (bpart) {  // q-bias gradient partial: column sums of this workgroup's dQ rows (fp32)
    const float v = colsum_wg(a0, a1, qscale, qok, (float*)smem, wave, lane, tid);  // the ring is idle
    if (tid < hd) bpart[((long long)b * gridDim.y + qtile) * ldp + (long long)hh * hd + tid] = v;
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
                                                             const float* __restrict__ nlse2,
                                                             bf16_t* __restrict__ dqkv, long long lddq, int T, int H,
                                                             int KV, int hd_rt, int window, uint32_t seed, uint32_t thr,
                                                             float dscale, float scale,
                                                             const uint32_t* __restrict__ qmask, int wpr,
                                                             float* __restrict__ bpart, long long ldp,
                                                             const float* __restrict__ rcos,
                                                             const float* __restrict__ rsin) {
  using namespace fa;
  constexpr int hd = HD;
  (void)hd_rt;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // per buffer: Q image | dO image | lse2[64] | delta[64] | lo[64] | rowhash[64]
  //             (+ DROP 2: the keep words of the tile's 64 queries x 128 keys, [key word][query])
  //             | a 64-word slot wave 3's row DMA fills (keeps every wave's DMA count equal)
  constexpr int BUF = 2 * IMG + 4 * 64 * 4 + (DROP == 2 ? 4 * 64 * 4 : 0) + 64 * 4;
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
  const float c = scale * 1.4426950408889634f;  // K is pre-multiplied by it (exp2 domain)
  v8bf kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = scale_frag(frag_global(krow, kok, ks, hd, lane), c);
    vf[ks] = frag_global(vrow, kok, ks, hd, lane);
  }
  // dS is accumulated divided by the dropout scale (see nd): dK = kscale * (Q^T . dS/dscale)
  const float kscale = DROP ? scale * dscale : scale;
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
  // Three LDS buffers: everything iteration it+2 reads -- the Q / dO images and the per-query rows
  // (-lse2 and nd, both written by the dQ kernel; segment starts; keep words) -- streams in by
  // LDS-DMA while iteration it computes, so the wait at the end of iteration it (a counted vmcnt
  // that leaves the newest iteration's DMAs in flight) is for data issued one iteration earlier.
  // Per wave and iteration: 4 image pieces + 1 row (wave 0: -lse2, 1: nd, 2: segment starts,
  // 3: the segment starts again, into a slot of its own that nothing reads)
  // + (DROP == 2) its 64 keep words.
  constexpr int NBUF = 3;
  constexpr int NV = 5 + (DROP == 2 ? 1 : 0);
  const int mw_idx = kt0 / 32 + wave;  // this wave's key word of a query's keep bits
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const TileDma qsrc = tile_dma_src(qkv + rowbase * ld, ld, T, hd, wave_u, lane);
  const TileDma dsrc = tile_dma_src(dy + rowbase * lddy, lddy, T, hd, wave_u, lane);
  const uint32_t qstride = (uint32_t)(KT * ld * 2), dstride = (uint32_t)(KT * lddy * 2);
  constexpr uint32_t OORD = 0x80000000u;  // past every record: the DMA writes 0
  const long long bh0 = (long long)b * H * T;  // (b, head 0, query 0) of the per-query rows
  const float* rowsrc = wave_u == 0 ? nlse2 : delta;
  const __amdgpu_buffer_rsrc_t rrow =
      wave_u < 2 ? __builtin_amdgcn_make_buffer_rsrc((void*)(rowsrc + bh0), (short)0, H * T * 4, 0x00020000)
                 : __builtin_amdgcn_make_buffer_rsrc((void*)(seg ? seg + rowbase : nullptr), (short)0,
                                                     seg ? T * 4 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rqm = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(DROP == 2 ? qmask + bh0 * wpr : nullptr), (short)0, DROP == 2 ? H * T * wpr * 4 : 0, 0x00020000);
  // this wave's word of key tile mw_idx/2 in the tile-major array: + ((h2*nt + tile)*T + q)*2 + half
  const uint32_t row_lds = (uint32_t)(wave_u < 3 ? 2 * IMG + wave_u * 64 * 4 : BUF - 64 * 4);  // -lse2 | nd | seg
  // iteration cursor: (query head, query tile), advanced without divisions
  struct Cur { int h2, qt; };
  auto next_of = [&](Cur c) { return c.qt < qt_end ? Cur{c.h2, c.qt + 1} : Cur{c.h2 + 1, qt_begin}; };
  auto stage_dma = [&](Cur cu, int nb) {
    const int h2 = cu.h2, qt = cu.qt;
    const uint32_t buf = lds0 + nb * BUF;
    tile_dma(buf, qsrc, qt * qstride + (uint32_t)(h2 * hd * 2), wave_u);
    tile_dma(buf + IMG, dsrc, qt * dstride + (uint32_t)(h2 * hd * 2), wave_u);
    const int q = qt * KT + lane;
    dma4(rrow, buf + row_lds, q < T ? (uint32_t)(((wave_u < 2 ? h2 * T : 0) + q) * 4) : OORD);
    if constexpr (DROP == 2)
      dma4(rqm, buf + (uint32_t)(2 * IMG + 4 * 64 * 4 + wave_u * 64 * 4),
           (q < T && mw_idx < wpr)
               ? (uint32_t)((((h2 * (wpr >> 1) + (mw_idx >> 1)) * T + q) * 2 + (mw_idx & 1)) * 4)
               : OORD);
  };
  // DROP == 1: the row hashes of cu into its buffer's hash slot (after that buffer's DMAs landed)
  auto stage_hash = [&](Cur cu, char* bufp) {
    if constexpr (DROP == 1) {
      if (tid < 64)
        ((uint32_t*)(bufp + 2 * IMG + 3 * 64 * 4))[tid] =
            cg_row_hash(seed, (uint32_t)(((long long)b * H + cu.h2) * T + cu.qt * KT + tid));
    }
  };
  Cur cur{kvh * rep, qt_begin};
  Cur n1 = next_of(cur);
  Cur n2 = next_of(n1);
  if (total > 0) {
    stage_dma(cur, 0);
    if (total > 1) {
      stage_dma(n1, 1);
      dma_wait<NV>();
    } else {
      dma_wait<0>();
    }
    stage_hash(cur, smem);
  }
  __syncthreads();
  const RowOff ro = row_offsets(lane);
  const TrOff to = tr_offsets(lane);
  // one iteration on LDS buffer CUR (compile-time: every image read is lane offset + immediate)
  auto iter = [&](auto cur_c, int it) __attribute__((always_inline)) {
    constexpr int CUR = decltype(cur_c)::value;
    const char* buf = smem + CUR * BUF;
    const char* Qi = buf;
    const char* Di = buf + IMG;
    const float* lse2s = (const float*)(buf + 2 * IMG);
    const float* nds = lse2s + 64;
    const int* los = (const int*)(buf + 2 * IMG + 2 * 64 * 4);
    const uint32_t* hrs = (const uint32_t*)(buf + 2 * IMG + 3 * 64 * 4);
    const bool more1 = it + 1 < total, more2 = it + 2 < total;
    // this wave's key word of the tile's keep bits, [query]
    const uint32_t* mws = (const uint32_t*)(buf + 2 * IMG + 4 * 64 * 4) + wave * 64;
    if (more2) stage_dma(n2, (CUR + 2) % NBUF);  // that buffer was last read before the previous barrier
    const int q0 = cur.qt * KT;
    // wave activity: some query q in [q0, q0+63] sees some key in [kw0, kw0+31]
    const int qlast = min(T - 1, q0 + KT - 1);
    // segment start of query q0 + i raised by the local window (the rows hold the raw segment starts)
    auto lo_at = [&](int i) { return window > 0 ? max(los[i], q0 + i - window + 1) : los[i]; };
    const bool active = (qlast >= kw0) && (lo_at(0) <= kw0 + 31);
    // full: every (query, key) of the wave's tile visible.  Otherwise the invisible scores are
    // set to -inf before the exponent (the branch touches only s: the dK/dV accumulators keep
    // their registers across it)
    // phases of one 32-query half: S and dP (accumulators seeded with -lse2 / nd), the softmax,
    // keep and dS in registers, then dV and dK
    auto phase_sdp = [&](int qb, v16f& s, v16f& dp, v16f& nd) __attribute__((always_inline)) {
      // dP starts from -delta/dscale (the rows' nd values): the accumulator then holds
      // dP - delta/dscale, and dS/dscale = p * (keep ? acc : nd) is one bit-select and a multiply
      // S starts from -lse2 (K is pre-multiplied by c = scale*log2(e)): the accumulator is the
      // exp2 argument itself
#pragma unroll
      for (int rg = 0; rg < 16; rg += 4) {
        const float4 n4 = *(const float4*)(nds + qb * 32 + acc_row(rg, lane));
        nd[rg] = n4.x; nd[rg + 1] = n4.y; nd[rg + 2] = n4.z; nd[rg + 3] = n4.w;
        const float4 l4 = *(const float4*)(lse2s + qb * 32 + acc_row(rg, lane));
        s[rg] = l4.x; s[rg + 1] = l4.y; s[rg + 2] = l4.z; s[rg + 3] = l4.w;
      }
      dp = nd;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (ks < nks) {
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row_o(Qi, ro, qb * 32, ks), kf[ks], s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row_o(Di, ro, qb * 32, ks), vf[ks], dp, 0, 0, 0);
        }
      }
    };
    auto phase_ds = [&](int qb, auto full_c, v16f& s, const v16f& dp, const v16f& nd, v8bf& pb0, v8bf& pb1, v8bf& sb0,
                        v8bf& sb1) __attribute__((always_inline)) {
      bool full;
      if constexpr (std::is_same_v<decltype(full_c), bool>) full = full_c;
      else full = decltype(full_c)::value;
      if (!full) {
#pragma unroll
        for (int rg = 0; rg < 16; rg += 4) {
          const int qi = qb * 32 + acc_row(rg, lane);
          const int4 lo4 = *(const int4*)(los + qi);
          const int lov[4] = {lo4.x, lo4.y, lo4.z, lo4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int q = q0 + qi + u;
            const int lq = window > 0 ? max(lov[u], q - window + 1) : lov[u];
            s[rg + u] = ((mykey > q) | (mykey < lq) | (q >= T)) ? -INFINITY : s[rg + u];
          }
        }
      }
      v16f pd;
#pragma unroll
      for (int rg = 0; rg < 16; rg += 4) {
        const int qi = qb * 32 + acc_row(rg, lane);  // 4 consecutive queries qi..qi+3
        uint4 hr4 = make_uint4(0, 0, 0, 0);
        if constexpr (DROP == 1) hr4 = *(const uint4*)(hrs + qi);
        uint4 mw4 = make_uint4(0, 0, 0, 0);
        if constexpr (DROP == 2) mw4 = *(const uint4*)(mws + qi);
        const uint32_t mwv[4] = {mw4.x, mw4.y, mw4.z, mw4.w};
        const uint32_t hrv[4] = {hr4.x, hr4.y, hr4.z, hr4.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = rg + u;
          const float p = __builtin_amdgcn_exp2f(s[r]);
          float pdr = p;  // the 1/(1-p) of P~ is applied to dV once at the end
          if constexpr (DROP == 1) {
            const uint32_t hsh = cg_pair_mix(hrv[u] + kcol);
            const uint32_t bits = (mykey & 1) ? (hsh >> 16) : (hsh & 0xFFFFu);
            const bool keep = bits >= thr;
            pdr = keep ? p : 0.f;
            s[r] = p * (keep ? dp[r] : nd[r]);
          } else if constexpr (DROP == 2) {
            const uint32_t m = (uint32_t)keep_mask(mwv[u], kpos);
            pdr = __uint_as_float(__float_as_uint(p) & m);
            s[r] = p * bsel(m, dp[r], nd[r]);
          } else {
            s[r] = p * dp[r];
          }
          pd[r] = pdr;
        }
      }
      pb0 = pack_b(pd, 0); pb1 = pack_b(pd, 1);
      sb0 = pack_b(s, 0); sb1 = pack_b(s, 1);
    };
    // the transposed dO / Q fragments the dV / dK products read: LDS only, so they are issued before
    // the half's softmax / keep VALU (a scheduling barrier keeps them there) and land under it
    struct TrFr { v8bf d[4], q[4]; };
    auto tr_frags = [&](int qb, TrFr& f) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < (hd > 32 ? 4 : 2); ++i) {
        f.d[i] = frag_tr_o(Di, to, qb * 32, i & 1, i >> 1);
        f.q[i] = frag_tr_o(Qi, to, qb * 32, i & 1, i >> 1);
      }
    };
    auto phase_dkdv = [&](const TrFr& f, const v8bf& pb0, const v8bf& pb1, const v8bf& sb0, const v8bf& sb1)
                          __attribute__((always_inline)) {
      dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.d[0], pb0, dv0, 0, 0, 0);
      dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.d[1], pb1, dv0, 0, 0, 0);
      dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.q[0], sb0, dk0, 0, 0, 0);
      dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.q[1], sb1, dk0, 0, 0, 0);
      if constexpr (hd > 32) {
        dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.d[2], pb0, dv1, 0, 0, 0);
        dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.d[3], pb1, dv1, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.q[2], sb0, dk1, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.q[3], sb1, dk1, 0, 0, 0);
      }
    };
    auto body = [&](auto full) __attribute__((always_inline)) {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        v16f s, dp, nd;
        v8bf x0, x1, x2, x3;
        TrFr f;
        phase_sdp(qb, s, dp, nd);
        tr_frags(qb, f);
        __builtin_amdgcn_sched_barrier(0);
        phase_ds(qb, full, s, dp, nd, x0, x1, x2, x3);
        phase_dkdv(f, x0, x1, x2, x3);
      }
    };
    if (active) {
      const bool full = (q0 >= kw0 + 31) && (q0 + KT - 1 < T) && (lo_at(qlast - q0) <= kw0);
      body(full);
    }
    if (more1) {  // n1's data (issued an iteration ago) landed; n2's DMAs may still be in flight
      if (more2) dma_wait<NV>();
      else dma_wait<0>();
      stage_hash(n1, smem + ((CUR + 1) % NBUF) * BUF);
    }
    cur = n1;
    n1 = n2;
    n2 = next_of(n2);
    // raw barrier: no vmcnt(0) (n2's DMAs stay in flight); the row stores and this wave's image
    // reads retired first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  for (int it = 0; it < total; it += NBUF) {
    iter(std::integral_constant<int, 0>{}, it);
    if (it + 1 < total) iter(std::integral_constant<int, 1>{}, it + 1);
    if (it + 2 < total) iter(std::integral_constant<int, 2>{}, it + 2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing in flight past the loop
  if (rcos) {  // RoPE: dK w.r.t. the rotated k, rotated back at the key's position
    const size_t ro = (size_t)(kok ? mykey : 0) * (hd / 2);
    rope_inv_blocks<hd>(dk0, dk1, rcos + ro, rsin + ro, lane >> 5);
  }
  {
    bf16_t* kr = dqkv + (rowbase + (kok ? mykey : 0)) * lddq + koff;
    bf16_t* vr = dqkv + (rowbase + (kok ? mykey : 0)) * lddq + voff;
    const float vs = DROP ? dscale : 1.0f;
    store_blk16(kr, dk0, kscale, kok, hd < 32 ? hd : 32, lane);
    store_blk16(vr, dv0, vs, kok, hd < 32 ? hd : 32, lane);
    if (hd > 32) {
      store_blk16(kr + 32, dk1, kscale, kok, hd - 32, lane);
      store_blk16(vr + 32, dv1, vs, kok, hd - 32, lane);
    }
  }
  if (bpart) {  // k / v bias gradient partials: column sums of this workgroup's dK, dV rows
    const float vs = DROP ? dscale : 1.0f;
    float* red = (float*)smem;  // the ring is idle after the last barrier
    const float vk = colsum_wg(dk0, dk1, kscale, kok, red, wave, lane, tid);
    const float vv = colsum_wg(dv0, dv1, vs, kok, red, wave, lane, tid);
    float* dst = bpart + ((long long)b * gridDim.y + ktile) * ldp;
    if (tid < hd) {
      dst[koff + tid] = vk;
      dst[voff + tid] = vv;
    }
  }
}

// ============================================================================
// fused backward: dK, dV AND dQ in one pass (five MFMA products per tile -- S, dP, dV, dK, dQ --
// against the two-kernel path's seven; Q, dO, the row statistics and the keep words streamed once).
// WG = 8 waves x 32 keys = one 256-key block at a time, and the WG owns ONE (b, kv head) for all of
// its key blocks and query heads.  So the dQ rows of the group's query heads have a single writer:
// the WG read-modify-writes fp32 dQ^T partials into dq_acc (layout fa::dqa_off), which no other
// workgroup touches -- no atomics, no cross-workgroup reduction, bitwise reproducible.
// Per iteration (one 64-query tile of one query head):
//   * waves 0-3 (one per SIMD) first finish the PREVIOUS tile's dQ^T block -- query half w >> 1,
//     head-dim block w & 1 -- = K^T[d][256 keys] dS^T[keys][q] (16 MFMAs, operands by
//     ds_read_b64_tr_b16 from the block's K image and the dS^T image), + the dq_acc value (plain
//     store on the tile's first visit);
//   * all waves, as attn_bwd_dkdv_mfma: S and dP (key on the lane, seeded with -lse2 / nd), P and
//     dS, dV += dO^T P, dK += Q^T dS; the wave's dS^T (bf16, the dK operand itself) goes into the
//     LDS image dsb[it & 1] ([256 keys][64 queries], dual layout).
// One barrier per iteration.  Before: attn_bwd_prep_kernel (the -lse2 and nd rows), after:
// attn_dq_finish_kernel (dq_acc -> the bf16 dqkv q columns, x scale, RoPE inverse, q-bias
// partials).  Keep bits from the forward's words only (DROP 0 / 2).
// ============================================================================
namespace fa {
constexpr int FB_KEYS = 256;     // keys per block (8 waves x 32)
constexpr int FB_DSB = 4 * IMG;  // one dS^T image set [256 keys][64 queries] bf16 (also the K image)
// ring buffer: Q image | dO image | -lse2 | nd | seg | (a slot the row DMAs of waves 3-7 fill) |
// (DROP 2) the 8 waves' keep words of the tile's 64 queries
__host__ __device__ constexpr int fb_buf(int drop) { return 2 * IMG + 4 * 64 * 4 + (drop == 2 ? 8 * 64 * 4 : 0); }
// LDS: 3 ring buffers (first: every per-iteration read is lane offset + a < 64 KiB immediate) | dsb[2] |
// K image; the first 68 KiB double as the bias column-sum scratch at the end of a key block
__host__ __device__ constexpr int fb_lds(int drop) { return 3 * FB_DSB + 3 * fb_buf(drop); }
// dq_acc: [b H + h][query block of 32][64 head dims][32 queries] fp32 -- one accumulator register
// of a dQ^T block is two 128-B runs (32 queries of one head dim), and its 16 registers sit at
// constant offsets from the lane's base (immediate-offset loads / stores)
__host__ __device__ inline long long dqa_off(long long bh, int nq32, int q32, int d) {
  return ((bh * nq32 + q32) * 64 + d) * 32;
}
// one 1-KiB LDS-DMA piece per wave: rows 8 wave .. 8 wave + 7 of a 64-row image (8 waves fill it);
// the dual_off swizzle on the per-lane source chunk as in tile_dma_src
struct PieceDma {
  __amdgpu_buffer_rsrc_t r;
  uint32_t off;
};
__device__ __forceinline__ PieceDma piece_dma_src(const bf16_t* batch_rows, long long ld, int T, int hd, int wave,
                                                  int lane) {
  PieceDma p;
  p.r = __builtin_amdgcn_make_buffer_rsrc((void*)batch_rows, (short)0, (int)((long long)T * ld * 2), 0x00020000);
  const int row = 8 * wave + (lane >> 3), j = row >> 1;
  const int ch = (lane & 7) ^ ((j & 7) ^ ((j & 1) << 2));
  p.off = ch * 8 < hd ? (uint32_t)(((long long)row * ld + ch * 8) * 2) : 0x80000000u;
  return p;
}
__device__ __forceinline__ void piece_dma(uint32_t img, const PieceDma& p, uint32_t ubase, int wave) {
  dma16(p.r, img + (uint32_t)(8 * wave * 128), p.off + ubase);
}
// column sums over the workgroup's 256 accumulator columns (8 waves x 32 lanes) of the 64 rows in
// x0 / x1 -- colsum_wg for 8 waves; `red` needs COLSUM8_LDS bytes; ends with a barrier
constexpr int COLSUM8_LDS = (8 * 64 * 33 + 8 * 64) * 4;
__device__ __forceinline__ float colsum_wg8(const v16f& x0, const v16f& x1, float s, bool ok, float* red, int wave,
                                            int lane, int tid) {
  float* t = red + wave * 64 * 33 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    t[acc_row(r, lane) * 33] = ok ? x0[r] * s : 0.f;
    t[(32 + acc_row(r, lane)) * 33] = ok ? x1[r] * s : 0.f;
  }
  __syncthreads();
  const float* run = red + (tid >> 6) * 64 * 33 + (tid & 63) * 33;
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int k = 0; k < 32; k += 2) {
    a += run[k];
    b += run[k + 1];
  }
  float* part = red + 8 * 64 * 33;
  part[tid] = a + b;
  __syncthreads();
  float v = 0.f;
  if (tid < 64)
    v = ((part[tid] + part[64 + tid]) + (part[128 + tid] + part[192 + tid])) +
        ((part[256 + tid] + part[320 + tid]) + (part[384 + tid] + part[448 + tid]));
  __syncthreads();
  return v;  // threads 0..63: the column sum of row tid
}
// sum over the 32 lanes of each half-wave, in every lane of that half (wave_reduce without its last
// v_permlane32_swap step)
__device__ __forceinline__ float half_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}
}  // namespace fa

// nd = -rowsum(dO o O) / dscale (the dP seed; delta of the FA2 preprocessing) and -lse * log2(e)
// (the S seed), one (b, query, head) per 8 lanes, 16-B loads of dO and O; consecutive groups take
// consecutive heads of one token, so a wave reads whole token rows
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const bf16_t* __restrict__ dy, long long lddy,
                                                            const bf16_t* __restrict__ yo, long long ldy,
                                                            const float* __restrict__ lse, float* __restrict__ nd,
                                                            float* __restrict__ nlse2, int T, int H, int hd,
                                                            float inv_dscale, long long nrows) {
  const long long g = (long long)blockIdx.x * 32 + (threadIdx.x >> 3);  // (b T + q) H + h
  const int j = threadIdx.x & 7;
  const long long row = g / H;                                          // b T + q
  const int h = (int)(g - row * H);
  const int b = (int)(row / T), q = (int)(row - (long long)b * T);
  const long long r = ((long long)b * H + h) * T + q;                   // the [b][h][q] row index
  float s = 0.f;
  if (g < nrows && 8 * j < hd) {
    const uint4 dv = *(const uint4*)(dy + row * lddy + (long long)h * hd + 8 * j);
    const uint4 ov = *(const uint4*)(yo + row * ldy + (long long)h * hd + 8 * j);
    const uint32_t dw[4] = {dv.x, dv.y, dv.z, dv.w}, ow[4] = {ov.x, ov.y, ov.z, ov.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s = fmaf(__uint_as_float(dw[i] << 16), __uint_as_float(ow[i] << 16), s);
      s = fmaf(__uint_as_float(dw[i] & 0xFFFF0000u), __uint_as_float(ow[i] & 0xFFFF0000u), s);
    }
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  if (g < nrows && j == 0) {
    nd[r] = -s * inv_dscale;
    nlse2[r] = -lse[r] * 1.4426950408889634f;
  }
}

template <int DROP, int HD>
__global__ __launch_bounds__(512, 2) void attn_bwd_fused_mfma(const bf16_t* __restrict__ qkv, long long ld,
                                                              const int32_t* __restrict__ seg,
                                                              const bf16_t* __restrict__ dy, long long lddy,
                                                              const float* __restrict__ ndrow,
                                                              const float* __restrict__ nlse2,
                                                              float* __restrict__ dq_acc, int nq32,
                                                              bf16_t* __restrict__ dqkv, long long lddq, int T, int H,
                                                              int KV, int window, float dscale, float scale,
                                                              const uint32_t* __restrict__ qmask, int wpr,
                                                              float* __restrict__ bpart, long long ldp,
                                                              const float* __restrict__ rcos,
                                                              const float* __restrict__ rsin) {
  using namespace fa;
  static_assert(DROP == 0 || DROP == 2, "fused backward: keep bits from the forward's words");
  constexpr int hd = HD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BUF = fb_buf(DROP);
  constexpr int NV = 3 + (DROP == 2 ? 1 : 0);  // DMAs per wave and ring stage
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int bk = blockIdx.x, b = bk / KV, kvh = bk % KV;
  const int rep = H / KV;
  const long long rowbase = (long long)b * T;
  const long long koff = (long long)H * hd + (long long)kvh * hd;
  const long long voff = (long long)(H + KV) * hd + (long long)kvh * hd;
  const float c = scale * 1.4426950408889634f;  // K is pre-multiplied by it (exp2 domain)
  const float kscale = DROP ? scale * dscale : scale;
  const float qscale = kscale;
  // MHA without RoPE: the last key block of each tile stores dQ itself, and the q-bias partials are
  // sum_key (sum_q dS[q][key]) K[key] (no per-query factor to apply); else dq_acc + the finish pass
  const bool direct = !rcos && rep == 1;
  const float vsc = DROP ? dscale : 1.0f;
  constexpr int nks = (hd + 15) >> 4;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const uint32_t ring_l = lds0, kimg_l = lds0 + 3 * BUF + 2 * FB_DSB;
  char* const dsb = smem + 3 * BUF;
  const char* const kimg = dsb + 2 * FB_DSB;
  const PieceDma qsrc = piece_dma_src(qkv + rowbase * ld, ld, T, hd, wave_u, lane);
  const PieceDma dsrc = piece_dma_src(dy + rowbase * lddy, lddy, T, hd, wave_u, lane);
  const uint32_t qstride = (uint32_t)(KT * ld * 2), dstride = (uint32_t)(KT * lddy * 2);
  const uint32_t kcol = (uint32_t)((H + kvh) * hd * 2);
  constexpr uint32_t OORD = 0x80000000u;  // past every record: the DMA writes 0
  const long long bh0 = (long long)b * H * T;  // (b, head 0, query 0) of the per-query rows
  const float* rowsrc = wave_u == 0 ? nlse2 : ndrow;
  const __amdgpu_buffer_rsrc_t rrow =
      wave_u < 2 ? __builtin_amdgcn_make_buffer_rsrc((void*)(rowsrc + bh0), (short)0, H * T * 4, 0x00020000)
                 : __builtin_amdgcn_make_buffer_rsrc((void*)(seg ? seg + rowbase : nullptr), (short)0,
                                                     seg ? T * 4 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rqm = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(DROP == 2 ? qmask + bh0 * wpr : nullptr), (short)0, DROP == 2 ? H * T * wpr * 4 : 0, 0x00020000);
  // -lse2 | nd | seg rows by waves 0 / 1 / 2; waves 3-7 load the seg row again into a slot nothing reads
  const uint32_t row_lds = (uint32_t)(2 * IMG + (wave_u < 3 ? wave_u : 3) * 64 * 4);
  const RowOff ro = row_offsets(lane);
  const TrOff to = tr_offsets(lane);
  // this lane's dS^T image row (key 32 wave + (lane & 31) of the block) and its XOR swizzle group;
  // its 8-byte stores go to columns 8 ch + 4 (lane >> 5) .. + 3
  const int srow = 32 * (wave & 1) + (lane & 31);
  const int sg = ((srow >> 1) & 7) ^ (((srow >> 1) & 1) << 2);
  const uint32_t sbase = (uint32_t)((wave >> 1) * IMG + srow * 128 + 8 * (lane >> 5));
  const int nkb = (T + FB_KEYS - 1) / FB_KEYS;
  const int ny = (T + 127) / 128;
  auto qt_end_of = [&](int kb) {
    const int qe = window > 0 ? min(T, kb * FB_KEYS + FB_KEYS - 1 + window) : T;
    return (qe - 1) / KT;
  };
  // the workgroup's whole sequence of (key block, query head, query tile) iterations: the LDS-DMA
  // ring runs across the key-block seams, so a new block starts on landed data
  const int h2_0 = kvh * rep;
  struct Cur {
    int kb, h2, qt;
  };
  auto next_of = [&](Cur cu) {
    if (cu.qt < qt_end_of(cu.kb)) return Cur{cu.kb, cu.h2, cu.qt + 1};
    if (cu.h2 + 1 < h2_0 + rep) return Cur{cu.kb, cu.h2 + 1, cu.kb * (FB_KEYS / KT)};
    return Cur{cu.kb + 1, h2_0, (cu.kb + 1) * (FB_KEYS / KT)};
  };
  int total = 0;
  for (int k = 0; k < nkb; ++k) total += (qt_end_of(k) - k * (FB_KEYS / KT) + 1) * rep;
  // the previous iteration's tile, finished (dQ) by waves 0-3 in the next iteration
  struct Prev {
    int h2, qt, first, last;  // the tile's first / last visiting key block is this one
  };
  auto stage_dma = [&](Cur cu, int nb) {
    const uint32_t buf = ring_l + nb * BUF;
    const int mw = cu.kb * (FB_KEYS / 32) + wave_u;  // this wave's key word of a query's keep bits
    piece_dma(buf, qsrc, cu.qt * qstride + (uint32_t)(cu.h2 * hd * 2), wave_u);
    piece_dma(buf + IMG, dsrc, cu.qt * dstride + (uint32_t)(cu.h2 * hd * 2), wave_u);
    const int q = cu.qt * KT + lane;
    dma4(rrow, buf + row_lds, q < T ? (uint32_t)(((wave_u < 2 ? cu.h2 * T : 0) + q) * 4) : OORD);
    if constexpr (DROP == 2)
      dma4(rqm, buf + (uint32_t)(2 * IMG + 4 * 64 * 4 + wave_u * 64 * 4),
           (q < T && mw < wpr) ? (uint32_t)((((cu.h2 * (wpr >> 1) + (mw >> 1)) * T + q) * 2 + (mw & 1)) * 4)
                               : OORD);
  };
  // a key block's K image (rows 256 kb .. + 255, unscaled) for the dQ product: 4 pieces per wave
  auto kimg_dma = [&](int k) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      piece_dma(kimg_l + i * IMG, qsrc, (uint32_t)((k * FB_KEYS + 64 * i) * ld * 2) + kcol, wave_u);
  };
  // the lane's key of block k, and its K (x c) / V fragments
  v8bf kf[4], vf[4];
  auto load_kv = [&](int k) {
    const int key = k * FB_KEYS + wave * 32 + (lane & 31);
    const bool ok = key < T;
    const bf16_t* krow = qkv + (rowbase + (ok ? key : 0)) * ld + koff;
    const bf16_t* vrow = qkv + (rowbase + (ok ? key : 0)) * ld + voff;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      kf[ks] = scale_frag(frag_global(krow, ok, ks, hd, lane), c);
      vf[ks] = frag_global(vrow, ok, ks, hd, lane);
    }
  };
  v16f dk0 = zero16(), dk1 = zero16(), dv0 = zero16(), dv1 = zero16();
  float dscol = 0.f;  // (direct, bias) sum over the block's queries of dS/dscale for the lane's key
  int kb = 0;
  load_kv(0);
  kimg_dma(0);
  Cur cur{0, h2_0, 0};
  Cur n1 = next_of(cur);
  Cur n2 = next_of(n1);
  stage_dma(cur, 0);
  if (total > 1) {
    stage_dma(n1, 1);
    dma_wait<NV>();
  } else {
    dma_wait<0>();
  }
  __syncthreads();
  Prev pv{0, 0, 0, 0};
  bool have_prev = false;
  // waves 0-3: the dq_acc block of tile (h2, qt) this wave owns -- query half w >> 1, head dims
  // 32 (w & 1) + acc_row(r): element r at + ((r & 3) + 8 (r >> 2)) * 32
  // (a wave-uniform base and a 32-bit lane offset: per-lane 64-bit pointers would be kept -- or
  // spilled -- across the loop)
  auto dq_base = [&](int h2, int qt) {
    return dq_acc + dqa_off((long long)b * H + h2, nq32, qt * 2 + (wave_u >> 1), (wave_u & 1) * 32);
  };
  const uint32_t dq_lane = (uint32_t)(4 * (lane >> 5) * 32 + (lane & 31));
  // its old value, loaded at the top of the tile's own iteration: the load latency runs under the
  // tile's phase A instead of stalling phase B.  Every wave loads on every iteration (waves 4-7 and
  // first visits a line they ignore), so the registers are written on every path.
  v16f oldv;
  // waves 0-3: dQ^T block of tile pv from the dS^T images, accumulated onto oldv.  Straight-line
  // (inactive key waves wrote zero rows), operand reads one 4-k-step group ahead of the MFMAs
  auto phase_b = [&](const char* dsimg, const Prev& p) __attribute__((always_inline)) {
    const int qb = wave_u >> 1, cb = wave_u & 1;
    const uint32_t ka0 = cb ? to.o[1][0] : to.o[0][0], ka1 = cb ? to.o[1][1] : to.o[0][1];
    const uint32_t sb0 = qb ? to.o[1][0] : to.o[0][0], sb1 = qb ? to.o[1][1] : to.o[0][1];
    float* dst = dq_base(p.h2, p.qt);
    v16f acc = p.first ? zero16() : oldv;  // the running sum, landed under the previous phase A
    v8bf fa[2][4], fb[2][4];
    auto rd = [&](int g) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kk = 4 * g + i, rb = 32 * ((kk >> 1) & 1), st = kk & 1;
        fa[g & 1][i] = frag_tr_p(kimg + g * IMG, ka0, ka1, rb, st);
        fb[g & 1][i] = frag_tr_p(dsimg + g * IMG, sb0, sb1, rb, st);
      }
    };
    rd(0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (g < 3) rd(g + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[g & 1][i], fb[g & 1][i], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (!p.last || !direct) {  // a later key block adds to it (or the finish pass converts it)
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[dq_lane + ((r & 3) + 8 * (r >> 2)) * 32] = acc[r];
    } else if (cb * 32 < hd) {  // the tile's last key block: dQ = qscale (dS/dscale . K) into dqkv
      const int q0b = p.qt * KT + qb * 32;
      const bool qok = q0b + (lane & 31) < T;
      bf16_t* dbase = dqkv + (rowbase + q0b) * lddq + (long long)p.h2 * hd + cb * 32;
      store_blk16(dbase + (uint32_t)(qok ? (lane & 31) * (uint32_t)lddq : 0u), acc, qscale, qok,
                  hd - cb * 32 < 32 ? hd - cb * 32 : 32, lane);
    }
  };
  // end of key block k (its last tile's dQ done, every wave past the barrier that follows it): dK,
  // dV (and, direct, the q-bias partial) out; the bias column sums use the dS^T / K image region
  // (the ring may hold the next block's first tiles in flight)
  auto block_epilogue = [&](int k) __attribute__((always_inline)) {
    const int mykey = k * FB_KEYS + wave * 32 + (lane & 31);
    const bool kok = mykey < T;
    if (rcos) {  // RoPE: dK w.r.t. the rotated k, rotated back at the key's position
      const size_t ro2 = (size_t)(kok ? mykey : 0) * (hd / 2);
      rope_inv_blocks<hd>(dk0, dk1, rcos + ro2, rsin + ro2, lane >> 5);
    }
    {
      bf16_t* kr = dqkv + (rowbase + (kok ? mykey : 0)) * lddq + koff;
      bf16_t* vr = dqkv + (rowbase + (kok ? mykey : 0)) * lddq + voff;
      store_blk16(kr, dk0, kscale, kok, hd < 32 ? hd : 32, lane);
      store_blk16(vr, dv0, vsc, kok, hd < 32 ? hd : 32, lane);
      if (hd > 32) {
        store_blk16(kr + 32, dk1, kscale, kok, hd - 32, lane);
        store_blk16(vr + 32, dv1, vsc, kok, hd - 32, lane);
      }
    }
    if (bpart) {  // k / v (and q) bias partials of the block into row 2 k of the batch's 128-row tiles
      float* red = (float*)dsb;
      v16f x0, x1;
      if (direct) {  // sum_key dscol[key] K[key][d], K from the block's image (raw bf16) -- read
        // before the column sums write over it (COLSUM8_LDS reaches into the K image)
        uint32_t kr_o = (uint32_t)((wave >> 1) * IMG + srow * 128 + 8 * (lane >> 5));
        int sg_k = sg;
        asm volatile("" : "+v"(kr_o), "+v"(sg_k));  // (not hoisted out of the iteration loop)
        const char* krow_l = kimg + kr_o;
        // lanes l and l + 32 hold the same key's two halves of the query rows: the whole column sum
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(dscol), __float_as_uint(dscol), false, false);
        const float dsall = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int cbk = 0; cbk < 2; ++cbk) {  // head dims 32 cbk + 8 j + 4 (lane >> 5) .. + 3
            const int ch = 4 * cbk + j;
            const uint2 kv = *(const uint2*)(krow_l + 16 * (ch ^ sg_k));
            const float k4[4] = {__uint_as_float(kv.x << 16), __uint_as_float(kv.x & 0xFFFF0000u),
                                 __uint_as_float(kv.y << 16), __uint_as_float(kv.y & 0xFFFF0000u)};
#pragma unroll
            for (int t = 0; t < 4; ++t) (cbk ? x1 : x0)[4 * j + t] = dsall * k4[t];
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();  // every wave's K row read before the first column sum writes over it
      }
      const float vk = colsum_wg8(dk0, dk1, kscale, kok, red, wave, lane, tid);
      const float vv = colsum_wg8(dv0, dv1, vsc, kok, red, wave, lane, tid);
      const float vq = direct ? colsum_wg8(x0, x1, qscale, kok, red, wave, lane, tid) : 0.f;
      float* dst = bpart + ((long long)b * ny + 2 * k) * ldp;
      const long long qoff = (long long)kvh * hd;  // (direct: rep == 1, the query head is kvh)
      if (tid < hd) {
        dst[koff + tid] = vk;
        dst[voff + tid] = vv;
        if (direct) dst[qoff + tid] = vq;
        if (2 * k + 1 < ny) {  // the block's second 128-row tile: its sums are in row 2 k
          dst[ldp + koff + tid] = 0.f;
          dst[ldp + voff + tid] = 0.f;
          if (direct) dst[ldp + qoff + tid] = 0.f;
        }
      }
    }
  };
  // one iteration on ring buffer CUR (compile-time: every image read is lane offset + immediate)
  auto iter = [&](auto cur_c, int it) __attribute__((always_inline)) {
    constexpr int CUR = decltype(cur_c)::value;
    const char* buf = smem + CUR * BUF;
    const char* Qi = buf;
    const char* Di = buf + IMG;
    const float* lse2s = (const float*)(buf + 2 * IMG);
    const float* nds = lse2s + 64;
    const int* los = (const int*)(buf + 2 * IMG + 2 * 64 * 4);
    const uint32_t* mws = (const uint32_t*)(buf + 2 * IMG + 4 * 64 * 4) + wave * 64;
    const int kt0 = kb * FB_KEYS, kw0 = kt0 + wave * 32;
    const int mykey = kw0 + (lane & 31);
    // the lane's key bit in a pair-split word: key 2c -> bit c, key 2c+1 -> bit 16 + c
    const uint32_t kpos = (uint32_t)(((mykey & 31) >> 1) + 16 * (mykey & 1));
    // the dS^T store offsets are rebuilt each iteration from (sbase, sg), which the empty asm makes
    // opaque: hoisted out of the loop, the eight per-lane offsets would stay live through phase A
    uint32_t sb_i = sbase;
    int sg_i = sg;
    asm volatile("" : "+v"(sb_i), "+v"(sg_i));
    char* dsw = dsb + (it & 1) * FB_DSB + sb_i;
    const bool more1 = it + 1 < total, more2 = it + 2 < total;
    // the previous tile's dQ first: its stores precede this iteration's DMAs in vmcnt order, so the
    // counted waits below leave exactly the newest stage (and the oldv loads) in flight
    if (wave_u < 4 && have_prev) phase_b(dsb + ((it - 1) & 1) * FB_DSB, pv);
    __builtin_amdgcn_sched_barrier(0);
    if (more2) stage_dma(n2, (CUR + 2) % 3);  // that buffer was last read before the previous barrier
    {  // this tile's dq_acc value for its phase B in the next iteration: in flight under phase A
      const float* src = wave_u < 4 ? dq_base(cur.h2, cur.qt) : dq_acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) oldv[r] = src[dq_lane + ((r & 3) + 8 * (r >> 2)) * 32];
    }
    const int q0 = cur.qt * KT;
    const int qlast = min(T - 1, q0 + KT - 1);
    auto lo_at = [&](int i) { return window > 0 ? max(los[i], q0 + i - window + 1) : los[i]; };
    const int lo0 = lo_at(0);
    // wave activity: some query of the tile sees some key of the wave (lo is monotone in q)
    const bool active = (qlast >= kt0 + 32 * wave_u) && (lo0 <= kt0 + 32 * wave_u + 31);
    auto phase_sdp = [&](int qb, v16f& s, v16f& dp, v16f& nd) __attribute__((always_inline)) {
#pragma unroll
      for (int rg = 0; rg < 16; rg += 4) {
        const float4 n4 = *(const float4*)(nds + qb * 32 + acc_row(rg, lane));
        nd[rg] = n4.x; nd[rg + 1] = n4.y; nd[rg + 2] = n4.z; nd[rg + 3] = n4.w;
        const float4 l4 = *(const float4*)(lse2s + qb * 32 + acc_row(rg, lane));
        s[rg] = l4.x; s[rg + 1] = l4.y; s[rg + 2] = l4.z; s[rg + 3] = l4.w;
      }
      dp = nd;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (ks < nks) {
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row_o(Qi, ro, qb * 32, ks), kf[ks], s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_row_o(Di, ro, qb * 32, ks), vf[ks], dp, 0, 0, 0);
        }
      }
    };
    auto phase_ds = [&](int qb, auto full_c, v16f& s, const v16f& dp, const v16f& nd, v8bf& pb0, v8bf& pb1,
                        v8bf& sb0, v8bf& sb1) __attribute__((always_inline)) {
      bool full;
      if constexpr (std::is_same_v<decltype(full_c), bool>) full = full_c;
      else full = decltype(full_c)::value;
      if (!full) {
#pragma unroll
        for (int rg = 0; rg < 16; rg += 4) {
          const int qi = qb * 32 + acc_row(rg, lane);
          const int4 lo4 = *(const int4*)(los + qi);
          const int lov[4] = {lo4.x, lo4.y, lo4.z, lo4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int q = q0 + qi + u;
            const int lq = window > 0 ? max(lov[u], q - window + 1) : lov[u];
            s[rg + u] = ((mykey > q) | (mykey < lq) | (q >= T)) ? -INFINITY : s[rg + u];
          }
        }
      }
      v16f pd;
#pragma unroll
      for (int rg = 0; rg < 16; rg += 4) {
        const int qi = qb * 32 + acc_row(rg, lane);
        uint4 mw4 = make_uint4(0, 0, 0, 0);
        if constexpr (DROP == 2) mw4 = *(const uint4*)(mws + qi);
        const uint32_t mwv[4] = {mw4.x, mw4.y, mw4.z, mw4.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = rg + u;
          const float p = __builtin_amdgcn_exp2f(s[r]);
          float pdr = p;  // the 1/(1-p) of P~ is applied to dV once at the end
          if constexpr (DROP == 2) {
            const uint32_t m = (uint32_t)keep_mask(mwv[u], kpos);
            pdr = __uint_as_float(__float_as_uint(p) & m);
            s[r] = p * bsel(m, dp[r], nd[r]);
          } else {
            s[r] = p * dp[r];
          }
          pd[r] = pdr;
        }
      }
      pb0 = pack_b(pd, 0); pb1 = pack_b(pd, 1);
      sb0 = pack_b(s, 0); sb1 = pack_b(s, 1);
    };
    struct TrFr { v8bf d[4], q[4]; };
    auto tr_frags = [&](int qb, TrFr& f) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < (hd > 32 ? 4 : 2); ++i) {
        f.d[i] = frag_tr_o(Di, to, qb * 32, i & 1, i >> 1);
        f.q[i] = frag_tr_o(Qi, to, qb * 32, i & 1, i >> 1);
      }
    };
    auto phase_dkdv = [&](const TrFr& f, const v8bf& pb0, const v8bf& pb1, const v8bf& sb0, const v8bf& sb1)
                          __attribute__((always_inline)) {
      dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.d[0], pb0, dv0, 0, 0, 0);
      dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.d[1], pb1, dv0, 0, 0, 0);
      dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.q[0], sb0, dk0, 0, 0, 0);
      dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.q[1], sb1, dk0, 0, 0, 0);
      if constexpr (hd > 32) {
        dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.d[2], pb0, dv1, 0, 0, 0);
        dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.d[3], pb1, dv1, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.q[2], sb0, dk1, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.q[3], sb1, dk1, 0, 0, 0);
      }
    };
    auto body = [&](auto full) __attribute__((always_inline)) {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        v16f s, dp, nd;
        v8bf x0, x1, x2, x3;
        TrFr f;
        phase_sdp(qb, s, dp, nd);
        phase_ds(qb, full, s, dp, nd, x0, x1, x2, x3);
        tr_frags(qb, f);  // (after the VALU: the registers hold oldv through phase A)
        if (direct && bpart) {
          float t = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) t += s[r];
          dscol += t;
        }
        // dS^T rows of this wave's keys: x2 = queries 4h + {0..3, 8..11}, x3 = 4h + {16..19, 24..27}
        // of the half, i.e. chunks 4 qb + 0..3 of the image row, 8 bytes at 8 (lane >> 5) in each
        const v4u_a w0 = __builtin_bit_cast(v4u_a, x2), w1 = __builtin_bit_cast(v4u_a, x3);
        *(uint2*)(dsw + 16 * ((4 * qb + 0) ^ sg_i)) = make_uint2(w0[0], w0[1]);
        *(uint2*)(dsw + 16 * ((4 * qb + 1) ^ sg_i)) = make_uint2(w0[2], w0[3]);
        *(uint2*)(dsw + 16 * ((4 * qb + 2) ^ sg_i)) = make_uint2(w1[0], w1[1]);
        *(uint2*)(dsw + 16 * ((4 * qb + 3) ^ sg_i)) = make_uint2(w1[2], w1[3]);
        phase_dkdv(f, x0, x1, x2, x3);
      }
    };
    if (active) {
      const bool full = (q0 >= kw0 + 31) && (q0 + KT - 1 < T) && (lo_at(qlast - q0) <= kw0);
      body(full);
    } else {  // no visible pair: zero dS^T rows, so the dQ product runs straight through
#pragma unroll
      for (int c8 = 0; c8 < 8; ++c8) *(uint2*)(dsw + 16 * (c8 ^ sg_i)) = make_uint2(0u, 0u);
    }
    pv = Prev{cur.h2, cur.qt, (kb == 0 || cur.qt > qt_end_of(kb - 1)) ? 1 : 0, (cur.qt >> 2) == kb ? 1 : 0};
    have_prev = true;
    // n1's data (issued an iteration ago) landed; n2's DMAs -- and the 16 oldv loads issued after
    // them -- may still be in flight
    if (more1) {
      if (more2) dma_wait<NV + 16>();
      else dma_wait<16>();
    }
    cur = n1;
    n1 = n2;
    n2 = next_of(n2);
    // raw barrier: no vmcnt(0) (n2's DMAs stay in flight); the dS^T stores and this wave's image
    // reads retired first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (more1 && cur.kb != kb) {  // key-block seam (the next tile's data already landed)
      load_kv(cur.kb);            // the new block's fragments, in flight under the epilogue
      if (wave_u < 4) phase_b(dsb + (it & 1) * FB_DSB, pv);  // the finished block's last tile
      __syncthreads();            // its dS^T / K images are free
      block_epilogue(kb);
      dk0 = zero16(); dk1 = zero16(); dv0 = zero16(); dv1 = zero16();
      dscol = 0.f;
      kimg_dma(cur.kb);           // lands before the new block's first phase B (two waits ahead)
      kb = cur.kb;
      have_prev = false;
    }
  };
  for (int it = 0; it < total; it += 3) {
    iter(std::integral_constant<int, 0>{}, it);
    if (it + 1 < total) iter(std::integral_constant<int, 1>{}, it + 1);
    if (it + 2 < total) iter(std::integral_constant<int, 2>{}, it + 2);
  }
  if (wave_u < 4) phase_b(dsb + ((total - 1) & 1) * FB_DSB, pv);  // the last tile's dQ
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing in flight past the loop
  __syncthreads();
  block_epilogue(kb);
}

// dq_acc (fp32 sums of dS/dscale . K over all keys, fa::dqa_off layout) -> the bf16 dqkv q columns:
// x qscale, RoPE inverse at the query's position (rcos != NULL), and the q-bias partial row of the
// 128-query tile (column sums of the unrounded values).  WG: one (b, h) x 128 queries.
template <int HD>
__global__ __launch_bounds__(256) void attn_dq_finish_kernel(const float* __restrict__ dq_acc, int nq32,
                                                             bf16_t* __restrict__ dqkv, long long lddq, int T, int H,
                                                             float qscale, float* __restrict__ bpart, long long ldp,
                                                             const float* __restrict__ rcos,
                                                             const float* __restrict__ rsin) {
  constexpr int hd = HD, PITCH = 65;
  __shared__ float t[128 * PITCH];
  const int tid = threadIdx.x;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int q0 = blockIdx.y * 128;
  // 4 query blocks of 32 x 64 head dims x 32 queries: 8 float4 per thread, coalesced
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = i * 256 + tid;             // float4 index in the 128-query slab
    const int blk = e >> 9, d = (e >> 3) & 63, q4 = (e & 7) * 4;
    const int q32 = (q0 >> 5) + blk;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q32 < nq32) v = *(const float4*)(dq_acc + fa::dqa_off(bh, nq32, q32, d) + q4);
    float* row = t + (blk * 32 + q4) * PITCH + d;
    row[0] = v.x; row[PITCH] = v.y; row[2 * PITCH] = v.z; row[3 * PITCH] = v.w;
  }
  __syncthreads();
  {
    // thread (query tid >> 1, half tid & 1): pairs i of [half hd/4, (half + 1) hd/4), dims i, i + hd/2
    const int ql = tid >> 1, half = tid & 1, q = q0 + ql;
    float* row = t + ql * PITCH;
    constexpr int hh = hd / 2, np = hd / 4;
    const float* cs = rcos ? rcos + (size_t)(q < T ? q : 0) * hh : nullptr;
    const float* sn = rcos ? rsin + (size_t)(q < T ? q : 0) * hh : nullptr;
#pragma unroll
    for (int k = 0; k < np; ++k) {
      const int i = half * np + k;
      const float g = row[i], gp = row[i + hh];
      if (cs) {
        row[i] = qscale * fmaf(cs[i], g, sn[i] * gp);
        row[i + hh] = qscale * fmaf(cs[i], gp, -sn[i] * g);
      } else {
        row[i] = qscale * g;
        row[i + hh] = qscale * gp;
      }
    }
  }
  __syncthreads();
  const int nq = min(128, T - q0);
  if (bpart && tid < hd) {  // the q-bias partial of this 128-query tile (fixed order)
    float a = 0.f, c2 = 0.f;
    int k = 0;
    for (; k + 1 < nq; k += 2) {
      a += t[k * PITCH + tid];
      c2 += t[(k + 1) * PITCH + tid];
    }
    if (k < nq) a += t[k * PITCH + tid];
    bpart[((long long)b * gridDim.y + blockIdx.y) * ldp + (long long)h * hd + tid] = a + c2;
  }
  // bf16 rows, 16 B per thread-chunk
  constexpr int CH = hd / 8;
  for (int e = tid; e < 128 * CH; e += 256) {
    const int ql = e / CH, ch = e - ql * CH;
    if (ql >= nq) continue;
    const float* src = t + ql * PITCH + ch * 8;
    uint4 o;
    o.x = fa::pk2bf(src[0], src[1]);
    o.y = fa::pk2bf(src[2], src[3]);
    o.z = fa::pk2bf(src[4], src[5]);
    o.w = fa::pk2bf(src[6], src[7]);
    *(uint4*)(dqkv + ((long long)b * T + q0 + ql) * lddq + (long long)h * hd + ch * 8) = o;
  }
}

// ----------------------------------------------------------------------------
static inline bool attn_mfma_supported(int hd, long long ld_in, long long ld_out) {
  return (hd == 32 || hd == 48 || hd == 64) && (ld_in % 8 == 0) && (ld_out % 8 == 0);
}

// words per (bh, row) of the keep-bit array
static inline int attn_drop_wpr(int T) { return 2 * cg_cdiv(T, 64); }
static inline size_t attn_drop_mask_words(int B, int T, int H) { return (size_t)B * H * T * attn_drop_wpr(T); }

static inline int attn_drop_mask_launch(uint32_t* mask, int B, int T, int H, uint32_t seed, uint32_t thr,
                                        hipStream_t s) {
  const int nb = cg_cdiv(T, 64);
  const int nbt = nb * (nb + 1) / 2;
  hipLaunchKernelGGL(attn_drop_mask_kernel, dim3(cg_cdiv(nbt, 4), B * H), dim3(256), 0, s, mask, T,
                     attn_drop_wpr(T), seed, thr, nbt);
  CG_LAUNCH_CHECK();
  return CG_OK;
}

// dmask_out (with thr): the keep words are made by the forward itself (DROP 3) instead of read
static inline int attn_fwd_mfma_launch(const bf16_t* qkv, long long ld, const int32_t* seg, bf16_t* y, long long ldy,
                                       float* lse, int B, int T, int H, int KV, int hd, int window, uint32_t seed,
                                       uint32_t thr, float dscale, float scale, const uint32_t* dmask, hipStream_t s,
                                       uint32_t* dmask_out = nullptr) {
  dim3 g(B * H, cg_cdiv(T, 128));
  const size_t sh = 4 * fa::IMG;
  const int wpr = attn_drop_wpr(T);
  // causal-exact products: QK^T and PV over the T(T+1)/2 visible (q, key) pairs
  const double tri = 2.0 * (double)B * H * hd * ((double)T * (T + 1) / 2.0);
  cg_probe_begin(CG_PROBE_ATTN_FWD, s);
#define FWD(D, HDv)                                                                                          \
  hipLaunchKernelGGL((attn_fwd_mfma<D, HDv>), g, dim3(256), sh, s, qkv, ld, seg, y, ldy, lse, T, H, KV, hd, window, \
                     seed, thr, dscale, scale, D == 3 ? dmask_out : const_cast<uint32_t*>(dmask), wpr)
  if (thr && dmask_out) {
    if (hd == 64) FWD(3, 64); else if (hd == 48) FWD(3, 48); else FWD(3, 32);
  } else if (thr && dmask) {
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

// fused backward workspace after the two per-query rows: dq_acc, [B H][Tp / 32][64][32] fp32
static inline int attn_dq_nq32(int T) { return cg_cdiv(T, 64) * 2; }
static inline size_t attn_dq_acc_floats(int B, int T, int H) {
  return (size_t)B * H * attn_dq_nq32(T) * 64 * 32;
}
// the fused pass when every CU gets a (batch, kv head) workgroup (it runs one per CU); the
// two-kernel pass spreads small batches over more workgroups.  Hash-in-kernel dropout (no keep
// words) stays on the two-kernel pass.
static inline bool attn_bwd_fused_ok(int algo, int B, int KV, int mode) {
  if (mode == 1 || algo == CG_ATTN_BWD_SPLIT) return false;
  if (algo == CG_ATTN_BWD_FUSED) return true;
  (void)B; (void)KV;
  return false;  // AUTO: the split pass until the fused one measures faster
}

static inline int attn_bwd_fused_launch(const bf16_t* qkv, long long ld, const int32_t* seg, const bf16_t* y,
                                        long long ldy, const bf16_t* dy, long long lddy, const float* lse,
                                        float* ws, bf16_t* dqkv, long long lddq, int B, int T, int H, int KV, int hd,
                                        int window, float dscale, float scale, const uint32_t* dmask, float* bpart,
                                        long long ldp, hipStream_t s, const float* rcos, const float* rsin) {
  const long long nbt = (long long)B * H * T;
  float* nd = ws;
  float* nlse2 = ws + nbt;
  float* dq_acc = ws + 2 * nbt;
  const int nq32 = attn_dq_nq32(T);
  const int wpr = attn_drop_wpr(T);
  const int mode = dmask ? 2 : 0;
  hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3(cg_cdiv(nbt, 32)), dim3(256), 0, s, dy, lddy, y, ldy, lse, nd, nlse2,
                     T, H, hd, mode ? 1.0f / dscale : 1.0f, nbt);
  CG_LAUNCH_CHECK();
  const double tri = 2.0 * (double)B * H * hd * ((double)T * (T + 1) / 2.0);
  const int sh = fa::fb_lds(mode);
  cg_probe_begin(CG_PROBE_ATTN_BWD, s);
#define FB(D, HDv)                                                                                              \
  do {                                                                                                          \
    cg_func_lds((const void*)attn_bwd_fused_mfma<D, HDv>, sh);                                                  \
    hipLaunchKernelGGL((attn_bwd_fused_mfma<D, HDv>), dim3(B * KV), dim3(512), sh, s, qkv, ld, seg, dy, lddy, nd, \
                       nlse2, dq_acc, nq32, dqkv, lddq, T, H, KV, window, dscale, scale, dmask, wpr, bpart, ldp,  \
                       rcos, rsin);                                                                             \
  } while (0)
#define FBH(D) if (hd == 64) FB(D, 64); else if (hd == 48) FB(D, 48); else FB(D, 32)
  if (mode == 2) { FBH(2); } else { FBH(0); }
#undef FBH
#undef FB
  cg_probe_end(CG_PROBE_ATTN_BWD, s, 5.0 * tri);  // S, dP recomputed + dV, dK, dQ
  CG_LAUNCH_CHECK();
  if (!rcos && H == KV) return CG_OK;  // MHA without RoPE: the last key block of each tile stored dQ
  const float qscale = mode ? scale * dscale : scale;
  const dim3 gf(B * H, cg_cdiv(T, 128));
  if (hd == 64)
    hipLaunchKernelGGL(attn_dq_finish_kernel<64>, gf, dim3(256), 0, s, dq_acc, nq32, dqkv, lddq, T, H, qscale, bpart,
                       ldp, rcos, rsin);
  else if (hd == 48)
    hipLaunchKernelGGL(attn_dq_finish_kernel<48>, gf, dim3(256), 0, s, dq_acc, nq32, dqkv, lddq, T, H, qscale, bpart,
                       ldp, rcos, rsin);
  else
    hipLaunchKernelGGL(attn_dq_finish_kernel<32>, gf, dim3(256), 0, s, dq_acc, nq32, dqkv, lddq, T, H, qscale, bpart,
                       ldp, rcos, rsin);
  CG_LAUNCH_CHECK();
  return CG_OK;
}

static inline int attn_bwd_mfma_launch(const bf16_t* qkv, long long ld, const int32_t* seg, const bf16_t* y,
                                       long long ldy, const bf16_t* dy, long long lddy, const float* lse,
                                       float* delta, bf16_t* dqkv, long long lddq, int B, int T, int H, int KV,
                                       int hd, int window, uint32_t seed, uint32_t thr, float dscale, float scale,
                                       const uint32_t* dmask, float* bpart, long long ldp, hipStream_t s,
                                       const float* rcos = nullptr, const float* rsin = nullptr, int algo = 0) {
  if (attn_bwd_fused_ok(algo, B, KV, thr ? (dmask ? 2 : 1) : 0))
    return attn_bwd_fused_launch(qkv, ld, seg, y, ldy, dy, lddy, lse, delta, dqkv, lddq, B, T, H, KV, hd, window,
                                 dscale, scale, thr ? dmask : nullptr, bpart, ldp, s, rcos, rsin);
  dim3 gq(B * H, cg_cdiv(T, 128));
  const int wpr = attn_drop_wpr(T);
  float* nlse2 = delta + (long long)B * H * T;  // second half of the workspace
  const int mode = thr ? (dmask ? 2 : 1) : 0;
  const double tri = 2.0 * (double)B * H * hd * ((double)T * (T + 1) / 2.0);
  // the K/V ring, or the bias-partial reduction buffer when it is larger
  const size_t shq = bpart ? std::max<size_t>(4 * fa::IMG, fa::COLSUM_LDS) : 4 * fa::IMG;
  cg_probe_begin(CG_PROBE_ATTN_DQ, s);
#define DQ(D, HDv)                                                                                             \
  hipLaunchKernelGGL((attn_bwd_dq_mfma<D, HDv>), gq, dim3(256), shq, s, qkv, ld, seg, dy, lddy, y, ldy, lse, \
                     delta, nlse2, dqkv, lddq, T, H, KV, hd, window, seed, thr, dscale, scale, dmask, wpr, bpart, ldp, \
                     rcos, rsin)
#define DQH(D) if (hd == 64) DQ(D, 64); else if (hd == 48) DQ(D, 48); else DQ(D, 32)
  if (mode == 2) { DQH(2); } else if (mode == 1) { DQH(1); } else { DQH(0); }
#undef DQH
#undef DQ
  cg_probe_end(CG_PROBE_ATTN_DQ, s, 3.0 * tri);  // S, dP recomputed + dQ
  CG_LAUNCH_CHECK();
  dim3 gk(B * KV, cg_cdiv(T, 128));
  const size_t shk = std::max<size_t>(3 * (2 * fa::IMG + 5 * 64 * 4 + (mode == 2 ? 4 * 64 * 4 : 0)),
                                      bpart ? fa::COLSUM_LDS : 0);
  cg_probe_begin(CG_PROBE_ATTN_DKDV, s);
#define DKDV(D, HDv)                                                                                            \
  hipLaunchKernelGGL((attn_bwd_dkdv_mfma<D, HDv>), gk, dim3(256), shk, s, qkv, ld, seg, dy, lddy, lse, delta, nlse2, dqkv, \
                     lddq, T, H, KV, hd, window, seed, thr, dscale, scale, dmask, wpr, bpart, ldp, rcos, rsin)
#define DKH(D) if (hd == 64) DKDV(D, 64); else if (hd == 48) DKDV(D, 48); else DKDV(D, 32)
  if (mode == 2) { DKH(2); } else if (mode == 1) { DKH(1); } else { DKH(0); }
#undef DKH
#undef DKDV
  cg_probe_end(CG_PROBE_ATTN_DKDV, s, 4.0 * tri);  // S, dP recomputed + dV, dK
  CG_LAUNCH_CHECK();
  return CG_OK;
}
