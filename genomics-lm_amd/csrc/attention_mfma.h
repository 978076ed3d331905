// bf16 MFMA flash-attention kernels (gfx950).  Included by attention.hip.
#pragma once

static inline bool attn_mfma_supported(int hd, long long ld_in, long long ld_out) {
  (void)hd; (void)ld_in; (void)ld_out;
  return false;  // enabled once the MFMA kernels land
}

static inline int attn_fwd_mfma_launch(const bf16_t*, long long, const int32_t*, bf16_t*, long long, float*, int, int,
                                       int, int, int, int, uint32_t, uint32_t, float, float, hipStream_t) {
  return CG_EUNSUPPORTED;
}
static inline int attn_bwd_mfma_launch(const bf16_t*, long long, const int32_t*, const bf16_t*, long long,
                                       const float*, const float*, bf16_t*, long long, int, int, int, int, int, int,
                                       uint32_t, uint32_t, float, float, hipStream_t) {
  return CG_EUNSUPPORTED;
}
