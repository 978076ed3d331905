// Per-CU operand-fetch bandwidth from L2 on gfx950: LDS-DMA (buffer_load_dwordx4 ... lds, the GEMM
// ring's path) vs buffer_load_dwordx4 into VGPRs.  Every workgroup (one per CU, 512 threads) streams
// the same 64 KiB region (L2-resident, L1 too small to hold it) ITERS times; 16 B per lane per
// instruction.  Prints GB/s per CU and B/clk at the measured clock.
//   hipcc --offload-arch=gfx950 -O3 -o l2bw tools/l2bw.hip && ./l2bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((address_space(3))) void* lds_ptr_t;
constexpr int REGION = 64 * 1024, ITERS = 400, THREADS = 512;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}

// VGPR loads: each wave keeps 8 loads in flight
__global__ __launch_bounds__(THREADS, 1) void vgpr_kernel(const char* src, uint32_t* out, long long* clk) {
  const __amdgpu_buffer_rsrc_t r = rsrc(src, REGION);
  const int tid = threadIdx.x;
  uint32_t x = 0;
  const long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < REGION / (THREADS * 16); ++j) {
      const uint32_t off = (uint32_t)((j * THREADS + tid) * 16);
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
      x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
  }
  const long long t1 = clock64();
  if (x == 0x12345678u) out[tid] = x;
  if (tid == 0) clk[blockIdx.x] = t1 - t0;
}

// LDS-DMA: the same bytes into a 64 KiB LDS ring, 8 instructions per wave in flight
__global__ __launch_bounds__(THREADS, 1) void dma_kernel(const char* src, uint32_t* out, long long* clk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const __amdgpu_buffer_rsrc_t r = rsrc(src, REGION);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < REGION / (THREADS * 16); ++j) {
      const int piece = j * (THREADS / 64) + wave;  // 1 KiB pieces
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(smem + piece * 1024), 16,
                                               (uint32_t)(piece * 1024 + 16 * lane), 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const long long t1 = clock64();
  if (tid == 0) clk[blockIdx.x] = t1 - t0;
  if (smem[tid] == 123) out[tid] = 1;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  char* src;
  uint32_t* out;
  long long* clk;
  hipMalloc(&src, REGION);
  hipMemset(src, 1, REGION);
  hipMalloc(&out, THREADS * 4);
  hipMalloc(&clk, cus * sizeof(long long));
  hipFuncSetAttribute((const void*)dma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, REGION);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    for (int k = 0; k < 2; ++k) {
      hipEventRecord(a);
      if (k == 0) hipLaunchKernelGGL(vgpr_kernel, dim3(cus), dim3(THREADS), 0, 0, src, out, clk);
      else hipLaunchKernelGGL(dma_kernel, dim3(cus), dim3(THREADS), REGION, 0, src, out, clk);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      long long c[1024];
      hipMemcpy(c, clk, cus * sizeof(long long), hipMemcpyDeviceToHost);
      double cmax = 0;
      for (int i = 0; i < cus; ++i) cmax = c[i] > cmax ? c[i] : cmax;
      const double bytes = (double)REGION * ITERS;  // per CU
      printf("%-5s %7.3f ms  %6.1f GB/s per CU  %5.1f B/clk (clock64 %.0f cycles)\n", k ? "dma" : "vgpr", ms,
             bytes / (ms * 1e-3) / 1e9, bytes / cmax, cmax);
    }
  }
  return 0;
}
