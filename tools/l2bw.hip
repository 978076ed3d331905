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

// VGPR loads (inline asm, so none is merged or hoisted): 8 per batch per wave, two batches in
// flight, each consumed after the next batch is issued (counted vmcnt)
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  u4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
  return v;
}
__global__ __launch_bounds__(THREADS, 1) void vgpr_kernel(const char* src, uint32_t* out, long long* clk) {
  const __amdgpu_buffer_rsrc_t r = rsrc(src, REGION);
  const int tid = threadIdx.x;
  constexpr int NB = REGION / (THREADS * 16);  // 8 loads per batch = the whole region
  u4 a[NB], b[NB];
  uint32_t x = 0;
  const long long t0 = clock64(), w0 = wall_clock64();
#pragma unroll
  for (int j = 0; j < NB; ++j) a[j] = ld16(r, (uint32_t)((j * THREADS + tid) * 16));
  for (int it = 0; it < ITERS; it += 2) {
#pragma unroll
    for (int j = 0; j < NB; ++j) b[j] = ld16(r, (uint32_t)((j * THREADS + tid) * 16));
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#pragma unroll
    for (int j = 0; j < NB; ++j) x ^= a[j][0] ^ a[j][3];
#pragma unroll
    for (int j = 0; j < NB; ++j) a[j] = ld16(r, (uint32_t)((j * THREADS + tid) * 16));
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#pragma unroll
    for (int j = 0; j < NB; ++j) x ^= b[j][0] ^ b[j][3];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < NB; ++j) x ^= a[j][1];
  const long long t1 = clock64(), w1 = wall_clock64();
  if (tid == 0) clk[gridDim.x + blockIdx.x] = w1 - w0;
  if (x == 0x12345678u) out[tid] = x;
  if (tid == 0) clk[blockIdx.x] = t1 - t0;
}

// LDS-DMA: the same bytes into a 64 KiB LDS ring, 8 instructions per wave in flight
__global__ __launch_bounds__(THREADS, 1) void dma_kernel(const char* src, uint32_t* out, long long* clk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const __amdgpu_buffer_rsrc_t r = rsrc(src, REGION);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long t0 = clock64(), w0 = wall_clock64();
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
  const long long t1 = clock64(), w1 = wall_clock64();
  if (tid == 0) clk[gridDim.x + blockIdx.x] = w1 - w0;
  if (tid == 0) clk[blockIdx.x] = t1 - t0;
  if (smem[tid] == 123) out[tid] = 1;
}

// mixed: per step each wave loads 4 KiB into VGPRs (the A fragments of a 32-row x 64-k slice, kept
// two steps ahead) and issues 2 KiB of LDS-DMA (its share of a 128 x 64 B tile): 48 KiB per
// workgroup step, as the 256x128x64 GEMM k-step
__global__ __launch_bounds__(THREADS, 1) void mixed_kernel(const char* src, uint32_t* out, long long* clk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const __amdgpu_buffer_rsrc_t r = rsrc(src, REGION);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  uint32_t x = 0;
  u4 a[4], b[4];
  constexpr int STEPS = ITERS * REGION / (48 * 1024);
  auto aoff = [&](int it, int j) { return (uint32_t)(16384 + (j * 8 + wave) * 1024 + 16 * lane) + 0u * it; };
  auto dma = [&](int it) {
    const uint32_t base = 0u * it;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int piece = j * 8 + wave;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(smem + (it & 1) * 16384 + piece * 1024), 16,
                                               base + (uint32_t)(piece * 1024 + 16 * lane), 0, 0, 0);
    }
  };
  const long long t0 = clock64(), w0 = wall_clock64();
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = ld16(r, aoff(0, j));
  dma(0);
  for (int it = 0; it < STEPS; it += 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = ld16(r, aoff(it + 1, j));
    dma(it + 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
#pragma unroll
    for (int j = 0; j < 4; ++j) x ^= a[j][0] ^ a[j][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = ld16(r, aoff(it + 2, j));
    dma(it + 2);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
#pragma unroll
    for (int j = 0; j < 4; ++j) x ^= b[j][0] ^ b[j][3];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < 4; ++j) x ^= a[j][1];
  const long long t1 = clock64(), w1 = wall_clock64();
  if (tid == 0) clk[gridDim.x + blockIdx.x] = w1 - w0;
  if (x == 0x12345678u) out[tid] = x;
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
  hipMalloc(&clk, 2 * cus * sizeof(long long));
  hipFuncSetAttribute((const void*)dma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, REGION);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    for (int k = 0; k < 3; ++k) {
      hipEventRecord(a);
      if (k == 0) hipLaunchKernelGGL(vgpr_kernel, dim3(cus), dim3(THREADS), 0, 0, src, out, clk);
      else if (k == 1) hipLaunchKernelGGL(dma_kernel, dim3(cus), dim3(THREADS), REGION, 0, src, out, clk);
      else hipLaunchKernelGGL(mixed_kernel, dim3(cus), dim3(THREADS), REGION, 0, src, out, clk);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      long long c[2048];
      hipMemcpy(c, clk, 2 * cus * sizeof(long long), hipMemcpyDeviceToHost);
      double cmax = 0, wmax = 0;
      for (int i = 0; i < cus; ++i) {
        cmax = c[i] > cmax ? c[i] : cmax;
        wmax = c[cus + i] > wmax ? c[cus + i] : wmax;
      }
      int wrate = 0;
      hipDeviceGetAttribute(&wrate, hipDeviceAttributeWallClockRate, 0);  // kHz
      const double bytes = (double)REGION * ITERS;  // per CU
      const char* name = k == 0 ? "vgpr" : k == 1 ? "dma" : "mixed";
      const double secs = wmax / (wrate * 1e3), ghz = cmax / secs / 1e9;
      printf("%-5s %7.3f ms  in-kernel %7.1f us  %6.1f GB/s per CU  clock64 %.2f GHz  %5.1f B/clock64-cycle\n",
             name, ms, secs * 1e6, bytes / secs / 1e9, ghz, bytes / cmax);
      (void)name;
    }
  }
  return 0;
}
