// Per-CU operand-fetch bandwidth on gfx950: LDS-DMA (buffer_load_dwordx4 ... lds, the GEMM ring's
// path) vs buffer_load_dwordx4 into VGPRs.  Every workgroup (one per CU, 512 threads) streams the
// same REGION bytes in 64-KiB chunks, PASSES times; 16 B per lane per instruction.  REGION 64 KiB
// keeps part of it in the CU's L1; 2 MiB is L2-resident only.  STRIDE > 0 reads each 1-KiB DMA
// piece as 8 rows of 128 B STRIDE bytes apart (a 256x128 GEMM tile's rows at K = STRIDE / 2).
//   hipcc --offload-arch=gfx950 -O3 -DREGION_KB=2048 -o l2bw tools/l2bw.hip && ./l2bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
#ifndef REGION_KB
#define REGION_KB 64
#endif
#ifndef STRIDE
#define STRIDE 0
#endif
constexpr int CHUNK = 64 * 1024, REGION = REGION_KB * 1024, NCH = REGION / CHUNK;
constexpr int PASSES = 400 * 64 / REGION_KB > 4 ? 400 * 64 / REGION_KB : 4, THREADS = 512;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}
// byte offset of lane `lane`'s 16 B in 1-KiB piece p of chunk c
__device__ __forceinline__ uint32_t src_off(int c, int p, int lane) {
  if (STRIDE == 0) return (uint32_t)(c * CHUNK + p * 1024 + 16 * lane);
  // piece p = 8 rows x 128 B: rows (p * 8 + lane / 8) at STRIDE apart, 16 B column lane % 8
  const int row = p * 8 + (lane >> 3);
  return (uint32_t)(((long long)c * 64 * 8 * 128 / 128 * 0 + (long long)(c * 64 * 8 + row) * STRIDE + 16 * (lane & 7)) % REGION);
}
__device__ __forceinline__ u4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  u4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
  return v;
}

// VGPR loads: 8 per batch per wave (one 64-KiB chunk per workgroup batch), two batches in flight
__global__ __launch_bounds__(THREADS, 1) void vgpr_kernel(const char* src, uint32_t* out, long long* clk) {
  const __amdgpu_buffer_rsrc_t r = rsrc(src, REGION);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  u4 a[8], b[8];
  uint32_t x = 0;
  const long long t0 = clock64(), w0 = wall_clock64();
  int c = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = ld16(r, src_off(c, j * 8 + wave, lane));
  for (int it = 0; it < PASSES * NCH; it += 2) {
    c = (it + 1) % NCH;
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = ld16(r, src_off(c, j * 8 + wave, lane));
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#pragma unroll
    for (int j = 0; j < 8; ++j) x ^= a[j][0] ^ a[j][3];
    c = (it + 2) % NCH;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = ld16(r, src_off(c, j * 8 + wave, lane));
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#pragma unroll
    for (int j = 0; j < 8; ++j) x ^= b[j][0] ^ b[j][3];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < 8; ++j) x ^= a[j][1];
  const long long t1 = clock64(), w1 = wall_clock64();
  if (x == 0x12345678u) out[tid] = x;
  if (tid == 0) {
    clk[blockIdx.x] = t1 - t0;
    clk[gridDim.x + blockIdx.x] = w1 - w0;
  }
}

// LDS-DMA: the same bytes into a 64 KiB LDS ring, 8-16 pieces per wave in flight
__global__ __launch_bounds__(THREADS, 1) void dma_kernel(const char* src, uint32_t* out, long long* clk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const __amdgpu_buffer_rsrc_t r = rsrc(src, REGION);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long t0 = clock64(), w0 = wall_clock64();
  for (int it = 0; it < PASSES * NCH; ++it) {
    const int c = it % NCH;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int piece = j * 8 + wave;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(smem + piece * 1024), 16, src_off(c, piece, lane), 0,
                                               0, 0);
    }
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const long long t1 = clock64(), w1 = wall_clock64();
  if (tid == 0) {
    clk[blockIdx.x] = t1 - t0;
    clk[gridDim.x + blockIdx.x] = w1 - w0;
  }
  if (smem[tid] == 123) out[tid] = 1;
}

int main() {
  int cus = 0, wrate = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipDeviceGetAttribute(&wrate, hipDeviceAttributeWallClockRate, 0);  // kHz
  char* src;
  uint32_t* out;
  long long* clk;
  (void)hipMalloc(&src, REGION);
  (void)hipMemset(src, 1, REGION);
  (void)hipMalloc(&out, THREADS * 4);
  (void)hipMalloc(&clk, 2 * cus * sizeof(long long));
  (void)hipFuncSetAttribute((const void*)dma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, CHUNK);
  printf("region %d KiB, stride %d, %d passes\n", REGION_KB, STRIDE, PASSES);
  for (int rep = 0; rep < 3; ++rep) {
    for (int k = 0; k < 2; ++k) {
      if (k == 0) hipLaunchKernelGGL(vgpr_kernel, dim3(cus), dim3(THREADS), 0, 0, src, out, clk);
      else hipLaunchKernelGGL(dma_kernel, dim3(cus), dim3(THREADS), CHUNK, 0, src, out, clk);
      (void)hipDeviceSynchronize();
      long long c[2048];
      (void)hipMemcpy(c, clk, 2 * cus * sizeof(long long), hipMemcpyDeviceToHost);
      double cmax = 0, wmax = 0;
      for (int i = 0; i < cus; ++i) {
        cmax = c[i] > cmax ? c[i] : cmax;
        wmax = c[cus + i] > wmax ? c[cus + i] : wmax;
      }
      const double bytes = (double)REGION * PASSES;  // per CU
      const double secs = wmax / (wrate * 1e3), ghz = cmax / secs / 1e9;
      printf("%-5s in-kernel %8.1f us  %6.1f GB/s per CU  clock %.2f GHz  %5.1f B/clk per CU  (chip %.1f TB/s)\n",
             k ? "dma" : "vgpr", secs * 1e6, bytes / secs / 1e9, ghz, bytes / cmax, bytes * cus / secs / 1e12);
    }
  }
  return 0;
}
