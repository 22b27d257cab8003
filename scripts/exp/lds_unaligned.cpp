// Experiment (not product code): do ds_write_b32 / ds_read_b32 at byte-unaligned
// LDS addresses store / load the right 4 bytes on gfx950, and what do they cost?
// Lane t writes K dwords at 71 t + 4 k + off (records ~71 B apart, as the encode
// record writer would), then reads them back; timed per offset 0..3 and checked
// against a host reference (the bytes between the records must stay untouched).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kWG = 256, K = 16, kMaxStride = 72;
constexpr int kLds = kWG * kMaxStride + 64;

__global__ __launch_bounds__(kWG) void wr(uint32_t kStride, uint32_t off, int iters, uint8_t* out, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
  const int t = threadIdx.x;
  for (int i = t; i < kLds; i += kWG) lds[i] = 0xEE;
  __syncthreads();
  uint32_t acc = 0;
  const uint32_t base = kStride * t + off;
  for (int it = 0; it < iters; ++it) {
    const uint32_t a0 = (uint32_t)(uintptr_t)lds + base;
#pragma unroll
    for (int k = 0; k < K; ++k)
      asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(a0), "v"((uint32_t)(t * 0x01010101u + k + it)), "i"(4 * k)
                   : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r[k]) : "v"(a0), "i"(4 * k) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < K; ++k) acc += r[k];
  }
  __syncthreads();
  sink[blockIdx.x * kWG + t] = acc;
  if (blockIdx.x == 0)
    for (int i = t; i < kLds; i += kWG) out[i] = lds[i];
}

int main() {
  uint8_t* dout; uint32_t* dsink;
  const int grid = 256 * 4, iters = 256;
  (void)hipMalloc(&dout, kLds); (void)hipMalloc(&dsink, 4 * grid * kWG);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const uint32_t cases[][2] = {{72, 0}, {72, 1}, {72, 2}, {72, 3}, {71, 0}, {68, 0}, {68, 1}, {64, 0}, {64, 1}};
  for (int rep = 0; rep < 2; ++rep)
    for (auto& c : cases) {
      const uint32_t stride = c[0], off = c[1];
      hipLaunchKernelGGL(wr, dim3(grid), dim3(kWG), 0, 0, stride, off, 1, dout, dsink);
      (void)hipDeviceSynchronize();
      std::vector<uint8_t> o(kLds);
      (void)hipMemcpy(o.data(), dout, kLds, hipMemcpyDeviceToHost);
      std::vector<uint8_t> ref(kLds, 0xEE);
      for (int t = 0; t < kWG; ++t)
        for (int k = 0; k < K; ++k) {
          const uint32_t v = (uint32_t)(t * 0x01010101u + k + 0);
          for (int b = 0; b < 4; ++b) ref[stride * t + off + 4 * k + b] = (uint8_t)(v >> (8 * b));
        }
      int bad = 0;
      for (int i = 0; i < kLds; ++i) bad += o[i] != ref[i];
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(wr, dim3(grid), dim3(kWG), 0, 0, stride, off, iters, dout, dsink);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      const double winstr = 2.0 * grid * (kWG / 64) * K * iters;  // wave-instructions (writes + reads)
      printf("stride %u off %u: %8.3f ms  %6.2f CU-cycles per wave-instr  %s (%d bytes differ)\n", stride, off, ms,
             ms * 1e-3 * 2.4e9 * 256 / winstr, bad ? "WRONG" : "ok", bad);
    }
  return 0;
}
