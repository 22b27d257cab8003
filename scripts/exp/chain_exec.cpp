// Experiment (not product code): does the XXH3 scramble step run faster when
// only lanes 0..7 of the wave are active (exec = 0xFF) than with all 64 lanes
// active?  One wave per workgroup, N dependent steps, contributions from
// registers (no memory in the loop); cycles per step from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint32_t P32_1 = 0x9E3779B1U;

template <int kLanes>
__global__ __launch_bounds__(64) void chain_exec(uint64_t n, uint64_t* out, uint64_t* cycles) {
  const uint32_t lane = threadIdx.x;
  const uint64_t s = 0x1234567890ABCDEFULL + lane;
  const uint32_t s_lo = (uint32_t)s, s_hi = (uint32_t)(s >> 32);
  const uint32_t p1 = __builtin_amdgcn_readfirstlane(P32_1);
  uint64_t y = lane + __builtin_amdgcn_mbcnt_lo(0, 0);
  uint64_t cn = 0x9E3779B185EBCA87ULL ^ lane;
  uint64_t t0 = 0, t1 = 0;
  if (lane < (uint32_t)kLanes) {
    t0 = __builtin_amdgcn_s_memtime();
    for (uint64_t i = 0; i < n; ++i) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const uint32_t hi = (uint32_t)(y >> 32);
        const uint32_t lo = (uint32_t)y ^ (hi >> 15) ^ s_lo;
        uint32_t hm;
        asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(hm) : "v"(hi ^ s_hi), "s"(p1));
        const uint64_t add = ((uint64_t)(hm + (uint32_t)(cn >> 32)) << 32) | (uint32_t)cn;
        uint64_t cc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(y), "=s"(cc) : "v"(lo), "s"(p1), "v"(add));
        cn += 0x1111;
      }
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  if (lane < (uint32_t)kLanes) out[blockIdx.x * 64 + lane] = y;
  if (lane == 0) cycles[blockIdx.x] = t1 - t0;
}

int main() {
  uint64_t *out, *cyc;
  hipMalloc(&out, 1024 * 64 * 8);
  hipMalloc(&cyc, 1024 * 8);
  const uint64_t n = 4096;  // x16 steps
  auto run = [&](auto kern, const char* name, int grid) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, n, out, cyc);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, n, out, cyc);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    uint64_t c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // s_memtime counts at the shader clock on gfx9 (100 MHz constant clock on some parts: print both)
    printf("%-10s grid %4d: %.3f ms, %.2f ns/step, memtime/step %.2f\n", name, grid, ms, ms * 1e6 / (n * 16),
           (double)c / (n * 16));
  };
  for (int g : {1, 256, 1024}) {
    run(chain_exec<64>, "lanes64", g);
    run(chain_exec<8>, "lanes8", g);
    run(chain_exec<16>, "lanes16", g);
    run(chain_exec<1>, "lanes1", g);
  }
  return 0;
}
