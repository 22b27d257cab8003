// lds_dma.hpp — LDS-DMA issue (global_load_lds_*) and counted vmcnt waits for
// loader waves on gfx950.
//
// The DMA is inline asm on purpose: hipcc's waitcnt pass drains an LDS-DMA it
// knows about (vmcnt(0)) before every later LDS access of the issuing wave,
// which would serialise a loader that polls LDS flags between issues.  Asm
// loads are invisible to that pass, so the issuing wave counts them itself
// (vm_wait_n) — cdna_hip_programming.md, "LDS-DMA recipe".
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lsmgpu {

// 16 bytes per lane HBM -> LDS (M0 = wave-uniform LDS base; lane l lands at +16 l).
// Inline asm so the compiler neither drains it nor counts it: the loader
// waits for it with its own counted vmcnt (cdna_hip_programming.md, LDS-DMA recipe).
template <bool kNt>
__device__ __forceinline__ void dma16(const uint8_t* src, uint32_t lds_dst) {
  uint32_t keep;
  if constexpr (kNt)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
}
// Same, global address = SGPR-pair base + per-lane VGPR offset (saddr form):
// stepping through a span costs SALU adds only.  The base may come straight
// from v_readfirstlane/v_readlane (a VALU write of an SGPR), which a VMEM
// instruction may read as its base only 5 wait states later: s_nop 4.
template <bool kNt>
__device__ __forceinline__ void dma16s(uint32_t voff, uint64_t sbase, uint32_t lds_dst) {
  uint32_t keep;
  if constexpr (kNt)
    asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_dst) : "memory");
  else
    asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void dma4(const uint8_t* src, uint32_t lds_dst) {  // 4 bytes per lane
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// s_waitcnt vmcnt(n) for a run-time n (clamped to 63: loads retire in order,
// so <= 63 outstanding also means every older load has landed).
__device__ __forceinline__ void vm_wait_n(uint32_t n) {
  n = n > 63 ? 63 : n;
  switch (n) {
#define LSM_VMW(i) case i: vm_wait<i>(); break;
#define LSM_VMW8(i) LSM_VMW(i) LSM_VMW(i + 1) LSM_VMW(i + 2) LSM_VMW(i + 3) LSM_VMW(i + 4) LSM_VMW(i + 5) LSM_VMW(i + 6) LSM_VMW(i + 7)
    LSM_VMW8(0) LSM_VMW8(8) LSM_VMW8(16) LSM_VMW8(24) LSM_VMW8(32) LSM_VMW8(40) LSM_VMW8(48) LSM_VMW8(56)
#undef LSM_VMW8
#undef LSM_VMW
    default: vm_wait<0>();
  }
}


}  // namespace lsmgpu
