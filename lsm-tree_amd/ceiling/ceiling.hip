// ceiling.hip — measurement-only kernels (liblsmceiling.so, NOT part of the
// product library or its header): the practical HBM ceilings the bench
// reports next to the 8 TB/s spec peak.
//   lsm_ceiling_copy   16 B/lane streaming copy (read + write): one 8 KiB tile
//                      per workgroup, 2 loads per lane then 2 stores (the
//                      fastest of the variants in scripts/copy_ceiling_sweep.py:
//                      5.88 TB/s vs 4.77 for a 4-deep grid-stride loop and
//                      4.1 for 8 per lane): the R+W ceiling.
//   lsm_ceiling_read   the decode kernel's read shape alone: 4-wave
//                      workgroups (four per CU) stage consecutive 32 KiB spans
//                      into LDS by LDS-DMA, nothing computed: the read ceiling.
//   lsm_ceiling_soa    WRITE_SIZE calibration for the decode output: the parsed
//                      SoA (u64, 3 x u32, 2 x u16, u8 per item) written either
//                      as the decode kernel writes it (thread = item, 1-8 B
//                      per lane) or as 16 B/lane stores of the same arrays.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                   uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// One tile of K x 4 KiB per workgroup (K x 16 B per lane, all loads then all
// stores), grid = the whole buffer: no grid-stride loop.  mode bit 0:
// non-temporal loads, bit 1: non-temporal stores.
template <int K>
__global__ __launch_bounds__(256) void copy_tile_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                        uint64_t n16, int mode) {
  const uint64_t base = (uint64_t)blockIdx.x * (256 * K) + threadIdx.x;
  u32x4 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (base + 256 * k < n16) v[k] = (mode & 1) ? __builtin_nontemporal_load(src + base + 256 * k) : src[base + 256 * k];
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (base + 256 * k < n16) {
      if (mode & 2) __builtin_nontemporal_store(v[k], dst + base + 256 * k);
      else dst[base + 256 * k] = v[k];
    }
}

constexpr uint32_t kSpan = 32768;

__global__ __launch_bounds__(256) void read_kernel(const uint8_t* __restrict__ src, uint64_t bytes,
                                                   uint32_t spans_per_wg, uint32_t* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kSpan];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const uint32_t lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (uint32_t s = 0; s < spans_per_wg; ++s) {
    const uint64_t base = ((uint64_t)blockIdx.x * spans_per_wg + s) * kSpan;
    if (base >= bytes) break;
    const uint32_t chunks = (uint32_t)((bytes - base < kSpan ? bytes - base : kSpan) >> 4);
    for (uint32_t i = wave; i * 64 < chunks; i += 4)
      if (i * 64 + lane < chunks)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + base + 1024 * i + 16 * lane),
                                         (lds_void_t*)(stage + 1024 * i), 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0)
    __syncthreads();
    acc ^= reinterpret_cast<const uint32_t*>(stage)[threadIdx.x];
    __syncthreads();
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the reads live
}

// mode 0: thread = item, one store per field (the decode kernel's shape);
// mode 1: every array as 16 B/lane stores (same bytes).
__global__ __launch_bounds__(256) void soa_kernel(uint8_t* __restrict__ out, uint64_t n, int mode) {
  uint64_t* seq = (uint64_t*)out;
  uint32_t* ko = (uint32_t*)(out + 8 * n);
  uint32_t* vo = ko + n;
  uint32_t* vl = vo + n;
  uint16_t* kl = (uint16_t*)(vl + n);
  uint16_t* pl = kl + n;
  uint8_t* vt = (uint8_t*)(pl + n);
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (mode == 0) {
    if (i >= n) return;
    const uint32_t x = (uint32_t)i;
    seq[i] = i;
    ko[i] = x;
    vo[i] = x + 1;
    vl[i] = x + 2;
    kl[i] = (uint16_t)x;
    pl[i] = (uint16_t)(x + 3);
    vt[i] = (uint8_t)x;
  } else {
    const uint64_t n16 = 25 * n / 16;  // (n a multiple of 16)
    const u32x4 v = {(uint32_t)i, (uint32_t)i + 1, (uint32_t)i + 2, (uint32_t)i + 3};
    if (i < n16) reinterpret_cast<u32x4*>(out)[i] = v;
  }
}

// FETCH_SIZE / WRITE_SIZE calibration for the encode kernels' narrow access
// shapes (the guide calibrates only 16 B/lane streams): each mode touches a
// known number of distinct bytes of `buf` once, in one access shape.
//   0  u64 per lane, lane-contiguous                  (E2 item fields)
//   1  u64, lane t reads elements 2t, 2t+1, 2t+2      (E1 key / value offsets)
//   2  u64, lane t reads elements 2t, 2t+1            (E1 seqnos)
//   3  u8, lane t reads bytes 2t, 2t+1                (E1 value types)
//   4  u8 per lane, lane-contiguous                   (E2 value types)
//   5  u32 per lane, lane-contiguous                  (E2 erec)
//   6  16 B per lane, lane-contiguous                 (the guide's calibrated shape)
//   7  u32 stores, lane t writes elements 2t, 2t+1    (E1 erec)
//   8  u32 stores per lane, lane-contiguous
// n = elements of the mode's type; the sum goes to sink[0] (reads kept live).
__global__ __launch_bounds__(256) void fetch_calib_kernel(const uint8_t* __restrict__ buf, uint8_t* __restrict__ wbuf,
                                                          uint64_t n, int mode, uint32_t* __restrict__ sink) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t acc = 0;
  const uint64_t* b64 = reinterpret_cast<const uint64_t*>(buf);
  switch (mode) {
    case 0:
      if (t < n) acc = b64[t];
      break;
    case 1:
      if (2 * t < n) acc = b64[2 * t] + b64[min(2 * t + 1, n - 1)] + b64[min(2 * t + 2, n - 1)];
      break;
    case 2:
      if (2 * t < n) acc = b64[2 * t] + b64[min(2 * t + 1, n - 1)];
      break;
    case 3:
      if (2 * t < n) acc = buf[2 * t] + buf[min(2 * t + 1, n - 1)];
      break;
    case 4:
      if (t < n) acc = buf[t];
      break;
    case 5:
      if (t < n) acc = reinterpret_cast<const uint32_t*>(buf)[t];
      break;
    case 6:
      if (t < n) {
        const u32x4 v = reinterpret_cast<const u32x4*>(buf)[t];
        acc = v.x ^ v.y ^ v.z ^ v.w;
      }
      break;
    case 7:
      if (2 * t < n) {
        reinterpret_cast<uint32_t*>(wbuf)[2 * t] = (uint32_t)t;
        if (2 * t + 1 < n) reinterpret_cast<uint32_t*>(wbuf)[2 * t + 1] = (uint32_t)t + 1;
      }
      break;
    case 8:
      if (t < n) reinterpret_cast<uint32_t*>(wbuf)[t] = (uint32_t)t;
      break;
  }
  if (acc == 0x9E3779B97F4A7C15ULL) sink[0] = (uint32_t)acc;  // keeps the reads live
}

}  // namespace

extern "C" int lsm_ceiling_fetch_calib(const void* buf, void* wbuf, uint64_t n, int mode, uint32_t* sink, void* stream) {
  const uint64_t threads = (mode == 1 || mode == 2 || mode == 3 || mode == 7) ? (n + 1) / 2 : n;
  hipLaunchKernelGGL(fetch_calib_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)buf, (uint8_t*)wbuf, n, mode, sink);
  return hipGetLastError() == hipSuccess ? 0 : 11;
}

extern "C" int lsm_ceiling_soa(void* out, uint64_t n_items, int mode, void* stream) {
  if (((uintptr_t)out & 15) || (n_items & 15)) return 10;
  const uint64_t threads = mode == 0 ? n_items : 25 * n_items / 16;
  hipLaunchKernelGGL(soa_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t*)out, n_items, mode);
  return hipGetLastError() == hipSuccess ? 0 : 11;
}

extern "C" int lsm_ceiling_copy_variant(const void* src, void* dst, uint64_t bytes, int variant, void* stream) {
  if (((uintptr_t)src | (uintptr_t)dst | bytes) & 15) return 10;
  const uint64_t n16 = bytes / 16;
  if (variant == 0)
    hipLaunchKernelGGL(copy_kernel, dim3(256 * 8), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src,
                       (u32x4*)dst, n16);
  else if (variant <= 4)  // 1..4: mode = variant - 1, 4 per lane
    hipLaunchKernelGGL(copy_tile_kernel<4>, dim3((unsigned)((n16 + 1023) / 1024)), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)src, (u32x4*)dst, n16, variant - 1);
  else if (variant <= 8)  // 5..8: mode = variant - 5, 8 per lane
    hipLaunchKernelGGL(copy_tile_kernel<8>, dim3((unsigned)((n16 + 2047) / 2048)), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)src, (u32x4*)dst, n16, variant - 5);
  else  // 9..12: 2 per lane
    hipLaunchKernelGGL(copy_tile_kernel<2>, dim3((unsigned)((n16 + 511) / 512)), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)src, (u32x4*)dst, n16, variant - 9);
  return hipGetLastError() == hipSuccess ? 0 : 11;
}

extern "C" int lsm_ceiling_copy(const void* src, void* dst, uint64_t bytes, void* stream) {
  return lsm_ceiling_copy_variant(src, dst, bytes, 9, stream);  // the fastest of scripts/copy_ceiling_sweep.py
}

extern "C" int lsm_ceiling_read(const void* src, uint64_t bytes, uint32_t* sink, void* stream) {
  if (((uintptr_t)src | bytes) & 15) return 10;
  const uint32_t spans_per_wg = 48 * 4096 / kSpan;  // the decode kernel's 48 blocks of 4 KiB per workgroup
  const uint64_t spans = (bytes + kSpan - 1) / kSpan;
  const uint32_t grid = (uint32_t)((spans + spans_per_wg - 1) / spans_per_wg);
  hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)src, bytes,
                     spans_per_wg, sink);
  return hipGetLastError() == hipSuccess ? 0 : 11;
}
