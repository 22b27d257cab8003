// Experiment (not product code): the encode record writer's value copy
// (LDS stage -> LDS image, lane = record, 64 B values at a 64 B source
// stride, destinations ~72-86 B apart at every byte alignment), timed at
// the group kernel's occupancy (4 workgroups x 4 waves per CU), several ways:
//   0 rot-wrap   the round-2 loop (32 rotation starts, wrap test per dword)
//   1 two-runs   rotation as two linear runs, 4 dwords per step
//   2 mskor      branch-free: every dest dword via ds_mskor_b32 (edges masked)
//   3 ub128      unaligned ds_read_b128 / ds_write_b128 (4-byte aligned) + alignbyte
//   4 plain      no rotation, linear 4-dword steps (conflicted source)
// Each variant's image is checked against a host reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kWG = 256, kRec = 256, kVal = 64;
constexpr int kStage = kRec * kVal + 64;     // 16 KiB of values
constexpr int kImg = kRec * 96 + 64;         // record slots

__device__ __forceinline__ uint32_t ab(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }

__device__ __forceinline__ void mskor(uint32_t addr, uint32_t mask, uint32_t data) {
  asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(addr), "v"(mask), "v"(data) : "memory");
}

template <int V>
__device__ __forceinline__ void copy(uint8_t* dst, uint32_t d, const uint8_t* src, uint32_t s, uint32_t n, uint32_t rot) {
  if (V == 0 || V == 1 || V == 4) {
    const uint32_t h = min(n, (4u - (d & 3u)) & 3u);
    uint32_t hb[3];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (k < h) hb[k] = src[s + k];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (k < h) dst[d + k] = (uint8_t)hb[k];
    if (n == h) return;
    const uint32_t d1 = d + h, e = d + n, body = ((e & ~3u) - d1) >> 2;
    const uint32_t sp = s + h, sh = sp & 3u;
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src + (sp & ~3u));
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + d1);
    if (V == 0) {
      uint32_t q = ((rot & 31u) * body) >> 5;
      const uint32_t w0 = body ? s32[0] : 0;
      uint32_t carry = body ? s32[q] : 0;
      for (uint32_t j0 = 0; j0 < body; j0 += 4) {
        uint32_t hi[4], at[4];
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) { uint32_t p = q + t; p = p >= body ? p - body : p; at[t] = p; if (j0 + t < body) hi[t] = s32[p + 1]; }
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) if (j0 + t < body) { const uint32_t lo = t == 0 ? carry : (at[t] == 0 ? w0 : hi[t - 1]); d32[at[t]] = ab(hi[t], lo, sh); }
        q += 4; q = q >= body ? q - body : q; carry = q == 0 ? w0 : hi[3];
      }
    } else {
      auto run = [&](uint32_t p, uint32_t p1) {
        if (p >= p1) return;
        uint32_t carry = s32[p];
        for (; p + 4 <= p1; p += 4) {
          const uint32_t w1 = s32[p + 1], w2 = s32[p + 2], w3 = s32[p + 3], w4 = s32[p + 4];
          d32[p] = ab(w1, carry, sh); d32[p + 1] = ab(w2, w1, sh); d32[p + 2] = ab(w3, w2, sh); d32[p + 3] = ab(w4, w3, sh);
          carry = w4;
        }
        if (p < p1) {
          const uint32_t w1 = s32[p + 1], w2 = s32[p + 2], w3 = s32[p + 3];
          d32[p] = ab(w1, carry, sh);
          if (p + 1 < p1) d32[p + 1] = ab(w2, w1, sh);
          if (p + 2 < p1) d32[p + 2] = ab(w3, w2, sh);
        }
      };
      const uint32_t q = V == 1 ? ((rot & 31u) * body) >> 5 : 0;
      run(q, body);
      run(0, q);
    }
    const uint32_t t0 = d1 + 4 * body;
    uint32_t tb[3];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (t0 + k < e) tb[k] = src[s + (t0 + k - d)];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (t0 + k < e) dst[t0 + k] = (uint8_t)tb[k];
  } else if (V == 2) {
    // dest dwords D0 .. D1 (inclusive); dest dword j holds src bytes s + 4j - d .. +4
    // (source dword index relative to floor((s - (d & 3)) / 4)); edges masked, all via mskor
    if (!n) return;
    const uint32_t D0 = d >> 2, D1 = (d + n - 1) >> 2, cnt = D1 - D0 + 1;
    const int32_t sb = (int32_t)s - (int32_t)(d & 3u);  // source byte of dest byte 4*D0
    const uint32_t sh = (uint32_t)sb & 3u;
    const int32_t sw = sb >> 2;                          // (may be -1: reads the dword before, masked)
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
    const uint32_t first_mask = 0xFFFFFFFFu << (8 * (d & 3u));
    const uint32_t end = (d + n) & 3u;
    const uint32_t last_mask = end ? 0xFFFFFFFFu >> (8 * (4 - end)) : 0xFFFFFFFFu;
    const uint32_t q = ((rot & 31u) * cnt) >> 5;
    auto run = [&](uint32_t p, uint32_t p1) {
      if (p >= p1) return;
      uint32_t carry = s32[sw + (int32_t)p];
      for (; p < p1; p += 4) {
        uint32_t w[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) w[t] = s32[sw + (int32_t)p + 1 + t];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t j = p + t;
          uint32_t m = j < p1 ? 0xFFFFFFFFu : 0u;
          if (j == 0) m &= first_mask;
          if (j == cnt - 1) m &= last_mask;
          const uint32_t v = ab(w[t], t ? w[t - 1] : carry, sh);
          mskor((uint32_t)(uintptr_t)dst + 4 * (D0 + j), m, v & m);
        }
        carry = w[3];
      }
    };
    run(q, cnt);
    run(0, q);
  } else if (V == 3) {
    // unaligned b128: dest dwords from d1 (4-aligned) in 16-byte pieces, 4-aligned b128 reads + carry
    const uint32_t h = min(n, (4u - (d & 3u)) & 3u);
    for (uint32_t k = 0; k < h; ++k) dst[d + k] = src[s + k];
    if (n == h) return;
    const uint32_t d1 = d + h, e = d + n, body = ((e & ~3u) - d1) >> 2;
    const uint32_t sp = s + h, sh = sp & 3u;
    const uint8_t* sa = src + (sp & ~3u);
    uint8_t* da = dst + d1;
    uint32_t p = 0;
    for (; p + 4 <= body; p += 4) {
      const u32x4 a = *reinterpret_cast<const u32x4*>(sa + 4 * p);  // 4-byte aligned
      const uint32_t x = *reinterpret_cast<const uint32_t*>(sa + 4 * p + 16);
      u32x4 o;
      o.x = ab(a.y, a.x, sh); o.y = ab(a.z, a.y, sh); o.z = ab(a.w, a.z, sh); o.w = ab(x, a.w, sh);
      *reinterpret_cast<u32x4*>(da + 4 * p) = o;
    }
    for (; p < body; ++p)
      *reinterpret_cast<uint32_t*>(da + 4 * p) = ab(*reinterpret_cast<const uint32_t*>(sa + 4 * p + 4), *reinterpret_cast<const uint32_t*>(sa + 4 * p), sh);
    for (uint32_t k = d1 + 4 * body; k < e; ++k) dst[k] = src[s + (k - d)];
  }
}


typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;
__device__ __forceinline__ void lds_or(uint32_t addr, uint32_t v) {
  asm volatile("ds_or_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
// up to 15 bytes b[0..n) (little-endian in w, bytes >= n zeroed by the caller) ORed at LDS byte address a
__device__ __forceinline__ void or_piece16(uint32_t a, u32x4 w) {
  const uint32_t s = a & 3u, base = a & ~3u;
  const uint32_t z = 0;
  lds_or(base, s ? w.x << (8 * s) : w.x);
  lds_or(base + 4, ab(w.y, w.x, 4 - s) * (s != 0) | (s ? 0u : w.y));
  lds_or(base + 8, s ? ab(w.z, w.y, 4 - s) : w.z);
  lds_or(base + 12, s ? ab(w.w, w.z, 4 - s) : w.w);
  lds_or(base + 16, s ? ab(z, w.w, 4 - s) : 0u);
}
__device__ __forceinline__ u32x4 mask_bytes(u32x4 w, uint32_t n) {  // keep bytes [0, n)
  auto m = [&](uint32_t i) { return n >= 4 * i + 4 ? 0xFFFFFFFFu : n <= 4 * i ? 0u : 0xFFFFFFFFu >> (8 * (4 * i + 4 - n)); };
  w.x &= m(0); w.y &= m(1); w.z &= m(2); w.w &= m(3);
  return w;
}
__device__ __forceinline__ u32x4 gload16(const uint8_t* p) { return *reinterpret_cast<const u32x4*>(p); }

template <int kMode>  // 5: map + DMA + or edges;  6: same without the DMA pass (edges only)
__global__ __launch_bounds__(kWG) void bench_dma(const uint8_t* vals, const uint32_t* dpos, uint8_t* out, int iters) {
  __shared__ __attribute__((aligned(16))) uint8_t img[kImg];
  __shared__ uint32_t map[kImg / 16];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t d = dpos[t];
  const uint8_t* src = vals + kVal * t;
  const uint32_t n = kVal;
  // this record's pieces: head [d, h1), interior chunks [c0, c1), tail [t0, e)
  const uint32_t e = d + n, h1 = min(e, (d + 15) & ~15u), c0 = (d + 15) >> 4, c1 = e >> 4;
  const uint32_t t0 = max(h1, e & ~15u);
  for (int it = 0; it < iters; ++it) {
    for (int i = t; i < kImg / 16; i += kWG) {
      reinterpret_cast<u32x4*>(img)[i] = u32x4{0, 0, 0, 0};
      map[i] = 0xFFFFFFFFu;
    }
    __syncthreads();
    // edges from global (in registers), interior chunk map entries
    const u32x4 hw = mask_bytes(gload16(src), h1 - d);
    const u32x4 tw = mask_bytes(gload16(src + (t0 - d)), e - t0);
    for (uint32_t c = c0; c < c1; ++c) map[c] = kVal * t + 16 * c - d;
    const uint32_t ib = (uint32_t)(uintptr_t)img;
    if (h1 > d) or_piece16(ib + d, hw);
    if (e > t0) or_piece16(ib + t0, tw);
    __syncthreads();
    if (kMode == 5) {
      for (uint32_t p = wave; p * 64 < kImg / 16; p += kWG / 64) {
        const uint32_t c = p * 64 + lane;
        const uint32_t m = c < kImg / 16 ? map[c] : 0xFFFFFFFFu;
        if (m != 0xFFFFFFFFu)
          __builtin_amdgcn_global_load_lds((gbl_void_t*)(vals + m), (lds_void_t*)(img + 1024 * p), 16, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0);
    }
    __syncthreads();
  }
  if (blockIdx.x == 0)
    for (int i = t; i < kImg; i += kWG) out[i] = img[i];
}


// 7: per-record LDS-DMA of the value's interior dwords (wave-uniform loop over the
// wave's 64 records, one global_load_lds_dword per record, unaligned global
// source), the <= 3 + 3 edge bytes as byte stores from two dword loads
__device__ __forceinline__ void dma4_m0(uint32_t voff_lo, uint32_t voff_hi, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, off\n\t" ::"v"(voff_lo), "v"(voff_hi), "s"(m0)
               : "memory");
}
template <int kMode>
__global__ __launch_bounds__(kWG) void bench_rec_dma(const uint8_t* vals, const uint32_t* dpos, uint8_t* out, int iters) {
  __shared__ __attribute__((aligned(16))) uint8_t img[kImg];
  const int t = threadIdx.x, lane = t & 63;
  const uint32_t d = dpos[t];
  const uint8_t* src = vals + kVal * t;
  const uint32_t n = kVal, e = d + n;
  const uint32_t i0 = (d + 3) & ~3u, i1 = e & ~3u;  // interior dwords [i0, i1)
  const uint32_t cnt = i1 > i0 ? (i1 - i0) >> 2 : 0;
  const uint32_t ib = (uint32_t)(uintptr_t)img;
  for (int it = 0; it < iters; ++it) {
    // edges: head bytes [d, i0), tail bytes [i1, e) (from unaligned dword loads)
    const uint32_t hv = *reinterpret_cast<const uint32_t*>(src);          // bytes 0..3
    const uint32_t tv = *reinterpret_cast<const uint32_t*>(src + n - 4);  // last 4 bytes
    const uint32_t nh = i0 - d, nt = e - i1;
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (k < nh) img[d + k] = (uint8_t)(hv >> (8 * k));
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (k < nt) img[i1 + k] = (uint8_t)(tv >> (8 * (4 - nt + k)));
    // interior: one DMA per record of this wave
    const uint64_t ga = (uint64_t)(uintptr_t)src + (i0 - d) + 4 * lane;
    for (int r = 0; r < 64; ++r) {
      const uint32_t c = __builtin_amdgcn_readlane(cnt, r);
      const uint32_t m0 = ib + __builtin_amdgcn_readlane(i0, r);
      const uint64_t a = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(uintptr_t)src, r) + 0;
      (void)a;
      const uint8_t* g = vals + kVal * (t - lane + r) + (__builtin_amdgcn_readlane(i0, r) - __builtin_amdgcn_readlane(d, r)) + 4 * lane;
      if ((uint32_t)lane < c)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(img + (m0 - ib)), 4, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  if (blockIdx.x == 0)
    for (int i = t; i < kImg; i += kWG) out[i] = img[i];
}

// each workgroup: stage 256 values, 256 records (thread t = record t) copied into the image,
// `iters` times (the image is rewritten every iteration), then the image goes to out
template <int V>
__global__ __launch_bounds__(kWG) void bench(const uint8_t* vals, const uint32_t* dpos, uint8_t* out, int iters) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kStage];
  __shared__ __attribute__((aligned(16))) uint8_t img[kImg];
  const int t = threadIdx.x;
  for (int i = t; i < kStage / 4; i += kWG) reinterpret_cast<uint32_t*>(stage)[i] = reinterpret_cast<const uint32_t*>(vals)[i];
  for (int i = t; i < kImg / 4; i += kWG) reinterpret_cast<uint32_t*>(img)[i] = 0;
  __syncthreads();
  const uint32_t d = dpos[t];
  for (int it = 0; it < iters; ++it) {
    copy<V>(img, d, stage, kVal * t, kVal, t & 63);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
  }
  __syncthreads();
  if (blockIdx.x == 0)
    for (int i = t; i < kImg; i += kWG) out[i] = img[i];
}

// 8: the body dwords by rows: 16-lane DPP row r copies record 16 r + k at step k (lane l =
// destination dword l of the body: consecutive banks), the record's params broadcast by
// row_newbcast; head / tail bytes by the record's own lane as in 0.
__device__ __forceinline__ uint32_t row_bcast(uint32_t v, int k) {
  switch (k) {
#define RB(K) case K: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + K, 0xF, 0xF, false);
    RB(0) RB(1) RB(2) RB(3) RB(4) RB(5) RB(6) RB(7) RB(8) RB(9) RB(10) RB(11) RB(12) RB(13) RB(14) RB(15)
#undef RB
  }
  return 0;
}
template <int V>
__global__ __launch_bounds__(kWG) void bench_row(const uint8_t* vals, const uint32_t* dpos, uint8_t* out, int iters) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kStage];
  __shared__ __attribute__((aligned(16))) uint8_t img[kImg];
  const int t = threadIdx.x, l = t & 15;
  for (int i = t; i < kStage / 4; i += kWG) reinterpret_cast<uint32_t*>(stage)[i] = reinterpret_cast<const uint32_t*>(vals)[i];
  for (int i = t; i < kImg / 4; i += kWG) reinterpret_cast<uint32_t*>(img)[i] = 0;
  __syncthreads();
  const uint32_t d = dpos[t];
  const uint32_t n = kVal, s = kVal * t;
  const uint32_t h = min(n, (4u - (d & 3u)) & 3u);
  const uint32_t d1 = d + h, e = d + n, body = ((e & ~3u) - d1) >> 2;
  const uint32_t sp = s + h, sh = sp & 3u;
  const uint32_t p_dst = d1 >> 2, p_src = sp >> 2, p_meta = body | (sh << 8);
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(stage);
  uint32_t* d32 = reinterpret_cast<uint32_t*>(img);
  for (int it = 0; it < iters; ++it) {
    uint32_t hb[3], tb[3];
    const uint32_t t0 = d1 + 4 * body;
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (k < h) hb[k] = stage[s + k];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (t0 + k < e) tb[k] = stage[s + (t0 + k - d)];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (k < h) img[d + k] = (uint8_t)hb[k];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) if (t0 + k < e) img[t0 + k] = (uint8_t)tb[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t rd = row_bcast(p_dst, k), rs = row_bcast(p_src, k), rm = row_bcast(p_meta, k);
      const uint32_t cnt = rm & 0xFF, rsh = rm >> 8;
      const uint32_t w0 = s32[rs + l], w1 = s32[rs + l + 1];
      if ((uint32_t)l < cnt) d32[rd + l] = __builtin_amdgcn_alignbyte(w1, w0, rsh);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
  }
  __syncthreads();
  if (blockIdx.x == 0)
    for (int i = t; i < kImg; i += kWG) out[i] = img[i];
}

int main() {
  std::vector<uint8_t> v(kStage);
  for (int i = 0; i < kStage; ++i) v[i] = (uint8_t)(i * 37 + 11);
  std::vector<uint32_t> dp(kRec);
  uint32_t pos = 5;
  for (int r = 0; r < kRec; ++r) { dp[r] = pos; pos += kVal + 6 + (r * 7) % 17; }  // 70..86 B apart
  std::vector<uint8_t> ref(kImg, 0);
  for (int r = 0; r < kRec; ++r) for (int i = 0; i < kVal; ++i) ref[dp[r] + i] = v[kVal * r + i];
  uint8_t *dv, *dout; uint32_t* ddp;
  hipMalloc(&dv, kStage); hipMalloc(&dout, kImg); hipMalloc(&ddp, 4 * kRec);
  hipMemcpy(dv, v.data(), kStage, hipMemcpyHostToDevice);
  hipMemcpy(ddp, dp.data(), 4 * kRec, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int grid = 256 * 4 * 4, iters = 64;
  auto run = [&](const char* name, auto k) {
    hipMemset(dout, 0, kImg);
    hipLaunchKernelGGL(k, dim3(grid), dim3(kWG), 0, 0, dv, ddp, dout, iters);
    hipDeviceSynchronize();
    std::vector<uint8_t> o(kImg);
    hipMemcpy(o.data(), dout, kImg, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < kImg; ++i) bad += o[i] != ref[i];
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(grid), dim3(kWG), 0, 0, dv, ddp, dout, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double recs = (double)grid * kRec * iters;
    printf("%-12s %8.3f ms  %7.2f ns/Mrec... %6.1f GB/s copied  %s\n", name, ms, ms * 1e6 / recs * 1e3, recs * kVal / (ms * 1e-3) / 1e9,
           bad ? "WRONG" : "ok");
  };
  run("0 rot-wrap", bench<0>);
  run("1 two-runs", bench<1>);
  run("2 mskor", bench<2>);
  run("3 ub128", bench<3>);
  run("4 plain", bench<4>);
  run("0 rot-wrap", bench<0>);
  run("1 two-runs", bench<1>);
  run("5 dma+or", bench_dma<5>);
  run("6 or-edges", bench_dma<6>);
  run("5 dma+or", bench_dma<5>);
  run("7 rec-dma", bench_rec_dma<7>);
  run("0 rot-wrap", bench<0>);
  run("7 rec-dma", bench_rec_dma<7>);
  run("8 rows", bench_row<8>);
  run("0 rot-wrap", bench<0>);
  run("8 rows", bench_row<8>);
  return 0;
}
