// Shared helpers for the gfx950 kernels behind include/gdino_amd.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "../../include/gdino_amd.h"

namespace gd {

// Per-thread message of the last failing call (gd_last_error()).
void set_error(const char* fmt, ...);

#define GD_REQUIRE(cond, ...)          \
  do {                                 \
    if (!(cond)) {                     \
      ::gd::set_error(__VA_ARGS__);    \
      return GD_ERR_INVALID;           \
    }                                  \
  } while (0)

#define GD_HIP_CHECK(expr)                                                    \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      ::gd::set_error("%s failed: %s", #expr, hipGetErrorString(_e));         \
      return GD_ERR_LAUNCH;                                                   \
    }                                                                         \
  } while (0)

// After a <<<>>> launch: surface launch-configuration errors as a status.
#define GD_LAUNCH_CHECK(name)                                                 \
  do {                                                                        \
    hipError_t _e = hipGetLastError();                                        \
    if (_e != hipSuccess) {                                                   \
      ::gd::set_error("launch of %s failed: %s", name, hipGetErrorString(_e)); \
      return GD_ERR_LAUNCH;                                                   \
    }                                                                         \
  } while (0)

inline hipStream_t as_hip(gd_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---- bf16 helpers (bit-level; the round-to-nearest-even store goes through
// the __bf16 cast, which hipcc lowers to v_cvt_pk_bf16_f32 on gfx950 and which
// keeps NaN a NaN) -----------------------------------------------------------
__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }
// c + a.lo * b.lo + a.hi * b.hi for two packed bf16 pairs: one
// v_dot2c_f32_bf16 (the bf16 products are exact in fp32) instead of two
// unpacks and two FMAs per channel pair
__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
  typedef __bf16 gd_bf16x2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(gd_bf16x2, a), __builtin_bit_cast(gd_bf16x2, b), c, false);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// Bijective XCD-contiguous remap: hardware deals blocks b, b+8, b+16, ... to
// one XCD; give that XCD a contiguous chunk of the logical grid instead.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int q = nb >> 3, r = nb & 7;
  const int xcd = b & 7, local = b >> 3;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + local;
}

// ---- DPP lane exchange inside 8/16-lane groups ----------------------------
// quad_perm [1,0,3,2] (xor 1), [2,3,0,1] (xor 2), row_half_mirror (i <-> 7-i),
// row_ror:8 (i <-> i^8 inside a 16-lane row).
enum : int {
  DPP_XOR1 = 0xB1,
  DPP_XOR2 = 0x4E,
  DPP_HALF_MIRROR = 0x141,
  DPP_ROR8 = 0x128,
};

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_amdgcn_update_dpp(0.f, v, CTRL, 0xf, 0xf, false);
}

// ---- fills as kernels ------------------------------------------------------
// Every buffer the kernels need pre-filled is filled by this kernel, not by
// hipMemsetAsync: inside a captured HIP graph a memset becomes a memset node,
// and the step graph's replays faulted (illegal address / hangs) while its
// eager warm-ups of the same work ran clean -- a kernel node is ordered like
// every other kernel of the stream.  bytes: a multiple of 4.
namespace {
__global__ void __launch_bounds__(256) fill_u32_kernel(uint32_t* __restrict__ p, int64_t n, uint32_t v, int vec) {
  const int64_t n4 = vec ? n / 4 : 0;
  const uint4 v4 = make_uint4(v, v, v, v);
  const int64_t stride = int64_t(gridDim.x) * 256;
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += stride)
    reinterpret_cast<uint4*>(p)[i] = v4;
  for (int64_t i = n4 * 4 + int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) p[i] = v;
}
}  // namespace

// fill bytes / 4 words at p with v (16-byte aligned p: vector stores)
inline hipError_t fill_u32_async(void* p, uint32_t v, size_t bytes, hipStream_t s) {
  const int64_t n = int64_t(bytes / 4);
  if (n == 0) return hipSuccess;
  const int vec = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  int64_t blocks = ((vec ? n / 4 : n) + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  hipLaunchKernelGGL(fill_u32_kernel, dim3(unsigned(blocks)), dim3(256), 0, s, static_cast<uint32_t*>(p), n, v, vec);
  return hipGetLastError();
}


// 16 bytes per lane from global memory straight into LDS (LDS-DMA,
// global_load_lds_dwordx4): lane l's bytes land at the wave-uniform `dst` +
// 16 l.  Inline asm rather than __builtin_amdgcn_global_load_lds: hipcc cannot
// tell which ring slot a builtin DMA writes, so after one it waits vmcnt(0)
// before every later ds_read (a multi-slot ring drains each step); an asm DMA
// is outside its wait bookkeeping and the kernel counts vmcnt itself
// (gd_wait_vmcnt).  M0 is written and restored in the same statement
// (cdna_hip_programming.md, "LDS-DMA recipe").  tests/emu's host header
// defines GD_LDS_DMA16 with a host emulation of the same data movement.
#ifndef GD_LDS_DMA16
namespace {
__device__ __forceinline__ void lds_dma16(const void* src, void* dst) {
  const uint32_t lds_addr = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)(dst))));
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_addr)
               : "memory");
}
}  // namespace
#define GD_LDS_DMA16(src, dst) ::gd::lds_dma16((src), (dst))
#endif
// s_waitcnt vmcnt(N) (expcnt, lgkmcnt left open), N < 64; and a bare
// s_barrier, which unlike __syncthreads() does not wait vmcnt(0) first
#define gd_wait_vmcnt(N)                                                      \
  do {                                                                        \
    __asm__ __volatile__("" ::: "memory");                                    \
    __builtin_amdgcn_s_waitcnt(((N) & 15) | (((N) >> 4) << 14) | 0x0F70);     \
  } while (0)
#define gd_raw_barrier()                      \
  do {                                        \
    __asm__ __volatile__("" ::: "memory");    \
    __builtin_amdgcn_s_barrier();             \
    __asm__ __volatile__("" ::: "memory");    \
  } while (0)
// An opaque copy of a per-lane integer: values derived from the copy cannot
// be computed once and kept live in registers from an earlier use of the
// original (a register-pressure valve for kernel epilogues)
#ifndef gd_opaque_i32
namespace {
__device__ __forceinline__ int gd_opaque_i32(int x) {
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
}  // namespace
#endif
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS (and
// scalar-memory) operations, then s_barrier -- NOT for its global loads and
// stores.  __syncthreads() waits vmcnt(0) as well, so a barrier inside a
// loop that prefetches the next iteration's global data (or has issued
// global stores) exposes their whole latency at every barrier.
#ifndef gd_lds_barrier
#define gd_lds_barrier()                                                     \
  do {                                                                       \
    __asm__ __volatile__("" ::: "memory");                                   \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0), vmcnt / expcnt open */ \
    __builtin_amdgcn_s_barrier();                                            \
    __asm__ __volatile__("" ::: "memory");                                   \
  } while (0)
#endif

// Wave-level ordering point for wave-private LDS: the wave runs in lock step
// and a wave's LDS instructions execute in order, so a ds_write by one lane
// is visible to a later ds_read by another lane of the same wave; this only
// keeps the compiler from moving LDS accesses across the point (no
// s_barrier, no wait).  tests/emu's header defines it as a wave-wide
// rendezvous of its lane fibers.
#ifndef gd_wave_sync
#define gd_wave_sync()                        \
  do {                                        \
    __asm__ __volatile__("" ::: "memory");    \
    __builtin_amdgcn_wave_barrier();          \
    __asm__ __volatile__("" ::: "memory");    \
  } while (0)
#endif
}  // namespace gd

// integer tuning / A-B switch from the environment (host side)
inline int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}

