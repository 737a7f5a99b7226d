// Host-side SIMT emulation of the HIP subset the gd kernels use.
//
// TEST INFRASTRUCTURE ONLY (tests/emu): the product's own csrc/*.hip files are
// compiled by the host clang++ against this header (it shadows
// <hip/hip_runtime.h> through -I), giving tests/emu/_build/libgd_emu.so with the
// same C ABI as libgdino_amd.so, operating on host pointers.  Tests use it to
// run the exact kernel sources -- indexing, LDS use, barriers, cross-lane
// exchanges, launch geometry -- on the CPU when no GPU is available, against
// the oracle.  It is never loaded by the product (gdino_amd._lib loads only
// the gfx950 library) and it says nothing about speed.
//
// Model: one workgroup at a time; each work-item is a ucontext fiber on one OS
// thread, scheduled round-robin.  A fiber runs until it has to wait:
//   * __syncthreads(): until every live work-item of the block has arrived;
//   * cross-lane reads (__shfl_xor, ds_swizzle, DPP) and MFMA (whose
//     operands come from all 64 lanes): until the source lane(s) have
//     published their value for the same exchange (each lane publishes into
//     an append-only log indexed by its exchange count, so a source never
//     overwrites a value a slower reader still needs).
// Wave = 64 consecutive work-items.  LDS (__shared__) is a static array,
// zero-initialised once, like uninitialised LDS it must be written before use.
// Global float atomics are plain read-modify-writes (one OS thread).
// GD_EMU_SCHED=rev | shuffle:<seed> changes the order in which the scheduler
// resumes work-items between synchronisation points (default: ascending):
// a kernel missing a barrier between an LDS producer and a consumer in
// another wave computes different results under another order.
#pragma once

#include <ucontext.h>

#include <climits>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
// LDS arrays live in their own section so the scheduler can poison them
// (0xFF bytes: NaN floats, -1 ints) before every workgroup: a kernel that
// reads LDS it has not written in the same workgroup sees garbage, as on the
// GPU, instead of the previous workgroup's values.
#define __shared__ static __attribute__((section("gd_emu_lds")))

struct dim3 {
  unsigned x, y, z;
  constexpr dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct float2 { float x, y; };
struct float4 { float x, y, z, w; };
struct uint2 { unsigned x, y; };
struct int2 { int x, y; };
struct int4 { int x, y, z, w; };
inline int2 make_int2(int a, int b) { return {a, b}; }
inline int4 make_int4(int a, int b, int c, int d) { return {a, b, c, d}; }
struct uint4 { unsigned x, y, z, w; };
inline float2 make_float2(float a, float b) { return {a, b}; }
inline float4 make_float4(float a, float b, float c, float d) { return {a, b, c, d}; }
inline uint2 make_uint2(unsigned a, unsigned b) { return {a, b}; }
inline uint4 make_uint4(unsigned a, unsigned b, unsigned c, unsigned d) { return {a, b, c, d}; }
inline float __logf(float x) { return logf(x); }
inline float __fadd_rn(float a, float b) { return a + b; }
inline float rsqrtf(float x) { return 1.0f / sqrtf(x); }
inline float __fmul_rn(float a, float b) { return a * b; }
inline float __fdiv_rn(float a, float b) { return a / b; }

typedef int hipError_t;
constexpr hipError_t hipSuccess = 0;
typedef struct ihipStream_t* hipStream_t;
#define HIP_VERSION 0

struct hipDeviceProp_t {
  char gcnArchName[256];
};
inline const char* hipGetErrorString(hipError_t) { return "emulated HIP error"; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) {
  memset(p, v, n);
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
constexpr int hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2;
#define HIP_SYMBOL(x) (&(x))
inline hipError_t hipMemcpyFromSymbol(void* dst, const void* sym, size_t n, size_t off = 0, int = 0) {
  std::memcpy(dst, static_cast<const char*>(sym) + off, n);
  return hipSuccess;
}
inline hipError_t hipMemcpyToSymbol(const void* sym, const void* src, size_t n, size_t off = 0, int = 0) {
  std::memcpy(const_cast<char*>(static_cast<const char*>(sym)) + off, src, n);
  return hipSuccess;
}
inline hipError_t hipRuntimeGetVersion(int* v) {
  *v = 0;
  return hipSuccess;
}
inline hipError_t hipGetDevice(int* d) {
  *d = 0;
  return hipSuccess;
}
inline hipError_t hipGetDeviceProperties(hipDeviceProp_t* p, int) {
  snprintf(p->gcnArchName, sizeof(p->gcnArchName), "host-emulator");
  return hipSuccess;
}

inline float __int_as_float(int v) { float f; memcpy(&f, &v, 4); return f; }
inline int __float_as_int(float f) { int v; memcpy(&v, &f, 4); return v; }
inline float __uint_as_float(unsigned v) { float f; memcpy(&f, &v, 4); return f; }
inline unsigned __float_as_uint(float f) { unsigned v; memcpy(&v, &f, 4); return v; }
inline float __expf(float x) { return expf(x); }
inline float __log2f(float x) { return log2f(x); }
#define __builtin_amdgcn_exp2f(x) exp2f(x)
inline int min(int a, int b) { return a < b ? a : b; }
inline int max(int a, int b) { return a > b ? a : b; }

namespace gd_emu {

struct Item {
  ucontext_t ctx;
  std::vector<char> stack;
  dim3 tid;
  bool done = false;
  bool at_barrier = false;
  unsigned barrier_gen = 0;
  size_t nxchg = 0;                  // cross-lane exchanges performed
  std::vector<uint64_t> published;   // value published at each exchange
};

struct Grid {
  dim3 grid, block, bid;
  std::vector<Item> items;
  size_t cur = 0;
  unsigned live = 0, arrived = 0, gen = 0;
  ucontext_t sched;
  void (*body)(void*) = nullptr;
  void* body_arg = nullptr;
};

Grid& grid();  // defined in gd_emu.cpp
void note_progress();
void yield();  // back to the scheduler
void run(dim3 g, dim3 b, void (*body)(void*), void* arg);

inline Item& self() { return grid().items[grid().cur]; }
inline unsigned flat_id() { return unsigned(grid().cur); }

// Publish `bits` as this lane's value for its next exchange; return the value
// lane `src` (flat work-item index) published for the same exchange.
inline uint64_t exchange(uint64_t bits, unsigned src) {
  Grid& g = grid();
  Item& me = g.items[g.cur];
  const size_t k = me.nxchg++;
  me.published.push_back(bits);
  note_progress();
  if (src >= g.items.size()) {
    fprintf(stderr, "gd_emu: lane exchange with work-item %u outside the block\n", src);
    abort();
  }
  for (;;) {
    Item& o = g.items[src];
    if (o.published.size() > k) return o.published[k];
    if (o.done) {
      fprintf(stderr, "gd_emu: work-item %u reads exited work-item %u (exchange %zu)\n", flat_id(), src, k);
      abort();
    }
    yield();
  }
}

template <typename V>
inline V xchg_from(V v, unsigned src) {
  static_assert(sizeof(V) <= 8, "exchange of at most 64 bits");
  uint64_t b = 0;
  memcpy(&b, &v, sizeof(V));
  const uint64_t r = exchange(b, src);
  V out;
  memcpy(&out, &r, sizeof(V));
  return out;
}

inline unsigned wave_base() { return flat_id() & ~63u; }
inline unsigned lane_id() { return flat_id() & 63u; }

// ds_swizzle, bitmask mode (offset bit 15 = 0) inside 32-lane groups
inline int ds_swizzle(int v, int pattern) {
  if (pattern & 0x8000) {
    fprintf(stderr, "gd_emu: ds_swizzle QDMode pattern 0x%x not emulated\n", pattern);
    abort();
  }
  const unsigned and_m = pattern & 0x1F, or_m = (pattern >> 5) & 0x1F, xor_m = (pattern >> 10) & 0x1F;
  const unsigned lane = lane_id();
  const unsigned src = (lane & ~31u) | ((((lane & 31u) & and_m) | or_m) ^ xor_m);
  return xchg_from(v, wave_base() + src);
}

// DPP (row_mask = bank_mask = 0xF): quad_perm, row_half_mirror, row_ror
template <typename V>
inline V update_dpp(V old, V src, int ctrl, int row_mask, int bank_mask, bool) {
  if (row_mask != 0xF || bank_mask != 0xF) {
    fprintf(stderr, "gd_emu: DPP with partial masks not emulated\n");
    abort();
  }
  (void)old;
  const unsigned lane = lane_id();
  unsigned from;
  if (ctrl >= 0 && ctrl <= 0xFF) {  // quad_perm
    from = (lane & ~3u) | ((unsigned(ctrl) >> (2 * (lane & 3u))) & 3u);
  } else if (ctrl == 0x141) {  // row_half_mirror
    from = (lane & ~7u) | (7u - (lane & 7u));
  } else if (ctrl >= 0x121 && ctrl <= 0x12F) {  // row_ror:n
    const unsigned n = unsigned(ctrl) & 0xF;
    from = (lane & ~15u) | (((lane & 15u) + n) & 15u);
  } else if ((ctrl >= 0x101 && ctrl <= 0x10F) || (ctrl >= 0x111 && ctrl <= 0x11F)) {
    // row_shl:n / row_shr:n (bound_ctrl off): a lane whose source lies
    // outside its 16-lane row keeps `old`
    const unsigned n = unsigned(ctrl) & 0xF;
    const int r = int(lane & 15u) + (ctrl <= 0x10F ? int(n) : -int(n));
    const bool inside = r >= 0 && r <= 15;
    from = inside ? (lane & ~15u) | unsigned(r) : lane;
    const V got = xchg_from(src, wave_base() + from);
    return inside ? got : old;
  } else {
    fprintf(stderr, "gd_emu: DPP control 0x%x not emulated\n", ctrl);
    abort();
  }
  return xchg_from(src, wave_base() + from);
}

template <typename V>
inline V shfl_xor(V v, int mask, int width) {
  const unsigned lane = lane_id();
  const unsigned w = unsigned(width);
  const unsigned src = (lane & ~(w - 1)) | (((lane & (w - 1)) ^ unsigned(mask)) & (w - 1));
  return xchg_from(v, wave_base() + src);
}

template <typename V>
inline V shfl(V v, int src, int width) {
  const unsigned lane = lane_id();
  const unsigned w = unsigned(width);
  return xchg_from(v, wave_base() + ((lane & ~(w - 1)) | (unsigned(src) & (w - 1))));
}

// v_readlane: lane `src` of the caller's wave (a wave-uniform result)
inline int readlane(int v, int src) { return xchg_from(v, wave_base() + unsigned(src)); }

// All 64 lanes of the caller's wave contribute `nbytes` (<= 64) and every
// lane receives the 64 contributions in lane order (MFMA operand exchange).
inline void wave_gather(const void* mine, size_t nbytes, void* all) {
  Grid& g = grid();
  const size_t nw = (nbytes + 7) / 8;
  uint64_t w[8] = {};
  memcpy(w, mine, nbytes);
  const size_t k0 = g.items[g.cur].nxchg;
  for (size_t i = 0; i < nw; ++i) g.items[g.cur].published.push_back(w[i]);
  g.items[g.cur].nxchg += nw;
  note_progress();
  const unsigned base = wave_base();
  if (base + 64 > g.items.size()) {
    fprintf(stderr, "gd_emu: MFMA in a partial wave (block of %zu work-items)\n", g.items.size());
    abort();
  }
  for (unsigned s = 0; s < 64; ++s) {
    for (;;) {
      Item& o = g.items[base + s];
      if (o.published.size() >= k0 + nw) {
        memcpy(static_cast<char*>(all) + s * nbytes, &o.published[k0], nbytes);
        break;
      }
      if (o.done) {
        fprintf(stderr, "gd_emu: MFMA of work-item %u waits for exited work-item %u\n", flat_id(), base + s);
        abort();
      }
      yield();
    }
  }
}

// __builtin_amdgcn_wave_barrier (gd_common.h gd_wave_sync): no lane of the
// wave continues before every lane has arrived (an exchange of nothing), so
// wave-private LDS written by one lane and read by another is ordered as the
// lock-stepped wave orders it on the GPU
inline void wave_sync() {
  const uint8_t z = 0;
  uint8_t all[64];
  wave_gather(&z, 1, all);
}

// __ballot: bit i = predicate of lane i (all 64 lanes of the wave take part)
inline unsigned long long ballot(int pred) {
  const uint8_t mine = pred ? 1 : 0;
  uint8_t all[64];
  wave_gather(&mine, 1, all);
  unsigned long long m = 0;
  for (unsigned i = 0; i < 64; ++i) m |= (unsigned long long)(all[i] & 1u) << i;
  return m;
}

// ds_read_b64_tr_b16 (gfx950): per 16-lane group, lane 4q+p supplies the
// address of row q, columns 4p..4p+3 of a 4 x 16 block of 16-bit elements;
// lane i receives column i of the 4 rows (row q in element q)
typedef short gd_emu_i16x4 __attribute__((ext_vector_type(4)));
inline gd_emu_i16x4 ds_read_tr16_b64(const void* p) {
  const uint64_t mine = uint64_t(uintptr_t(p));
  uint64_t all[64];
  wave_gather(&mine, sizeof(mine), all);
  const unsigned lane = lane_id(), base = lane & ~15u, i = lane & 15u;
  gd_emu_i16x4 r;
  for (unsigned q = 0; q < 4; ++q) {
    const int16_t* a = reinterpret_cast<const int16_t*>(uintptr_t(all[base + 4 * q + i / 4]));
    r[q] = a[i % 4];
  }
  return r;
}


inline float bf16_bits_to_f(uint16_t h) {
  uint32_t u = uint32_t(h) << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// v_mfma_f32_16x16x32_bf16 (cdna_hip_programming.md §3, lane maps [HW]):
// lane l holds A[l&15][8(l>>4)+j] and B[8(l>>4)+j][l&15] in element j, and
// receives D[4(l>>4)+r][l&15] in element r.  Products are exact; the sum is
// taken in double and rounded once.
// v_dot2c_f32_bf16: the two bf16 products are exact in fp32; modelled as
// the sum of both products and c in double rounded once to fp32
template <typename V2>
inline float fdot2_bf16(V2 a, V2 b, float c) {
  return float(double(float(a[0])) * double(float(b[0])) + double(float(a[1])) * double(float(b[1])) + double(c));
}

template <typename V8, typename C4>
inline C4 mfma_16x16x32_bf16(V8 a, V8 b, C4 c) {
  static_assert(sizeof(V8) == 16 && sizeof(C4) == 16, "bf16x8 / f32x4 operands");
  struct Ops { uint16_t a[8], b[8]; } mine, all[64];
  memcpy(mine.a, &a, 16);
  memcpy(mine.b, &b, 16);
  wave_gather(&mine, sizeof(Ops), all);
  const unsigned l = lane_id();
  C4 d;
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * int(l >> 4) + r, col = int(l & 15);
    double acc = 0.0;
    for (int k = 0; k < 32; ++k)
      acc += double(bf16_bits_to_f(all[row + 16 * (k >> 3)].a[k & 7])) *
             double(bf16_bits_to_f(all[col + 16 * (k >> 3)].b[k & 7]));
    d[r] = float(double(c[r]) + acc);
  }
  return d;
}

// v_mfma_f32_16x16x4_f32: lane l holds A[l&15][l>>4] and B[l>>4][l&15].
template <typename C4>
inline C4 mfma_16x16x4_f32(float a, float b, C4 c) {
  static_assert(sizeof(C4) == 16, "f32x4 accumulator");
  struct Ops { float a, b; } mine{a, b}, all[64];
  wave_gather(&mine, sizeof(Ops), all);
  const unsigned l = lane_id();
  C4 d;
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * int(l >> 4) + r, col = int(l & 15);
    double acc = 0.0;
    for (int k = 0; k < 4; ++k) acc += double(all[row + 16 * k].a) * double(all[col + 16 * k].b);
    d[r] = float(double(c[r]) + acc);
  }
  return d;
}

void syncthreads();

// global_load_lds_dwordx4 (gd_common.h GD_LDS_DMA16): the LDS destination is
// the wave-uniform base (M0, from the first lane) + 16 * lane; the source is
// per lane.  The emulator's memory is synchronous, so the data lands at once
// (an early ds_read of a slot still shows what the kernel's ordering allows:
// the poisoned or previous contents until a barrier-ordered DMA wrote it).
inline void lds_dma16(const void* src, void* dst) {
  const uint64_t mine = uint64_t(uintptr_t(dst));
  uint64_t all[64];
  wave_gather(&mine, sizeof(mine), all);
  memcpy(reinterpret_cast<char*>(uintptr_t(all[0])) + 16 * lane_id(), src, 16);
}

template <typename F>
void launch(dim3 g, dim3 b, F&& f) {
  auto thunk = [](void* p) { (*static_cast<F*>(p))(); };
  run(g, b, thunk, &f);
}

}  // namespace gd_emu

#define threadIdx (::gd_emu::self().tid)
#define blockIdx (::gd_emu::grid().bid)
#define gridDim (::gd_emu::grid().grid)
#define blockDim (::gd_emu::grid().block)
#define __syncthreads() ::gd_emu::syncthreads()
#define __ballot(pred) ::gd_emu::ballot(pred)
#define __threadfence() ((void)0)  // one OS thread: memory is coherent
#define __threadfence_block() ((void)0)
inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
inline int __ffsll(long long v) { return __builtin_ffsll(v); }
#define __shfl_xor(v, mask, width) ::gd_emu::shfl_xor((v), (mask), (width))
#define __shfl(v, src, width) ::gd_emu::shfl((v), (src), (width))
#define __builtin_amdgcn_readlane(v, src) ::gd_emu::readlane((v), (src))
#define __builtin_amdgcn_s_barrier() ::gd_emu::syncthreads()
#define gd_wave_sync() ::gd_emu::wave_sync()
#define __builtin_amdgcn_s_waitcnt(imm) ((void)(imm))  // memory is synchronous here
#define gd_opaque_i32(x) (x)  // gd_common.h: a register-allocation hint only
#define GD_LDS_DMA16(src, dst) ::gd_emu::lds_dma16((const void*)(src), (void*)(dst))
// compiler scheduling hints: no semantics to emulate
#define __builtin_amdgcn_sched_barrier(mask) ((void)(mask))
#define __builtin_amdgcn_ds_read_tr16_b64_v4i16(p) ::gd_emu::ds_read_tr16_b64((const void*)(uintptr_t)(p))
#define __builtin_amdgcn_ds_swizzle(v, pattern) ::gd_emu::ds_swizzle((v), (pattern))
#define __builtin_amdgcn_update_dpp(old, src, ctrl, rm, bm, bc) \
  ::gd_emu::update_dpp((old), (src), (ctrl), (rm), (bm), (bc))
#define __builtin_amdgcn_mov_dpp(src, ctrl, rm, bm, bc) ::gd_emu::update_dpp((src), (src), (ctrl), (rm), (bm), (bc))
#define __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, cbsz, abid, blgp) \
  ::gd_emu::mfma_16x16x32_bf16((a), (b), (c))
#define __builtin_amdgcn_fdot2_f32_bf16(a, b, c, clamp) ::gd_emu::fdot2_bf16((a), (b), (c))
#define __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, cbsz, abid, blgp) ::gd_emu::mfma_16x16x4_f32((a), (b), (c))
#define hipLaunchKernelGGL(kernel, g, b, shm, stream, ...) \
  ((void)(shm), (void)(stream), ::gd_emu::launch(dim3(g), dim3(b), [&]() { kernel(__VA_ARGS__); }))

template <typename T>
inline T atomicAdd(T* p, T v) {
  const T old = *p;
  *p = old + v;
  return old;
}

template <typename T>
inline T atomicOr(T* p, T v) {
  const T old = *p;
  *p = old | v;
  return old;
}

template <typename T>
inline T atomicMin(T* p, T v) {
  const T old = *p;
  *p = v < old ? v : old;
  return old;
}

template <typename T>
inline T atomicMax(T* p, T v) {
  const T old = *p;
  *p = v > old ? v : old;
  return old;
}
