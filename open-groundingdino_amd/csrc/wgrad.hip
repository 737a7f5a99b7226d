// Weight / bias gradients of the token-heavy Linear layers for gfx950:
//   dW[o][i] = sum_t dY[t][o] X[t][i]     db[o] = sum_t dY[t][o]
// over T = 44 446 tokens (800x1333 encoder, bs=2) with small outputs
// (O, I = 128..1024).  The library GEMM the autograd path runs here tiles
// only the O x I output (a 256 x 256 weight is 16 tiles of 64 x 64: 16 of
// 256 CUs busy for 158 us, round-1 profile "MT64x64x256"), so this kernel
// splits the token (K) dimension instead: grid (I/64, O/64, splits), each
// workgroup reduces its token range for one 64 x 64 tile into an fp32
// partial, and wgrad_reduce sums the partials -- deterministic, and dW / db
// come out in fp32 (the fp32 master parameters' gradient dtype) with no bf16
// rounding of the product.
//
// MFMA: contraction over t, the ROW index of both operands, so each 32-token
// chunk of dY and X is staged transposed in LDS ([feature][token], a 16-B
// ds_read per fragment; mfma_frag.inc's stage_t pattern) and every wave
// computes a 32 x 32 quarter of the tile with 2 x 2 v_mfma_f32_16x16x32_bf16
// (fp32 inputs: eight v_mfma_f32_16x16x4_f32 each) per chunk.
#include "gd_common.h"

#include <cmath>

namespace gd {
namespace {
#include "mfma_frag.inc"

__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void st4(uint16_t* p, float4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(uint32_t(f32_to_bf16(v.x)) | (uint32_t(f32_to_bf16(v.y)) << 16),
                                            uint32_t(f32_to_bf16(v.z)) | (uint32_t(f32_to_bf16(v.w)) << 16));
}

template <typename T> __device__ __forceinline__ float to_float(T v);
template <> __device__ __forceinline__ float to_float<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_float<uint16_t>(uint16_t v) { return bf16_to_f32(v); }

constexpr int kWgChunk = 32;             // tokens per staged chunk
constexpr int kWgRow = kWgChunk + 8;     // LDS row pitch (elements): 16-B aligned rows

template <typename T>
__device__ __forceinline__ WFrag<T> lds_row8(const T* p);
template <>
__device__ __forceinline__ WFrag<uint16_t> lds_row8<uint16_t>(const uint16_t* p) {
  WFrag<uint16_t> f;
  f.v = *reinterpret_cast<const gd_bf16x8*>(p);
  return f;
}
template <>
__device__ __forceinline__ WFrag<float> lds_row8<float>(const float* p) {
  WFrag<float> f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f.v[j] = p[j];
  return f;
}

// Stage rows [t0, t0+32) x features [f0, f0+64) of a row-major [T, ld]
// matrix into xt[64][kWgRow] (transposed), zero past T.  256 threads.
template <typename T>
__device__ __forceinline__ void stage_chunk(T* xt, const T* src, int64_t ld, int t0, int T_, int f0) {
  constexpr int VE = 16 / int(sizeof(T));  // elements per 16-B load
  constexpr int NV = 64 / VE;              // vectors per 64-feature row slice
  for (int i = threadIdx.x; i < kWgChunk * NV; i += 256) {
    const int tt = i / NV, f = (i % NV) * VE;
    const int t = t0 + tt;
    union {
      uint4 u;
      T e[VE];
    } buf;
    if (t < T_) {
      buf.u = *reinterpret_cast<const uint4*>(src + int64_t(t) * ld + f0 + f);
    } else {
      buf.u = make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int e = 0; e < VE; ++e) xt[(f + e) * kWgRow + tt] = buf.e[e];
  }
}

// grid (I/64, O/64, batch * splits); batch b reads dy + b*bsy, x + b*bsx
template <typename T>
__global__ void __launch_bounds__(256)
wgrad_kernel(const T* __restrict__ dy, int64_t ldy, int64_t bsy, const T* __restrict__ x, int64_t ldx, int64_t bsx,
             int T_, int O, int I, int splits, int tokens_per_split, float* __restrict__ part_w,
             float* __restrict__ part_b) {
  __shared__ __attribute__((aligned(16))) T ys[64 * kWgRow];  // dY^T chunk: [o][t]
  __shared__ __attribute__((aligned(16))) T xs[64 * kWgRow];  // X^T chunk:  [i][t]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int wo = wave >> 1, wi = wave & 1;  // the wave's 32 x 32 quarter
  const int i0 = blockIdx.x * 64, o0 = blockIdx.y * 64;
  const int bz = blockIdx.z / splits, split = blockIdx.z - bz * splits;
  dy += bz * bsy;
  x += bz * bsx;
  const int64_t part = int64_t(bz) * splits + split;  // partial slot
  const int tb = split * tokens_per_split;
  const int te = min(T_, tb + tokens_per_split);
  const bool do_bias = part_b != nullptr && blockIdx.x == 0;
  gd_f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = zero4();
  float bsum = 0.f;  // threads 0..63: column o0 + tid of dY

  for (int t0 = tb; t0 < te; t0 += kWgChunk) {
    __syncthreads();  // previous chunk consumed
    stage_chunk<T>(ys, dy, ldy, t0, te, o0);
    stage_chunk<T>(xs, x, ldx, t0, te, i0);
    __syncthreads();
    if (do_bias && threadIdx.x < 64) {
      const T* r = ys + threadIdx.x * kWgRow;
#pragma unroll 8
      for (int k = 0; k < kWgChunk; ++k) bsum += to_float(r[k]);
    }
    WFrag<T> af[2], bf[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) af[m] = lds_row8<T>(ys + (32 * wo + 16 * m + c) * kWgRow + 8 * g);
#pragma unroll
    for (int n = 0; n < 2; ++n) bf[n] = lds_row8<T>(xs + (32 * wi + 16 * n + c) * kWgRow + 8 * g);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) acc[m][n] = wmma(af[m], bf[n], acc[m][n]);
  }
  // partial tile: (o0 + 32wo + 16m + 4g + r, i0 + 32wi + 16n + c)
  float* pw = part_w + part * O * I;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + 32 * wo + 16 * m + 4 * g + r, i = i0 + 32 * wi + 16 * n + c;
        pw[int64_t(o) * I + i] = acc[m][n][r];
      }
  if (do_bias && threadIdx.x < 64) part_b[part * O + o0 + threadIdx.x] = bsum;
}

// out[b] = sum over splits of the partials (4 columns per thread), written in
// fp32 or bf16 with batch stride ob; db (batch 1) likewise
template <typename TO>
__global__ void __launch_bounds__(256)
wgrad_reduce_kernel(const float* __restrict__ part_w, const float* __restrict__ part_b, int splits, int batch,
                    int O, int I, TO* __restrict__ out, int64_t ob, float* __restrict__ db) {
  const int64_t t = int64_t(blockIdx.x) * 256 + threadIdx.x;
  const int64_t nw4 = int64_t(O) * I / 4;  // float4 groups per batch item
  if (t < nw4 * batch) {
    const int64_t b = t / nw4, e = t - b * nw4;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < splits; ++k) {
      const float4 v = reinterpret_cast<const float4*>(part_w)[(b * splits + k) * nw4 + e];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    TO* o = out + b * ob + e * 4;
    st4(o, s);
  } else if (db && t < nw4 * batch + O) {
    const int o = int(t - nw4 * batch);
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += part_b[int64_t(k) * O + o];
    db[o] = s;
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" size_t gd_wgrad_workspace_bytes(int O, int I, int splits) {
  return sizeof(float) * (size_t(splits) * O * I + size_t(splits) * O);
}

extern "C" int gd_wgrad_splits(int T, int O, int I) {
  // about 1024 workgroups, at least 256 tokens each
  const int tiles = (O / 64) * (I / 64);
  int s = tiles > 0 ? (1024 + tiles - 1) / tiles : 1;
  const int cap = T / 256 > 1 ? T / 256 : 1;
  return s < 1 ? 1 : (s > cap ? cap : s);
}

extern "C" gd_status gd_wgrad_batched(gd_dtype dt, const void* grad_y, int64_t ldy, int64_t batch_stride_y,
                                      const void* x, int64_t ldx, int64_t batch_stride_x, int T, int O, int I,
                                      int batch, int splits, void* workspace, gd_dtype out_dtype, void* out,
                                      int64_t batch_stride_out, float* grad_b, gd_stream_t stream) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "wgrad: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(out_dtype == GD_F32 || out_dtype == GD_BF16, "wgrad: out dtype %d not supported", int(out_dtype));
  GD_REQUIRE(T >= 0 && O > 0 && I > 0 && O % 64 == 0 && I % 64 == 0 && splits >= 1 && batch >= 1 &&
                 int64_t(batch) * splits < 65536 && O / 64 < 65536,
             "wgrad: bad sizes T=%d O=%d I=%d (multiples of 64) batch=%d splits=%d", T, O, I, batch, splits);
  GD_REQUIRE(!grad_b || batch == 1, "wgrad: bias gradient only for batch 1");
  GD_REQUIRE(grad_y && x && workspace && out, "wgrad: null pointer");
  const int64_t align = 16 / (dt == GD_BF16 ? 2 : 4);
  GD_REQUIRE(aligned16(grad_y) && aligned16(x) && ldy % align == 0 && ldx % align == 0 && ldy >= O && ldx >= I &&
                 batch_stride_y % align == 0 && batch_stride_x % align == 0,
             "wgrad: rows must be 16-byte aligned (ldy=%lld ldx=%lld)", (long long)ldy, (long long)ldx);
  GD_REQUIRE(aligned16(out) && aligned16(workspace) && batch_stride_out % 8 == 0 &&
                 (batch == 1 || batch_stride_out >= int64_t(O) * I),
             "wgrad: out / workspace must be 16-byte aligned, batch_stride_out >= O*I");
  hipStream_t s = as_hip(stream);
  float* part_w = static_cast<float*>(workspace);
  float* part_b = part_w + int64_t(batch) * splits * O * I;
  const int tps = ((T + splits - 1) / splits + kWgChunk - 1) / kWgChunk * kWgChunk;
  const dim3 grid(unsigned(I / 64), unsigned(O / 64), unsigned(batch * splits));
  if (dt == GD_BF16)
    hipLaunchKernelGGL((wgrad_kernel<uint16_t>), grid, dim3(256), 0, s, (const uint16_t*)grad_y, ldy, batch_stride_y,
                       (const uint16_t*)x, ldx, batch_stride_x, T, O, I, splits, tps, part_w,
                       grad_b ? part_b : nullptr);
  else
    hipLaunchKernelGGL((wgrad_kernel<float>), grid, dim3(256), 0, s, (const float*)grad_y, ldy, batch_stride_y,
                       (const float*)x, ldx, batch_stride_x, T, O, I, splits, tps, part_w,
                       grad_b ? part_b : nullptr);
  GD_LAUNCH_CHECK("wgrad");
  const int64_t n = int64_t(O) * I / 4 * batch + (grad_b ? O : 0);
  const dim3 rg(unsigned((n + 255) / 256));
  if (out_dtype == GD_F32)
    hipLaunchKernelGGL((wgrad_reduce_kernel<float>), rg, dim3(256), 0, s, part_w, part_b, splits, batch, O, I,
                       (float*)out, batch_stride_out, grad_b);
  else
    hipLaunchKernelGGL((wgrad_reduce_kernel<uint16_t>), rg, dim3(256), 0, s, part_w, part_b, splits, batch, O, I,
                       (uint16_t*)out, batch_stride_out, grad_b);
  GD_LAUNCH_CHECK("wgrad_reduce");
  return GD_OK;
}

extern "C" gd_status gd_wgrad(gd_dtype dt, const void* grad_y, int64_t ldy, const void* x, int64_t ldx, int T,
                              int O, int I, int splits, void* workspace, float* grad_w, float* grad_b,
                              gd_stream_t stream) {
  return gd_wgrad_batched(dt, grad_y, ldy, 0, x, ldx, 0, T, O, I, 1, splits, workspace, GD_F32, grad_w,
                          int64_t(O) * I, grad_b, stream);
}
