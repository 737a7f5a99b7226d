// Residual add + LayerNorm for gfx950: the post-norm sublayer ending
//   y = LayerNorm(x + r) * w + b
// of the deformable encoder / decoder layers and the text enhancer
// (reference transformer.py:789-808, 877-936, transformer_vanilla.py:83-110:
// `norm(src + dropout(src2))`).  Under bf16 autocast the reference runs an
// fp32 add of the bf16 sublayer output into the fp32 residual stream, then
// PyTorch's LayerNorm (fp32), and in the backward the LayerNorm input
// gradient, the gamma / beta partial sums and a bf16 cast of the gradient
// sent to the sublayer.  Here: one kernel forward (s = x + r, mean / rstd,
// y), one kernel backward (ds, dx = ds, dr = ds in r's dtype, per-wave
// gamma / beta partials) and a column reduction of the partials.
//
// One wave per row (grid-stride over rows); lane j owns columns j + 64e,
// e < E = C / 64, so every access is a coalesced 256-B (fp32) row segment and
// the row statistics are wave shuffles.  The variance is the two-pass
// mean((s - mean)^2) over the registers.  s is recomputed from x and r in the
// backward instead of being stored.
#include "gd_common.h"

#include <cmath>
#include <type_traits>

namespace gd {
namespace {

template <typename T> __device__ __forceinline__ float ldv(const T* p);
template <> __device__ __forceinline__ float ldv<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ldv<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }
template <typename T> __device__ __forceinline__ void stv(T* p, float v);
template <> __device__ __forceinline__ void stv<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void stv<uint16_t>(uint16_t* p, float v) { *p = f32_to_bf16(v); }

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// lane's column lane + 64 e exists (C not a multiple of 64: Swin-T's 96)
template <int C>
__device__ __forceinline__ bool col_ok(int lane, int e) {
  return C % 64 == 0 || lane + 64 * e < C;
}

// grid-stride: wave w of the grid handles rows w, w + nwaves, ...
template <typename TX, typename TR, int C>
__global__ void __launch_bounds__(256)
addln_fwd_kernel(const TX* __restrict__ x, const TR* __restrict__ r, const float* __restrict__ w,
                 const float* __restrict__ b, int64_t rows, float eps, float* __restrict__ y,
                 uint16_t* __restrict__ y16, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int E = (C + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = int64_t(gridDim.x) * 4;
  float wv[E], bv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const bool ok = col_ok<C>(lane, e);
    wv[e] = ok && w ? w[lane + 64 * e] : 1.f;
    bv[e] = ok && b ? b[lane + 64 * e] : 0.f;
  }
  for (int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); row < rows; row += nwaves) {
    float s[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t o = row * C + lane + 64 * e;
      s[e] = col_ok<C>(lane, e) ? ldv<TX>(x + o) + (r ? ldv<TR>(r + o) : 0.f) : 0.f;
    }
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) sum += s[e];
    const float mean = wsum(sum) / float(C);
    float sq = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float d = col_ok<C>(lane, e) ? s[e] - mean : 0.f;
      sq += d * d;
    }
    const float rstd = rsqrtf(wsum(sq) / float(C) + eps);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (!col_ok<C>(lane, e)) continue;
      const float v = (s[e] - mean) * rstd * wv[e] + bv[e];
      y[row * C + lane + 64 * e] = v;
      if (y16) y16[row * C + lane + 64 * e] = f32_to_bf16(v);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

// dy [rows, C] fp32 (+ dy2, the gradient of a second consumer of y, summed
// here instead of by an autograd add) -> dx (TX), dr (TR, optional),
// partial dw / db per wave
template <typename TX, typename TR, int C>
__global__ void __launch_bounds__(256)
addln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ dy2, const TX* __restrict__ x,
                 const TR* __restrict__ r,
                 const float* __restrict__ w, const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                 int64_t rows, TX* __restrict__ dx, TR* __restrict__ dr, float* __restrict__ part_w,
                 float* __restrict__ part_b) {
  constexpr int E = (C + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = int64_t(gridDim.x) * 4;
  float wv[E], gw[E], gb[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    wv[e] = col_ok<C>(lane, e) && w ? w[lane + 64 * e] : 1.f;
    gw[e] = gb[e] = 0.f;
  }
  for (int64_t row = wave_id; row < rows; row += nwaves) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[E], g[E];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t o = row * C + lane + 64 * e;
      const bool ok = col_ok<C>(lane, e);
      const float s = ok ? ldv<TX>(x + o) + (r ? ldv<TR>(r + o) : 0.f) : 0.f;
      xh[e] = ok ? (s - mean) * rstd : 0.f;
      const float d = ok ? dy[o] + (dy2 ? dy2[o] : 0.f) : 0.f;  // dy2: a second consumer's gradient
      gw[e] += d * xh[e];
      gb[e] += d;
      g[e] = d * wv[e];
      sg += g[e];
      sgx += g[e] * xh[e];
    }
    const float mg = wsum(sg) / float(C), mgx = wsum(sgx) / float(C);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (!col_ok<C>(lane, e)) continue;
      const int64_t o = row * C + lane + 64 * e;
      const float ds = rstd * (g[e] - mg - xh[e] * mgx);
      stv<TX>(dx + o, ds);
      if (dr) stv<TR>(dr + o, ds);
    }
  }
  if (part_w) {  // combine the block's 4 waves in LDS: one partial row per block
    __shared__ float red[2][4][C];
    const int wv_i = threadIdx.x >> 6;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (!col_ok<C>(lane, e)) continue;
      red[0][wv_i][lane + 64 * e] = gw[e];
      red[1][wv_i][lane + 64 * e] = gb[e];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      part_w[int64_t(blockIdx.x) * C + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
      part_b[int64_t(blockIdx.x) * C + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
    }
  }
}

// dw[c] = sum_k part_w[k][c], db likewise; grid ceil(C / 16), block 1024 =
// 16 columns x 64 row groups, combined through LDS
__global__ void __launch_bounds__(1024)
addln_reduce_kernel(const float* __restrict__ part_w, const float* __restrict__ part_b, int nparts, int C,
                    float* __restrict__ dw, float* __restrict__ db) {
  // 16 columns x 64 part groups per workgroup (C / 16 workgroups): each
  // thread sums nparts / 64 partials, four loads in flight per step; with 64
  // columns x 16 groups a C = 256 reduction ran on 4 CUs, 32 serial-ish
  // loads per thread and array (5.2 us per call, ~118 calls per step).
  // Fixed summation order (deterministic).
  constexpr int kCols = 16, kGroups = 64;
  __shared__ float red[2][kGroups][kCols];
  const int cx = threadIdx.x % kCols, grp = threadIdx.x / kCols;
  const int c = blockIdx.x * kCols + cx;
  float sw = 0.f, sb = 0.f;
  if (c < C) {
    int k = grp;
    for (; k + 3 * kGroups < nparts; k += 4 * kGroups) {
      const float w0 = part_w[int64_t(k) * C + c], w1 = part_w[int64_t(k + kGroups) * C + c];
      const float w2 = part_w[int64_t(k + 2 * kGroups) * C + c], w3 = part_w[int64_t(k + 3 * kGroups) * C + c];
      const float b0 = part_b[int64_t(k) * C + c], b1 = part_b[int64_t(k + kGroups) * C + c];
      const float b2 = part_b[int64_t(k + 2 * kGroups) * C + c], b3 = part_b[int64_t(k + 3 * kGroups) * C + c];
      sw += w0;
      sw += w1;
      sw += w2;
      sw += w3;
      sb += b0;
      sb += b1;
      sb += b2;
      sb += b3;
    }
    for (; k < nparts; k += kGroups) {
      sw += part_w[int64_t(k) * C + c];
      sb += part_b[int64_t(k) * C + c];
    }
  }
  red[0][grp][cx] = sw;
  red[1][grp][cx] = sb;
  __syncthreads();
  if (grp == 0 && c < C) {
    for (int k = 1; k < kGroups; ++k) {
      sw += red[0][k][cx];
      sb += red[1][k][cx];
    }
    dw[c] = sw;
    db[c] = sb;
  }
}

// ---------------------------------------------------------------------------
// Round 6: the same two kernels with 4 consecutive columns per lane (16-B
// fp32 / 8-B bf16 vector accesses): lane j owns columns 4j + 256e, e < E4.
// The one-column-per-lane kernels above issue C/64 scalar 4-B accesses per
// array and row (256 B per wave instruction) and ran at 1.7-1.9 TB/s in the
// step (bench hip_entry_points_one_step, round 5); host-checked alignment
// routes here (GD_ADDLN_V4=0: the scalar kernels, A/B).
template <typename T> __device__ __forceinline__ void ld4v(const T* p, float v[4]);
template <> __device__ __forceinline__ void ld4v<float>(const float* p, float v[4]) {
  const float4 t = *reinterpret_cast<const float4*>(p);
  v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
template <> __device__ __forceinline__ void ld4v<uint16_t>(const uint16_t* p, float v[4]) {
  const uint2 t = *reinterpret_cast<const uint2*>(p);
  v[0] = bf16_lo(t.x); v[1] = bf16_hi(t.x); v[2] = bf16_lo(t.y); v[3] = bf16_hi(t.y);
}
template <typename T> __device__ __forceinline__ void st4v(T* p, const float v[4]);
template <> __device__ __forceinline__ void st4v<float>(float* p, const float v[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> __device__ __forceinline__ void st4v<uint16_t>(uint16_t* p, const float v[4]) {
  const uint32_t lo = uint32_t(f32_to_bf16(v[0])) | (uint32_t(f32_to_bf16(v[1])) << 16);
  const uint32_t hi = uint32_t(f32_to_bf16(v[2])) | (uint32_t(f32_to_bf16(v[3])) << 16);
  *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}

template <int C>
__device__ __forceinline__ bool col4_ok(int lane, int e) {
  return C % 256 == 0 || 4 * lane + 256 * e < C;
}

template <typename TX, typename TR, int C>
__global__ void __launch_bounds__(256)
addln_fwd_v4_kernel(const TX* __restrict__ x, const TR* __restrict__ r, const float* __restrict__ w,
                    const float* __restrict__ b, int64_t rows, float eps, float* __restrict__ y,
                    uint16_t* __restrict__ y16, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int E4 = (C + 255) / 256;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = int64_t(gridDim.x) * 4;
  float wv[E4][4], bv[E4][4];
#pragma unroll
  for (int e = 0; e < E4; ++e) {
    const bool ok = col4_ok<C>(lane, e);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wv[e][i] = ok && w ? w[4 * lane + 256 * e + i] : 1.f;
      bv[e][i] = ok && b ? b[4 * lane + 256 * e + i] : 0.f;
    }
  }
  for (int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); row < rows; row += nwaves) {
    float s[E4][4];
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      if (col4_ok<C>(lane, e)) {
        const int64_t o = row * C + 4 * lane + 256 * e;
        float xv[4], rv[4] = {0.f, 0.f, 0.f, 0.f};
        ld4v<TX>(x + o, xv);
        if (r) ld4v<TR>(r + o, rv);
#pragma unroll
        for (int i = 0; i < 4; ++i) s[e][i] = xv[i] + rv[i];
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) s[e][i] = 0.f;
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < E4; ++e)
#pragma unroll
      for (int i = 0; i < 4; ++i) sum += s[e][i];
    const float mean = wsum(sum) / float(C);
    float sq = 0.f;
#pragma unroll
    for (int e = 0; e < E4; ++e)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = col4_ok<C>(lane, e) ? s[e][i] - mean : 0.f;
        sq += d * d;
      }
    const float rstd = rsqrtf(wsum(sq) / float(C) + eps);
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      if (!col4_ok<C>(lane, e)) continue;
      const int64_t o = row * C + 4 * lane + 256 * e;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (s[e][i] - mean) * rstd * wv[e][i] + bv[e][i];
      st4v<float>(y + o, v);
      if (y16) st4v<uint16_t>(y16 + o, v);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

template <typename TX, typename TR, int C>
__global__ void __launch_bounds__(256)
addln_bwd_v4_kernel(const float* __restrict__ dy, const float* __restrict__ dy2, const TX* __restrict__ x,
                    const TR* __restrict__ r, const float* __restrict__ w, const float* __restrict__ mean_in,
                    const float* __restrict__ rstd_in, int64_t rows, TX* __restrict__ dx, TR* __restrict__ dr,
                    float* __restrict__ part_w, float* __restrict__ part_b) {
  constexpr int E4 = (C + 255) / 256;
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = int64_t(gridDim.x) * 4;
  float wv[E4][4], gw[E4][4], gb[E4][4];
#pragma unroll
  for (int e = 0; e < E4; ++e)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wv[e][i] = col4_ok<C>(lane, e) && w ? w[4 * lane + 256 * e + i] : 1.f;
      gw[e][i] = gb[e][i] = 0.f;
    }
  for (int64_t row = wave_id; row < rows; row += nwaves) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[E4][4], g[E4][4];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      const bool ok = col4_ok<C>(lane, e);
      const int64_t o = row * C + 4 * lane + 256 * e;
      float xv[4] = {0.f, 0.f, 0.f, 0.f}, rv[4] = {0.f, 0.f, 0.f, 0.f}, d[4] = {0.f, 0.f, 0.f, 0.f},
            d2[4] = {0.f, 0.f, 0.f, 0.f};
      if (ok) {
        ld4v<TX>(x + o, xv);
        if (r) ld4v<TR>(r + o, rv);
        ld4v<float>(dy + o, d);
        if (dy2) ld4v<float>(dy2 + o, d2);  // a second consumer's gradient
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xh[e][i] = ok ? (xv[i] + rv[i] - mean) * rstd : 0.f;
        const float dd = d[i] + d2[i];
        gw[e][i] += dd * xh[e][i];
        gb[e][i] += dd;
        g[e][i] = dd * wv[e][i];
        sg += g[e][i];
        sgx += g[e][i] * xh[e][i];
      }
    }
    const float mg = wsum(sg) / float(C), mgx = wsum(sgx) / float(C);
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      if (!col4_ok<C>(lane, e)) continue;
      const int64_t o = row * C + 4 * lane + 256 * e;
      float ds[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) ds[i] = rstd * (g[e][i] - mg - xh[e][i] * mgx);
      st4v<TX>(dx + o, ds);
      if (dr) st4v<TR>(dr + o, ds);
    }
  }
  if (part_w) {  // combine the block's 4 waves in LDS: one partial row per block
    __shared__ float red[2][4][C];
    const int wv_i = threadIdx.x >> 6;
#pragma unroll
    for (int e = 0; e < E4; ++e) {
      if (!col4_ok<C>(lane, e)) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[0][wv_i][4 * lane + 256 * e + i] = gw[e][i];
        red[1][wv_i][4 * lane + 256 * e + i] = gb[e][i];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      part_w[int64_t(blockIdx.x) * C + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
      part_b[int64_t(blockIdx.x) * C + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
    }
  }
}

// ---------------------------------------------------------------------------
// Three-input variant for the deformable layers' attention sublayer (C = 256):
//   y = LayerNorm(x + (r + drop(r2)))
// x the fp32 residual stream, r the fp32 identity the MSDA module adds
// (reference ms_deform_attn.py `self.dropout(output) + identity`), r2 its
// bf16 output projection, drop() the module's dropout: the reference's
// bf16 dropout kernel, mixed bf16 + fp32 add and fp32 add + LayerNorm in one
// pass.  Dropout keeps element (row, col) when a counter-based hash of the
// seed (host value XOR the device word, graph-safe) clears p * 2^32; kept
// values are rounded to bf16 after the 1 / (1 - p) scale, as the reference's
// bf16 dropout output is.  The backward regenerates the mask: dx = dr = ds,
// dr2 = bf16(bf16(ds) * scale) where kept (autograd's cast of the gradient
// to the bf16 branch, then the dropout backward).
__device__ __forceinline__ uint32_t drop_hash(uint32_t seed, uint32_t row, uint32_t col) {
  uint32_t h = (col * 0x9E3779B1u) ^ (row * 0x85EBCA77u) ^ seed;
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}

struct Drop3 {
  float scale;        // 1 / (1 - p)
  uint32_t thresh;    // drop when hash < thresh (p * 2^32)
  uint32_t seed;
  const uint32_t* seed_dev;  // or NULL
};

template <bool DROP>
__device__ __forceinline__ float branch3(const uint16_t* r2, int64_t o, uint32_t row, int col, const Drop3& d) {
  const float v = bf16_to_f32(r2[o]);
  if constexpr (!DROP) {
    return v;
  } else {
    return drop_hash(d.seed, row, uint32_t(col)) >= d.thresh ? bf16_to_f32(f32_to_bf16(v * d.scale)) : 0.f;
  }
}

template <int C, bool DROP>
__global__ void __launch_bounds__(256)
addln3_fwd_kernel(const float* __restrict__ x, const float* __restrict__ r, const uint16_t* __restrict__ r2,
                  const float* __restrict__ w, const float* __restrict__ b, int64_t rows, float eps, Drop3 d,
                  float* __restrict__ y, uint16_t* __restrict__ y16, float* __restrict__ mean_out,
                  float* __restrict__ rstd_out) {
  constexpr int E = C / 64;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = int64_t(gridDim.x) * 4;
  if (DROP && d.seed_dev) d.seed ^= *d.seed_dev;
  float wv[E], bv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    wv[e] = w[lane + 64 * e];
    bv[e] = b[lane + 64 * e];
  }
  for (int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); row < rows; row += nwaves) {
    float s[E];
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t o = row * C + lane + 64 * e;
      s[e] = x[o] + (branch3<DROP>(r2, o, uint32_t(row), lane + 64 * e, d) + r[o]);
      sum += s[e];
    }
    const float mean = wsum(sum) / float(C);
    float sq = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) sq += (s[e] - mean) * (s[e] - mean);
    const float rstd = rsqrtf(wsum(sq) / float(C) + eps);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float v = (s[e] - mean) * rstd * wv[e] + bv[e];
      y[row * C + lane + 64 * e] = v;
      if (y16) y16[row * C + lane + 64 * e] = f32_to_bf16(v);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

template <int C, bool DROP>
__global__ void __launch_bounds__(256)
addln3_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ dy2, const float* __restrict__ x,
                  const float* __restrict__ r,
                  const uint16_t* __restrict__ r2, const float* __restrict__ w, const float* __restrict__ mean_in,
                  const float* __restrict__ rstd_in, int64_t rows, Drop3 d, float* __restrict__ dx,
                  uint16_t* __restrict__ dr2, float* __restrict__ part_w, float* __restrict__ part_b) {
  constexpr int E = C / 64;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = int64_t(gridDim.x) * 4;
  if (DROP && d.seed_dev) d.seed ^= *d.seed_dev;
  float wv[E], gw[E], gb[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    wv[e] = w[lane + 64 * e];
    gw[e] = gb[e] = 0.f;
  }
  for (int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); row < rows; row += nwaves) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[E], g[E];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t o = row * C + lane + 64 * e;
      const float s = x[o] + (branch3<DROP>(r2, o, uint32_t(row), lane + 64 * e, d) + r[o]);
      xh[e] = (s - mean) * rstd;
      const float dv = dy[o] + (dy2 ? dy2[o] : 0.f);
      gw[e] += dv * xh[e];
      gb[e] += dv;
      g[e] = dv * wv[e];
      sg += g[e];
      sgx += g[e] * xh[e];
    }
    const float mg = wsum(sg) / float(C), mgx = wsum(sgx) / float(C);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t o = row * C + lane + 64 * e;
      const float ds = rstd * (g[e] - mg - xh[e] * mgx);
      dx[o] = ds;
      if (dr2) {
        float v = bf16_to_f32(f32_to_bf16(ds));
        if (DROP) v = drop_hash(d.seed, uint32_t(row), uint32_t(lane + 64 * e)) >= d.thresh ? v * d.scale : 0.f;
        dr2[o] = f32_to_bf16(v);
      }
    }
  }
  __shared__ float red[2][4][C];
  const int wv_i = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    red[0][wv_i][lane + 64 * e] = gw[e];
    red[1][wv_i][lane + 64 * e] = gb[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part_w[int64_t(blockIdx.x) * C + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    part_b[int64_t(blockIdx.x) * C + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

// ---------------------------------------------------------------------------
// Pre-norm residual step of the Swin blocks (reference swin_transformer.py
// :295-296, `x = shortcut + drop_path(attn)` then `norm2(x)`):
//   s = x + branch * scale,  y = LayerNorm(s)
// with scale the per-sample drop-path factor (scale[row / n_per]) or one
// value, both outputs written (s is the residual stream the block adds the
// MLP to).  Backward takes both incoming gradients and sums them in the
// kernel: ds = g_s + LN'(g_y); dx = ds, d branch = ds * scale (branch dtype)
// -- the accumulation add autograd ran between the LayerNorm backward and
// the residual one, and that residual backward, folded away.
template <typename TB, int C>
__global__ void __launch_bounds__(256)
addsln_fwd_kernel(const float* __restrict__ x, const TB* __restrict__ br, const float* __restrict__ scale,
                  int64_t n_per, int per_sample, const float* __restrict__ w, const float* __restrict__ b,
                  int64_t rows, float eps, float* __restrict__ sum_out, float* __restrict__ y,
                  uint16_t* __restrict__ y16, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int E = (C + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = int64_t(gridDim.x) * 4;
  float wv[E], bv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const bool ok = col_ok<C>(lane, e);
    wv[e] = ok ? w[lane + 64 * e] : 1.f;
    bv[e] = ok ? b[lane + 64 * e] : 0.f;
  }
  for (int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); row < rows; row += nwaves) {
    const float sc = scale[per_sample ? row / n_per : 0];
    float s[E];
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t o = row * C + lane + 64 * e;
      s[e] = col_ok<C>(lane, e) ? x[o] + ldv<TB>(br + o) * sc : 0.f;
      sum += s[e];
    }
    const float mean = wsum(sum) / float(C);
    float sq = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float d = col_ok<C>(lane, e) ? s[e] - mean : 0.f;
      sq += d * d;
    }
    const float rstd = rsqrtf(wsum(sq) / float(C) + eps);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (!col_ok<C>(lane, e)) continue;
      const int64_t o = row * C + lane + 64 * e;
      const float v = (s[e] - mean) * rstd * wv[e] + bv[e];
      sum_out[o] = s[e];
      y[o] = v;
      if (y16) y16[o] = f32_to_bf16(v);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

template <typename TB, int C>
__global__ void __launch_bounds__(256)
addsln_bwd_kernel(const float* __restrict__ g_s, const float* __restrict__ g_y, const float* __restrict__ s_in,
                  const float* __restrict__ scale, int64_t n_per, int per_sample, const float* __restrict__ w,
                  const float* __restrict__ mean_in, const float* __restrict__ rstd_in, int64_t rows,
                  float* __restrict__ dx, TB* __restrict__ dbr, float* __restrict__ part_w,
                  float* __restrict__ part_b) {
  constexpr int E = (C + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = int64_t(gridDim.x) * 4;
  float wv[E], gw[E], gb[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    wv[e] = col_ok<C>(lane, e) ? w[lane + 64 * e] : 1.f;
    gw[e] = gb[e] = 0.f;
  }
  for (int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); row < rows; row += nwaves) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[E], g[E];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t o = row * C + lane + 64 * e;
      const bool ok = col_ok<C>(lane, e);
      xh[e] = ok ? (s_in[o] - mean) * rstd : 0.f;
      const float d = ok ? g_y[o] : 0.f;
      gw[e] += d * xh[e];
      gb[e] += d;
      g[e] = d * wv[e];
      sg += g[e];
      sgx += g[e] * xh[e];
    }
    const float mg = wsum(sg) / float(C), mgx = wsum(sgx) / float(C);
    const float sc = scale[per_sample ? row / n_per : 0];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (!col_ok<C>(lane, e)) continue;
      const int64_t o = row * C + lane + 64 * e;
      const float ds = rstd * (g[e] - mg - xh[e] * mgx) + (g_s ? g_s[o] : 0.f);
      dx[o] = ds;
      if (dbr) stv<TB>(dbr + o, ds * sc);
    }
  }
  __shared__ float red[2][4][C];
  const int wv_i = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (!col_ok<C>(lane, e)) continue;
    red[0][wv_i][lane + 64 * e] = gw[e];
    red[1][wv_i][lane + 64 * e] = gb[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part_w[int64_t(blockIdx.x) * C + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    part_b[int64_t(blockIdx.x) * C + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

template <typename Fn>
gd_status dispatch_sln(gd_dtype tb, int C, Fn&& fn) {
  GD_REQUIRE(tb == GD_F32 || tb == GD_BF16, "add_scaled_layernorm: branch dtype %d (F32, BF16)", int(tb));
  GD_REQUIRE(C == 96 || C == 192 || C == 256 || C == 384 || C == 768,
             "add_scaled_layernorm: C=%d not supported (96, 192, 256, 384, 768)", C);
  auto with_c = [&](auto tag) {
    switch (C) {
      case 96: fn(tag, std::integral_constant<int, 96>{}); break;
      case 192: fn(tag, std::integral_constant<int, 192>{}); break;
      case 256: fn(tag, std::integral_constant<int, 256>{}); break;
      case 384: fn(tag, std::integral_constant<int, 384>{}); break;
      default: fn(tag, std::integral_constant<int, 768>{}); break;
    }
  };
  if (tb == GD_BF16) with_c(uint16_t{});
  else with_c(float{});
  return GD_OK;
}

Drop3 make_drop3(float p, uint32_t seed, const uint32_t* seed_dev) {
  Drop3 d;
  d.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const double t = double(p) * 4294967296.0;
  d.thresh = p > 0.f ? uint32_t(t >= 4294967295.0 ? 4294967295.0 : t) : 0u;
  d.seed = seed;
  d.seed_dev = seed_dev;
  return d;
}

constexpr int kLnBlocks = 512;  // backward grid: 2048 waves, one partial row per block

// the 4-column vector kernels: a null pointer or one aligned to its 4-element
// vector (16 B fp32, 8 B bf16); GD_ADDLN_V4=0 keeps the scalar kernels (A/B)
bool v4_ok(const void* p, gd_dtype dt) {
  if (env_int("GD_ADDLN_V4", 1) == 0) return false;
  return !p || (reinterpret_cast<uintptr_t>(p) & (dt == GD_BF16 ? 7 : 15)) == 0;
}

template <typename Fn>
gd_status dispatch_types(gd_dtype tx, gd_dtype tr, bool has_r, int C, Fn&& fn) {
  GD_REQUIRE(tx == GD_F32 || tx == GD_BF16, "add_layernorm: x dtype %d (F32, BF16)", int(tx));
  GD_REQUIRE(!has_r || tr == GD_F32 || tr == GD_BF16, "add_layernorm: r dtype %d (F32, BF16)", int(tr));
  GD_REQUIRE(C == 64 || C == 96 || C == 128 || C == 192 || C == 256 || C == 384 || C == 512 || C == 768 ||
                 C == 1024 || C == 1536 || C == 2048,
             "add_layernorm: C=%d not supported (64, 96, 128, 192, 256, 384, 512, 768, 1024, 1536, 2048)", C);
  auto with_e = [&](auto tx_tag, auto tr_tag) {
    using TX = decltype(tx_tag);
    using TR = decltype(tr_tag);
    switch (C) {
      case 64: fn(TX{}, TR{}, std::integral_constant<int, 64>{}); break;
      case 96: fn(TX{}, TR{}, std::integral_constant<int, 96>{}); break;
      case 128: fn(TX{}, TR{}, std::integral_constant<int, 128>{}); break;
      case 192: fn(TX{}, TR{}, std::integral_constant<int, 192>{}); break;
      case 256: fn(TX{}, TR{}, std::integral_constant<int, 256>{}); break;
      case 384: fn(TX{}, TR{}, std::integral_constant<int, 384>{}); break;
      case 512: fn(TX{}, TR{}, std::integral_constant<int, 512>{}); break;
      case 768: fn(TX{}, TR{}, std::integral_constant<int, 768>{}); break;
      case 1024: fn(TX{}, TR{}, std::integral_constant<int, 1024>{}); break;
      case 1536: fn(TX{}, TR{}, std::integral_constant<int, 1536>{}); break;
      default: fn(TX{}, TR{}, std::integral_constant<int, 2048>{}); break;
    }
  };
  const bool xb = tx == GD_BF16, rb = has_r && tr == GD_BF16;
  if (xb && rb) with_e(uint16_t{}, uint16_t{});
  else if (xb) with_e(uint16_t{}, float{});
  else if (rb) with_e(float{}, uint16_t{});
  else with_e(float{}, float{});
  return GD_OK;
}

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" size_t gd_add_layernorm_workspace_bytes(int C) { return sizeof(float) * size_t(kLnBlocks) * C * 2; }

extern "C" gd_status gd_add_layernorm_forward(gd_dtype x_dtype, const void* x, gd_dtype r_dtype, const void* r,
                                             const float* weight, const float* bias, int64_t rows, int C,
                                             float eps, float* y, float* mean, float* rstd, gd_stream_t stream) {
  return gd_add_layernorm_forward2(x_dtype, x, r_dtype, r, weight, bias, rows, C, eps, y, nullptr, mean, rstd,
                                   stream);
}

extern "C" gd_status gd_add_layernorm_forward2(gd_dtype x_dtype, const void* x, gd_dtype r_dtype, const void* r,
                                              const float* weight, const float* bias, int64_t rows, int C,
                                              float eps, float* y, void* y_bf16, float* mean, float* rstd,
                                              gd_stream_t stream) {
  GD_REQUIRE(rows >= 0, "add_layernorm: rows < 0");
  if (rows == 0) return gd_status(GD_OK);
  GD_REQUIRE(x && y && mean && rstd, "add_layernorm_forward: null pointer");
  hipStream_t s = as_hip(stream);
  const int64_t blocks64 = (rows + 3) / 4;
  const unsigned blocks = unsigned(blocks64 < 8192 ? blocks64 : 8192);
  const bool v4 = v4_ok(x, x_dtype) && v4_ok(r, r_dtype) && v4_ok(y, GD_F32) && v4_ok(y_bf16, GD_BF16);
  gd_status st = dispatch_types(x_dtype, r_dtype, r != nullptr, C, [&](auto tx, auto tr, auto e) {
    using TX = decltype(tx);
    using TR = decltype(tr);
    if (v4)
      hipLaunchKernelGGL((addln_fwd_v4_kernel<TX, TR, decltype(e)::value>), dim3(blocks), dim3(256), 0, s,
                         (const TX*)x, (const TR*)r, weight, bias, rows, eps, y, (uint16_t*)y_bf16, mean, rstd);
    else
      hipLaunchKernelGGL((addln_fwd_kernel<TX, TR, decltype(e)::value>), dim3(blocks), dim3(256), 0, s,
                         (const TX*)x, (const TR*)r, weight, bias, rows, eps, y, (uint16_t*)y_bf16, mean, rstd);
  });
  if (st != GD_OK) return st;
  GD_LAUNCH_CHECK("add_layernorm_fwd");
  return GD_OK;
}

extern "C" gd_status gd_add_layernorm_backward2(gd_dtype x_dtype, const void* x, gd_dtype r_dtype, const void* r,
                                               const float* weight, const float* grad_y, const float* grad_y2,
                                               const float* mean, const float* rstd, int64_t rows, int C,
                                               void* grad_x, void* grad_r, float* grad_weight, float* grad_bias,
                                               void* workspace, gd_stream_t stream);

extern "C" gd_status gd_add_layernorm_backward(gd_dtype x_dtype, const void* x, gd_dtype r_dtype, const void* r,
                                              const float* weight, const float* grad_y, const float* mean,
                                              const float* rstd, int64_t rows, int C, void* grad_x, void* grad_r,
                                              float* grad_weight, float* grad_bias, void* workspace,
                                              gd_stream_t stream) {
  return gd_add_layernorm_backward2(x_dtype, x, r_dtype, r, weight, grad_y, nullptr, mean, rstd, rows, C, grad_x,
                                    grad_r, grad_weight, grad_bias, workspace, stream);
}

extern "C" gd_status gd_add_layernorm_backward2(gd_dtype x_dtype, const void* x, gd_dtype r_dtype, const void* r,
                                               const float* weight, const float* grad_y, const float* grad_y2,
                                               const float* mean, const float* rstd, int64_t rows, int C,
                                               void* grad_x, void* grad_r, float* grad_weight, float* grad_bias,
                                               void* workspace, gd_stream_t stream) {
  GD_REQUIRE(rows >= 0, "add_layernorm: rows < 0");
  GD_REQUIRE((grad_weight == nullptr) == (grad_bias == nullptr),
             "add_layernorm_backward: grad_weight and grad_bias are requested together");
  if (rows == 0) {
    hipStream_t s = as_hip(stream);
    if (grad_weight) GD_HIP_CHECK(fill_u32_async(grad_weight, 0u, sizeof(float) * C, s));
    if (grad_bias) GD_HIP_CHECK(fill_u32_async(grad_bias, 0u, sizeof(float) * C, s));
    return GD_OK;
  }
  GD_REQUIRE(x && grad_y && mean && rstd && grad_x, "add_layernorm_backward: null pointer");
  GD_REQUIRE(!grad_r || r, "add_layernorm_backward: grad_r without r");
  GD_REQUIRE(!grad_weight || workspace, "add_layernorm_backward: workspace missing");
  hipStream_t s = as_hip(stream);
  float* part_w = grad_weight ? static_cast<float*>(workspace) : nullptr;
  float* part_b = grad_weight ? part_w + int64_t(kLnBlocks) * C : nullptr;
  const bool v4 = v4_ok(x, x_dtype) && v4_ok(r, r_dtype) && v4_ok(grad_y, GD_F32) && v4_ok(grad_y2, GD_F32) &&
                  v4_ok(grad_x, x_dtype) && v4_ok(grad_r, r_dtype);
  gd_status st = dispatch_types(x_dtype, r_dtype, r != nullptr, C, [&](auto tx, auto tr, auto e) {
    using TX = decltype(tx);
    using TR = decltype(tr);
    if (v4)
      hipLaunchKernelGGL((addln_bwd_v4_kernel<TX, TR, decltype(e)::value>), dim3(kLnBlocks), dim3(256), 0, s,
                         grad_y, grad_y2, (const TX*)x, (const TR*)r, weight, mean, rstd, rows, (TX*)grad_x,
                         (TR*)grad_r, part_w, part_b);
    else
      hipLaunchKernelGGL((addln_bwd_kernel<TX, TR, decltype(e)::value>), dim3(kLnBlocks), dim3(256), 0, s, grad_y,
                         grad_y2, (const TX*)x, (const TR*)r, weight, mean, rstd, rows, (TX*)grad_x, (TR*)grad_r,
                         part_w, part_b);
  });
  if (st != GD_OK) return st;
  GD_LAUNCH_CHECK("add_layernorm_bwd");
  if (grad_weight) {
    hipLaunchKernelGGL(addln_reduce_kernel, dim3(unsigned((C + 15) / 16)), dim3(1024), 0, s, part_w, part_b,
                       kLnBlocks, C, grad_weight, grad_bias);
    GD_LAUNCH_CHECK("add_layernorm_reduce");
  }
  return GD_OK;
}

extern "C" gd_status gd_add_layernorm3_forward(const float* x, const float* r, const void* r2_bf16,
                                              const float* weight, const float* bias, int64_t rows, int C,
                                              float eps, float drop_p, uint32_t seed, const uint32_t* seed_dev,
                                              float* y, void* y_bf16, float* mean, float* rstd,
                                              gd_stream_t stream) {
  GD_REQUIRE(rows >= 0 && C == 256, "add_layernorm3: rows=%lld C=%d (C = 256)", (long long)rows, C);
  GD_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "add_layernorm3: dropout p=%f", double(drop_p));
  if (rows == 0) return GD_OK;
  GD_REQUIRE(x && r && r2_bf16 && weight && bias && y && mean && rstd, "add_layernorm3_forward: null pointer");
  const int64_t blocks64 = (rows + 3) / 4;
  const unsigned blocks = unsigned(blocks64 < 8192 ? blocks64 : 8192);
  const Drop3 d = make_drop3(drop_p, seed, seed_dev);
  if (drop_p > 0.f)
    hipLaunchKernelGGL((addln3_fwd_kernel<256, true>), dim3(blocks), dim3(256), 0, as_hip(stream), x, r,
                       (const uint16_t*)r2_bf16, weight, bias, rows, eps, d, y, (uint16_t*)y_bf16, mean, rstd);
  else
    hipLaunchKernelGGL((addln3_fwd_kernel<256, false>), dim3(blocks), dim3(256), 0, as_hip(stream), x, r,
                       (const uint16_t*)r2_bf16, weight, bias, rows, eps, d, y, (uint16_t*)y_bf16, mean, rstd);
  GD_LAUNCH_CHECK("add_layernorm3_fwd");
  return GD_OK;
}

extern "C" gd_status gd_add_layernorm3_backward(const float* x, const float* r, const void* r2_bf16,
                                               const float* weight, const float* grad_y, const float* grad_y2,
                                               const float* mean,
                                               const float* rstd, int64_t rows, int C, float drop_p, uint32_t seed,
                                               const uint32_t* seed_dev, float* grad_x, void* grad_r2_bf16,
                                               float* grad_weight, float* grad_bias, void* workspace,
                                               gd_stream_t stream) {
  GD_REQUIRE(rows >= 0 && C == 256, "add_layernorm3: rows=%lld C=%d (C = 256)", (long long)rows, C);
  GD_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "add_layernorm3: dropout p=%f", double(drop_p));
  GD_REQUIRE(grad_weight && grad_bias && workspace, "add_layernorm3_backward: grad_weight / grad_bias / workspace");
  hipStream_t s = as_hip(stream);
  if (rows == 0) {
    GD_HIP_CHECK(fill_u32_async(grad_weight, 0u, sizeof(float) * C, s));
    GD_HIP_CHECK(fill_u32_async(grad_bias, 0u, sizeof(float) * C, s));
    return GD_OK;
  }
  GD_REQUIRE(x && r && r2_bf16 && weight && grad_y && mean && rstd && grad_x,
             "add_layernorm3_backward: null pointer");
  float* part_w = static_cast<float*>(workspace);
  float* part_b = part_w + int64_t(kLnBlocks) * C;
  const Drop3 d = make_drop3(drop_p, seed, seed_dev);
  if (drop_p > 0.f)
    hipLaunchKernelGGL((addln3_bwd_kernel<256, true>), dim3(kLnBlocks), dim3(256), 0, s, grad_y, grad_y2, x, r,
                       (const uint16_t*)r2_bf16, weight, mean, rstd, rows, d, grad_x, (uint16_t*)grad_r2_bf16,
                       part_w, part_b);
  else
    hipLaunchKernelGGL((addln3_bwd_kernel<256, false>), dim3(kLnBlocks), dim3(256), 0, s, grad_y, grad_y2, x, r,
                       (const uint16_t*)r2_bf16, weight, mean, rstd, rows, d, grad_x, (uint16_t*)grad_r2_bf16,
                       part_w, part_b);
  GD_LAUNCH_CHECK("add_layernorm3_bwd");
  hipLaunchKernelGGL(addln_reduce_kernel, dim3(unsigned((C + 15) / 16)), dim3(1024), 0, s, part_w, part_b, kLnBlocks,
                     C, grad_weight, grad_bias);
  GD_LAUNCH_CHECK("add_layernorm3_reduce");
  return GD_OK;
}

extern "C" gd_status gd_add_scaled_layernorm_forward(const float* x, gd_dtype branch_dtype, const void* branch,
                                                    const float* scale, int64_t tokens_per_sample, int per_sample,
                                                    const float* weight, const float* bias, int64_t rows, int C,
                                                    float eps, float* sum, float* y, void* y_bf16, float* mean,
                                                    float* rstd, gd_stream_t stream) {
  GD_REQUIRE(rows >= 0 && (!per_sample || tokens_per_sample > 0), "add_scaled_layernorm: rows=%lld n=%lld",
             (long long)rows, (long long)tokens_per_sample);
  if (rows == 0) return GD_OK;
  GD_REQUIRE(x && branch && scale && weight && bias && sum && y && mean && rstd,
             "add_scaled_layernorm_forward: null pointer");
  const int64_t blocks64 = (rows + 3) / 4;
  const unsigned blocks = unsigned(blocks64 < 8192 ? blocks64 : 8192);
  hipStream_t s = as_hip(stream);
  gd_status st = dispatch_sln(branch_dtype, C, [&](auto tb, auto c) {
    using TB = decltype(tb);
    hipLaunchKernelGGL((addsln_fwd_kernel<TB, decltype(c)::value>), dim3(blocks), dim3(256), 0, s, x,
                       (const TB*)branch, scale, tokens_per_sample, per_sample, weight, bias, rows, eps, sum, y,
                       (uint16_t*)y_bf16, mean, rstd);
  });
  if (st != GD_OK) return st;
  GD_LAUNCH_CHECK("add_scaled_layernorm_fwd");
  return GD_OK;
}

extern "C" gd_status gd_add_scaled_layernorm_backward(const float* grad_sum, const float* grad_y, const float* sum,
                                                     gd_dtype branch_dtype, const float* scale,
                                                     int64_t tokens_per_sample, int per_sample, const float* weight,
                                                     const float* mean, const float* rstd, int64_t rows, int C,
                                                     float* grad_x, void* grad_branch, float* grad_weight,
                                                     float* grad_bias, void* workspace, gd_stream_t stream) {
  GD_REQUIRE(rows >= 0, "add_scaled_layernorm: rows < 0");
  GD_REQUIRE(grad_weight && grad_bias && workspace, "add_scaled_layernorm_backward: grad_weight / grad_bias");
  hipStream_t s = as_hip(stream);
  if (rows == 0) {
    GD_HIP_CHECK(fill_u32_async(grad_weight, 0u, sizeof(float) * C, s));
    GD_HIP_CHECK(fill_u32_async(grad_bias, 0u, sizeof(float) * C, s));
    return GD_OK;
  }
  GD_REQUIRE(grad_y && sum && scale && weight && mean && rstd && grad_x, "add_scaled_layernorm_backward: null pointer");
  float* part_w = static_cast<float*>(workspace);
  float* part_b = part_w + int64_t(kLnBlocks) * C;
  gd_status st = dispatch_sln(branch_dtype, C, [&](auto tb, auto c) {
    using TB = decltype(tb);
    hipLaunchKernelGGL((addsln_bwd_kernel<TB, decltype(c)::value>), dim3(kLnBlocks), dim3(256), 0, s, grad_sum,
                       grad_y, sum, scale, tokens_per_sample, per_sample, weight, mean, rstd, rows, grad_x,
                       (TB*)grad_branch, part_w, part_b);
  });
  if (st != GD_OK) return st;
  GD_LAUNCH_CHECK("add_scaled_layernorm_bwd");
  hipLaunchKernelGGL(addln_reduce_kernel, dim3(unsigned((C + 15) / 16)), dim3(1024), 0, s, part_w, part_b, kLnBlocks,
                     C, grad_weight, grad_bias);
  GD_LAUNCH_CHECK("add_scaled_layernorm_reduce");
  return GD_OK;
}
