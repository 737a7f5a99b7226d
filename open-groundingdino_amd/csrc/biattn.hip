// Bidirectional softmax of BiMultiHeadAttention for gfx950.
//
// Reference: models/GroundingDINO/fuse_modules.py:174-217.  One score matrix
// s = q.k^T [BH, S, T] (S image tokens, T text tokens; produced by a
// hipBLASLt GEMM) feeds two softmaxes:
//   P_v = softmax over T of (s + mask_l)     (image queries attend text)
//   P_l = softmax over S of (s + mask_v)     (text queries attend image),
//         stored in the same [BH, S, T] layout (column-normalised), so the
//         text-side output is the GEMM P_l^T . v_v.
// The reference's global-max shift, column-max shift and +-5e4 clamps are
// shift/clamp guards that leave softmax unchanged for any score spread below
// 5e4 (fp32 statistics here); see DESIGN.md.
//
// Forward  (3 launches, S read twice, P_v / P_l written once):
//   colstats  : per (column block of rows) online max / sum-exp per column t
//   colmerge  : merge the row-chunk partials -> m_t, 1/l_t
//   rows      : one wave per row: row max / sum over T by wave shuffles,
//               writes P_v and P_l = exp(s - m_t) / l_t.
// Backward (3 launches):
//   colsum    : c_t partials of sum_s dP_l * P_l
//   colmerge  : -> c_t
//   rows      : r_s = sum_t dP_v * P_v by wave shuffles,
//               dS = P_v (dP_v - r_s) + P_l (dP_l - c_t).
// Padding: pad_v[b, s] masks image row s out of every column softmax (P_l = 0),
// pad_l[b, t] masks text column t out of every row softmax (P_v = 0).
#include "gd_common.h"

namespace gd {
namespace {

constexpr int kRowsPerChunk = 128;

template <typename T> __device__ __forceinline__ float ldf(const T* p);
template <> __device__ __forceinline__ float ldf<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ldf<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }
template <typename T> __device__ __forceinline__ void stf(T* p, float v);
template <> __device__ __forceinline__ void stf<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void stf<uint16_t>(uint16_t* p, float v) { *p = f32_to_bf16(v); }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// grid (nchunk, BH), block 256: thread owns columns t = tid, tid+256, ...
// and walks the chunk's rows (coalesced across the block).
template <typename T>
__global__ void __launch_bounds__(256)
colstats_kernel(const T* __restrict__ s, const uint8_t* __restrict__ pad_v, int H, int S, int Tn,
                float* __restrict__ pm, float* __restrict__ pl) {
  const int chunk = blockIdx.x, bh = blockIdx.y, b = bh / H;
  const int r0 = chunk * kRowsPerChunk;
  const int r1 = min(S, r0 + kRowsPerChunk);
  const size_t nchunk = gridDim.x;
  for (int t = threadIdx.x; t < Tn; t += blockDim.x) {
    float m = -INFINITY, l = 0.f;
    for (int r = r0; r < r1; ++r) {
      if (pad_v && pad_v[size_t(b) * S + r]) continue;
      const float x = ldf<T>(s + (size_t(bh) * S + r) * Tn + t);
      if (x > m) {
        l = l * __expf(m - x) + 1.f;
        m = x;
      } else {
        l += __expf(x - m);
      }
    }
    pm[(size_t(bh) * nchunk + chunk) * Tn + t] = m;
    pl[(size_t(bh) * nchunk + chunk) * Tn + t] = l;
  }
}

// grid BH, block 256: merge nchunk partials of each column.
__global__ void __launch_bounds__(256)
colmerge_kernel(const float* __restrict__ pm, const float* __restrict__ pl, int nchunk, int Tn,
                float* __restrict__ col_m, float* __restrict__ col_inv) {
  const int bh = blockIdx.x;
  for (int t = threadIdx.x; t < Tn; t += blockDim.x) {
    float m = -INFINITY;
    for (int c = 0; c < nchunk; ++c) m = fmaxf(m, pm[(size_t(bh) * nchunk + c) * Tn + t]);
    float l = 0.f;
    if (m != -INFINITY)
      for (int c = 0; c < nchunk; ++c) {
        const float mc = pm[(size_t(bh) * nchunk + c) * Tn + t];
        if (mc != -INFINITY) l += pl[(size_t(bh) * nchunk + c) * Tn + t] * __expf(mc - m);
      }
    col_m[size_t(bh) * Tn + t] = m;
    col_inv[size_t(bh) * Tn + t] = l > 0.f ? 1.f / l : 0.f;
  }
}

// one wave per row of [BH*S, T]
template <typename T>
__global__ void __launch_bounds__(256)
rows_fwd_kernel(const T* __restrict__ s, const uint8_t* __restrict__ pad_v, const uint8_t* __restrict__ pad_l,
                const float* __restrict__ col_m, const float* __restrict__ col_inv, int H, int S, int Tn,
                int64_t nrows, T* __restrict__ pv, T* __restrict__ plo) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const int bh = int(row / S), r = int(row % S), b = bh / H;
  const T* sr = s + row * Tn;
  const bool row_pad = pad_v && pad_v[size_t(b) * S + r];
  constexpr int MAXE = 16;  // T <= 1024
  float x[MAXE];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    const int t = lane + 64 * j;
    x[j] = -INFINITY;
    if (t < Tn) {
      const float v = ldf<T>(sr + t);
      const bool cp = pad_l && pad_l[size_t(b) * Tn + t];
      x[j] = cp ? -INFINITY : v;
      mx = fmaxf(mx, x[j]);
      // column softmax output (independent of the row statistics)
      const float ci = col_inv[size_t(bh) * Tn + t];
      const float pcol = (row_pad || ci == 0.f) ? 0.f : __expf(v - col_m[size_t(bh) * Tn + t]) * ci;
      stf<T>(plo + row * Tn + t, pcol);
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    const int t = lane + 64 * j;
    if (t < Tn) {
      x[j] = (mx == -INFINITY) ? 0.f : __expf(x[j] - mx);
      sum += x[j];
    }
  }
  sum = wave_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    const int t = lane + 64 * j;
    if (t < Tn) stf<T>(pv + row * Tn + t, x[j] * inv);
  }
}

// backward: column partial sums of dP_l * P_l
template <typename T>
__global__ void __launch_bounds__(256)
colsum_kernel(const T* __restrict__ plo, const T* __restrict__ dpl, int S, int Tn, float* __restrict__ part) {
  const int chunk = blockIdx.x, bh = blockIdx.y;
  const int r0 = chunk * kRowsPerChunk;
  const int r1 = min(S, r0 + kRowsPerChunk);
  const size_t nchunk = gridDim.x;
  for (int t = threadIdx.x; t < Tn; t += blockDim.x) {
    float acc = 0.f;
    for (int r = r0; r < r1; ++r) {
      const size_t o = (size_t(bh) * S + r) * Tn + t;
      acc += ldf<T>(plo + o) * ldf<T>(dpl + o);
    }
    part[(size_t(bh) * nchunk + chunk) * Tn + t] = acc;
  }
}

__global__ void __launch_bounds__(256)
colsum_merge_kernel(const float* __restrict__ part, int nchunk, int Tn, float* __restrict__ csum) {
  const int bh = blockIdx.x;
  for (int t = threadIdx.x; t < Tn; t += blockDim.x) {
    float acc = 0.f;
    for (int c = 0; c < nchunk; ++c) acc += part[(size_t(bh) * nchunk + c) * Tn + t];
    csum[size_t(bh) * Tn + t] = acc;
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
rows_bwd_kernel(const T* __restrict__ pv, const T* __restrict__ plo, const T* __restrict__ dpv,
                const T* __restrict__ dpl, const float* __restrict__ csum, int S, int Tn, int64_t nrows,
                T* __restrict__ ds) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const int bh = int(row / S);
  constexpr int MAXE = 16;
  float p[MAXE], g[MAXE];
  float r = 0.f;
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    const int t = lane + 64 * j;
    p[j] = g[j] = 0.f;
    if (t < Tn) {
      p[j] = ldf<T>(pv + row * Tn + t);
      g[j] = ldf<T>(dpv + row * Tn + t);
      r += p[j] * g[j];
    }
  }
  r = wave_sum(r);
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    const int t = lane + 64 * j;
    if (t < Tn) {
      const float q = ldf<T>(plo + row * Tn + t);
      const float gq = ldf<T>(dpl + row * Tn + t);
      const float v = p[j] * (g[j] - r) + q * (gq - csum[size_t(bh) * Tn + t]);
      stf<T>(ds + row * Tn + t, v);
    }
  }
}

inline int nchunks(int S) { return (S + kRowsPerChunk - 1) / kRowsPerChunk; }

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" size_t gd_biattn_workspace_bytes(int B, int H, int S, int T) {
  const size_t bh = size_t(B) * H;
  return sizeof(float) * (bh * nchunks(S) * T * 2 + bh * T * 2);
}

extern "C" gd_status gd_biattn_softmax_fwd(gd_dtype dt, const void* s, const uint8_t* pad_v,
                                           const uint8_t* pad_l, int B, int H, int S, int T, void* pv,
                                           void* pl, void* workspace, gd_stream_t stream) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "biattn: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(B >= 0 && H > 0 && S >= 0 && T > 0 && T <= 1024, "biattn: bad sizes B=%d H=%d S=%d T=%d", B, H, S,
             T);
  if (B == 0 || S == 0) return GD_OK;
  GD_REQUIRE(s && pv && pl && workspace, "biattn_fwd: null pointer");
  hipStream_t st = as_hip(stream);
  const int bh = B * H, nc = nchunks(S);
  float* pm = static_cast<float*>(workspace);
  float* plp = pm + size_t(bh) * nc * T;
  float* col_m = plp + size_t(bh) * nc * T;
  float* col_inv = col_m + size_t(bh) * T;
  const int64_t nrows = int64_t(bh) * S;
  const int rblocks = int((nrows + 3) / 4);
  if (dt == GD_BF16) {
    colstats_kernel<uint16_t><<<dim3(nc, bh), 256, 0, st>>>((const uint16_t*)s, pad_v, H, S, T, pm, plp);
    GD_LAUNCH_CHECK("biattn colstats");
    colmerge_kernel<<<bh, 256, 0, st>>>(pm, plp, nc, T, col_m, col_inv);
    GD_LAUNCH_CHECK("biattn colmerge");
    rows_fwd_kernel<uint16_t><<<rblocks, 256, 0, st>>>((const uint16_t*)s, pad_v, pad_l, col_m, col_inv, H, S,
                                                      T, nrows, (uint16_t*)pv, (uint16_t*)pl);
    GD_LAUNCH_CHECK("biattn rows_fwd");
  } else {
    colstats_kernel<float><<<dim3(nc, bh), 256, 0, st>>>((const float*)s, pad_v, H, S, T, pm, plp);
    GD_LAUNCH_CHECK("biattn colstats");
    colmerge_kernel<<<bh, 256, 0, st>>>(pm, plp, nc, T, col_m, col_inv);
    GD_LAUNCH_CHECK("biattn colmerge");
    rows_fwd_kernel<float><<<rblocks, 256, 0, st>>>((const float*)s, pad_v, pad_l, col_m, col_inv, H, S, T,
                                                   nrows, (float*)pv, (float*)pl);
    GD_LAUNCH_CHECK("biattn rows_fwd");
  }
  return GD_OK;
}

extern "C" gd_status gd_biattn_softmax_bwd(gd_dtype dt, const void* pv, const void* pl, const void* dpv,
                                           const void* dpl, int B, int H, int S, int T, void* ds,
                                           void* workspace, gd_stream_t stream) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "biattn: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(B >= 0 && H > 0 && S >= 0 && T > 0 && T <= 1024, "biattn: bad sizes B=%d H=%d S=%d T=%d", B, H, S,
             T);
  if (B == 0 || S == 0) return GD_OK;
  GD_REQUIRE(pv && pl && dpv && dpl && ds && workspace, "biattn_bwd: null pointer");
  hipStream_t st = as_hip(stream);
  const int bh = B * H, nc = nchunks(S);
  float* part = static_cast<float*>(workspace);
  float* csum = part + size_t(bh) * nc * T * 2;
  const int64_t nrows = int64_t(bh) * S;
  const int rblocks = int((nrows + 3) / 4);
  if (dt == GD_BF16) {
    colsum_kernel<uint16_t><<<dim3(nc, bh), 256, 0, st>>>((const uint16_t*)pl, (const uint16_t*)dpl, S, T, part);
    GD_LAUNCH_CHECK("biattn colsum");
    colsum_merge_kernel<<<bh, 256, 0, st>>>(part, nc, T, csum);
    GD_LAUNCH_CHECK("biattn colsum_merge");
    rows_bwd_kernel<uint16_t><<<rblocks, 256, 0, st>>>((const uint16_t*)pv, (const uint16_t*)pl,
                                                      (const uint16_t*)dpv, (const uint16_t*)dpl, csum, S, T,
                                                      nrows, (uint16_t*)ds);
    GD_LAUNCH_CHECK("biattn rows_bwd");
  } else {
    colsum_kernel<float><<<dim3(nc, bh), 256, 0, st>>>((const float*)pl, (const float*)dpl, S, T, part);
    GD_LAUNCH_CHECK("biattn colsum");
    colsum_merge_kernel<<<bh, 256, 0, st>>>(part, nc, T, csum);
    GD_LAUNCH_CHECK("biattn colsum_merge");
    rows_bwd_kernel<float><<<rblocks, 256, 0, st>>>((const float*)pv, (const float*)pl, (const float*)dpv,
                                                   (const float*)dpl, csum, S, T, nrows, (float*)ds);
    GD_LAUNCH_CHECK("biattn rows_bwd");
  }
  return GD_OK;
}
