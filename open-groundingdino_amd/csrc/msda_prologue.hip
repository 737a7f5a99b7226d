// MSDA prologue for gfx950: the projections' outputs -> sampling locations
// and attention weights, forward and backward, one kernel each.
//
// Reference math (models/GroundingDINO/ms_deform_attn.py:274-363, the mmcv
// module it mirrors): for each unit (n, q, head m) and sample s = (l, p),
//   attn[s] = softmax over the unit's L*P logits
//   loc[s]  = ref[l].xy + off[s] / (W_l, H_l)                  (2-d refs)
//           = ref[l].xy + off[s] / P * ref[l].wh * 0.5         (4-d refs)
// The reference composes this from a cast, a softmax, a cast, a division
// and an addition over [N, Lq, M, L, P, 2] fp32 tensors (and their
// backward); here one thread owns one sample and the softmax over a unit's
// 16 samples is a 16-lane shuffle reduction.  The element arithmetic keeps
// the reference's operation order with round-to-nearest intrinsics (no FMA
// contraction), so loc matches the fp32 composition bit for bit.
//
// Layouts: off [N, Lq, M*L*P*2] and logits [N, Lq, M*L*P] rows with their own
// row strides (the two column blocks of the fused offsets / attention
// Linear, read in place); ref [N, Lq, L, 2|4] fp32; loc [N, Lq, M, L, P, 2],
// attn [N, Lq, M, L, P] fp32.  Backward writes grad_off / grad_logits
// contiguous in the projection dtype.  L*P == 16.
#include "gd_common.h"

#include <cmath>

namespace gd {
namespace {

template <typename T> __device__ __forceinline__ float ld1(const T* p);
template <> __device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld1<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }
template <typename T> __device__ __forceinline__ void st1(T* p, float v);
template <> __device__ __forceinline__ void st1<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st1<uint16_t>(uint16_t* p, float v) { *p = f32_to_bf16(v); }

__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 1, 16);
  v += __shfl_xor(v, 2, 16);
  v += __shfl_xor(v, 4, 16);
  v += __shfl_xor(v, 8, 16);
  return v;
}
__device__ __forceinline__ float max16(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 16));
  v = fmaxf(v, __shfl_xor(v, 2, 16));
  v = fmaxf(v, __shfl_xor(v, 4, 16));
  v = fmaxf(v, __shfl_xor(v, 8, 16));
  return v;
}

// one thread per (unit, sample); 16 consecutive threads = one unit
template <typename T>
__global__ void __launch_bounds__(256)
prologue_fwd_kernel(const T* __restrict__ off, int64_t ors, const T* __restrict__ logits, int64_t lrs,
                    const float* __restrict__ ref, int rdim, const int64_t* __restrict__ shapes, int M, int L,
                    int P, int64_t units, float* __restrict__ loc, float* __restrict__ attn) {
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t unit = t >> 4;
  const bool live = unit < units;
  const int s = int(t & 15);
  const int64_t u = live ? unit : 0;
  const int64_t row = u / M;
  const int m = int(u - row * M);
  const int l = s / P;
  // softmax over the unit's 16 logits (every lane of the 16-group takes part)
  const float x = ld1<T>(logits + row * lrs + m * 16 + s);
  const float mx = max16(x);
  const float e = expf(x - mx);
  const float a = e / sum16(e);
  if (!live) return;
  attn[unit * 16 + s] = a;
  const T* op = off + row * ors + (m * 16 + s) * 2;
  const float ox = ld1<T>(op), oy = ld1<T>(op + 1);
  float lx, ly;
  if (rdim == 2) {
    const float* rp = ref + (row * L + l) * 2;
    lx = __fadd_rn(rp[0], __fdiv_rn(ox, float(shapes[2 * l + 1])));
    ly = __fadd_rn(rp[1], __fdiv_rn(oy, float(shapes[2 * l])));
  } else {
    const float* rp = ref + (row * L + l) * 4;
    const float fp = float(P);
    lx = __fadd_rn(rp[0], __fmul_rn(__fmul_rn(__fdiv_rn(ox, fp), rp[2]), 0.5f));
    ly = __fadd_rn(rp[1], __fmul_rn(__fmul_rn(__fdiv_rn(oy, fp), rp[3]), 0.5f));
  }
  *reinterpret_cast<float2*>(loc + (unit * 16 + s) * 2) = make_float2(lx, ly);
}

template <typename T>
__global__ void __launch_bounds__(256)
prologue_bwd_kernel(const float* __restrict__ grad_loc, const float* __restrict__ grad_attn,
                    const float* __restrict__ attn, const float* __restrict__ ref, int rdim,
                    const int64_t* __restrict__ shapes, int M, int L, int P, int64_t units, T* __restrict__ grad_off,
                    T* __restrict__ grad_logits) {
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t unit = t >> 4;
  const bool live = unit < units;
  const int s = int(t & 15);
  const int64_t e = (live ? unit : 0) * 16 + s;
  const int64_t row = (live ? unit : 0) / M;
  const int l = s / P;
  // softmax backward: a (g - sum_s' a g)
  const float a = attn[e], g = grad_attn[e];
  const float dot = sum16(a * g);
  if (!live) return;
  st1<T>(grad_logits + e, a * (g - dot));
  const float2 gl = *reinterpret_cast<const float2*>(grad_loc + e * 2);
  float gx, gy;
  if (rdim == 2) {
    gx = __fdiv_rn(gl.x, float(shapes[2 * l + 1]));
    gy = __fdiv_rn(gl.y, float(shapes[2 * l]));
  } else {  // autograd of ((off / P) * wh) * 0.5: ((g * 0.5) * wh) / P
    const float* rp = ref + (row * L + l) * 4;
    const float fp = float(P);
    gx = __fdiv_rn(__fmul_rn(__fmul_rn(gl.x, 0.5f), rp[2]), fp);
    gy = __fdiv_rn(__fmul_rn(__fmul_rn(gl.y, 0.5f), rp[3]), fp);
  }
  st1<T>(grad_off + e * 2, gx);
  st1<T>(grad_off + e * 2 + 1, gy);
}

}  // namespace
}  // namespace gd

using namespace gd;

static gd_status prologue_check(gd_dtype dt, int N, int Lq, int M, int L, int P, int rdim) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "msda_prologue: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(N >= 0 && Lq >= 0 && M > 0 && L > 0 && P > 0 && L * P == 16,
             "msda_prologue: bad sizes N=%d Lq=%d M=%d L=%d P=%d (L*P must be 16)", N, Lq, M, L, P);
  GD_REQUIRE(rdim == 2 || rdim == 4, "msda_prologue: reference points must have 2 or 4 coordinates, got %d",
             rdim);
  return GD_OK;
}

extern "C" gd_status gd_msda_prologue_forward(gd_dtype dt, const void* offsets, int64_t offsets_row_stride,
                                             const void* logits, int64_t logits_row_stride,
                                             const float* reference_points, int ref_dim,
                                             const int64_t* spatial_shapes, int N, int Lq, int M, int L, int P,
                                             float* sampling_loc, float* attn_weight, gd_stream_t stream) {
  const gd_status st = prologue_check(dt, N, Lq, M, L, P, ref_dim);
  if (st != GD_OK) return st;
  const int64_t units = int64_t(N) * Lq * M;
  if (units == 0) return GD_OK;
  GD_REQUIRE(offsets && logits && reference_points && spatial_shapes && sampling_loc && attn_weight,
             "msda_prologue_forward: null pointer");
  GD_REQUIRE(offsets_row_stride >= int64_t(M) * 32 && logits_row_stride >= int64_t(M) * 16,
             "msda_prologue_forward: row strides too small");
  const int64_t blocks = (units * 16 + 255) / 256;
  GD_REQUIRE(blocks < (int64_t(1) << 31), "msda_prologue_forward: grid too large");
  hipStream_t s = as_hip(stream);
  if (dt == GD_BF16)
    hipLaunchKernelGGL((prologue_fwd_kernel<uint16_t>), dim3(unsigned(blocks)), dim3(256), 0, s,
                       (const uint16_t*)offsets, offsets_row_stride, (const uint16_t*)logits, logits_row_stride,
                       reference_points, ref_dim, spatial_shapes, M, L, P, units, sampling_loc, attn_weight);
  else
    hipLaunchKernelGGL((prologue_fwd_kernel<float>), dim3(unsigned(blocks)), dim3(256), 0, s,
                       (const float*)offsets, offsets_row_stride, (const float*)logits, logits_row_stride,
                       reference_points, ref_dim, spatial_shapes, M, L, P, units, sampling_loc, attn_weight);
  GD_LAUNCH_CHECK("msda_prologue_fwd");
  return GD_OK;
}

extern "C" gd_status gd_msda_prologue_backward(gd_dtype dt, const float* grad_loc, const float* grad_attn,
                                              const float* attn_weight, const float* reference_points,
                                              int ref_dim, const int64_t* spatial_shapes, int N, int Lq, int M,
                                              int L, int P, void* grad_offsets, void* grad_logits,
                                              gd_stream_t stream) {
  const gd_status st = prologue_check(dt, N, Lq, M, L, P, ref_dim);
  if (st != GD_OK) return st;
  const int64_t units = int64_t(N) * Lq * M;
  if (units == 0) return GD_OK;
  GD_REQUIRE(grad_loc && grad_attn && attn_weight && reference_points && spatial_shapes && grad_offsets &&
                 grad_logits,
             "msda_prologue_backward: null pointer");
  const int64_t blocks = (units * 16 + 255) / 256;
  GD_REQUIRE(blocks < (int64_t(1) << 31), "msda_prologue_backward: grid too large");
  hipStream_t s = as_hip(stream);
  if (dt == GD_BF16)
    hipLaunchKernelGGL((prologue_bwd_kernel<uint16_t>), dim3(unsigned(blocks)), dim3(256), 0, s, grad_loc,
                       grad_attn, attn_weight, reference_points, ref_dim, spatial_shapes, M, L, P, units,
                       (uint16_t*)grad_offsets, (uint16_t*)grad_logits);
  else
    hipLaunchKernelGGL((prologue_bwd_kernel<float>), dim3(unsigned(blocks)), dim3(256), 0, s, grad_loc, grad_attn,
                       attn_weight, reference_points, ref_dim, spatial_shapes, M, L, P, units,
                       (float*)grad_offsets, (float*)grad_logits);
  GD_LAUNCH_CHECK("msda_prologue_bwd");
  return GD_OK;
}
