// Box refinement  out = sigmoid(delta + inverse_sigmoid(ref))  for gfx950:
// the anchor update of every decoder layer (reference transformer.py:728-731)
// and the per-layer box heads (reference groundingdino.py:325-327), with
// inverse_sigmoid as util/misc.py:614-618:
//     rc = clamp(ref, 0, 1);  logit = log(max(rc, eps) / max(1 - rc, eps))
// The composition is 8 elementwise kernels forward and ~12 backward on
// [2, 900, 4] tensors (clamps, rsub, div, log, add, sigmoid and their
// backward masks), each a few microseconds of launch for 7 200 elements; here
// one kernel each way.
//
// Operands are 3-D [n0, n1, n2] with element strides (the heads read the
// decoder's reference points through a transposed view); out, grad_out and
// the gradients are contiguous in that logical order.  Backward, as autograd
// differentiates the composition:
//     g_z     = g * (1 - out) * out                      (sigmoid)
//     g_delta = g_z                                      (delta's dtype)
//     g_ref   = [0 <= ref <= 1] * ( [rc >= eps] g_z / max(rc, eps)
//                                 + [1 - rc >= eps] g_z / max(1 - rc, eps) )
// NaN in ref propagates forward (clamp keeps NaN) and gets a zero gradient
// (every clamp mask is false), as in the composition.
#include "gd_common.h"

#include <cmath>

namespace gd {
namespace {

struct Geo3 {
  int64_t n1, n2;          // logical shape (n0 implied by n)
  int64_t d0, d1, d2;      // delta strides
  int64_t r0, r1, r2;      // ref strides
};

template <typename T> __device__ __forceinline__ float ldf(const T* p);
template <> __device__ __forceinline__ float ldf<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ldf<uint16_t>(const uint16_t* p) { return bf16_lo(uint32_t(*p)); }
template <typename T> __device__ __forceinline__ void stf(T* p, float v);
template <> __device__ __forceinline__ void stf<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void stf<uint16_t>(uint16_t* p, float v) { *p = f32_to_bf16(v); }

__device__ __forceinline__ float clamp01(float v) { return v < 0.f ? 0.f : (v > 1.f ? 1.f : v); }  // NaN stays
__device__ __forceinline__ float atleast(float v, float lo) { return v < lo ? lo : v; }            // NaN stays

template <typename TD>
__global__ void __launch_bounds__(256)
box_refine_fwd_kernel(const TD* __restrict__ delta, const float* __restrict__ ref, Geo3 g, int64_t n, float eps,
                      float* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const int64_t i2 = i % g.n2, i1 = (i / g.n2) % g.n1, i0 = i / (g.n2 * g.n1);
    const float d = ldf(delta + i0 * g.d0 + i1 * g.d1 + i2 * g.d2);
    const float rc = clamp01(ref[i0 * g.r0 + i1 * g.r1 + i2 * g.r2]);
    const float z = d + logf(atleast(rc, eps) / atleast(1.f - rc, eps));
    out[i] = 1.f / (1.f + expf(-z));
  }
}

template <typename TD>
__global__ void __launch_bounds__(256)
box_refine_bwd_kernel(const float* __restrict__ grad_out, const float* __restrict__ out,
                      const float* __restrict__ ref, Geo3 g, int64_t n, float eps, TD* __restrict__ grad_delta,
                      float* __restrict__ grad_ref) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const float y = out[i];
    const float gz = grad_out[i] * (1.f - y) * y;
    if (grad_delta) stf(grad_delta + i, gz);
    if (grad_ref) {
      const int64_t i2 = i % g.n2, i1 = (i / g.n2) % g.n1, i0 = i / (g.n2 * g.n1);
      const float r = ref[i0 * g.r0 + i1 * g.r1 + i2 * g.r2];
      const float rc = clamp01(r);
      float gr = 0.f;
      if (rc >= eps) gr += gz / rc;
      if (1.f - rc >= eps) gr += gz / (1.f - rc);
      grad_ref[i] = (r >= 0.f && r <= 1.f) ? gr : 0.f;
    }
  }
}


// Decoder query anchors, per layer (reference transformer.py:660-672 via
// utils.py:204-230): from the layer's reference boxes ref [nq, bs, 4]
// (strided) and the valid ratios vr [bs, L, 4]
//     ref_input[q, b, l, :] = ref[q, b, :] * vr[b, l, :]
//     sine[q, b, 128 c + j]  = (j even ? sin : cos)(p_c * 2 pi / dim_t[j])
// with p = ref_input[q, b, 0, :] taken in the order (y, x, w, h) = (1, 0, 2, 3)
// and dim_t = 10000^(2 (j / 2) / 128) (the caller's device table).  The
// composition is seven launches per decoder layer (mul, index_select, div,
// two strided sin / cos, stack, the ratio product); here one, no gradient
// (the anchors are detached).  One thread per output feature of a (q, b) row.
__global__ void __launch_bounds__(256)
query_anchor_kernel(const float* __restrict__ ref, int64_t r0, int64_t r1, int64_t r2, int64_t nq, int64_t bs,
                    const float* __restrict__ vr, int L, const float* __restrict__ dim_t,
                    float* __restrict__ ref_input, float* __restrict__ sine) {
  const int64_t rows = nq * bs;
  const float two_pi = 6.283185307179586f;  // (float)(2 * math.pi), as the composition's scalar
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < rows * 512; i += int64_t(gridDim.x) * 256) {
    const int64_t row = i / 512;
    const int f = int(i - row * 512);
    const int64_t q = row / bs, b = row - q * bs;
    const int c = f / 128, j = f - c * 128;
    const int src = c == 0 ? 1 : (c == 1 ? 0 : c);
    const float p = ref[q * r0 + b * r1 + src * r2] * vr[b * L * 4 + src];
    const float v = (p * two_pi) / dim_t[j];
    sine[i] = (j & 1) ? cosf(v) : sinf(v);
    if (f < L * 4) {
      const int l = f / 4, k = f - l * 4;
      ref_input[row * L * 4 + f] = ref[q * r0 + b * r1 + k * r2] * vr[(b * L + l) * 4 + k];
    }
  }
}

template <typename Fn>
bool with_delta_type(gd_dtype d, Fn&& fn) {
  if (d == GD_F32) fn(float{});
  else if (d == GD_BF16) fn(uint16_t{});
  else return false;
  return true;
}

unsigned grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return unsigned(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" gd_status gd_box_refine_forward(gd_dtype delta_dtype, const void* delta, int64_t ds0, int64_t ds1,
                                           int64_t ds2, const float* ref, int64_t rs0, int64_t rs1, int64_t rs2,
                                           int64_t n0, int64_t n1, int64_t n2, float eps, float* out,
                                           gd_stream_t stream) {
  GD_REQUIRE(n0 >= 0 && n1 > 0 && n2 > 0, "box_refine: shape %lld x %lld x %lld", (long long)n0, (long long)n1,
             (long long)n2);
  GD_REQUIRE(delta_dtype == GD_F32 || delta_dtype == GD_BF16, "box_refine: delta dtype %d (F32, BF16)",
             int(delta_dtype));
  const int64_t n = n0 * n1 * n2;
  if (n == 0) return GD_OK;
  GD_REQUIRE(delta && ref && out, "box_refine_forward: null pointer");
  const Geo3 g{n1, n2, ds0, ds1, ds2, rs0, rs1, rs2};
  hipStream_t st = as_hip(stream);
  with_delta_type(delta_dtype, [&](auto td) {
    using TD = decltype(td);
    hipLaunchKernelGGL((box_refine_fwd_kernel<TD>), dim3(grid_for(n)), dim3(256), 0, st, (const TD*)delta, ref, g,
                       n, eps, out);
  });
  GD_LAUNCH_CHECK("box_refine_forward");
  return GD_OK;
}

extern "C" gd_status gd_box_refine_backward(gd_dtype delta_dtype, const float* grad_out, const float* out,
                                            const float* ref, int64_t rs0, int64_t rs1, int64_t rs2, int64_t n0,
                                            int64_t n1, int64_t n2, float eps, void* grad_delta, float* grad_ref,
                                            gd_stream_t stream) {
  GD_REQUIRE(n0 >= 0 && n1 > 0 && n2 > 0, "box_refine: shape %lld x %lld x %lld", (long long)n0, (long long)n1,
             (long long)n2);
  GD_REQUIRE(delta_dtype == GD_F32 || delta_dtype == GD_BF16, "box_refine: delta dtype %d (F32, BF16)",
             int(delta_dtype));
  const int64_t n = n0 * n1 * n2;
  if (n == 0 || (!grad_delta && !grad_ref)) return GD_OK;
  GD_REQUIRE(grad_out && out && (!grad_ref || ref), "box_refine_backward: null pointer");
  const Geo3 g{n1, n2, 0, 0, 0, rs0, rs1, rs2};
  hipStream_t st = as_hip(stream);
  with_delta_type(delta_dtype, [&](auto td) {
    using TD = decltype(td);
    hipLaunchKernelGGL((box_refine_bwd_kernel<TD>), dim3(grid_for(n)), dim3(256), 0, st, grad_out, out, ref, g, n,
                       eps, (TD*)grad_delta, grad_ref);
  });
  GD_LAUNCH_CHECK("box_refine_backward");
  return GD_OK;
}

extern "C" gd_status gd_query_anchor_forward(const float* ref, int64_t rs0, int64_t rs1, int64_t rs2, int64_t nq,
                                            int64_t bs, const float* valid_ratios, int L, const float* dim_t,
                                            float* ref_input, float* sine, gd_stream_t stream) {
  GD_REQUIRE(nq >= 0 && bs > 0 && L > 0 && L * 4 <= 512, "query_anchor: nq=%lld bs=%lld L=%d", (long long)nq,
             (long long)bs, L);
  if (nq == 0) return GD_OK;
  GD_REQUIRE(ref && valid_ratios && dim_t && ref_input && sine, "query_anchor: null pointer");
  hipLaunchKernelGGL(query_anchor_kernel, dim3(grid_for(nq * bs * 512)), dim3(256), 0, as_hip(stream), ref, rs0, rs1,
                     rs2, nq, bs, valid_ratios, L, dim_t, ref_input, sine);
  GD_LAUNCH_CHECK("query_anchor_forward");
  return GD_OK;
}
