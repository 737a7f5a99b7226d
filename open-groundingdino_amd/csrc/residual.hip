// Scaled residual ending  out = x + branch * s  for gfx950, s broadcast per
// (sample, channel) -- the layer-scale + stochastic-depth residuals of the
// BiAttention fusion block (reference fuse_modules.py:285-286:
// `v = v + drop_path(gamma_v * delta_v)`) and the drop-path residuals of the
// Swin blocks (swin_transformer.py:295-296).  The composition runs them as a
// broadcast addcmul forward and three passes backward (g * s, g * branch, a
// token reduction of that product); here one streaming kernel forward and one
// backward (d branch = g * s stored in branch's dtype, plus per-chunk column
// partials of g * branch) and a fixed-order merge of the partials
// (deterministic).
//
// Layout: x / branch / out / g are [B, N, C] contiguous, C % 4 == 0; s is
// fp32 at s[b * s_bstride + c * s_cstride] (strides 0 broadcast).  Each thread
// moves 4 consecutive channels (16-B fp32 / 8-B bf16 vectors); every
// iteration of a block covers whole rows so a thread keeps the same 4
// channels and its partial sums stay in registers.
#include "gd_common.h"

namespace gd {
namespace {

struct f4 {
  float v[4];
};

template <typename T> __device__ __forceinline__ f4 ld4(const T* p);
template <> __device__ __forceinline__ f4 ld4<float>(const float* p) {
  const float4 q = *reinterpret_cast<const float4*>(p);
  return {{q.x, q.y, q.z, q.w}};
}
template <> __device__ __forceinline__ f4 ld4<uint16_t>(const uint16_t* p) {
  const uint2 q = *reinterpret_cast<const uint2*>(p);
  return {{bf16_lo(q.x), bf16_hi(q.x), bf16_lo(q.y), bf16_hi(q.y)}};
}
template <typename T> __device__ __forceinline__ void st4(T* p, const f4& a);
template <> __device__ __forceinline__ void st4<float>(float* p, const f4& a) {
  *reinterpret_cast<float4*>(p) = make_float4(a.v[0], a.v[1], a.v[2], a.v[3]);
}
template <> __device__ __forceinline__ void st4<uint16_t>(uint16_t* p, const f4& a) {
  uint2 q;
  q.x = uint32_t(f32_to_bf16(a.v[0])) | (uint32_t(f32_to_bf16(a.v[1])) << 16);
  q.y = uint32_t(f32_to_bf16(a.v[2])) | (uint32_t(f32_to_bf16(a.v[3])) << 16);
  *reinterpret_cast<uint2*>(p) = q;
}

__device__ __forceinline__ f4 ld_s(const float* s, int64_t b, int c, int64_t sbs, int scs) {
  const float* p = s + b * sbs;
  if (scs == 0) {
    const float v = p[0];
    return {{v, v, v, v}};
  }
  return {{p[c], p[c + 1], p[c + 2], p[c + 3]}};
}

// flat grid-stride over the 4-channel vectors of [B, N, C]
template <typename TX, typename TB, typename TO>
__global__ void __launch_bounds__(256)
add_scaled_fwd_kernel(const TX* __restrict__ x, const TB* __restrict__ br, const float* __restrict__ s, int64_t N,
                      int C, int64_t sbs, int scs, int64_t nvec, TO* __restrict__ out) {
  const int64_t per_sample = N * C;
  for (int64_t v = int64_t(blockIdx.x) * 256 + threadIdx.x; v < nvec; v += int64_t(gridDim.x) * 256) {
    const int64_t e = v * 4;
    const int64_t b = e / per_sample;
    const int c = int(e % C);
    const f4 xv = ld4<TX>(x + e), bv = ld4<TB>(br + e), sv = ld_s(s, b, c, sbs, scs);
    f4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o.v[k] = xv.v[k] + bv.v[k] * sv.v[k];
    st4<TO>(out + e, o);
  }
}

// grid (chunks, B): block (chunk, b) walks rows chunk*rows_per_chunk ... of
// sample b, rows_per_it = 256 / (C / 4) rows per iteration.  Writes
// d branch = g * s and part[b][chunk][c] = sum over its rows of g * branch.
template <typename TG, typename TB>
__global__ void __launch_bounds__(256)
add_scaled_bwd_kernel(const TG* __restrict__ g, const TB* __restrict__ br, const float* __restrict__ s, int64_t N,
                      int C, int64_t sbs, int scs, int64_t rows_per_chunk, TB* __restrict__ gbr,
                      float* __restrict__ part) {
  const int V = C >> 2;
  const int rows_per_it = 256 / V;
  const int t = threadIdx.x;
  const int r0 = t / V, c = (t % V) * 4;
  const bool active = r0 < rows_per_it;
  const int64_t b = blockIdx.y;
  const int64_t row_lo = int64_t(blockIdx.x) * rows_per_chunk;
  const int64_t row_hi = row_lo + rows_per_chunk < N ? row_lo + rows_per_chunk : N;
  f4 acc = {{0.f, 0.f, 0.f, 0.f}};
  if (active) {
    const f4 sv = ld_s(s, b, c, sbs, scs);
    for (int64_t row = row_lo + r0; row < row_hi; row += rows_per_it) {
      const int64_t e = (b * N + row) * C + c;
      const f4 gv = ld4<TG>(g + e);
      if (part) {
        const f4 bv = ld4<TB>(br + e);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc.v[k] += gv.v[k] * bv.v[k];
      }
      if (gbr) {
        f4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o.v[k] = gv.v[k] * sv.v[k];
        st4<TB>(gbr + e, o);
      }
    }
  }
  if (!part) return;
  __shared__ float red[256 * 4];
#pragma unroll
  for (int k = 0; k < 4; ++k) red[t * 4 + k] = acc.v[k];
  __syncthreads();
  if (t < V) {  // fixed order over the rows of the iteration
    f4 sum = {{0.f, 0.f, 0.f, 0.f}};
    for (int r = 0; r < rows_per_it; ++r) {
#pragma unroll
      for (int k = 0; k < 4; ++k) sum.v[k] += red[(r * V + t) * 4 + k];
    }
    float* dst = part + (b * gridDim.x + blockIdx.x) * int64_t(C) + t * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = sum.v[k];
  }
}

// gs[b][c] = sum over chunks of part[b][chunk][c]; grid (ceil(C/64), B),
// block 1024 = 64 channels x 16 chunk groups, combined in LDS in fixed order
__global__ void __launch_bounds__(1024)
add_scaled_merge_kernel(const float* __restrict__ part, int chunks, int C, float* __restrict__ gs) {
  __shared__ float red[16][64];
  const int cx = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cx;
  const int64_t b = blockIdx.y;
  float acc = 0.f;
  if (c < C)
    for (int k = grp; k < chunks; k += 16) acc += part[(b * chunks + k) * C + c];
  red[grp][cx] = acc;
  __syncthreads();
  if (grp == 0 && c < C) {
#pragma unroll
    for (int k = 1; k < 16; ++k) acc += red[k][cx];
    gs[b * C + c] = acc;
  }
}

// out = a + b (fp32) with the bf16 copies of out and of a written in the
// same pass (either copy optional): the encoder's query = src + pos, whose
// two Linears (sampling offsets / attention weights on the query, value_proj
// on src) read bf16 -- one pass instead of the add and two cast kernels
__global__ void __launch_bounds__(256)
add_twin_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t nvec, float* __restrict__ out,
                uint16_t* __restrict__ out16, uint16_t* __restrict__ a16) {
  for (int64_t v = int64_t(blockIdx.x) * 256 + threadIdx.x; v < nvec; v += int64_t(gridDim.x) * 256) {
    const int64_t e = v * 4;
    const f4 av = ld4<float>(a + e), bv = ld4<float>(b + e);
    f4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o.v[k] = av.v[k] + bv.v[k];
    st4<float>(out + e, o);
    if (out16) st4<uint16_t>(out16 + e, o);
    if (a16) st4<uint16_t>(a16 + e, av);
  }
}

constexpr int kScaledChunks = 256;  // backward chunks per sample (max)

template <typename Fn>
bool with_type(gd_dtype d, Fn&& fn) {
  if (d == GD_F32) fn(float{});
  else if (d == GD_BF16) fn(uint16_t{});
  else return false;
  return true;
}

int64_t chunks_for(int64_t N, int C) {
  const int64_t rows_per_it = 256 / (C / 4);
  const int64_t its = (N + rows_per_it - 1) / rows_per_it;
  // >= 4 iterations per block, at most kScaledChunks chunks per sample
  int64_t ch = (its + 3) / 4;
  return ch < 1 ? 1 : (ch > kScaledChunks ? kScaledChunks : ch);
}

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" size_t gd_add_scaled_workspace_bytes(int64_t B, int64_t N, int C) {
  if (C <= 0 || C % 4 != 0) return 0;
  return sizeof(float) * size_t(B) * size_t(chunks_for(N, C)) * size_t(C);
}

extern "C" gd_status gd_add_scaled_forward(gd_dtype x_dtype, const void* x, gd_dtype branch_dtype,
                                          const void* branch, const float* s, int64_t s_bstride, int s_cstride,
                                          int64_t B, int64_t N, int C, gd_dtype out_dtype, void* out,
                                          gd_stream_t stream) {
  GD_REQUIRE(B >= 0 && N >= 0, "add_scaled: B=%lld N=%lld", (long long)B, (long long)N);
  GD_REQUIRE(C > 0 && C % 4 == 0 && C <= 1024, "add_scaled: C=%d (a multiple of 4, <= 1024)", C);
  GD_REQUIRE(s_cstride == 0 || s_cstride == 1, "add_scaled: s channel stride %d (0 or 1)", s_cstride);
  if (B * N == 0) return GD_OK;
  GD_REQUIRE(x && branch && s && out, "add_scaled_forward: null pointer");
  const int64_t nvec = B * N * C / 4;
  const int64_t blocks64 = (nvec + 255) / 256;
  const unsigned blocks = unsigned(blocks64 < 16384 ? blocks64 : 16384);
  GD_REQUIRE((x_dtype == GD_F32 || x_dtype == GD_BF16) && (branch_dtype == GD_F32 || branch_dtype == GD_BF16)
                 && (out_dtype == GD_F32 || out_dtype == GD_BF16),
             "add_scaled_forward: dtypes %d/%d/%d (F32, BF16)", int(x_dtype), int(branch_dtype), int(out_dtype));
  hipStream_t st = as_hip(stream);
  with_type(x_dtype, [&](auto tx) {
    using TX = decltype(tx);
    with_type(branch_dtype, [&](auto tb) {
      using TB = decltype(tb);
      with_type(out_dtype, [&](auto to) {
        using TO = decltype(to);
        hipLaunchKernelGGL((add_scaled_fwd_kernel<TX, TB, TO>), dim3(blocks), dim3(256), 0, st, (const TX*)x,
                           (const TB*)branch, s, N, C, s_bstride, s_cstride, nvec, (TO*)out);
      });
    });
  });
  GD_LAUNCH_CHECK("add_scaled_fwd");
  return GD_OK;
}

extern "C" gd_status gd_add_scaled_backward(gd_dtype g_dtype, const void* grad_out, gd_dtype branch_dtype,
                                           const void* branch, const float* s, int64_t s_bstride, int s_cstride,
                                           int64_t B, int64_t N, int C, void* grad_branch, float* grad_s_bc,
                                           void* workspace, gd_stream_t stream) {
  GD_REQUIRE(B >= 0 && N >= 0, "add_scaled: B=%lld N=%lld", (long long)B, (long long)N);
  GD_REQUIRE(C > 0 && C % 4 == 0 && C <= 1024, "add_scaled: C=%d (a multiple of 4, <= 1024)", C);
  GD_REQUIRE(s_cstride == 0 || s_cstride == 1, "add_scaled: s channel stride %d (0 or 1)", s_cstride);
  GD_REQUIRE((g_dtype == GD_F32 || g_dtype == GD_BF16) && (branch_dtype == GD_F32 || branch_dtype == GD_BF16),
             "add_scaled_backward: dtypes %d/%d (F32, BF16)", int(g_dtype), int(branch_dtype));
  hipStream_t st = as_hip(stream);
  if (B * N == 0) {
    if (grad_s_bc) GD_HIP_CHECK(fill_u32_async(grad_s_bc, 0u, sizeof(float) * size_t(B) * C, st));
    return GD_OK;
  }
  GD_REQUIRE(grad_out && s && (grad_branch || grad_s_bc), "add_scaled_backward: null pointer");
  GD_REQUIRE(!grad_s_bc || (branch && workspace), "add_scaled_backward: grad_s needs branch and workspace");
  const int64_t chunks = chunks_for(N, C);
  const int64_t rows_per_chunk = (N + chunks - 1) / chunks;
  float* part = grad_s_bc ? static_cast<float*>(workspace) : nullptr;
  with_type(g_dtype, [&](auto tg) {
    using TG = decltype(tg);
    with_type(branch_dtype, [&](auto tb) {
      using TB = decltype(tb);
      hipLaunchKernelGGL((add_scaled_bwd_kernel<TG, TB>), dim3(unsigned(chunks), unsigned(B)), dim3(256), 0, st,
                         (const TG*)grad_out, (const TB*)branch, s, N, C, s_bstride, s_cstride, rows_per_chunk,
                         (TB*)grad_branch, part);
    });
  });
  GD_LAUNCH_CHECK("add_scaled_bwd");
  if (grad_s_bc) {
    hipLaunchKernelGGL(add_scaled_merge_kernel, dim3(unsigned((C + 63) / 64), unsigned(B)), dim3(1024), 0, st, part,
                       int(chunks), C, grad_s_bc);
    GD_LAUNCH_CHECK("add_scaled_merge");
  }
  return GD_OK;
}

extern "C" gd_status gd_add_twin_forward(const float* a, const float* b, int64_t n, float* out, void* out_bf16,
                                        void* a_bf16, gd_stream_t stream) {
  GD_REQUIRE(n >= 0 && n % 4 == 0, "add_twin: n=%lld (a multiple of 4)", (long long)n);
  if (n == 0) return GD_OK;
  GD_REQUIRE(a && b && out, "add_twin: null pointer");
  const int64_t nvec = n / 4;
  const int64_t blocks64 = (nvec + 255) / 256;
  const unsigned blocks = unsigned(blocks64 < 16384 ? blocks64 : 16384);
  hipLaunchKernelGGL(add_twin_kernel, dim3(blocks), dim3(256), 0, as_hip(stream), a, b, nvec, out,
                     static_cast<uint16_t*>(out_bf16), static_cast<uint16_t*>(a_bf16));
  GD_LAUNCH_CHECK("add_twin");
  return GD_OK;
}
