// Multi-scale deformable attention (MSDA) forward + backward for gfx950.
//
// Replaces the reference's CUDA extension
//   models/GroundingDINO/ops/src/cuda/ms_deform_attn_cuda.cu:20-153   (host)
//   models/GroundingDINO/ops/src/cuda/ms_deform_im2col_cuda.cuh:34-84 (bilinear)
//   ms_deform_im2col_cuda.cuh:88-159                                (bilinear grad)
//   ms_deform_im2col_cuda.cuh:238-299                               (im2col fwd)
//   ms_deform_im2col_cuda.cuh:302-403 (the D=32 backward variant the reference
//   launches with 32-thread blocks and a serial 32-way shared-memory sum)
//
// Layout (all contiguous, row-major):
//   value [N, S, M, D]   loc [N, Lq, M, L, P, 2]   attn [N, Lq, M, L, P]
//   out   [N, Lq, M*D]
// A "unit" is one (n, q, m) triple: L*P samples, each a 4-corner bilinear
// gather of a D-channel row slice of `value`.
//
// Forward (msda_fwd_vec): every lane owns one 16-byte channel vector of one
// unit (4 fp32 or 8 bf16 channels), so each corner gather is a single
// global_load_dwordx4 and a unit's D channels are D/VE adjacent lanes.  The
// unit's 16 sampling locations / weights are read as 12 dwordx4 broadcast
// loads.  Accumulation is fp32; the output row is one coalesced 16-B store
// per lane.
//
// Backward (msda_bwd_lane): one lane per channel (D = 32 -> 2 units per
// wave).  Per corner the unit's 32 lanes issue one 128-B contiguous
// global_atomic_add_f32 for grad_value (the shape the memory-side atomic unit
// runs at full rate, MI355X_MICROARCH "Global float atomics").  The
// 48 per-unit partial sums (grad_attn, grad_loc_w, grad_loc_h per sample) are
// reduced with a reduce-scatter butterfly (ds_swizzle xor16, DPP row_ror8,
// row_half_mirror, quad xor2, quad xor1): 48 lane exchanges instead of the
// reference's shared-memory round trip + serial thread-0 sum per sample.
//
// Both kernels remap blockIdx so that each XCD gets a contiguous range of
// queries (neighbouring encoder queries sample neighbouring value rows, so
// this keeps the gathered rows in one XCD's L2).
#include "gd_common.h"

namespace gd {
namespace {

// Bijective XCD-contiguous remap: hardware deals blocks b, b+8, b+16, ... to
// one XCD; give that XCD a contiguous chunk of the logical grid instead.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int q = nb >> 3, r = nb & 7;
  const int xcd = b & 7, local = b >> 3;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + local;
}

// --------------------------------------------------------------------------
// 16-byte vector IO
// --------------------------------------------------------------------------
template <typename T>
struct Vec;

template <>
struct Vec<float> {
  static constexpr int N = 4;
  __device__ static __forceinline__ void load(const float* p, float (&v)[4]) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  __device__ static __forceinline__ void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};

// bf16 storage as uint16_t.
template <>
struct Vec<uint16_t> {
  static constexpr int N = 8;
  __device__ static __forceinline__ void load(const uint16_t* p, float (&v)[8]) {
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    v[0] = bf16_lo(t.x); v[1] = bf16_hi(t.x);
    v[2] = bf16_lo(t.y); v[3] = bf16_hi(t.y);
    v[4] = bf16_lo(t.z); v[5] = bf16_hi(t.z);
    v[6] = bf16_lo(t.w); v[7] = bf16_hi(t.w);
  }
  __device__ static __forceinline__ void store(uint16_t* p, const float (&v)[8]) {
    uint4 t;
    t.x = uint32_t(f32_to_bf16(v[0])) | (uint32_t(f32_to_bf16(v[1])) << 16);
    t.y = uint32_t(f32_to_bf16(v[2])) | (uint32_t(f32_to_bf16(v[3])) << 16);
    t.z = uint32_t(f32_to_bf16(v[4])) | (uint32_t(f32_to_bf16(v[5])) << 16);
    t.w = uint32_t(f32_to_bf16(v[6])) | (uint32_t(f32_to_bf16(v[7])) << 16);
    *reinterpret_cast<uint4*>(p) = t;
  }
};

template <typename T> __device__ __forceinline__ float to_f(T x);
template <> __device__ __forceinline__ float to_f<float>(float x) { return x; }
template <> __device__ __forceinline__ float to_f<uint16_t>(uint16_t x) { return bf16_to_f32(x); }

// --------------------------------------------------------------------------
// Forward, vectorised fast path (fp32 / bf16 value, fp32 loc/attn)
// --------------------------------------------------------------------------
template <typename T, int D, int L, int P>
__global__ void __launch_bounds__(256)
msda_fwd_vec(const T* __restrict__ value, const int64_t* __restrict__ shapes,
             const int64_t* __restrict__ lsi, const float* __restrict__ loc,
             const float* __restrict__ attn, T* __restrict__ out, int S, int Lq,
             int M, int num_units) {
  constexpr int VE = Vec<T>::N;       // channels per lane
  constexpr int LPU = D / VE;         // lanes per unit
  constexpr int UPW = 64 / LPU;       // units per wave
  constexpr int NS = L * P;           // samples per unit
  static_assert(D % VE == 0 && 64 % LPU == 0, "bad D");
  static_assert((NS * 2) % 4 == 0 && NS % 4 == 0, "bad L*P");

  const int lane = threadIdx.x & 63;
  const int sub = lane % LPU;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int u = (blk * 4 + int(threadIdx.x >> 6)) * UPW + lane / LPU;
  if (u >= num_units) return;

  const int m = u % M;
  const int n = (u / M) / Lq;
  const int qstride = M * D;  // elements between consecutive positions
  const T* vb = value + (size_t(n) * S * M + m) * D + sub * VE;

  // Sampling locations and weights of this unit (broadcast loads).
  float lw[NS * 2], aw[NS];
  {
    const float4* lp = reinterpret_cast<const float4*>(loc + size_t(u) * NS * 2);
#pragma unroll
    for (int i = 0; i < NS / 2; ++i) {
      const float4 t = lp[i];
      lw[4 * i + 0] = t.x; lw[4 * i + 1] = t.y; lw[4 * i + 2] = t.z; lw[4 * i + 3] = t.w;
    }
    const float4* ap = reinterpret_cast<const float4*>(attn + size_t(u) * NS);
#pragma unroll
    for (int i = 0; i < NS / 4; ++i) {
      const float4 t = ap[i];
      aw[4 * i + 0] = t.x; aw[4 * i + 1] = t.y; aw[4 * i + 2] = t.z; aw[4 * i + 3] = t.w;
    }
  }

  float acc[VE];
#pragma unroll
  for (int c = 0; c < VE; ++c) acc[c] = 0.f;

#pragma unroll
  for (int l = 0; l < L; ++l) {
    const int Hl = int(shapes[2 * l]);
    const int Wl = int(shapes[2 * l + 1]);
    const T* vl = vb + size_t(lsi[l]) * qstride;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int s = l * P + p;
      const float h_im = lw[2 * s + 1] * float(Hl) - 0.5f;
      const float w_im = lw[2 * s + 0] * float(Wl) - 0.5f;
      if (h_im > -1.f && w_im > -1.f && h_im < float(Hl) && w_im < float(Wl)) {
        const float hf = floorf(h_im), wf = floorf(w_im);
        const int h_low = int(hf), w_low = int(wf);
        const int h_high = h_low + 1, w_high = w_low + 1;
        const float lh = h_im - hf, lwt = w_im - wf;
        const float hh = 1.f - lh, hw = 1.f - lwt;
        const float w1 = hh * hw, w2 = hh * lwt, w3 = lh * hw, w4 = lh * lwt;
        float v1[VE], v2[VE], v3[VE], v4[VE];
#pragma unroll
        for (int c = 0; c < VE; ++c) v1[c] = v2[c] = v3[c] = v4[c] = 0.f;
        const int r_lo = h_low * Wl, r_hi = h_high * Wl;
        if (h_low >= 0 && w_low >= 0) Vec<T>::load(vl + (r_lo + w_low) * qstride, v1);
        if (h_low >= 0 && w_high <= Wl - 1) Vec<T>::load(vl + (r_lo + w_high) * qstride, v2);
        if (h_high <= Hl - 1 && w_low >= 0) Vec<T>::load(vl + (r_hi + w_low) * qstride, v3);
        if (h_high <= Hl - 1 && w_high <= Wl - 1) Vec<T>::load(vl + (r_hi + w_high) * qstride, v4);
        const float a = aw[s];
#pragma unroll
        for (int c = 0; c < VE; ++c)
          acc[c] += (w1 * v1[c] + w2 * v2[c] + w3 * v3[c] + w4 * v4[c]) * a;
      }
    }
  }
  Vec<T>::store(out + size_t(u) * D + sub * VE, acc);
}

// --------------------------------------------------------------------------
// Forward, generic (any D/L/P; float, double or bf16 value)
// one thread per (unit, channel) — mirrors .cuh:238-299 index decomposition
// --------------------------------------------------------------------------
template <typename T, typename A>
__device__ __forceinline__ A ld(const T* p);
template <> __device__ __forceinline__ float ld<float, float>(const float* p) { return *p; }
template <> __device__ __forceinline__ double ld<double, double>(const double* p) { return *p; }
template <> __device__ __forceinline__ float ld<uint16_t, float>(const uint16_t* p) { return bf16_to_f32(*p); }

template <typename T, typename A>
__device__ __forceinline__ void st(T* p, A v);
template <> __device__ __forceinline__ void st<float, float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st<double, double>(double* p, double v) { *p = v; }
template <> __device__ __forceinline__ void st<uint16_t, float>(uint16_t* p, float v) { *p = f32_to_bf16(v); }

template <typename T, typename A>
__global__ void __launch_bounds__(256)
msda_fwd_generic(const T* __restrict__ value, const int64_t* __restrict__ shapes,
                 const int64_t* __restrict__ lsi, const A* __restrict__ loc,
                 const A* __restrict__ attn, T* __restrict__ out, int S, int Lq,
                 int M, int D, int L, int P, int64_t total) {
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int c = int(idx % D);
    const int64_t u = idx / D;
    const int m = int(u % M);
    const int64_t n = (u / M) / Lq;
    const int qstride = M * D;
    const T* vb = value + (n * S * M + m) * D + c;
    const A* lp = loc + u * L * P * 2;
    const A* ap = attn + u * L * P;
    A col = 0;
    for (int l = 0; l < L; ++l) {
      const int Hl = int(shapes[2 * l]), Wl = int(shapes[2 * l + 1]);
      const T* vl = vb + lsi[l] * qstride;
      for (int p = 0; p < P; ++p) {
        const A loc_w = lp[0], loc_h = lp[1], wgt = ap[0];
        lp += 2; ap += 1;
        const A h_im = loc_h * A(Hl) - A(0.5);
        const A w_im = loc_w * A(Wl) - A(0.5);
        if (h_im > A(-1) && w_im > A(-1) && h_im < A(Hl) && w_im < A(Wl)) {
          const int h_low = int(floor(h_im)), w_low = int(floor(w_im));
          const int h_high = h_low + 1, w_high = w_low + 1;
          const A lh = h_im - A(h_low), lw = w_im - A(w_low);
          const A hh = A(1) - lh, hw = A(1) - lw;
          A v1 = 0, v2 = 0, v3 = 0, v4 = 0;
          if (h_low >= 0 && w_low >= 0) v1 = ld<T, A>(vl + int64_t(h_low * Wl + w_low) * qstride);
          if (h_low >= 0 && w_high <= Wl - 1) v2 = ld<T, A>(vl + int64_t(h_low * Wl + w_high) * qstride);
          if (h_high <= Hl - 1 && w_low >= 0) v3 = ld<T, A>(vl + int64_t(h_high * Wl + w_low) * qstride);
          if (h_high <= Hl - 1 && w_high <= Wl - 1) v4 = ld<T, A>(vl + int64_t(h_high * Wl + w_high) * qstride);
          const A w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
          col += (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4) * wgt;
        }
      }
    }
    st<T, A>(out + u * D + c, col);
  }
}

// --------------------------------------------------------------------------
// Backward, lane-per-channel fast path (D = 32, fp32 / bf16 value)
// --------------------------------------------------------------------------
__device__ __forceinline__ float swz_xor16(float v) {
  // ds_swizzle bitmask mode: and 0x1f, or 0, xor 0x10 (inside 32-lane halves)
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));
}

// One butterfly stage of the reduce-scatter: lanes whose `bit` is clear keep
// the lower half of v[0..2K), the others the upper half; each adds its
// partner's copy of the half it keeps.
template <int K, typename Xchg>
__device__ __forceinline__ void rs_stage(float* v, bool upper, Xchg xchg) {
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const float keep = upper ? v[K + i] : v[i];
    const float send = upper ? v[i] : v[K + i];
    v[i] = keep + xchg(send);
  }
}

template <typename T, int L, int P>
__global__ void __launch_bounds__(256)
msda_bwd_lane32(const T* __restrict__ value, const int64_t* __restrict__ shapes,
                const int64_t* __restrict__ lsi, const float* __restrict__ loc,
                const float* __restrict__ attn, const T* __restrict__ grad_out,
                float* __restrict__ grad_value, float* __restrict__ grad_loc,
                float* __restrict__ grad_attn, int S, int Lq, int M, int num_units) {
  constexpr int D = 32;
  constexpr int NS = L * P;
  constexpr int K = NS * 3;  // partials per lane: (attn, loc_w, loc_h) x NS
  static_assert(NS == 16, "reduce-scatter below is laid out for 16 samples on 32 lanes");

  const int lane = threadIdx.x & 63;
  const int c = lane & 31;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  int u = (blk * 4 + int(threadIdx.x >> 6)) * 2 + (lane >> 5);
  // A whole 32-lane unit is in or out together: the butterfly only mixes
  // lanes of one unit, so out-of-range units can leave.
  if (u >= num_units) return;

  const int m = u % M;
  const int n = (u / M) / Lq;
  const int qstride = M * D;
  const size_t vofs = (size_t(n) * S * M + m) * D + c;
  const T* vb = value + vofs;
  float* gvb = grad_value + vofs;
  const float top_grad = to_f<T>(grad_out[size_t(u) * D + c]);

  const float* lp = loc + size_t(u) * NS * 2;
  const float* ap = attn + size_t(u) * NS;

  float part[K];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const int Hl = int(shapes[2 * l]);
    const int Wl = int(shapes[2 * l + 1]);
    const T* vl = vb + size_t(lsi[l]) * qstride;
    float* gl = gvb + size_t(lsi[l]) * qstride;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int s = l * P + p;
      const float2 lwh = *reinterpret_cast<const float2*>(lp + 2 * s);
      const float a = ap[s];
      const float h_im = lwh.y * float(Hl) - 0.5f;
      const float w_im = lwh.x * float(Wl) - 0.5f;
      float g_attn = 0.f, g_w = 0.f, g_h = 0.f;
      if (h_im > -1.f && w_im > -1.f && h_im < float(Hl) && w_im < float(Wl)) {
        const float hf = floorf(h_im), wf = floorf(w_im);
        const int h_low = int(hf), w_low = int(wf);
        const int h_high = h_low + 1, w_high = w_low + 1;
        const float lh = h_im - hf, lwt = w_im - wf;
        const float hh = 1.f - lh, hw = 1.f - lwt;
        const float w1 = hh * hw, w2 = hh * lwt, w3 = lh * hw, w4 = lh * lwt;
        const float tgv = top_grad * a;
        float gh = 0.f, gw = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f, v4 = 0.f;
        const int r_lo = h_low * Wl, r_hi = h_high * Wl;
        if (h_low >= 0 && w_low >= 0) {
          const int o = (r_lo + w_low) * qstride;
          v1 = to_f<T>(vl[o]);
          gh -= hw * v1; gw -= hh * v1;
          atomicAdd(gl + o, w1 * tgv);
        }
        if (h_low >= 0 && w_high <= Wl - 1) {
          const int o = (r_lo + w_high) * qstride;
          v2 = to_f<T>(vl[o]);
          gh -= lwt * v2; gw += hh * v2;
          atomicAdd(gl + o, w2 * tgv);
        }
        if (h_high <= Hl - 1 && w_low >= 0) {
          const int o = (r_hi + w_low) * qstride;
          v3 = to_f<T>(vl[o]);
          gh += hw * v3; gw -= lh * v3;
          atomicAdd(gl + o, w3 * tgv);
        }
        if (h_high <= Hl - 1 && w_high <= Wl - 1) {
          const int o = (r_hi + w_high) * qstride;
          v4 = to_f<T>(vl[o]);
          gh += lwt * v4; gw += lh * v4;
          atomicAdd(gl + o, w4 * tgv);
        }
        const float val = w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4;
        g_attn = top_grad * val;
        g_w = float(Wl) * gw * tgv;
        g_h = float(Hl) * gh * tgv;
      }
      part[3 * s + 0] = g_attn;
      part[3 * s + 1] = g_w;
      part[3 * s + 2] = g_h;
    }
  }

  // Reduce-scatter over the unit's 32 lanes: 48 -> 24 -> 12 -> 6 -> 3, then
  // an all-reduce of the final 3 over the lane pair.  Lane c ends up owning
  // sample c >> 1 (see DESIGN.md "MSDA backward").
  rs_stage<24>(part, (c & 16) != 0, [](float x) { return swz_xor16(x); });
  rs_stage<12>(part, (c & 8) != 0, [](float x) { return dpp<DPP_ROR8>(x); });
  rs_stage<6>(part, (c & 4) != 0, [](float x) { return dpp<DPP_HALF_MIRROR>(x); });
  rs_stage<3>(part, (c & 2) != 0, [](float x) { return dpp<DPP_XOR2>(x); });
#pragma unroll
  for (int i = 0; i < 3; ++i) part[i] += dpp<DPP_XOR1>(part[i]);

  if ((c & 1) == 0) {
    const int s = c >> 1;
    grad_attn[size_t(u) * NS + s] = part[0];
    *reinterpret_cast<float2*>(grad_loc + (size_t(u) * NS + s) * 2) = make_float2(part[1], part[2]);
  }
}

// --------------------------------------------------------------------------
// Backward, generic: one thread per (unit, channel), global atomics for all
// three gradients (the reference's _gm variant, .cuh:846-920).  Used for the
// odd shapes of ops/test.py (D = 2, 30, 64, 71) and for fp64 gradcheck.
// --------------------------------------------------------------------------
template <typename T, typename A>
__global__ void __launch_bounds__(256)
msda_bwd_generic(const T* __restrict__ value, const int64_t* __restrict__ shapes,
                 const int64_t* __restrict__ lsi, const A* __restrict__ loc,
                 const A* __restrict__ attn, const T* __restrict__ grad_out,
                 A* __restrict__ grad_value, A* __restrict__ grad_loc,
                 A* __restrict__ grad_attn, int S, int Lq, int M, int D, int L,
                 int P, int64_t total) {
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int c = int(idx % D);
    const int64_t u = idx / D;
    const int m = int(u % M);
    const int64_t n = (u / M) / Lq;
    const int qstride = M * D;
    const int64_t vofs = (n * S * M + m) * D + c;
    const T* vb = value + vofs;
    A* gvb = grad_value + vofs;
    const A top_grad = ld<T, A>(grad_out + u * D + c);
    const A* lp = loc + u * L * P * 2;
    const A* ap = attn + u * L * P;
    A* glp = grad_loc + u * L * P * 2;
    A* gap = grad_attn + u * L * P;
    for (int l = 0; l < L; ++l) {
      const int Hl = int(shapes[2 * l]), Wl = int(shapes[2 * l + 1]);
      const T* vl = vb + lsi[l] * qstride;
      A* gl = gvb + lsi[l] * qstride;
      for (int p = 0; p < P; ++p) {
        const A loc_w = lp[0], loc_h = lp[1], wgt = ap[0];
        const A h_im = loc_h * A(Hl) - A(0.5);
        const A w_im = loc_w * A(Wl) - A(0.5);
        if (h_im > A(-1) && w_im > A(-1) && h_im < A(Hl) && w_im < A(Wl)) {
          const int h_low = int(floor(h_im)), w_low = int(floor(w_im));
          const int h_high = h_low + 1, w_high = w_low + 1;
          const A lh = h_im - A(h_low), lw = w_im - A(w_low);
          const A hh = A(1) - lh, hw = A(1) - lw;
          const A w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
          const A tgv = top_grad * wgt;
          A gh = 0, gw = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0;
          if (h_low >= 0 && w_low >= 0) {
            const int64_t o = int64_t(h_low * Wl + w_low) * qstride;
            v1 = ld<T, A>(vl + o); gh -= hw * v1; gw -= hh * v1;
            atomicAdd(gl + o, w1 * tgv);
          }
          if (h_low >= 0 && w_high <= Wl - 1) {
            const int64_t o = int64_t(h_low * Wl + w_high) * qstride;
            v2 = ld<T, A>(vl + o); gh -= lw * v2; gw += hh * v2;
            atomicAdd(gl + o, w2 * tgv);
          }
          if (h_high <= Hl - 1 && w_low >= 0) {
            const int64_t o = int64_t(h_high * Wl + w_low) * qstride;
            v3 = ld<T, A>(vl + o); gh += hw * v3; gw -= lh * v3;
            atomicAdd(gl + o, w3 * tgv);
          }
          if (h_high <= Hl - 1 && w_high <= Wl - 1) {
            const int64_t o = int64_t(h_high * Wl + w_high) * qstride;
            v4 = ld<T, A>(vl + o); gh += lw * v4; gw += lh * v4;
            atomicAdd(gl + o, w4 * tgv);
          }
          const A val = w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4;
          atomicAdd(gap, top_grad * val);
          atomicAdd(glp, A(Wl) * gw * tgv);
          atomicAdd(glp + 1, A(Hl) * gh * tgv);
        }
        lp += 2; ap += 1; glp += 2; gap += 1;
      }
    }
  }
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

inline int grid_for(int64_t total, int block) {
  int64_t g = (total + block - 1) / block;
  const int64_t cap = 256 * 32;  // grid-stride beyond 8192 blocks
  return int(g < cap ? (g < 1 ? 1 : g) : cap);
}

}  // namespace
}  // namespace gd

using namespace gd;

static gd_status check_common(gd_dtype dt, int N, int S, int M, int D, int L, int Lq, int P) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_F64 || dt == GD_BF16,
             "msda: value dtype %d not supported (F32, F64, BF16)", int(dt));
  GD_REQUIRE(N >= 0 && S >= 0 && M > 0 && D > 0 && L > 0 && Lq >= 0 && P > 0,
             "msda: bad sizes N=%d S=%d M=%d D=%d L=%d Lq=%d P=%d", N, S, M, D, L, Lq, P);
  // int32 index math inside one batch element (as the reference, .cuh uses int)
  GD_REQUIRE(int64_t(S) * M * D < (int64_t(1) << 31), "msda: S*M*D overflows int32");
  return GD_OK;
}

extern "C" gd_status gd_msda_forward(gd_dtype dt, const void* value,
                                     const int64_t* shapes, const int64_t* lsi,
                                     const void* loc, const void* attn, int N, int S,
                                     int M, int D, int L, int Lq, int P, void* out,
                                     gd_stream_t stream) {
  gd_status st0 = check_common(dt, N, S, M, D, L, Lq, P);
  if (st0 != GD_OK) return st0;
  const int64_t units = int64_t(N) * Lq * M;
  if (units == 0) return GD_OK;
  GD_REQUIRE(out && loc && attn && shapes && lsi, "msda_forward: null pointer");
  GD_REQUIRE(value || S == 0, "msda_forward: null value");
  hipStream_t s = as_hip(stream);
  const int64_t total = units * D;

  const bool vec_ok = D == 32 && L == 4 && P == 4 && units < (int64_t(1) << 31) &&
                      aligned16(value) && aligned16(loc) && aligned16(attn) && aligned16(out);
  if (dt == GD_F32 && vec_ok) {
    constexpr int UPW = 64 / (32 / 4);
    const int blocks = int((units + 4 * UPW - 1) / (4 * UPW));
    msda_fwd_vec<float, 32, 4, 4><<<blocks, 256, 0, s>>>(
        (const float*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (float*)out, S, Lq, M, int(units));
    GD_LAUNCH_CHECK("msda_fwd_vec<f32>");
  } else if (dt == GD_BF16 && vec_ok) {
    constexpr int UPW = 64 / (32 / 8);
    const int blocks = int((units + 4 * UPW - 1) / (4 * UPW));
    msda_fwd_vec<uint16_t, 32, 4, 4><<<blocks, 256, 0, s>>>(
        (const uint16_t*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (uint16_t*)out, S, Lq, M, int(units));
    GD_LAUNCH_CHECK("msda_fwd_vec<bf16>");
  } else if (dt == GD_F32) {
    msda_fwd_generic<float, float><<<grid_for(total, 256), 256, 0, s>>>(
        (const float*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (float*)out, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_fwd_generic<f32>");
  } else if (dt == GD_BF16) {
    msda_fwd_generic<uint16_t, float><<<grid_for(total, 256), 256, 0, s>>>(
        (const uint16_t*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (uint16_t*)out, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_fwd_generic<bf16>");
  } else {
    msda_fwd_generic<double, double><<<grid_for(total, 256), 256, 0, s>>>(
        (const double*)value, shapes, lsi, (const double*)loc, (const double*)attn,
        (double*)out, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_fwd_generic<f64>");
  }
  return GD_OK;
}

extern "C" gd_status gd_msda_backward(gd_dtype dt, const void* value,
                                      const int64_t* shapes, const int64_t* lsi,
                                      const void* loc, const void* attn,
                                      const void* grad_out, int N, int S, int M, int D,
                                      int L, int Lq, int P, void* grad_value,
                                      void* grad_loc, void* grad_attn,
                                      gd_stream_t stream) {
  gd_status st0 = check_common(dt, N, S, M, D, L, Lq, P);
  if (st0 != GD_OK) return st0;
  hipStream_t s = as_hip(stream);
  const size_t acc = dt == GD_F64 ? 8 : 4;
  const int64_t units = int64_t(N) * Lq * M;
  const size_t nval = size_t(N) * S * M * D;
  if (nval) {
    GD_REQUIRE(grad_value && value, "msda_backward: null value / grad_value");
    GD_HIP_CHECK(hipMemsetAsync(grad_value, 0, nval * acc, s));
  }
  if (units == 0) return GD_OK;
  GD_REQUIRE(grad_out && loc && attn && grad_loc && grad_attn && shapes && lsi,
             "msda_backward: null pointer");
  const int64_t total = units * D;
  const bool lane_ok = D == 32 && L == 4 && P == 4 && units < (int64_t(1) << 31) &&
                       aligned16(loc) && aligned16(grad_loc);
  if ((dt == GD_F32 || dt == GD_BF16) && lane_ok) {
    const int blocks = int((units + 7) / 8);  // 4 waves x 2 units
    if (dt == GD_F32) {
      msda_bwd_lane32<float, 4, 4><<<blocks, 256, 0, s>>>(
          (const float*)value, shapes, lsi, (const float*)loc, (const float*)attn,
          (const float*)grad_out, (float*)grad_value, (float*)grad_loc,
          (float*)grad_attn, S, Lq, M, int(units));
      GD_LAUNCH_CHECK("msda_bwd_lane32<f32>");
    } else {
      msda_bwd_lane32<uint16_t, 4, 4><<<blocks, 256, 0, s>>>(
          (const uint16_t*)value, shapes, lsi, (const float*)loc, (const float*)attn,
          (const uint16_t*)grad_out, (float*)grad_value, (float*)grad_loc,
          (float*)grad_attn, S, Lq, M, int(units));
      GD_LAUNCH_CHECK("msda_bwd_lane32<bf16>");
    }
    return GD_OK;
  }
  const size_t nloc = size_t(units) * L * P;
  GD_HIP_CHECK(hipMemsetAsync(grad_loc, 0, nloc * 2 * acc, s));
  GD_HIP_CHECK(hipMemsetAsync(grad_attn, 0, nloc * acc, s));
  if (dt == GD_F32) {
    msda_bwd_generic<float, float><<<grid_for(total, 256), 256, 0, s>>>(
        (const float*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (const float*)grad_out, (float*)grad_value, (float*)grad_loc, (float*)grad_attn,
        S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_bwd_generic<f32>");
  } else if (dt == GD_BF16) {
    msda_bwd_generic<uint16_t, float><<<grid_for(total, 256), 256, 0, s>>>(
        (const uint16_t*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (const uint16_t*)grad_out, (float*)grad_value, (float*)grad_loc,
        (float*)grad_attn, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_bwd_generic<bf16>");
  } else {
    msda_bwd_generic<double, double><<<grid_for(total, 256), 256, 0, s>>>(
        (const double*)value, shapes, lsi, (const double*)loc, (const double*)attn,
        (const double*)grad_out, (double*)grad_value, (double*)grad_loc,
        (double*)grad_attn, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_bwd_generic<f64>");
  }
  return GD_OK;
}
