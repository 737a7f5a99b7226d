// CPU backend of the MSDA op under the same C-ABI as the gfx950 library
// (include/gdino_amd.h: gd_msda_forward / gd_msda_backward /
// gd_msda_backward_geom), built by g++ into libgdino_cpu.so.
//
// The reference's CPU backend is a stub that raises "Not implemented on the
// CPU" (models/GroundingDINO/ops/src/cpu/ms_deform_attn_cpu.cpp:26,39, reached
// through the device dispatch of ops/src/ms_deform_attn.h:20-61); this is a
// real implementation of the same semantics, for host tensors:
//   forward  ms_deform_attn_im2col_bilinear + ms_deformable_im2col_gpu_kernel
//            (ops/src/cuda/ms_deform_im2col_cuda.cuh:34-84, 238-299): sample
//            at loc*(W,H) - 0.5, bilinear over the in-bounds corners
//            (val = w1 v1 + w2 v2 + w3 v3 + w4 v4), out += attn * val;
//   backward ms_deform_attn_col2im_bilinear (.cuh:88-159): grad_value +=
//            w_k * attn * g per corner, grad_attn = sum_c g * val,
//            grad_loc = (W, H) * sum_c attn * g * d(val)/d(w, h).
// Host pointers everywhere (spatial_shapes / level_start_index too); the
// stream argument must be NULL.  Work is split over OpenMP threads: the
// forward over (n, q, m) units, the backward over (n, m) pairs -- each pair
// owns the grad_value rows of its head, so the scatter needs no atomics and
// the summation order is fixed (deterministic, unlike the GPU atomics).
#include <omp.h>

#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../../include/gdino_amd.h"

#define GD_CPU_API extern "C" __attribute__((visibility("default")))

namespace {

thread_local char g_err[512];

gd_status fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return GD_ERR_INVALID;
}

inline float bf16_to_f32(uint16_t h) {
  uint32_t u = uint32_t(h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f32_to_bf16(float f) {  // round to nearest even, NaN stays NaN
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return uint16_t((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

template <typename T> struct Acc { typedef float type; };
template <> struct Acc<double> { typedef double type; };

template <typename T> inline typename Acc<T>::type ld(const T* p) { return *p; }
template <> inline float ld<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }
template <typename T> inline void st(T* p, typename Acc<T>::type v) { *p = T(v); }
template <> inline void st<uint16_t>(uint16_t* p, float v) { *p = f32_to_bf16(v); }

// bilinear corners of one sample (the reference's index math, .cuh:34-84)
template <typename A>
struct Corners {
  int64_t off[4];  // element offset of (row, head m, channel 0) or -1
  A w[4];
  A hh, hw, lh, lw;
  bool any;
};

template <typename A>
inline Corners<A> corners(A loc_w, A loc_h, int H, int W, int64_t row0, int M, int m, int D) {
  Corners<A> k;
  const A h_im = loc_h * H - A(0.5), w_im = loc_w * W - A(0.5);
  k.any = h_im > A(-1) && w_im > A(-1) && h_im < A(H) && w_im < A(W);
  if (!k.any) return k;
  const int h_low = int(std::floor(h_im)), w_low = int(std::floor(w_im));
  const int h_high = h_low + 1, w_high = w_low + 1;
  k.lh = h_im - h_low;
  k.lw = w_im - w_low;
  k.hh = A(1) - k.lh;
  k.hw = A(1) - k.lw;
  k.w[0] = k.hh * k.hw;
  k.w[1] = k.hh * k.lw;
  k.w[2] = k.lh * k.hw;
  k.w[3] = k.lh * k.lw;
  const int ys[4] = {h_low, h_low, h_high, h_high}, xs[4] = {w_low, w_high, w_low, w_high};
  for (int i = 0; i < 4; ++i) {
    const bool ok = ys[i] >= 0 && xs[i] >= 0 && ys[i] <= H - 1 && xs[i] <= W - 1;
    k.off[i] = ok ? ((row0 + int64_t(ys[i]) * W + xs[i]) * M + m) * D : -1;
  }
  return k;
}

struct Dims {
  int N, S, M, D, L, Lq, P;
};

gd_status check(gd_dtype dt, const void* value, const int64_t* shapes, const int64_t* lsi, const void* loc,
                const void* attn, const Dims& d, gd_stream_t stream) {
  if (stream) return fail("gd_msda (CPU backend): stream must be NULL");
  if (dt != GD_F32 && dt != GD_F64 && dt != GD_BF16)
    return fail("gd_msda (CPU backend): value dtype %d not supported (F32, F64, BF16)", int(dt));
  if (d.N < 0 || d.S < 0 || d.M <= 0 || d.D <= 0 || d.L <= 0 || d.Lq < 0 || d.P <= 0)
    return fail("gd_msda (CPU backend): bad sizes N=%d S=%d M=%d D=%d L=%d Lq=%d P=%d", d.N, d.S, d.M, d.D, d.L,
                d.Lq, d.P);
  if (!shapes || !lsi) return fail("gd_msda (CPU backend): null spatial_shapes / level_start_index");
  if ((d.N > 0 && d.S > 0 && !value) || (d.N > 0 && d.Lq > 0 && (!loc || !attn)))
    return fail("gd_msda (CPU backend): null pointer");
  for (int l = 0; l < d.L; ++l) {
    if (shapes[2 * l] < 0 || shapes[2 * l + 1] < 0 || lsi[l] < 0 ||
        lsi[l] + shapes[2 * l] * shapes[2 * l + 1] > d.S)
      return fail("gd_msda (CPU backend): level %d (%lld x %lld at %lld) outside spatial_size %d", l,
                  (long long)shapes[2 * l], (long long)shapes[2 * l + 1], (long long)lsi[l], d.S);
  }
  return GD_OK;
}

template <typename T>
void forward(const T* value, const int64_t* shapes, const int64_t* lsi, const typename Acc<T>::type* loc,
             const typename Acc<T>::type* attn, const Dims& d, T* out) {
  typedef typename Acc<T>::type A;
  const int64_t units = int64_t(d.N) * d.Lq * d.M;
#pragma omp parallel
  {
    std::vector<A> acc(d.D), val(d.D);
#pragma omp for schedule(static)
    for (int64_t u = 0; u < units; ++u) {
      const int m = int(u % d.M);
      const int64_t nq = u / d.M;
      const int n = int(nq / d.Lq);
      std::fill(acc.begin(), acc.end(), A(0));
      const A* lp = loc + u * d.L * d.P * 2;
      const A* ap = attn + u * d.L * d.P;
      for (int l = 0; l < d.L; ++l) {
        const int H = int(shapes[2 * l]), W = int(shapes[2 * l + 1]);
        const int64_t row0 = int64_t(n) * d.S + lsi[l];
        for (int p = 0; p < d.P; ++p, lp += 2, ++ap) {
          const Corners<A> k = corners<A>(lp[0], lp[1], H, W, row0, d.M, m, d.D);
          if (!k.any) continue;
          std::fill(val.begin(), val.end(), A(0));
          for (int i = 0; i < 4; ++i) {
            if (k.off[i] < 0) continue;
            const T* v = value + k.off[i];
            const A w = k.w[i];
            for (int c = 0; c < d.D; ++c) val[c] += w * ld(v + c);
          }
          const A a = *ap;
          for (int c = 0; c < d.D; ++c) acc[c] += a * val[c];
        }
      }
      T* o = out + u * d.D;
      for (int c = 0; c < d.D; ++c) st(o + c, acc[c]);
    }
  }
}

template <typename T>
void backward(const T* value, const int64_t* shapes, const int64_t* lsi, const typename Acc<T>::type* loc,
              const typename Acc<T>::type* attn, const T* gout, const Dims& d, typename Acc<T>::type* gval,
              typename Acc<T>::type* gloc, typename Acc<T>::type* gattn) {
  typedef typename Acc<T>::type A;
  std::memset(gval, 0, sizeof(A) * size_t(d.N) * d.S * d.M * d.D);
  const int pairs = d.N * d.M;
#pragma omp parallel
  {
    std::vector<A> g(d.D), tg(d.D);
#pragma omp for schedule(dynamic, 1)
    for (int nm = 0; nm < pairs; ++nm) {
      const int n = nm / d.M, m = nm % d.M;
      for (int q = 0; q < d.Lq; ++q) {
        const int64_t u = (int64_t(n) * d.Lq + q) * d.M + m;
        const T* go = gout + u * d.D;
        for (int c = 0; c < d.D; ++c) g[c] = ld(go + c);
        const A* lp = loc + u * d.L * d.P * 2;
        const A* ap = attn + u * d.L * d.P;
        A* glp = gloc + u * d.L * d.P * 2;
        A* gap = gattn + u * d.L * d.P;
        for (int l = 0; l < d.L; ++l) {
          const int H = int(shapes[2 * l]), W = int(shapes[2 * l + 1]);
          const int64_t row0 = int64_t(n) * d.S + lsi[l];
          for (int p = 0; p < d.P; ++p, lp += 2, ++ap, glp += 2, ++gap) {
            glp[0] = glp[1] = A(0);
            *gap = A(0);
            const Corners<A> k = corners<A>(lp[0], lp[1], H, W, row0, d.M, m, d.D);
            if (!k.any) continue;
            const A a = *ap;
            for (int c = 0; c < d.D; ++c) tg[c] = g[c] * a;
            // d(val)/dh and d(val)/dw coefficients of the four corners (.cuh:110-146)
            const A ch[4] = {-k.hw, -k.lw, k.hw, k.lw};
            const A cw[4] = {-k.hh, k.hh, -k.lh, k.lh};
            A s_attn = 0, s_h = 0, s_w = 0;
            for (int i = 0; i < 4; ++i) {
              if (k.off[i] < 0) continue;
              const T* v = value + k.off[i];
              A* gv = gval + k.off[i];
              A sv = 0, svt = 0;
              for (int c = 0; c < d.D; ++c) {
                const A x = ld(v + c);
                sv += g[c] * x;   // contributes to grad_attn through val
                svt += tg[c] * x;  // contributes to grad_loc
                gv[c] += k.w[i] * tg[c];
              }
              s_attn += k.w[i] * sv;
              s_h += ch[i] * svt;
              s_w += cw[i] * svt;
            }
            *gap = s_attn;
            glp[0] = W * s_w;
            glp[1] = H * s_h;
          }
        }
      }
    }
  }
}

template <typename T>
gd_status run_backward(const void* value, const int64_t* shapes, const int64_t* lsi, const void* loc,
                       const void* attn, const void* gout, const Dims& d, void* gval, void* gloc, void* gattn) {
  typedef typename Acc<T>::type A;
  backward<T>((const T*)value, shapes, lsi, (const A*)loc, (const A*)attn, (const T*)gout, d, (A*)gval, (A*)gloc,
              (A*)gattn);
  return GD_OK;
}

}  // namespace

GD_CPU_API const char* gd_last_error(void) { return g_err; }
GD_CPU_API int gd_abi_version(void) { return 1; }
GD_CPU_API const char* gd_runtime_info(void) {
  static char buf[128];
  snprintf(buf, sizeof(buf), "gdino_amd CPU backend (C++/OpenMP, %d threads)", omp_get_max_threads());
  return buf;
}

GD_CPU_API gd_status gd_msda_forward(gd_dtype dt, const void* value, const int64_t* shapes, const int64_t* lsi,
                                     const void* loc, const void* attn, int N, int S, int M, int D, int L, int Lq,
                                     int P, void* out, gd_stream_t stream) {
  const Dims d{N, S, M, D, L, Lq, P};
  const gd_status st = check(dt, value, shapes, lsi, loc, attn, d, stream);
  if (st != GD_OK) return st;
  if (int64_t(N) * Lq == 0) return GD_OK;
  if (!out) return fail("gd_msda_forward (CPU backend): null output");
  if (dt == GD_F64) {
    forward<double>((const double*)value, shapes, lsi, (const double*)loc, (const double*)attn, d, (double*)out);
  } else if (dt == GD_F32) {
    forward<float>((const float*)value, shapes, lsi, (const float*)loc, (const float*)attn, d, (float*)out);
  } else {
    forward<uint16_t>((const uint16_t*)value, shapes, lsi, (const float*)loc, (const float*)attn, d,
                      (uint16_t*)out);
  }
  return GD_OK;
}

GD_CPU_API gd_status gd_msda_backward(gd_dtype dt, const void* value, const int64_t* shapes, const int64_t* lsi,
                                      const void* loc, const void* attn, const void* gout, int N, int S, int M,
                                      int D, int L, int Lq, int P, void* gval, void* gloc, void* gattn,
                                      gd_stream_t stream) {
  const Dims d{N, S, M, D, L, Lq, P};
  const gd_status st = check(dt, value, shapes, lsi, loc, attn, d, stream);
  if (st != GD_OK) return st;
  if (int64_t(N) * S * M * D > 0 && !gval) return fail("gd_msda_backward (CPU backend): null grad_value");
  if (int64_t(N) * Lq > 0 && (!gout || !gloc || !gattn)) return fail("gd_msda_backward (CPU backend): null pointer");
  if (dt == GD_F64) return run_backward<double>(value, shapes, lsi, loc, attn, gout, d, gval, gloc, gattn);
  if (dt == GD_F32) return run_backward<float>(value, shapes, lsi, loc, attn, gout, d, gval, gloc, gattn);
  return run_backward<uint16_t>(value, shapes, lsi, loc, attn, gout, d, gval, gloc, gattn);
}

// the host level shapes only select GPU tilings; the CPU result is the same
GD_CPU_API gd_status gd_msda_backward_geom(gd_dtype dt, const void* value, const int64_t* shapes,
                                           const int64_t* lsi, const void* loc, const void* attn, const void* gout,
                                           int N, int S, int M, int D, int L, int Lq, int P, void* gval, void* gloc,
                                           void* gattn, const int64_t* /*shapes_host*/, gd_stream_t stream) {
  return gd_msda_backward(dt, value, shapes, lsi, loc, attn, gout, N, S, M, D, L, Lq, P, gval, gloc, gattn,
                          stream);
}
