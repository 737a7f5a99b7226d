// Contrastive text-alignment head for gfx950 (ContrastiveEmbed, reference
// models/GroundingDINO/utils.py:242-273, used at groundingdino.py:332-337 and
// for the two-stage selection transformer.py:292-296):
//   logits[b, q, t] = x[b, q] . text[b, t]   (t < T and text_mask[b, t])
//                   = -inf                   (masked token, or T <= t < Tout)
// as one MFMA kernel writing the fp32 [B, Q, Tout] logits directly (the
// reference: matmul, masked_fill, a -inf [B, Q, 256] fill and a slice copy),
// and/or the row maxima max_t logits[b, q, t] -- the two-stage proposal score
// (enc_outputs_class_unselected.max(-1)) without materialising the
// [B, S, 256] logits of every image token.
//
// A wave owns 64 rows of x and walks the Tout columns in 64-token tiles;
// every product is a 16x16x32 MFMA step with natural operands (mfma_frag.inc):
// A = x rows (row q on the lane), B = text rows (column t on the lane), K = C.
#include "gd_common.h"

#include <cmath>

namespace gd {
namespace {
#include "mfma_frag.inc"

template <typename T>
__global__ void __launch_bounds__(256)
contrastive_kernel(const T* __restrict__ x, int64_t xsb, int64_t xsq, const T* __restrict__ text, int64_t tsb,
                   int64_t tst, const uint8_t* __restrict__ tmask, int Q, int Tn, int C, int Tout,
                   float* __restrict__ out, float* __restrict__ rowmax) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.y;
  const int q0 = (blockIdx.x * 4 + wave) * 64;
  if (q0 >= Q) return;  // no barriers in this kernel
  const T* xb = x + b * xsb;
  const T* tb = text + b * tsb;
  float mx[4][4];
#pragma unroll
  for (int qt = 0; qt < 4; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[qt][r] = -INFINITY;

  for (int t0 = 0; t0 < Tout; t0 += 64) {
    gd_f32x4 acc[4][4];  // (row q0 + 16qt + 4g + r, token t0 + 16tt + c)
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) acc[qt][tt] = zero4();
    if (t0 < Tn) {
      for (int ch = 0; ch < C / 32; ++ch) {
        WFrag<T> tf[4];
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const int t = t0 + 16 * tt + c;
          tf[tt] = ld_frag<T>(tb + int64_t(t < Tn ? t : 0) * tst + 32 * ch + 8 * g, t < Tn);
        }
#pragma unroll
        for (int qt = 0; qt < 4; ++qt) {
          const int q = q0 + 16 * qt + c;
          const WFrag<T> xf = ld_frag<T>(xb + int64_t(q < Q ? q : 0) * xsq + 32 * ch + 8 * g, q < Q);
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) acc[qt][tt] = wmma(xf, tf[tt], acc[qt][tt]);
        }
      }
    }
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int t = t0 + 16 * tt + c;
      const bool live = t < Tn && tmask[int64_t(b) * Tn + t] != 0;
#pragma unroll
      for (int qt = 0; qt < 4; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = q0 + 16 * qt + 4 * g + r;
          const float v = live ? acc[qt][tt][r] : -INFINITY;
          mx[qt][r] = fmaxf(mx[qt][r], v);
          if (out && q < Q && t < Tout) out[(int64_t(b) * Q + q) * Tout + t] = v;
        }
    }
  }
  if (!rowmax) return;
#pragma unroll
  for (int qt = 0; qt < 4; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float m = mx[qt][r];
      m = fmaxf(m, __shfl_xor(m, 1, 64));
      m = fmaxf(m, __shfl_xor(m, 2, 64));
      m = fmaxf(m, __shfl_xor(m, 4, 64));
      m = fmaxf(m, __shfl_xor(m, 8, 64));
      const int q = q0 + 16 * qt + 4 * g + r;
      if (c == 0 && q < Q) rowmax[int64_t(b) * Q + q] = m;
    }
}

// v2 (round 4): the round-3 kernel gave a wave 64 rows x every token, so
// the decoder call (B = 2, Q = 900) ran 32 waves on a 1024-SIMD chip and
// each wave walked 8 dependent load -> MFMA rounds per token tile: 47 us of
// latency for 2.7 MB.  Here a workgroup owns 16 * QT rows and its 4 waves
// split the token tiles (wave w: tokens 64w .. 64w + 63, then + 256 ...), so
// the decoder call is 456 waves (QT = 1) and the encoder's row-max call 2 784
// (QT = 4); the next K chunk's operands are loaded while the current
// chunk's MFMAs run, and the row maxima of the 4 waves meet in LDS.
template <typename T, int QT>
__global__ void __launch_bounds__(256)
contrastive_v2_kernel(const T* __restrict__ x, int64_t xsb, int64_t xsq, const T* __restrict__ text, int64_t tsb,
                      int64_t tst, const uint8_t* __restrict__ tmask, int Q, int Tn, int C, int Tout,
                      float* __restrict__ out, float* __restrict__ rowmax) {
  __shared__ float smax[4][16 * QT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.y;
  const int q0 = blockIdx.x * 16 * QT;
  const T* xb = x + b * xsb;
  const T* tb = text + b * tsb;
  float mx[QT][4];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[qt][r] = -INFINITY;
  const int nch = C / 32;
  for (int t0 = 64 * wave; t0 < Tout; t0 += 256) {
    gd_f32x4 acc[QT][4];  // (row q0 + 16qt + 4g + r, token t0 + 16tt + c)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) acc[qt][tt] = zero4();
    if (t0 < Tn) {
      auto load = [&](int ch, WFrag<T>* tf, WFrag<T>* xf) {
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const int t = t0 + 16 * tt + c;
          tf[tt] = ld_frag<T>(tb + int64_t(t < Tn ? t : 0) * tst + 32 * ch + 8 * g, t < Tn);
        }
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
          const int q = q0 + 16 * qt + c;
          xf[qt] = ld_frag<T>(xb + int64_t(q < Q ? q : 0) * xsq + 32 * ch + 8 * g, q < Q);
        }
      };
      // two register sets, the loop unrolled by two so that every index
      // into them is a compile-time constant: a runtime-indexed [2][...]
      // fragment array is placed in scratch (private memory), and this
      // kernel then needs a scratch allocation on every queue it runs on
      WFrag<T> tf0[4], xf0[QT], tf1[4], xf1[QT];
      auto mma = [&](const WFrag<T>* tf, const WFrag<T>* xf) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) acc[qt][tt] = wmma(xf[qt], tf[tt], acc[qt][tt]);
      };
      load(0, tf0, xf0);
      for (int ch = 0; ch < nch; ch += 2) {
        if (ch + 1 < nch) load(ch + 1, tf1, xf1);  // next chunk in flight
        mma(tf0, xf0);
        if (ch + 1 < nch) {
          if (ch + 2 < nch) load(ch + 2, tf0, xf0);
          mma(tf1, xf1);
        }
      }
    }
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int t = t0 + 16 * tt + c;
      const bool live = t < Tn && tmask[int64_t(b) * Tn + t] != 0;
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = q0 + 16 * qt + 4 * g + r;
          const float v = live ? acc[qt][tt][r] : -INFINITY;
          mx[qt][r] = fmaxf(mx[qt][r], v);
          if (out && q < Q && t < Tout) out[(int64_t(b) * Q + q) * Tout + t] = v;
        }
    }
  }
  if (!rowmax) return;  // uniform over the workgroup: no barrier skipped by part of it
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float m = mx[qt][r];
      m = fmaxf(m, __shfl_xor(m, 1, 64));
      m = fmaxf(m, __shfl_xor(m, 2, 64));
      m = fmaxf(m, __shfl_xor(m, 4, 64));
      m = fmaxf(m, __shfl_xor(m, 8, 64));
      if (c == 0) smax[wave][16 * qt + 4 * g + r] = m;
    }
  __syncthreads();
  if (threadIdx.x < 16 * QT) {
    const int q = q0 + threadIdx.x;
    const float m = fmaxf(fmaxf(smax[0][threadIdx.x], smax[1][threadIdx.x]),
                          fmaxf(smax[2][threadIdx.x], smax[3][threadIdx.x]));
    if (q < Q) rowmax[int64_t(b) * Q + q] = m;
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" gd_status gd_contrastive_forward(gd_dtype dt, const void* x, const int64_t* x_strides, const void* text,
                                           const int64_t* text_strides, const uint8_t* text_mask, int B, int Q,
                                           int T, int C, int Tout, float* logits, float* rowmax,
                                           gd_stream_t stream) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "contrastive: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(B >= 0 && Q >= 0 && T > 0 && C > 0 && C % 32 == 0 && Tout >= T && B < 65536,
             "contrastive: bad sizes B=%d Q=%d T=%d C=%d (multiple of 32) Tout=%d (>= T)", B, Q, T, C, Tout);
  GD_REQUIRE(logits || rowmax, "contrastive: neither logits nor rowmax requested");
  if (B == 0 || Q == 0) return GD_OK;
  GD_REQUIRE(x && text && text_mask && x_strides && text_strides, "contrastive: null pointer");
  const int64_t align = 16 / (dt == GD_BF16 ? 2 : 4);
  GD_REQUIRE(aligned16(x) && aligned16(text) && x_strides[0] % align == 0 && x_strides[1] % align == 0 &&
                 text_strides[0] % align == 0 && text_strides[1] % align == 0,
             "contrastive: x / text rows must be contiguous and 16-byte aligned");
  hipStream_t s = as_hip(stream);
  // GD_CONTRASTIVE_V=1: the round-3 kernel (64 rows x all tokens per wave), A/B
  if (env_int("GD_CONTRASTIVE_V", 2) == 1) {
    const dim3 grid(unsigned((Q + 255) / 256), unsigned(B));
    if (dt == GD_BF16) {
      hipLaunchKernelGGL((contrastive_kernel<uint16_t>), grid, dim3(256), 0, s, (const uint16_t*)x, x_strides[0],
                         x_strides[1], (const uint16_t*)text, text_strides[0], text_strides[1], text_mask, Q, T, C,
                         Tout, logits, rowmax);
    } else {
      hipLaunchKernelGGL((contrastive_kernel<float>), grid, dim3(256), 0, s, (const float*)x, x_strides[0],
                         x_strides[1], (const float*)text, text_strides[0], text_strides[1], text_mask, Q, T, C,
                         Tout, logits, rowmax);
    }
    GD_LAUNCH_CHECK("contrastive");
    return GD_OK;
  }
  // 4 row tiles per workgroup when that still leaves >= 2 workgroups per CU
  // (GD_CONTRASTIVE_WIDE=0 / 1 forces the 16- / 64-row workgroups: tests)
  const int wide_env = env_int("GD_CONTRASTIVE_WIDE", -1);
  const bool wide = wide_env >= 0 ? wide_env == 1 : int64_t(B) * ((Q + 63) / 64) >= 512;
  const int rows = wide ? 64 : 16;
  const dim3 grid(unsigned((Q + rows - 1) / rows), unsigned(B));
  auto launch = [&](auto tag) {
    using E = decltype(tag);
    const E* xp = static_cast<const E*>(x);
    const E* tp = static_cast<const E*>(text);
    if (wide)
      hipLaunchKernelGGL((contrastive_v2_kernel<E, 4>), grid, dim3(256), 0, s, xp, x_strides[0], x_strides[1], tp,
                         text_strides[0], text_strides[1], text_mask, Q, T, C, Tout, logits, rowmax);
    else
      hipLaunchKernelGGL((contrastive_v2_kernel<E, 1>), grid, dim3(256), 0, s, xp, x_strides[0], x_strides[1], tp,
                         text_strides[0], text_strides[1], text_mask, Q, T, C, Tout, logits, rowmax);
  };
  if (dt == GD_BF16)
    launch(uint16_t{});
  else
    launch(float{});
  GD_LAUNCH_CHECK("contrastive_v2");
  return GD_OK;
}
