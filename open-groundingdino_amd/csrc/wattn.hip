// Swin window attention (W-MSA / SW-MSA) forward + backward for gfx950.
//
// Replaces the eager chain of the reference's WindowAttention.forward
//   models/GroundingDINO/backbone/swin_transformer.py:134-174
// (q.scale.k^T -> + relative_position_bias_table[relative_position_index]
//  -> + shift mask (-100 / 0, :416-443) -> softmax -> .v), and its autograd
// backward including the scatter-add into relative_position_bias_table.
// One MFMA kernel per direction; the qkv Linear output is read in place
// ([B_, N, 3, nH, hd], no permute copy) and the output is written in the
// layout the proj Linear reads ([B_, N, nH*hd], no transpose copy).
// The _image entry points also absorb the SwinTransformerBlock's pad, cyclic
// shift and window partition / reverse (swin_transformer.py:238-292): they
// read the qkv Linear output of the unpartitioned image [B, H*W, 3C] through
// a row map and write [B, H*W, C].
// Device code and its design notes: wattn_kernels.inc.
#include "gd_common.h"

#include <cmath>

namespace gd {
namespace {
#include "wattn_kernels.inc"

constexpr int kWpw = 4;  // backward: windows per wave (one head per block)

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

gd_status check(gd_dtype dt, const void* qkv, const float* table, const int64_t* ridx, int B_, int N, int nH,
                int hd, int nW) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "window_attn: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(B_ >= 0 && N > 0 && N <= kWTok && nH > 0 && nW > 0,
             "window_attn: bad sizes B_=%d N=%d (1..%d) nH=%d nW=%d", B_, N, kWTok, nH, nW);
  GD_REQUIRE(hd == 32, "window_attn: head_dim %d not supported (32: Swin-T/S/B/L)", hd);
  GD_REQUIRE(B_ % nW == 0, "window_attn: B_=%d is not a multiple of nW=%d", B_, nW);
  GD_REQUIRE(int64_t(B_) * N * 3 * nH * hd < (int64_t(1) << 31), "window_attn: qkv too large for int32 offsets");
  GD_REQUIRE(B_ == 0 || (qkv && table && ridx), "window_attn: null pointer");
  GD_REQUIRE(aligned16(qkv), "window_attn: qkv must be 16-byte aligned");
  return GD_OK;
}

template <typename T>
void launch_fwd(const void* qkv, const void* padv, const WinGeo& geo, const float* table, const int64_t* ridx,
                const float* mask, int B_, int N, int nH, int nW, float scale, void* out, float* lse, hipStream_t s) {
  const dim3 grid(unsigned((B_ + 3) / 4), unsigned(nH));
  hipLaunchKernelGGL((wattn_fwd_kernel<T, 32>), grid, dim3(256), 0, s, (const T*)qkv, (const T*)padv, geo, table,
                     ridx, mask, B_, N, nH, nW, scale, (T*)out, lse);
}

template <typename T>
void launch_bwd(const void* qkv, const void* padv, const WinGeo& geo, const float* table, const int64_t* ridx,
                const float* mask, const void* out, const void* dout, const float* lse, int B_, int N, int nH,
                int nW, float scale, void* dqkv, float* grad_pad, float* dtable, hipStream_t s) {
  const dim3 grid(unsigned((B_ + 4 * kWpw - 1) / (4 * kWpw)), unsigned(nH));
  hipLaunchKernelGGL((wattn_bwd_kernel<T, 32, kWpw>), grid, dim3(256), 0, s, (const T*)qkv, (const T*)padv, geo,
                     table, ridx, mask, (const T*)out, (const T*)dout, lse, B_, N, nH, nW, scale, (T*)dqkv,
                     grad_pad, dtable);
}

// image geometry -> WinGeo + window count; validates the sizes
gd_status image_geo(int B, int H, int W, int ws, int sh, WinGeo* geo, int* B_) {
  GD_REQUIRE(B >= 0 && H > 0 && W > 0, "window_attn_image: bad sizes B=%d H=%d W=%d", B, H, W);
  GD_REQUIRE(ws > 0 && ws * ws <= kWTok, "window_attn_image: window %d not supported (ws*ws <= %d)", ws, kWTok);
  GD_REQUIRE(sh >= 0 && sh < ws, "window_attn_image: shift %d not in [0, window %d)", sh, ws);
  GD_REQUIRE(int64_t(B) * H * W < (int64_t(1) << 31), "window_attn_image: too many tokens");
  geo->img = 1;
  geo->H = H;
  geo->W = W;
  geo->ws = ws;
  geo->sh = sh;
  geo->Hp = (H + ws - 1) / ws * ws;
  geo->Wp = (W + ws - 1) / ws * ws;
  geo->nWw = geo->Wp / ws;
  geo->nWi = (geo->Hp / ws) * geo->nWw;
  GD_REQUIRE(int64_t(B) * geo->nWi * ws * ws < (int64_t(1) << 31), "window_attn_image: too many windows");
  *B_ = B * geo->nWi;
  return GD_OK;
}

WinGeo window_geo() {
  WinGeo g{};
  return g;
}

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" gd_status gd_window_attn_forward(gd_dtype dt, const void* qkv, const float* table,
                                           const int64_t* rel_index, const float* mask, int B_, int N, int nH,
                                           int head_dim, int nW, float scale, void* out, float* lse,
                                           gd_stream_t stream) {
  const gd_status st = check(dt, qkv, table, rel_index, B_, N, nH, head_dim, nW);
  if (st != GD_OK) return st;
  if (B_ == 0) return GD_OK;
  GD_REQUIRE(out && lse, "window_attn_forward: null output");
  hipStream_t s = as_hip(stream);
  if (dt == GD_BF16) {
    launch_fwd<uint16_t>(qkv, nullptr, window_geo(), table, rel_index, mask, B_, N, nH, nW, scale, out, lse, s);
  } else {
    launch_fwd<float>(qkv, nullptr, window_geo(), table, rel_index, mask, B_, N, nH, nW, scale, out, lse, s);
  }
  GD_LAUNCH_CHECK("wattn_fwd");
  return GD_OK;
}

extern "C" gd_status gd_window_attn_backward(gd_dtype dt, const void* qkv, const float* table,
                                            const int64_t* rel_index, const float* mask, const void* out,
                                            const void* grad_out, const float* lse, int B_, int N, int nH,
                                            int head_dim, int nW, float scale, void* grad_qkv,
                                            float* grad_table, gd_stream_t stream) {
  const gd_status st = check(dt, qkv, table, rel_index, B_, N, nH, head_dim, nW);
  if (st != GD_OK) return st;
  if (B_ == 0) return GD_OK;
  GD_REQUIRE(out && grad_out && lse && grad_qkv && grad_table, "window_attn_backward: null pointer");
  GD_REQUIRE(aligned16(out) && aligned16(grad_out) && aligned16(grad_qkv),
             "window_attn_backward: out / grad_out / grad_qkv must be 16-byte aligned");
  hipStream_t s = as_hip(stream);
  if (dt == GD_BF16) {
    launch_bwd<uint16_t>(qkv, nullptr, window_geo(), table, rel_index, mask, out, grad_out, lse, B_, N, nH, nW,
                         scale, grad_qkv, nullptr, grad_table, s);
  } else {
    launch_bwd<float>(qkv, nullptr, window_geo(), table, rel_index, mask, out, grad_out, lse, B_, N, nH, nW,
                      scale, grad_qkv, nullptr, grad_table, s);
  }
  GD_LAUNCH_CHECK("wattn_bwd");
  return GD_OK;
}

extern "C" gd_status gd_window_attn_image_forward(gd_dtype dt, const void* qkv, const void* qkv_bias,
                                                 const float* table, const int64_t* rel_index, const float* mask,
                                                 int B, int H, int W, int window, int shift, int nH,
                                                 int head_dim, float scale, void* out, float* lse,
                                                 gd_stream_t stream) {
  WinGeo geo;
  int B_ = 0;
  gd_status st = image_geo(B, H, W, window, shift, &geo, &B_);
  if (st != GD_OK) return st;
  st = check(dt, qkv, table, rel_index, B_, window * window, nH, head_dim, mask ? geo.nWi : 1);
  if (st != GD_OK) return st;
  if (B_ == 0) return GD_OK;
  GD_REQUIRE(out && lse, "window_attn_image_forward: null output");
  GD_REQUIRE(aligned16(qkv_bias), "window_attn_image_forward: qkv_bias must be 16-byte aligned");
  hipStream_t s = as_hip(stream);
  const int N = window * window, nW = mask ? geo.nWi : 1;
  if (dt == GD_BF16) {
    launch_fwd<uint16_t>(qkv, qkv_bias, geo, table, rel_index, mask, B_, N, nH, nW, scale, out, lse, s);
  } else {
    launch_fwd<float>(qkv, qkv_bias, geo, table, rel_index, mask, B_, N, nH, nW, scale, out, lse, s);
  }
  GD_LAUNCH_CHECK("wattn_image_fwd");
  return GD_OK;
}

extern "C" gd_status gd_window_attn_image_backward(gd_dtype dt, const void* qkv, const void* qkv_bias,
                                                  const float* table, const int64_t* rel_index, const float* mask,
                                                  const void* out, const void* grad_out, const float* lse, int B,
                                                  int H, int W, int window, int shift, int nH, int head_dim,
                                                  float scale, void* grad_qkv, float* grad_qkv_bias,
                                                  float* grad_table, gd_stream_t stream) {
  WinGeo geo;
  int B_ = 0;
  gd_status st = image_geo(B, H, W, window, shift, &geo, &B_);
  if (st != GD_OK) return st;
  st = check(dt, qkv, table, rel_index, B_, window * window, nH, head_dim, mask ? geo.nWi : 1);
  if (st != GD_OK) return st;
  if (B_ == 0) return GD_OK;
  GD_REQUIRE(out && grad_out && lse && grad_qkv && grad_table, "window_attn_image_backward: null pointer");
  GD_REQUIRE(aligned16(out) && aligned16(grad_out) && aligned16(grad_qkv) && aligned16(qkv_bias),
             "window_attn_image_backward: out / grad_out / grad_qkv / qkv_bias must be 16-byte aligned");
  hipStream_t s = as_hip(stream);
  const int N = window * window, nW = mask ? geo.nWi : 1;
  if (dt == GD_BF16) {
    launch_bwd<uint16_t>(qkv, qkv_bias, geo, table, rel_index, mask, out, grad_out, lse, B_, N, nH, nW, scale,
                         grad_qkv, qkv_bias ? grad_qkv_bias : nullptr, grad_table, s);
  } else {
    launch_bwd<float>(qkv, qkv_bias, geo, table, rel_index, mask, out, grad_out, lse, B_, N, nH, nW, scale,
                      grad_qkv, qkv_bias ? grad_qkv_bias : nullptr, grad_table, s);
  }
  GD_LAUNCH_CHECK("wattn_image_bwd");
  return GD_OK;
}
