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

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace gd {
namespace {
#include "wattn_kernels.inc"

constexpr int kMaxTokens = 144;  // 12x12 windows (Swin-B/L at 384)

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int isqrt_exact(int n) {  // ws with ws*ws == n, else 0
  for (int w = 1; w * w <= n; ++w)
    if (w * w == n) return w;
  return 0;
}

gd_status check(gd_dtype dt, const void* qkv, const float* table, const int64_t* ridx, int B_, int N, int nH,
                int hd, int nW, int ws) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "window_attn: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(B_ >= 0 && N > 0 && N <= kMaxTokens && nH > 0 && nW > 0,
             "window_attn: bad sizes B_=%d N=%d (1..%d) nH=%d nW=%d", B_, N, kMaxTokens, nH, nW);
  GD_REQUIRE(hd == 32, "window_attn: head_dim %d not supported (32: Swin-T/S/B/L)", hd);
  GD_REQUIRE(B_ % nW == 0, "window_attn: B_=%d is not a multiple of nW=%d", B_, nW);
  GD_REQUIRE(ridx || (ws > 0 && ws * ws == N && ws <= 12),
             "window_attn: rel_index NULL needs a square window of <= 12x12 tokens (N=%d)", N);
  GD_REQUIRE(int64_t(B_) * N * 3 * nH * hd < (int64_t(1) << 31), "window_attn: qkv too large for int32 offsets");
  GD_REQUIRE(B_ == 0 || (qkv && table), "window_attn: null pointer");
  GD_REQUIRE(aligned16(qkv), "window_attn: qkv must be 16-byte aligned");
  return GD_OK;
}

// windows per block: about GD_WATTN_BLOCKS workgroups over the launch
// (default 1024: 3-4 resident per CU, so every block runs several windows
// with the next one's loads in flight -- at 2048 the later Swin stages got
// one window per block, whose loads and prologue nothing overlapped), at
// most 8
int windows_per_block(int B_, int nH) {
  const int64_t tasks = int64_t(B_) * nH;
  const int64_t target = std::max(64, env_int("GD_WATTN_BLOCKS", 1024));
  return int(std::max<int64_t>(1, std::min<int64_t>(8, (tasks + target - 1) / target)));
}

WinCtx make_ctx(const float* table, const int64_t* ridx, const float* mask, int N, int nH, int nW, int ws,
                float scale) {
  WinCtx X{};
  X.table = table;
  X.ridx = ridx;
  X.mask = mask;
  X.N = N;
  X.nH = nH;
  X.nW = nW;
  X.h = 0;
  X.c0 = ws > 0 ? (ws - 1) * (2 * ws - 1) + ws - 1 : 0;
  X.scale = scale;
  return X;
}

template <typename T, int NT, int MODE>
void launch_fwd_nt(const void* qkv, const void* padv, const WinGeo& geo, const WinCtx& X, int B_, void* out,
                   float* lse, hipStream_t s) {
  const int wpb = windows_per_block(B_, X.nH);
  const unsigned nblk = unsigned((B_ + wpb - 1) / wpb) * unsigned(X.nH);
  hipLaunchKernelGGL((wattn_fwd_kernel<T, NT, MODE>), dim3(nblk), dim3(64 * NT), 0, s, (const T*)qkv, (const T*)padv,
                     geo, X, B_, wpb, (T*)out, lse);
}

template <typename T, int NT>
void launch_fwd_mode(int mode, const void* qkv, const void* padv, const WinGeo& geo, const WinCtx& X, int B_,
                     void* out, float* lse, hipStream_t s) {
  if (mode == kModeStd) {
    launch_fwd_nt<T, NT, kModeStd>(qkv, padv, geo, X, B_, out, lse, s);
  } else if (mode == kModeRegion) {
    launch_fwd_nt<T, NT, kModeRegion>(qkv, padv, geo, X, B_, out, lse, s);
  } else {
    launch_fwd_nt<T, NT, kModeAny>(qkv, padv, geo, X, B_, out, lse, s);
  }
}

template <typename T>
void launch_fwd(int mode, const void* qkv, const void* padv, const WinGeo& geo, const WinCtx& X, int B_, void* out,
                float* lse, hipStream_t s) {
  if (X.N <= 64) {
    launch_fwd_mode<T, 4>(mode, qkv, padv, geo, X, B_, out, lse, s);
  } else {
    launch_fwd_mode<T, 9>(mode, qkv, padv, geo, X, B_, out, lse, s);
  }
}

// backward dS-over-windows sums for 7x7 windows: registers (default) or LDS
// atomics per window (GD_WATTN_REGSUM=0)
bool bwd_regsum() {
  static const bool on = [] {
    const char* e = std::getenv("GD_WATTN_REGSUM");
    return !(e && e[0] == '0');
  }();
  return on;
}

// the single-pass-softmax backward (wattn_bwd2_kernel) for N <= 64 with a
// computed index / mask (GD_WATTN_BWD2=0: the round-5 kernel, A/B)
bool bwd_v2() { return env_int("GD_WATTN_BWD2", 1) != 0; }

template <typename T, int NT, int MODE>
void launch_bwd_nt(const void* qkv, const void* padv, const WinGeo& geo, const WinCtx& X, const void* out,
                   const void* dout, const float* lse, int B_, void* dqkv, float* grad_pad, float* dtable,
                   hipStream_t s) {
  const int wpb = windows_per_block(B_, X.nH);
  const unsigned nblk = unsigned((B_ + wpb - 1) / wpb) * unsigned(X.nH);
  if constexpr (NT <= 4 && MODE != kModeAny) {
    if (bwd_v2()) {
      hipLaunchKernelGGL((wattn_bwd2_kernel<T, MODE>), dim3(nblk), dim3(256), 0, s, (const T*)qkv, (const T*)padv,
                         geo, X, (const T*)out, (const T*)dout, lse, B_, wpb, (T*)dqkv, grad_pad, dtable);
      return;
    }
  }
  if constexpr (NT <= 4) {
    if (bwd_regsum()) {
      hipLaunchKernelGGL((wattn_bwd_kernel<T, NT, MODE, true>), dim3(nblk), dim3(64 * NT), 0, s, (const T*)qkv,
                         (const T*)padv, geo, X, (const T*)out, (const T*)dout, lse, B_, wpb, (T*)dqkv, grad_pad,
                         dtable);
      return;
    }
  }
  {
    hipLaunchKernelGGL((wattn_bwd_kernel<T, NT, MODE, false>), dim3(nblk), dim3(64 * NT), 0, s, (const T*)qkv,
                       (const T*)padv, geo, X, (const T*)out, (const T*)dout, lse, B_, wpb, (T*)dqkv, grad_pad,
                       dtable);
  }
}

template <typename T, int NT>
void launch_bwd_mode(int mode, const void* qkv, const void* padv, const WinGeo& geo, const WinCtx& X,
                     const void* out, const void* dout, const float* lse, int B_, void* dqkv, float* grad_pad,
                     float* dtable, hipStream_t s) {
  if (mode == kModeStd) {
    launch_bwd_nt<T, NT, kModeStd>(qkv, padv, geo, X, out, dout, lse, B_, dqkv, grad_pad, dtable, s);
  } else if (mode == kModeRegion) {
    launch_bwd_nt<T, NT, kModeRegion>(qkv, padv, geo, X, out, dout, lse, B_, dqkv, grad_pad, dtable, s);
  } else {
    launch_bwd_nt<T, NT, kModeAny>(qkv, padv, geo, X, out, dout, lse, B_, dqkv, grad_pad, dtable, s);
  }
}

template <typename T>
void launch_bwd(int mode, const void* qkv, const void* padv, const WinGeo& geo, const WinCtx& X, const void* out,
                const void* dout, const float* lse, int B_, void* dqkv, float* grad_pad, float* dtable,
                hipStream_t s) {
  if (X.N <= 64) {
    launch_bwd_mode<T, 4>(mode, qkv, padv, geo, X, out, dout, lse, B_, dqkv, grad_pad, dtable, s);
  } else {
    launch_bwd_mode<T, 9>(mode, qkv, padv, geo, X, out, dout, lse, B_, dqkv, grad_pad, dtable, s);
  }
}

// image geometry -> WinGeo + window count; validates the sizes
gd_status image_geo(int B, int H, int W, int ws, int sh, WinGeo* geo, int* B_) {
  GD_REQUIRE(B >= 0 && H > 0 && W > 0, "window_attn_image: bad sizes B=%d H=%d W=%d", B, H, W);
  GD_REQUIRE(ws > 0 && ws * ws <= kMaxTokens, "window_attn_image: window %d not supported (ws*ws <= %d)", ws,
             kMaxTokens);
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

// kernel variant: a given rel_index or mask tensor is read as given; with
// both NULL the index is computed, and in the image layout a shift > 0
// computes the reference's region mask (window-major: no mask)
int win_mode(const int64_t* ridx, const float* mask, bool region) {
  if (ridx || mask) return kModeAny;
  return region ? kModeRegion : kModeStd;
}

WinGeo window_geo(int N) {
  WinGeo g{};
  g.ws = isqrt_exact(N);
  return g;
}

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" gd_status gd_window_attn_forward(gd_dtype dt, const void* qkv, const float* table,
                                           const int64_t* rel_index, const float* mask, int B_, int N, int nH,
                                           int head_dim, int nW, float scale, void* out, float* lse,
                                           gd_stream_t stream) {
  const WinGeo geo = window_geo(N);
  const gd_status st = check(dt, qkv, table, rel_index, B_, N, nH, head_dim, nW, geo.ws);
  if (st != GD_OK) return st;
  if (B_ == 0) return GD_OK;
  GD_REQUIRE(out && lse, "window_attn_forward: null output");
  GD_REQUIRE(aligned16(out), "window_attn_forward: out must be 16-byte aligned");
  const WinCtx X = make_ctx(table, rel_index, mask, N, nH, nW, geo.ws, scale);
  hipStream_t s = as_hip(stream);
  if (dt == GD_BF16) {
    launch_fwd<uint16_t>(win_mode(rel_index, mask, false), qkv, nullptr, geo, X, B_, out, lse, s);
  } else {
    launch_fwd<float>(win_mode(rel_index, mask, false), qkv, nullptr, geo, X, B_, out, lse, s);
  }
  GD_LAUNCH_CHECK("wattn_fwd");
  return GD_OK;
}

extern "C" gd_status gd_window_attn_backward(gd_dtype dt, const void* qkv, const float* table,
                                            const int64_t* rel_index, const float* mask, const void* out,
                                            const void* grad_out, const float* lse, int B_, int N, int nH,
                                            int head_dim, int nW, float scale, void* grad_qkv,
                                            float* grad_table, gd_stream_t stream) {
  const WinGeo geo = window_geo(N);
  const gd_status st = check(dt, qkv, table, rel_index, B_, N, nH, head_dim, nW, geo.ws);
  if (st != GD_OK) return st;
  if (B_ == 0) return GD_OK;
  GD_REQUIRE(out && grad_out && lse && grad_qkv && grad_table, "window_attn_backward: null pointer");
  GD_REQUIRE(aligned16(out) && aligned16(grad_out) && aligned16(grad_qkv),
             "window_attn_backward: out / grad_out / grad_qkv must be 16-byte aligned");
  const WinCtx X = make_ctx(table, rel_index, mask, N, nH, nW, geo.ws, scale);
  hipStream_t s = as_hip(stream);
  if (dt == GD_BF16) {
    launch_bwd<uint16_t>(win_mode(rel_index, mask, false), qkv, nullptr, geo, X, out, grad_out, lse, B_, grad_qkv, nullptr, grad_table, s);
  } else {
    launch_bwd<float>(win_mode(rel_index, mask, false), qkv, nullptr, geo, X, out, grad_out, lse, B_, grad_qkv, nullptr, grad_table, s);
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
  const int N = window * window, nW = mask ? geo.nWi : 1;
  st = check(dt, qkv, table, rel_index, B_, N, nH, head_dim, nW, window);
  if (st != GD_OK) return st;
  if (B_ == 0) return GD_OK;
  GD_REQUIRE(out && lse, "window_attn_image_forward: null output");
  GD_REQUIRE(aligned16(qkv_bias) && aligned16(out), "window_attn_image_forward: qkv_bias / out must be 16-byte aligned");
  const WinCtx X = make_ctx(table, rel_index, mask, N, nH, nW, window, scale);
  hipStream_t s = as_hip(stream);
  if (dt == GD_BF16) {
    launch_fwd<uint16_t>(win_mode(rel_index, mask, shift > 0), qkv, qkv_bias, geo, X, B_, out, lse, s);
  } else {
    launch_fwd<float>(win_mode(rel_index, mask, shift > 0), qkv, qkv_bias, geo, X, B_, out, lse, s);
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
  const int N = window * window, nW = mask ? geo.nWi : 1;
  st = check(dt, qkv, table, rel_index, B_, N, nH, head_dim, nW, window);
  if (st != GD_OK) return st;
  if (B_ == 0) return GD_OK;
  GD_REQUIRE(out && grad_out && lse && grad_qkv && grad_table, "window_attn_image_backward: null pointer");
  GD_REQUIRE(aligned16(out) && aligned16(grad_out) && aligned16(grad_qkv) && aligned16(qkv_bias),
             "window_attn_image_backward: out / grad_out / grad_qkv / qkv_bias must be 16-byte aligned");
  const WinCtx X = make_ctx(table, rel_index, mask, N, nH, nW, window, scale);
  hipStream_t s = as_hip(stream);
  if (dt == GD_BF16) {
    launch_bwd<uint16_t>(win_mode(rel_index, mask, shift > 0), qkv, qkv_bias, geo, X, out, grad_out, lse, B_, grad_qkv, qkv_bias ? grad_qkv_bias : nullptr,
                         grad_table, s);
  } else {
    launch_bwd<float>(win_mode(rel_index, mask, shift > 0), qkv, qkv_bias, geo, X, out, grad_out, lse, B_, grad_qkv, qkv_bias ? grad_qkv_bias : nullptr,
                      grad_table, s);
  }
  GD_LAUNCH_CHECK("wattn_image_bwd");
  return GD_OK;
}
