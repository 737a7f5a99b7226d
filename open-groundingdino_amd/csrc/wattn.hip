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
  const dim3 grid(unsigned((B_ + 3) / 4), unsigned(nH));
#define GD_WF(T, HD)                                                                                     \
  hipLaunchKernelGGL((wattn_fwd_kernel<T, HD>), grid, dim3(256), 0, s, (const T*)qkv, table,            \
                     rel_index, mask, B_, N, nH, nW, scale, (T*)out, lse)
  if (dt == GD_BF16) {
    GD_WF(uint16_t, 32);
  } else {
    GD_WF(float, 32);
  }
#undef GD_WF
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
  const dim3 grid(unsigned((B_ + 4 * kWpw - 1) / (4 * kWpw)), unsigned(nH));
#define GD_WB(T, HD)                                                                                        \
  hipLaunchKernelGGL((wattn_bwd_kernel<T, HD, kWpw>), grid, dim3(256), 0, s, (const T*)qkv, table,         \
                     rel_index, mask, (const T*)out, (const T*)grad_out, lse, B_, N, nH, nW, scale,        \
                     (T*)grad_qkv, grad_table)
  if (dt == GD_BF16) {
    GD_WB(uint16_t, 32);
  } else {
    GD_WB(float, 32);
  }
#undef GD_WB
  GD_LAUNCH_CHECK("wattn_bwd");
  return GD_OK;
}
