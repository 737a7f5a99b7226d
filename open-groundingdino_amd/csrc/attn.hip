// Masked multi-head attention (forward + backward) for gfx950: flash-style
// MFMA kernels (attn_kernels.inc) for the attention cores the reference runs
// as eager matmul / softmax / matmul chains:
//   BERT self-attention     HF BertSelfAttention via bertwarper.py:31-166
//                           (masks :224-273)
//   text enhancer           transformer_vanilla.py:83 (nn.MultiheadAttention)
//   decoder self / text     transformer.py:839,844 (nn.MultiheadAttention)
//   cross attention
// Scores never reach HBM: per 64-query block the softmax statistics stay in
// registers and only lse [B, H, Lq] is written for the backward.
#include "gd_common.h"

#include <cmath>

namespace gd {
namespace {
#include "attn_kernels.inc"
#include "attn_ks.inc"

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

gd_status fill(AttnArgs& a, gd_dtype dt, int B, int H, int Lq, int Lk, int hd, const void* q, const int64_t* qs,
               const void* k, const int64_t* ks, const void* v, const int64_t* vs, const void* mask, int mask_kind,
               const int64_t* ms, float scale, float dropout_p, uint32_t seed) {
  GD_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "attn: dropout_p %g outside [0, 1)", double(dropout_p));
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "attn: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(B >= 0 && H > 0 && Lq > 0 && Lk > 0, "attn: bad sizes B=%d H=%d Lq=%d Lk=%d", B, H, Lq, Lk);
  GD_REQUIRE(int64_t(B) * H < 65536, "attn: B*H=%lld exceeds the grid's y dimension", (long long)B * H);
  GD_REQUIRE(hd == 32 || hd == 64, "attn: head_dim %d not supported (32, 64)", hd);
  GD_REQUIRE(mask_kind >= 0 && mask_kind <= 2, "attn: mask_kind %d (0 none, 1 bool, 2 additive f32)", mask_kind);
  GD_REQUIRE(mask_kind == 0 || (mask && ms), "attn: mask pointer / strides missing");
  GD_REQUIRE(q && k && v && qs && ks && vs, "attn: null pointer");
  const int64_t align = 16 / (dt == GD_BF16 ? 2 : 4);
  for (const int64_t* st : {qs, ks, vs})
    for (int i = 0; i < 3; ++i) GD_REQUIRE(st[i] % align == 0, "attn: q/k/v strides must keep rows 16-byte aligned");
  GD_REQUIRE(aligned16(q) && aligned16(k) && aligned16(v), "attn: q/k/v must be 16-byte aligned");
  a = AttnArgs{};
  a.q = q;
  a.k = k;
  a.v = v;
  a.mask = mask;
  a.mask_kind = mask_kind;
  for (int i = 0; i < 3; ++i) {
    a.qs[i] = qs[i];
    a.ks[i] = ks[i];
    a.vs[i] = vs[i];
  }
  for (int i = 0; i < 3; ++i) a.ms[i] = mask_kind ? ms[i] : 0;
  {
    const uintptr_t mal = mask_kind == 2 ? 15 : 3;
    a.mvec = mask_kind != 0 && (reinterpret_cast<uintptr_t>(mask) & mal) == 0 && a.ms[0] % 4 == 0 &&
             a.ms[1] % 4 == 0 && a.ms[2] % 4 == 0;
  }
  a.B = B;
  a.H = H;
  a.Lq = Lq;
  a.Lk = Lk;
  a.scale = scale;
  a.dropout = dropout_p > 0.f;
  a.drop_thresh = uint32_t(fmin(double(dropout_p) * 4294967296.0, 4294967295.0));
  a.drop_scale = dropout_p > 0.f ? 1.f / (1.f - dropout_p) : 1.f;
  a.seed = seed;
  a.seed_dev = nullptr;
  return GD_OK;
}

gd_status take_strides(int64_t dst[3], const int64_t* src, const void* p, gd_dtype dt, const char* what) {
  GD_REQUIRE(p && src, "attn: null %s", what);
  GD_REQUIRE(aligned16(p), "attn: %s must be 16-byte aligned", what);
  const int64_t align = 16 / (dt == GD_BF16 ? 2 : 4);
  for (int i = 0; i < 3; ++i) {
    GD_REQUIRE(src[i] % align == 0, "attn: %s strides must keep rows 16-byte aligned", what);
    dst[i] = src[i];
  }
  return GD_OK;
}

// Query tiles of 16 per wave: 4 (64-query waves, the K / V fragments of a
// key block amortised over the most queries) unless that leaves fewer than
// 1024 waves (4 per CU) -- BERT (24 (b, h) x 256 queries: 96 waves), the text
// enhancer (32) and the decoder (240) -- then 1.  GD_ATTN_QT=1|4 forces it.
int query_tiles(int Lq, int bh) {
  const int f = env_int("GD_ATTN_QT", 0);
  if (f == 1 || f == 4) return f;
  return int64_t((Lq + 63) / 64) * bh >= 1024 ? 4 : 1;
}
// Key tiles of 16 per wave in the dK / dV kernel: 2, or 1 below 1024 waves.
int key_tiles(int Lk, int bh) {
  const int f = env_int("GD_ATTN_KT", 0);
  if (f == 1 || f == 2) return f;
  return int64_t((Lk + 31) / 32) * bh >= 1024 ? 2 : 1;
}

// The split kernels (attn_ks.inc: a workgroup per 16-query / 16-key tile,
// its waves splitting the other dimension) where the one-walk kernels would
// run 16-token waves -- the small (b, h) x L problems of the train step:
// decoder self / text cross-attention, BERT, text enhancer.  GD_ATTN_SPLIT=0
// keeps the round-5 kernels (A/B).
bool use_split(int L, int bh) {
  if (env_int("GD_ATTN_SPLIT", 1) == 0) return false;
  return int64_t((L + 63) / 64) * bh < 1024;
}

}  // namespace
}  // namespace gd

using namespace gd;

#define GD_RET(expr)                 \
  do {                               \
    const gd_status _s = (expr);     \
    if (_s != GD_OK) return _s;      \
  } while (0)

extern "C" gd_status gd_attn_forward_dev(gd_dtype dt, int B, int H, int Lq, int Lk, int head_dim, const void* q,
                                         const int64_t* q_strides, const void* k, const int64_t* k_strides,
                                         const void* v, const int64_t* v_strides, const void* mask, int mask_kind,
                                         const int64_t* mask_strides, float scale, float dropout_p, uint32_t seed,
                                         const uint32_t* seed_dev, void* out, const int64_t* out_strides,
                                         float* lse, gd_stream_t stream) {
  AttnArgs a;
  GD_RET(fill(a, dt, B, H, Lq, Lk, head_dim, q, q_strides, k, k_strides, v, v_strides, mask, mask_kind,
              mask_strides, scale, dropout_p, seed));
  a.seed_dev = seed_dev;
  if (B == 0) return GD_OK;
  GD_RET(take_strides(a.os, out_strides, out, dt, "out"));
  GD_REQUIRE(lse, "attn: null lse");
  a.o = out;
  a.lse = lse;
  hipStream_t s = as_hip(stream);
  if (use_split(Lq, B * H)) {
    const dim3 g16(unsigned((Lq + 15) / 16), unsigned(B * H));
#define GD_AS2(T, HD, KS, MK)                                                                     \
  do {                                                                                            \
    if (a.dropout)                                                                                \
      hipLaunchKernelGGL((attn_fwd_ks_kernel<T, HD, true, KS, MK>), g16, dim3(64 * KS), 0, s, a);  \
    else                                                                                          \
      hipLaunchKernelGGL((attn_fwd_ks_kernel<T, HD, false, KS, MK>), g16, dim3(64 * KS), 0, s, a); \
  } while (0)
#define GD_AS1(T, HD, KS)                                  \
  do {                                                     \
    if (a.mask_kind == 1) GD_AS2(T, HD, KS, 1);            \
    else if (a.mask_kind == 2) GD_AS2(T, HD, KS, 2);       \
    else GD_AS2(T, HD, KS, 0);                             \
  } while (0)
    if (dt == GD_BF16) {
      if (head_dim == 32) GD_AS1(uint16_t, 32, 4); else GD_AS1(uint16_t, 64, 4);
    } else {
      if (head_dim == 32) GD_AS1(float, 32, 2); else GD_AS1(float, 64, 2);
    }
#undef GD_AS1
#undef GD_AS2
    GD_LAUNCH_CHECK("attn_fwd_ks");
    return GD_OK;
  }
  const int qt = query_tiles(Lq, B * H);
  const dim3 grid(unsigned((Lq + 64 * qt - 1) / (64 * qt)), unsigned(B * H));
#define GD_AF1(T, HD, QT)                                                                    \
  do {                                                                                       \
    if (a.dropout)                                                                           \
      hipLaunchKernelGGL((attn_fwd_kernel<T, HD, true, QT>), grid, dim3(256), 0, s, a);      \
    else                                                                                     \
      hipLaunchKernelGGL((attn_fwd_kernel<T, HD, false, QT>), grid, dim3(256), 0, s, a);     \
  } while (0)
#define GD_AF(T, HD)                       \
  do {                                     \
    if (qt == 4) GD_AF1(T, HD, 4);         \
    else GD_AF1(T, HD, 1);                 \
  } while (0)
  if (dt == GD_BF16) {
    if (head_dim == 32) GD_AF(uint16_t, 32); else GD_AF(uint16_t, 64);
  } else {
    if (head_dim == 32) GD_AF(float, 32); else GD_AF(float, 64);
  }
#undef GD_AF1
#undef GD_AF
  GD_LAUNCH_CHECK("attn_fwd");
  return GD_OK;
}

extern "C" gd_status gd_attn_forward(gd_dtype dt, int B, int H, int Lq, int Lk, int head_dim, const void* q,
                                     const int64_t* q_strides, const void* k, const int64_t* k_strides,
                                     const void* v, const int64_t* v_strides, const void* mask, int mask_kind,
                                     const int64_t* mask_strides, float scale, float dropout_p, uint32_t seed,
                                     void* out, const int64_t* out_strides, float* lse, gd_stream_t stream) {
  return gd_attn_forward_dev(dt, B, H, Lq, Lk, head_dim, q, q_strides, k, k_strides, v, v_strides, mask,
                             mask_kind, mask_strides, scale, dropout_p, seed, nullptr, out, out_strides, lse,
                             stream);
}

extern "C" gd_status gd_attn_backward_dev(gd_dtype dt, int B, int H, int Lq, int Lk, int head_dim, const void* q,
                                          const int64_t* q_strides, const void* k, const int64_t* k_strides,
                                          const void* v, const int64_t* v_strides, const void* mask,
                                          int mask_kind, const int64_t* mask_strides, float scale, float dropout_p,
                                          uint32_t seed, const uint32_t* seed_dev, const void* out,
                                      const int64_t* out_strides, const void* grad_out,
                                      const int64_t* grad_out_strides, const float* lse, float* dsum,
                                      void* grad_q, const int64_t* grad_q_strides, void* grad_k,
                                      const int64_t* grad_k_strides, void* grad_v, const int64_t* grad_v_strides,
                                      gd_stream_t stream) {
  AttnArgs a;
  GD_RET(fill(a, dt, B, H, Lq, Lk, head_dim, q, q_strides, k, k_strides, v, v_strides, mask, mask_kind,
              mask_strides, scale, dropout_p, seed));
  a.seed_dev = seed_dev;
  if (B == 0) return GD_OK;
  GD_RET(take_strides(a.os, out_strides, out, dt, "out"));
  GD_RET(take_strides(a.gs, grad_out_strides, grad_out, dt, "grad_out"));
  GD_RET(take_strides(a.dqs, grad_q_strides, grad_q, dt, "grad_q"));
  GD_RET(take_strides(a.dks, grad_k_strides, grad_k, dt, "grad_k"));
  GD_RET(take_strides(a.dvs, grad_v_strides, grad_v, dt, "grad_v"));
  GD_REQUIRE(lse && dsum, "attn: null lse / dsum");
  a.o = const_cast<void*>(out);
  a.dout = grad_out;
  a.dq = grad_q;
  a.dk = grad_k;
  a.dv = grad_v;
  a.lse = const_cast<float*>(lse);
  a.dsum = dsum;
  a.lvec = Lq % 4 == 0 && aligned16(lse) && aligned16(dsum);
  hipStream_t s = as_hip(stream);
  const bool split_q = use_split(Lq, B * H), split_k = use_split(Lk, B * H);
  if (split_q && split_k) {
    const dim3 gq16(unsigned((Lq + 15) / 16), unsigned(B * H)), gk16(unsigned((Lk + 15) / 16), unsigned(B * H));
#define GD_BS2(T, HD, DR, KS, MK)                                                                          \
  do {                                                                                                     \
    hipLaunchKernelGGL((attn_bwd_dq_ks_kernel<T, HD, DR, KS, MK>), gq16, dim3(64 * KS), 0, s, a);          \
    GD_LAUNCH_CHECK("attn_bwd_dq_ks");                                                                     \
    hipLaunchKernelGGL((attn_bwd_dkv_qs_kernel<T, HD, DR, KS, MK>), gk16, dim3(64 * KS), 0, s, a);         \
    GD_LAUNCH_CHECK("attn_bwd_dkv_qs");                                                                    \
  } while (0)
#define GD_BS1(T, HD, DR, KS)                              \
  do {                                                     \
    if (a.mask_kind == 1) GD_BS2(T, HD, DR, KS, 1);        \
    else if (a.mask_kind == 2) GD_BS2(T, HD, DR, KS, 2);   \
    else GD_BS2(T, HD, DR, KS, 0);                         \
  } while (0)
#define GD_BS(T, HD, KS)                     \
  do {                                       \
    if (a.dropout) GD_BS1(T, HD, true, KS);  \
    else GD_BS1(T, HD, false, KS);           \
  } while (0)
    if (dt == GD_BF16) {
      if (head_dim == 32) GD_BS(uint16_t, 32, 4); else GD_BS(uint16_t, 64, 4);
    } else {
      if (head_dim == 32) GD_BS(float, 32, 2); else GD_BS(float, 64, 2);
    }
#undef GD_BS1
#undef GD_BS2
#undef GD_BS
    return GD_OK;
  }
  const int qt = query_tiles(Lq, B * H), kt = key_tiles(Lk, B * H);
  const dim3 gq(unsigned((Lq + 64 * qt - 1) / (64 * qt)), unsigned(B * H));
  const dim3 gk(unsigned((Lk + 64 * kt - 1) / (64 * kt)), unsigned(B * H));
#define GD_AB1(T, HD, DR)                                                                                  \
  do {                                                                                                     \
    if (qt == 4) hipLaunchKernelGGL((attn_bwd_dq_kernel<T, HD, DR, 4>), gq, dim3(256), 0, s, a);           \
    else hipLaunchKernelGGL((attn_bwd_dq_kernel<T, HD, DR, 1>), gq, dim3(256), 0, s, a);                   \
    GD_LAUNCH_CHECK("attn_bwd_dq");                                                                        \
    if (kt == 2) hipLaunchKernelGGL((attn_bwd_dkv_kernel<T, HD, DR, 2>), gk, dim3(256), 0, s, a);          \
    else hipLaunchKernelGGL((attn_bwd_dkv_kernel<T, HD, DR, 1>), gk, dim3(256), 0, s, a);                  \
    GD_LAUNCH_CHECK("attn_bwd_dkv");                                                                       \
  } while (0)
#define GD_AB(T, HD)                       \
  do {                                     \
    if (a.dropout) GD_AB1(T, HD, true);    \
    else GD_AB1(T, HD, false);             \
  } while (0)
  if (dt == GD_BF16) {
    if (head_dim == 32) GD_AB(uint16_t, 32); else GD_AB(uint16_t, 64);
  } else {
    if (head_dim == 32) GD_AB(float, 32); else GD_AB(float, 64);
  }
#undef GD_AB1
#undef GD_AB
  return GD_OK;
}

extern "C" gd_status gd_attn_backward(gd_dtype dt, int B, int H, int Lq, int Lk, int head_dim, const void* q,
                                      const int64_t* q_strides, const void* k, const int64_t* k_strides,
                                      const void* v, const int64_t* v_strides, const void* mask, int mask_kind,
                                      const int64_t* mask_strides, float scale, float dropout_p, uint32_t seed,
                                      const void* out, const int64_t* out_strides, const void* grad_out,
                                      const int64_t* grad_out_strides, const float* lse, float* dsum,
                                      void* grad_q, const int64_t* grad_q_strides, void* grad_k,
                                      const int64_t* grad_k_strides, void* grad_v, const int64_t* grad_v_strides,
                                      gd_stream_t stream) {
  return gd_attn_backward_dev(dt, B, H, Lq, Lk, head_dim, q, q_strides, k, k_strides, v, v_strides, mask,
                              mask_kind, mask_strides, scale, dropout_p, seed, nullptr, out, out_strides, grad_out,
                              grad_out_strides, lse, dsum, grad_q, grad_q_strides, grad_k, grad_k_strides, grad_v,
                              grad_v_strides, stream);
}
