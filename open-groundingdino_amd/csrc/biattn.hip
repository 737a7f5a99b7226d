// Bidirectional softmax of BiMultiHeadAttention for gfx950.
//
// Reference: models/GroundingDINO/fuse_modules.py:174-217.  One score matrix
// s = q.k^T [BH, S, T] (S image tokens, T text tokens; produced by a
// hipBLASLt GEMM) feeds two softmaxes:
//   P_v = softmax over T of (s + mask_l)     (image queries attend text)
//   P_l = softmax over S of (s + mask_v)     (text queries attend image),
//         stored in the same [BH, S, T] layout (column-normalised), so the
//         text-side output is the GEMM P_l^T . v_v.
// The reference's global-max shift, column-max shift and +-5e4 clamps are
// shift/clamp guards that leave softmax unchanged for any score spread below
// 5e4 (fp32 statistics here); see DESIGN.md.
//
// Forward  (3 launches, S read twice, P_v / P_l written once):
//   colstats  : per (column block of rows) online max / sum-exp per column t
//   colmerge  : merge the row-chunk partials -> m_t, 1/l_t
//   rows      : one wave per row: row max / sum over T by wave shuffles,
//               writes P_v and P_l = exp(s - m_t) / l_t.
// Backward (3 launches):
//   colsum    : c_t partials of sum_s dP_l * P_l
//   colmerge  : -> c_t
//   rows      : r_s = sum_t dP_v * P_v by wave shuffles,
//               dS = P_v (dP_v - r_s) + P_l (dP_l - c_t).
// Padding: pad_v[b, s] masks image row s out of every column softmax (P_l = 0),
// pad_l[b, t] masks text column t out of every row softmax (P_v = 0).
#include "gd_common.h"

#include <algorithm>
#include <initializer_list>
#include <type_traits>

namespace gd {
namespace {
#include "biattn_kernels.inc"

inline int nchunks(int S) { return (S + kRowsPerChunk - 1) / kRowsPerChunk; }

inline bool aligned_to(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

// Slots per lane: smallest power of two E with 64*E >= T (T <= 1024).
inline int slots_for(int Tn) {
  int e = 1;
  while (64 * e < Tn) e <<= 1;
  return e;
}

// Contiguous slots need T == 64*E and every row operand aligned to its
// E-element vector (capped at 16 B: wider slots are several dwordx4 loads).
inline bool contig_ok(int Tn, size_t elem, std::initializer_list<const void*> ptrs) {
  const int e = slots_for(Tn);
  if (Tn != 64 * e) return false;
  const size_t a = std::min<size_t>(16, size_t(e) * elem);
  for (const void* p : ptrs)
    if (!aligned_to(p, a)) return false;
  return true;
}

// Calls fn(integral_constant<int, E>, bool_constant<CONTIG>) for the run-time
// (slots_for(T), contig) pair.
template <typename Fn>
void with_slots(int Tn, bool contig, Fn&& fn) {
  using std::integral_constant;
  using std::true_type;
  using std::false_type;
  switch (slots_for(Tn)) {
    case 1: contig ? fn(integral_constant<int, 1>{}, true_type{}) : fn(integral_constant<int, 1>{}, false_type{}); break;
    case 2: contig ? fn(integral_constant<int, 2>{}, true_type{}) : fn(integral_constant<int, 2>{}, false_type{}); break;
    case 4: contig ? fn(integral_constant<int, 4>{}, true_type{}) : fn(integral_constant<int, 4>{}, false_type{}); break;
    case 8: contig ? fn(integral_constant<int, 8>{}, true_type{}) : fn(integral_constant<int, 8>{}, false_type{}); break;
    default: contig ? fn(integral_constant<int, 16>{}, true_type{}) : fn(integral_constant<int, 16>{}, false_type{}); break;
  }
}

template <typename T>
gd_status softmax_fwd(const void* s, const uint8_t* pad_v, const uint8_t* pad_l, int B, int H, int S, int Tn,
                      void* pv, void* pl, void* workspace, hipStream_t st) {
  const int bh = B * H, nc = nchunks(S);
  float* pm = static_cast<float*>(workspace);
  float* plp = pm + size_t(bh) * nc * Tn;
  float* col_m = plp + size_t(bh) * nc * Tn;
  float* col_inv = col_m + size_t(bh) * Tn;
  const int64_t nrows = int64_t(bh) * S;
  const int rblocks = int((nrows + 3) / 4);
  constexpr int VE = 16 / int(sizeof(T));
  const int lpr = Tn / VE;
  if (Tn % VE == 0 && lpr >= 2 && 256 % lpr == 0 && aligned_to(s, 16)) {
    hipLaunchKernelGGL((colstats_vec_kernel<T>), dim3(nc, bh), dim3(256), 0, st,
                       (const T*)s, pad_v, H, S, Tn, pm, plp);
  } else {
    hipLaunchKernelGGL((colstats_kernel<T>), dim3(nc, bh), dim3(256), 0, st,
                       (const T*)s, pad_v, H, S, Tn, pm, plp);
  }
  GD_LAUNCH_CHECK("biattn colstats");
  hipLaunchKernelGGL((colmerge_kernel), dim3((Tn + 63) / 64, bh), dim3(1024), 0, st,
                     pm, plp, nc, Tn, col_m, col_inv);
  GD_LAUNCH_CHECK("biattn colmerge");
  const bool contig = contig_ok(Tn, sizeof(T), {s, pv, pl}) && aligned_to(col_m, 16) && aligned_to(col_inv, 16);
  with_slots(Tn, contig, [&](auto e, auto c) {
    hipLaunchKernelGGL((rows_fwd_kernel<T, decltype(e)::value, decltype(c)::value>),
                       dim3(unsigned((nrows + 4 * kRowsPerWave - 1) / (4 * kRowsPerWave))), dim3(256), 0, st,
                     (const T*)s, pad_v, pad_l, col_m, col_inv, H, S, Tn, nrows, (T*)pv, (T*)pl);
  });
  GD_LAUNCH_CHECK("biattn rows_fwd");
  return GD_OK;
}

template <typename T>
gd_status softmax_bwd(const void* pv, const void* pl, const void* dpv, const void* dpl, int B, int H, int S, int Tn,
                      void* ds, void* workspace, hipStream_t st) {
  const int bh = B * H, nc = nchunks(S);
  float* part = static_cast<float*>(workspace);
  float* csum = part + size_t(bh) * nc * Tn * 2;
  const int64_t nrows = int64_t(bh) * S;
  const int rblocks = int((nrows + 3) / 4);
  constexpr int VE = 16 / int(sizeof(T));
  const int lpr = Tn / VE;
  if (Tn % VE == 0 && lpr >= 2 && 256 % lpr == 0 && aligned_to(pl, 16) && aligned_to(dpl, 16)) {
    hipLaunchKernelGGL((colsum_vec_kernel<T>), dim3(nc, bh), dim3(256), 0, st,
                       (const T*)pl, (const T*)dpl, S, Tn, part);
  } else {
    hipLaunchKernelGGL((colsum_kernel<T>), dim3(nc, bh), dim3(256), 0, st,
                       (const T*)pl, (const T*)dpl, S, Tn, part);
  }
  GD_LAUNCH_CHECK("biattn colsum");
  hipLaunchKernelGGL((colsum_merge_kernel), dim3((Tn + 63) / 64, bh), dim3(1024), 0, st,
                     part, nc, Tn, csum);
  GD_LAUNCH_CHECK("biattn colsum_merge");
  const bool contig = contig_ok(Tn, sizeof(T), {pv, pl, dpv, dpl, ds}) && aligned_to(csum, 16);
  with_slots(Tn, contig, [&](auto e, auto c) {
    hipLaunchKernelGGL((rows_bwd_kernel<T, decltype(e)::value, decltype(c)::value>), dim3(rblocks), dim3(256), 0, st,
                     (const T*)pv, (const T*)pl, (const T*)dpv, (const T*)dpl, csum, S, Tn, nrows, (T*)ds);
  });
  GD_LAUNCH_CHECK("biattn rows_bwd");
  return GD_OK;
}

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" size_t gd_biattn_workspace_bytes(int B, int H, int S, int T) {
  const size_t bh = size_t(B) * H;
  return sizeof(float) * (bh * nchunks(S) * T * 2 + bh * T * 2);
}

extern "C" gd_status gd_biattn_softmax_fwd(gd_dtype dt, const void* s, const uint8_t* pad_v,
                                           const uint8_t* pad_l, int B, int H, int S, int T, void* pv,
                                           void* pl, void* workspace, gd_stream_t stream) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "biattn: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(B >= 0 && H > 0 && S >= 0 && T > 0 && T <= 1024, "biattn: bad sizes B=%d H=%d S=%d T=%d", B, H, S,
             T);
  if (B == 0 || S == 0) return GD_OK;
  GD_REQUIRE(s && pv && pl && workspace, "biattn_fwd: null pointer");
  hipStream_t st = as_hip(stream);
  return dt == GD_BF16 ? softmax_fwd<uint16_t>(s, pad_v, pad_l, B, H, S, T, pv, pl, workspace, st)
                       : softmax_fwd<float>(s, pad_v, pad_l, B, H, S, T, pv, pl, workspace, st);
}

extern "C" gd_status gd_biattn_softmax_bwd(gd_dtype dt, const void* pv, const void* pl, const void* dpv,
                                           const void* dpl, int B, int H, int S, int T, void* ds,
                                           void* workspace, gd_stream_t stream) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "biattn: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(B >= 0 && H > 0 && S >= 0 && T > 0 && T <= 1024, "biattn: bad sizes B=%d H=%d S=%d T=%d", B, H, S,
             T);
  if (B == 0 || S == 0) return GD_OK;
  GD_REQUIRE(pv && pl && dpv && dpl && ds && workspace, "biattn_bwd: null pointer");
  hipStream_t st = as_hip(stream);
  return dt == GD_BF16 ? softmax_bwd<uint16_t>(pv, pl, dpv, dpl, B, H, S, T, ds, workspace, st)
                       : softmax_bwd<float>(pv, pl, dpv, dpl, B, H, S, T, ds, workspace, st);
}
