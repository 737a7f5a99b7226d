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

#include <algorithm>
#include <cmath>

#include <climits>
#include <cstdlib>
#include <cstring>

namespace gd {
namespace {
// Device-side check word of the MSDA kernels (gd_device_status): a bit per
// check, set with a vector atomic OR, read and cleared by the host.
__device__ int g_device_err;
constexpr int kErrMsdaSlot = 1;  // a sorted-backward record slot past the record buffer
__device__ __forceinline__ void flag_device_error(int code) { atomicOr(&g_device_err, code); }
#include "msda_kernels.inc"
#include "msda_enc.inc"
#include "msda_sorted.inc"

constexpr int kTileQ = 32;      // queries per workgroup (one head)
constexpr int kTileRows = 384;  // LDS accumulator rows (48 KB): 3 workgroups per CU

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Encoder-shape backward selection, read per call so a test can compare the
// kernels in one process (GD_MSDA_BWD):
//   lane32  direct 128-B atomics for every corner (msda_bwd_lane32);
//   tiled   round-1 LDS pre-aggregation over 4 x 8 pixel blocks
//           (msda_bwd_tiled; 3.77 ms vs lane32's 2.19 ms on the box);
//   enc     2-D query tiles per level, vector lanes, packed LDS boxes
//           (msda_bwd_enc, msda_enc.inc);
//   auto / unset: enc when the host passes the level shapes (the model's
//           encoder does), else lane32.  Measured at 800x1333 bs=2: enc
//           0.82 ms on the reference-init geometry the bench runs at and
//           1.90 ms on a 2-px random spread, lane32 2.19 / 2.09 ms.
enum class BwdVariant { kLane32, kTiled, kEnc };
inline BwdVariant bwd_variant() {
  const char* e = getenv("GD_MSDA_BWD");
  if (e && strcmp(e, "tiled") == 0) return BwdVariant::kTiled;
  if (e && strcmp(e, "lane32") == 0) return BwdVariant::kLane32;
  return BwdVariant::kEnc;  // "enc", "auto", unset: msda_bwd_enc when the level shapes are known
}

// msda_bwd_enc geometry (tuning overrides, default below):
//   GD_MSDA_ENC_TILE="THxTW,THxTW,THxTW,THxTW"  query tile extents per query level
//   GD_MSDA_ENC_CAP="r0,r1,r2,r3"               LDS rows of each sampled level's box
inline void enc_geometry(int (&th)[4], int (&tw)[4], int (&cap)[4]) {
  // 4 x 4 query tiles on every level and 64 / 40 / 24 / 28 box rows (+ one
  // spare row each: 160 rows, 20 KB of LDS per 2-wave workgroup, so the
  // 122-VGPR waves, not LDS, limit occupancy): the fastest of the tilings
  // measured by tools/msda_microbench.py --enc-variants
  static const int dth[4] = {4, 4, 4, 4}, dtw[4] = {4, 4, 4, 4}, dcap[4] = {64, 40, 24, 28};
  for (int l = 0; l < 4; ++l) { th[l] = dth[l]; tw[l] = dtw[l]; cap[l] = dcap[l]; }
  if (const char* e = getenv("GD_MSDA_ENC_TILE")) {
    int v[8];
    if (sscanf(e, "%dx%d,%dx%d,%dx%d,%dx%d", &v[0], &v[1], &v[2], &v[3], &v[4], &v[5], &v[6], &v[7]) == 8)
      for (int l = 0; l < 4; ++l)
        if (v[2 * l] > 0 && v[2 * l + 1] > 0) { th[l] = v[2 * l]; tw[l] = v[2 * l + 1]; }
  }
  if (const char* e = getenv("GD_MSDA_ENC_CAP")) {
    int v[4];
    if (sscanf(e, "%d,%d,%d,%d", &v[0], &v[1], &v[2], &v[3]) == 4)
      for (int l = 0; l < 4; ++l)
        if (v[l] >= 0) cap[l] = v[l];
  }
}

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

  // 32-bit byte offsets from the value base inside msda_fwd_vec
  const size_t vbytes = size_t(N) * S * M * D * (dt == GD_BF16 ? 2 : 4);
  const bool vec_ok = D == 32 && L == 4 && P == 4 && units < (int64_t(1) << 31) && vbytes < (size_t(1) << 32) &&
                      aligned16(value) && aligned16(loc) && aligned16(attn) && aligned16(out);
  // gather batching: SB samples' corner loads issued together (GD_MSDA_FWD_SB
  // 4, 8, or 40 / 80 = 4 / 8 with the next batch in flight while one is
  // consumed).  Measured at 800x1333 bs=2 (tools/msda_microbench.py
  // --fwd-variants): bf16 encoder 99 / 91 / 96 / 85 us
  // (round 1: 128 us), fp32 120 / 120 / 127 / 138 us.
  const int sb = env_int("GD_MSDA_FWD_SB", dt == GD_BF16 ? 80 : 4);
  if (dt == GD_F32 && vec_ok) {
    constexpr int UPW = 64 / (32 / 4);
    const int blocks = int((units + 4 * UPW - 1) / (4 * UPW));
#define GD_FWD_LAUNCH(T, SB)                                                                               \
  hipLaunchKernelGGL((msda_fwd_vec<T, 32, 4, 4, (SB >= 10 ? SB / 10 : SB), (SB >= 10)>), dim3(blocks), dim3(256), 0, s, (const T*)value, shapes, \
                     lsi, (const float*)loc, (const float*)attn, (T*)out, S, Lq, M, int(units))
    if (sb == 8) GD_FWD_LAUNCH(float, 8); else if (sb == 40) GD_FWD_LAUNCH(float, 40);
    else if (sb == 80) GD_FWD_LAUNCH(float, 80); else GD_FWD_LAUNCH(float, 4);
    GD_LAUNCH_CHECK("msda_fwd_vec<f32>");
  } else if (dt == GD_BF16 && vec_ok && env_int("GD_MSDA_FWD_GS", 1) == 1) {
    // geometry shared across the unit's quad + packed fp32 math (round 5);
    // GD_MSDA_FWD_GS=0: msda_fwd_vec (A/B)
    const int blocks = int((units + 63) / 64);
    hipLaunchKernelGGL(msda_fwd_gs, dim3(blocks), dim3(256), 0, s, (const uint16_t*)value, shapes, lsi,
                       (const float*)loc, (const float*)attn, (uint16_t*)out, S, Lq, M, int(units));
    GD_LAUNCH_CHECK("msda_fwd_gs");
  } else if (dt == GD_BF16 && vec_ok) {
    constexpr int UPW = 64 / (32 / 8);
    const int blocks = int((units + 4 * UPW - 1) / (4 * UPW));
    if (sb == 8) GD_FWD_LAUNCH(uint16_t, 8); else if (sb == 40) GD_FWD_LAUNCH(uint16_t, 40);
    else if (sb == 80) GD_FWD_LAUNCH(uint16_t, 80); else GD_FWD_LAUNCH(uint16_t, 4);
#undef GD_FWD_LAUNCH
    GD_LAUNCH_CHECK("msda_fwd_vec<bf16>");
  } else if (dt == GD_F32) {
    hipLaunchKernelGGL((msda_fwd_generic<float, float>), dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const float*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (float*)out, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_fwd_generic<f32>");
  } else if (dt == GD_BF16) {
    hipLaunchKernelGGL((msda_fwd_generic<uint16_t, float>), dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const uint16_t*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (uint16_t*)out, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_fwd_generic<bf16>");
  } else {
    hipLaunchKernelGGL((msda_fwd_generic<double, double>), dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const double*)value, shapes, lsi, (const double*)loc, (const double*)attn,
        (double*)out, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_fwd_generic<f64>");
  }
  return GD_OK;
}

extern "C" gd_status gd_msda_backward_geom(gd_dtype dt, const void* value,
                                           const int64_t* shapes, const int64_t* lsi,
                                           const void* loc, const void* attn,
                                           const void* grad_out, int N, int S, int M, int D,
                                           int L, int Lq, int P, void* grad_value,
                                           void* grad_loc, void* grad_attn,
                                           const int64_t* shapes_host, gd_stream_t stream) {
  gd_status st0 = check_common(dt, N, S, M, D, L, Lq, P);
  if (st0 != GD_OK) return st0;
  hipStream_t s = as_hip(stream);
  const size_t acc = dt == GD_F64 ? 8 : 4;
  const int64_t units = int64_t(N) * Lq * M;
  const size_t nval = size_t(N) * S * M * D;
  if (nval) {
    GD_REQUIRE(grad_value && value, "msda_backward: null value / grad_value");
    GD_HIP_CHECK(fill_u32_async(grad_value, 0u, nval * acc, s));
  }
  if (units == 0) return GD_OK;
  GD_REQUIRE(grad_out && loc && attn && grad_loc && grad_attn && shapes && lsi,
             "msda_backward: null pointer");
  const int64_t total = units * D;
  const bool lane_ok = D == 32 && L == 4 && P == 4 && units < (int64_t(1) << 31) &&
                       aligned16(loc) && aligned16(grad_loc) && aligned16(attn);
  // Self-attention (Lq == S: every value position is also a query, ordered as
  // the value rows, so consecutive queries sample neighbouring rows): tiled
  // backward with LDS pre-aggregation.  Cross-attention (the decoder's 900
  // score-sorted queries) keeps the direct-atomic kernel.
  const BwdVariant variant = bwd_variant();
  if ((dt == GD_F32 || dt == GD_BF16) && lane_ok && Lq == S && M == 8 && variant == BwdVariant::kEnc && shapes_host &&
      aligned16(value) && aligned16(grad_out) && aligned16(attn) && aligned16(grad_attn)) {
    EncTiles tl{};
    int th[4], tw[4], cap[4];
    enc_geometry(th, tw, cap);
    int64_t cover = 0, nt = 0;
    int rows = 0;
    bool ok = true;
    for (int l = 0; l < L; ++l) {
      const int64_t h = shapes_host[2 * l], w = shapes_host[2 * l + 1];
      ok = ok && h > 0 && w > 0;
      cover += h * w;
      tl.th[l] = th[l];
      tl.tw[l] = tw[l];
      tl.tx[l] = int((w + tw[l] - 1) / tw[l]);
      tl.tstart[l] = int(nt);
      nt += ((h + th[l] - 1) / th[l]) * tl.tx[l];
      tl.rbase[l] = rows;
      tl.rcap[l] = cap[l];
      rows += cap[l] + 1;  // + the region's spare row
    }
    tl.tstart[4] = int(nt);
    const int64_t blocks = int64_t(N) * nt * M;
    // the kernel's 32-bit byte offsets into value (msda_enc.inc) need
    // N*S*M*D*sizeof(T) < 2^32, as the forward checks
    const size_t vbytes = size_t(N) * S * M * D * (dt == GD_BF16 ? 2 : 4);
    if (ok && cover == S && blocks < (int64_t(1) << 31) && rows <= 1024 && vbytes < (size_t(1) << 32)) {
      const int rmax = env_int("GD_MSDA_ENC_RMAX", 8);
      const int mode = env_int("GD_MSDA_ENC_MODE", 0);  // 1: ds_add_f32 instead of read-modify-write
      // gathers of 1 unit in flight (default, measured 0.84 ms) or 2
      // (GD_MSDA_ENC_DEPTH=2: 152 VGPR, 3 waves/SIMD; A/B in
      // tools/msda_microbench.py --enc-probes)
      const bool deep = env_int("GD_MSDA_ENC_DEPTH", 1) >= 2;
#define GD_ENC_LAUNCH1(T, NR, DP)                                                                          \
  hipLaunchKernelGGL((msda_bwd_enc<T, NR, DP>), dim3(int(blocks)), dim3(128), 0, s, (const T*)value, shapes, \
                     lsi, (const float*)loc, (const float*)attn, (const T*)grad_out, (float*)grad_value,       \
                     (float*)grad_loc, (float*)grad_attn, S, M, tl, rmax, mode)
#define GD_ENC_LAUNCH(T, NR)                                             \
  do {                                                                   \
    if (deep) GD_ENC_LAUNCH1(T, NR, true); else GD_ENC_LAUNCH1(T, NR, false); \
  } while (0)
#define GD_ENC_LAUNCH_ROWS(T)                  \
  if (rows <= 160) GD_ENC_LAUNCH(T, 160);      \
  else if (rows <= 224) GD_ENC_LAUNCH(T, 224); \
  else if (rows <= 288) GD_ENC_LAUNCH(T, 288); \
  else if (rows <= 352) GD_ENC_LAUNCH(T, 352); \
  else if (rows <= 512) GD_ENC_LAUNCH(T, 512); \
  else GD_ENC_LAUNCH(T, 1024)
      if (dt == GD_F32) {
        GD_ENC_LAUNCH_ROWS(float);
        GD_LAUNCH_CHECK("msda_bwd_enc<f32>");
      } else {
        GD_ENC_LAUNCH_ROWS(uint16_t);
        GD_LAUNCH_CHECK("msda_bwd_enc<bf16>");
      }
#undef GD_ENC_LAUNCH_ROWS
#undef GD_ENC_LAUNCH
#undef GD_ENC_LAUNCH1
      return GD_OK;
    }
  }
  if ((dt == GD_F32 || dt == GD_BF16) && lane_ok && Lq == S && variant == BwdVariant::kTiled) {
    // 2-D pixel tiles when the host knows the level grid (and it covers the
    // S queries exactly); otherwise strips of kTileQ consecutive queries
    int tiles_per_n = (Lq + kTileQ - 1) / kTileQ, tiles2d = 0;
    if (shapes_host) {
      int64_t cover = 0, nt = 0;
      bool ok = true;
      for (int l = 0; l < L; ++l) {
        const int64_t h = shapes_host[2 * l], w = shapes_host[2 * l + 1];
        ok = ok && h > 0 && w > 0;
        cover += h * w;
        nt += ((h + 3) / 4) * ((w + 7) / 8);
      }
      if (ok && cover == S && nt < (int64_t(1) << 30)) {
        tiles_per_n = int(nt);
        tiles2d = 1;
      }
    }
    const int64_t blocks = int64_t(N) * tiles_per_n * M;
    GD_REQUIRE(blocks < (int64_t(1) << 31), "msda_backward: grid too large");
    if (dt == GD_F32) {
      hipLaunchKernelGGL((msda_bwd_tiled<float, kTileQ, kTileRows>), dim3(int(blocks)), dim3(256), 0, s,
                     (const float*)value, shapes, lsi, (const float*)loc, (const float*)attn,
          (const float*)grad_out, (float*)grad_value, (float*)grad_loc, (float*)grad_attn,
          S, Lq, M, tiles_per_n, tiles2d);
      GD_LAUNCH_CHECK("msda_bwd_tiled<f32>");
    } else {
      hipLaunchKernelGGL((msda_bwd_tiled<uint16_t, kTileQ, kTileRows>), dim3(int(blocks)), dim3(256), 0, s,
                     (const uint16_t*)value, shapes, lsi, (const float*)loc, (const float*)attn,
          (const uint16_t*)grad_out, (float*)grad_value, (float*)grad_loc, (float*)grad_attn,
          S, Lq, M, tiles_per_n, tiles2d);
      GD_LAUNCH_CHECK("msda_bwd_tiled<bf16>");
    }
    return GD_OK;
  }
  if ((dt == GD_F32 || dt == GD_BF16) && lane_ok) {
    const int blocks = int((units + 7) / 8);  // 4 waves x 2 units
    if (dt == GD_F32) {
      hipLaunchKernelGGL((msda_bwd_lane32<float, 4, 4>), dim3(blocks), dim3(256), 0, s,
                     (const float*)value, shapes, lsi, (const float*)loc, (const float*)attn,
          (const float*)grad_out, (float*)grad_value, (float*)grad_loc,
          (float*)grad_attn, S, Lq, M, int(units));
      GD_LAUNCH_CHECK("msda_bwd_lane32<f32>");
    } else {
      hipLaunchKernelGGL((msda_bwd_lane32<uint16_t, 4, 4>), dim3(blocks), dim3(256), 0, s,
                     (const uint16_t*)value, shapes, lsi, (const float*)loc, (const float*)attn,
          (const uint16_t*)grad_out, (float*)grad_value, (float*)grad_loc,
          (float*)grad_attn, S, Lq, M, int(units));
      GD_LAUNCH_CHECK("msda_bwd_lane32<bf16>");
    }
    return GD_OK;
  }
  const size_t nloc = size_t(units) * L * P;
  GD_HIP_CHECK(fill_u32_async(grad_loc, 0u, nloc * 2 * acc, s));
  GD_HIP_CHECK(fill_u32_async(grad_attn, 0u, nloc * acc, s));
  if (dt == GD_F32) {
    hipLaunchKernelGGL((msda_bwd_generic<float, float>), dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const float*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (const float*)grad_out, (float*)grad_value, (float*)grad_loc, (float*)grad_attn,
        S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_bwd_generic<f32>");
  } else if (dt == GD_BF16) {
    hipLaunchKernelGGL((msda_bwd_generic<uint16_t, float>), dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const uint16_t*)value, shapes, lsi, (const float*)loc, (const float*)attn,
        (const uint16_t*)grad_out, (float*)grad_value, (float*)grad_loc,
        (float*)grad_attn, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_bwd_generic<bf16>");
  } else {
    hipLaunchKernelGGL((msda_bwd_generic<double, double>), dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const double*)value, shapes, lsi, (const double*)loc, (const double*)attn,
        (const double*)grad_out, (double*)grad_value, (double*)grad_loc,
        (double*)grad_attn, S, Lq, M, D, L, P, total);
    GD_LAUNCH_CHECK("msda_bwd_generic<f64>");
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
  return gd_msda_backward_geom(dt, value, shapes, lsi, loc, attn, grad_out, N, S, M, D, L, Lq, P,
                               grad_value, grad_loc, grad_attn, nullptr, stream);
}

// ---------------------------------------------------------------------------
// Sorted backward (msda_sorted.inc): plan, workspace, launches
// ---------------------------------------------------------------------------
namespace gd {
namespace {

struct SortedPlan {
  SortGeo G;
  SweepGeo W;
  int ncells = 0, nsamples = 0, nb = 0, k1_blocks = 0;
  size_t o_sweep = 0;  // K4 sweep: partial rows of the chunked levels
  size_t o_cnt = 0, o_off = 0, o_cur = 0, o_bsum = 0, o_ids = 0, o_part = 0, o_scr = 0, o_stat = 0, bytes = 0;
};

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// false: the sorted backward does not apply (the caller uses another kernel)
bool plan_sorted(gd_dtype dt, int N, int S, int M, int D, int L, int Lq, int P, const int64_t* hs, int flags,
                 SortedPlan& pl) {
  if (!((dt == GD_F32 || dt == GD_BF16) && D == 32 && L == 4 && P == 4 && hs && N > 0 && M > 0 && Lq >= 0))
    return false;
  SortGeo& G = pl.G;
  int64_t cover = 0, cpn = 0;
  for (int l = 0; l < 4; ++l) {
    const int64_t h = hs[2 * l], w = hs[2 * l + 1];
    if (h <= 0 || w <= 0 || h > (1 << 20) || w > (1 << 20)) return false;
    G.H[l] = int(h);
    G.W[l] = int(w);
    G.lsi[l] = int(cover);
    G.cofs[l] = int(cpn);
    cover += h * w;
    cpn += (h + 1) * (w + 1);
  }
  if (cover != S) return false;
  const int64_t units = int64_t(N) * Lq * M;
  const int64_t ncells = int64_t(N) * M * cpn;
  const size_t vbytes = size_t(N) * S * M * D * (dt == GD_BF16 ? 2 : 4);
  if (units * 16 >= (int64_t(1) << 31) || ncells + 1 >= (int64_t(1) << 31) || vbytes >= (size_t(1) << 32))
    return false;
  G.cpn = int(cpn);
  G.N = N;
  // K4a splits: ~16 samples per lane group (a level-l cell holds about
  // Lq * P / (H W) samples of each (n, m))
  const int lpu = dt == GD_BF16 ? 4 : 8, upb = 4 * (64 / lpu);  // K1 units per block
  const int gpb = 256 / lpu, maxF = 64 / lpu;
  int64_t bl = 0;
  for (int l = 0; l < 4; ++l) {
    const double e = double(Lq) * P / (double(G.H[l]) * G.W[l]);
    int F = 1;
    while (F < maxF && e / F > 16.0) F *= 2;
    if (const char* ev = getenv("GD_MSDA_SORTED_F")) {  // A/B: fixed split for every level
      const int f = atoi(ev);
      if (f >= 1 && f <= maxF && (f & (f - 1)) == 0) F = f;
    }
    G.F[l] = F;
    G.cstart[l] = int(bl);
    bl += (int64_t(N) * M * (G.H[l] + 1) * (G.W[l] + 1) * F + gpb - 1) / gpb;
  }
  if (bl >= (int64_t(1) << 31)) return false;
  G.cstart[4] = int(bl);
  if (int64_t(N) * M * S >= (int64_t(1) << 31)) return false;  // K4 item index
  pl.ncells = int(ncells);
  pl.nsamples = int(units * 16);
  pl.nb = int((ncells + kScanBlock - 1) / kScanBlock);
  if (pl.nb > 256 * kScanPer) return false;
  pl.k1_blocks = int((units + upb - 1) / upb);
  size_t o = 0;
  pl.o_cnt = o; o = align_up(o + sizeof(int) * size_t(ncells + 2));    // cell counts + 2 run statistics
  pl.o_off = o; o = align_up(o + sizeof(int) * size_t(ncells + 1));    // segment offsets
  pl.o_bsum = o; o = align_up(o + sizeof(int) * size_t(pl.nb));
  pl.o_cur = o; o = align_up(o + sizeof(int) * size_t(ncells));        // segment cursors (K1)
  pl.o_ids = o; o = align_up(o + 16 * size_t(pl.nsamples));            // sample records by cell
  // K4 sweep geometry (msda_sorted.inc): a wave = GPW - 1 pixel columns x R
  // rows of one (n, m, level) [x Gs record chunks].  lam = samples per cell
  // of one (n, m) on level l; chunks keep <= 32 records per cell and wave,
  // rows ~128 records per lane group and task.
  {
    SweepGeo& W = pl.W;
    const int gpw = 64 / lpu;
    int64_t tasks = 0, items = 0, pfl = 0;
    for (int l = 0; l < 4; ++l) {
      const int H = G.H[l], Wd = G.W[l];
      const double lam = double(Lq) * P / (double(H) * Wd);
      int Gs = 1;
      while (Gs < 64 && lam / Gs > 32.0) Gs *= 2;
      const double per = std::max(lam / Gs, 1.0);
      // ~128 records per lane group and task; levels with < 2 samples per
      // cell (the decoder's 900 queries on the fine levels) walk mostly empty
      // cells -- a chain of dependent offset loads per row -- so their tasks
      // stop at 8 rows (measured: decoder 203 -> 117 us; the encoder's level 0
      // keeps 24 rows: 373 us there vs 410 us at 8)
      const int rmax = lam < 2.0 ? 8 : H;
      const int R = int(std::min<double>(std::min(H, rmax), std::max(2.0, std::floor(128.0 / per))));
      W.Gs[l] = Gs;
      W.R[l] = R;
      W.bands[l] = (Wd + gpw - 2) / (gpw - 1);
      W.rblk[l] = (H + R - 1) / R;
      W.tstart[l] = int(tasks);
      tasks += int64_t(W.bands[l]) * W.rblk[l] * Gs;  // per (n, m)
      W.cstart[l] = int(items);
      W.pbase[l] = pfl;
      if (Gs > 1) {
        items += int64_t(N) * M * H * Wd;
        pfl += int64_t(N) * M * H * Wd * Gs * D;
      }
    }
    W.tstart[4] = int(tasks);
    W.cstart[4] = int(items);
    if (tasks * N * M >= (int64_t(1) << 30) || items >= (int64_t(1) << 30)) return false;
    W.ntasks = int(tasks * N * M);
    W.hp = (M % 2 == 0 && env_int("GD_MSDA_SORTED_HP", 2) == 2) ? 2 : 1;
    pl.o_sweep = o;
    o = align_up(o + sizeof(float) * size_t(pfl));
  }
  pl.o_part = o;
  if (env_int("GD_MSDA_SORTED_K4", 0) == 1) o = align_up(o + sizeof(float) * 128 * size_t(ncells));  // cellsum
  pl.o_scr = o;
  if (flags & GD_MSDA_DETERMINISTIC) o = align_up(o + 16 * size_t(pl.nsamples));
  pl.bytes = o;
  return true;
}

}  // namespace
}  // namespace gd

extern "C" size_t gd_msda_backward_workspace_bytes(gd_dtype dt, int N, int S, int M, int D, int L, int Lq, int P,
                                                   const int64_t* shapes_host, int flags) {
  SortedPlan pl;
  return plan_sorted(dt, N, S, M, D, L, Lq, P, shapes_host, flags, pl) ? pl.bytes : 0;
}

extern "C" gd_status gd_msda_backward_sorted(gd_dtype dt, const void* value, const int64_t* shapes,
                                             const int64_t* lsi, const void* loc, const void* attn,
                                             const void* grad_out, int N, int S, int M, int D, int L, int Lq,
                                             int P, void* grad_value, gd_dtype gv_dt, void* grad_loc,
                                             void* grad_attn, const int64_t* shapes_host, void* ws,
                                             size_t ws_bytes, int flags, gd_stream_t stream) {
  gd_status st0 = check_common(dt, N, S, M, D, L, Lq, P);
  if (st0 != GD_OK) return st0;
  (void)shapes;
  (void)lsi;  // the level geometry comes from the host shapes (lsi = their cumulative sums)
  SortedPlan pl;
  if (!plan_sorted(dt, N, S, M, D, L, Lq, P, shapes_host, flags, pl)) {
    set_error("msda_backward_sorted: not applicable (value F32/BF16, D=32, L=P=4, host shapes tiling "
              "spatial_size, 32-bit offsets)");
    return GD_ERR_UNSUPPORTED;
  }
  GD_REQUIRE(gv_dt == GD_F32 || (gv_dt == GD_BF16 && dt == GD_BF16),
             "msda_backward_sorted: grad_value dtype %d (F32, or BF16 for a BF16 value)", int(gv_dt));
  GD_REQUIRE(ws && ws_bytes >= pl.bytes, "msda_backward_sorted: workspace of %zu bytes needed", pl.bytes);
  GD_REQUIRE(grad_value && (Lq == 0 || (value && loc && attn && grad_out && grad_loc && grad_attn)),
             "msda_backward_sorted: null pointer");
  GD_REQUIRE(aligned16(value) && aligned16(loc) && aligned16(attn) && aligned16(grad_out) && aligned16(grad_loc) &&
                 aligned16(grad_attn) && aligned16(grad_value),
             "msda_backward_sorted: operands must be 16-byte aligned");
  hipStream_t s = as_hip(stream);
  char* w = static_cast<char*>(ws);
  int* cnt = reinterpret_cast<int*>(w + pl.o_cnt);
  int* off = reinterpret_cast<int*>(w + pl.o_off);
  int* bsum = reinterpret_cast<int*>(w + pl.o_bsum);
  int* cur = reinterpret_cast<int*>(w + pl.o_cur);
  int4* ids = reinterpret_cast<int4*>(w + pl.o_ids);
  int4* scr = reinterpret_cast<int4*>(w + pl.o_scr);
  float* part = reinterpret_cast<float*>(w + pl.o_part);
  const int units = pl.nsamples / 16;
  GD_HIP_CHECK(fill_u32_async(cnt, 0u, sizeof(int) * size_t(pl.ncells + 2), s));
  int* stat = cnt + pl.ncells;  // coarse runs / coarse samples of the first count blocks
  if (units > 0) {
    // coarse-level counts through a per-workgroup LDS histogram when both
    // (n, m) slots of it fit (GD_MSDA_COUNT_PRIV=0: all global atomics, A/B)
    const int c23 = (pl.G.H[2] + 1) * (pl.G.W[2] + 1) + (pl.G.H[3] + 1) * (pl.G.W[3] + 1);
    const bool priv = Lq >= 64 && 2 * c23 <= kCountBins && env_int("GD_MSDA_COUNT_PRIV", 1) != 0;
    // 4 rounds of 64 units per workgroup when a workgroup's 256 units still
    // span at most two (n, m) (GD_MSDA_COUNT_R=1: one round, =8: eight
    // rounds when Lq >= 512 -- A/B)
    const int renv = env_int("GD_MSDA_COUNT_R", 4);
    const int rr = (renv == 8 && Lq >= 512) ? 8 : (renv >= 4 && Lq >= 256) ? 4 : 1;
    const dim3 cg((units + 64 * rr - 1) / (64 * rr));
#define GD_COUNT(PRIV, R)                                                                                      \
  hipLaunchKernelGGL((msda_bwd_count<PRIV, R>), cg, dim3(256), 0, s, (const float*)loc, cnt, stat, pl.G, Lq, M, \
                     units)
    if (priv) {
      if (rr == 8) GD_COUNT(true, 8);
      else if (rr == 4) GD_COUNT(true, 4);
      else GD_COUNT(true, 1);
    } else {
      if (rr == 8) GD_COUNT(false, 8);
      else if (rr == 4) GD_COUNT(false, 4);
      else GD_COUNT(false, 1);
    }
#undef GD_COUNT
    GD_LAUNCH_CHECK("msda_bwd_count");
  }
  hipLaunchKernelGGL(scan_block_sums, dim3(pl.nb), dim3(256), 0, s, (const int*)cnt, pl.ncells, bsum);
  hipLaunchKernelGGL(scan_finish, dim3(pl.nb), dim3(256), 0, s, (const int*)cnt, pl.ncells, (const int*)bsum, off,
                     cur);
  GD_LAUNCH_CHECK("msda_bwd scan");
  if (units > 0) {
    // K1 gathers one level at a time (default; fewer VGPRs: 169 vs 192 us at
    // the encoder's init geometry, 379 vs 397 us on a 2-px spread) or with
    // the next level in flight (GD_MSDA_SORTED_K1PIPE=1)
    const bool pipe = env_int("GD_MSDA_SORTED_K1PIPE", 0) != 0;
    // GD_MSDA_SORTED_K1=2: the level-by-level variant (103 VGPRs, 4 waves
    // per SIMD; measured 380 vs 367 us at the init geometry, 846 vs 884 on
    // a 2-px spread -- twice the waves in flight double its L2 misses)
    if (env_int("GD_MSDA_SORTED_K1", 1) == 2) {
      if (dt == GD_BF16)
        hipLaunchKernelGGL((msda_bwd_samples_lv<uint16_t>), dim3(pl.k1_blocks), dim3(256), 0, s,
                           (const uint16_t*)value, (const float*)loc, (const float*)attn, (const uint16_t*)grad_out,
                           (float*)grad_loc, (float*)grad_attn, cur, ids, pl.G, S, Lq, M, units);
      else
        hipLaunchKernelGGL((msda_bwd_samples_lv<float>), dim3(pl.k1_blocks), dim3(256), 0, s, (const float*)value,
                           (const float*)loc, (const float*)attn, (const float*)grad_out, (float*)grad_loc,
                           (float*)grad_attn, cur, ids, pl.G, S, Lq, M, units);
    } else {
#define GD_K1(T, P, HP, LL)                                                                                      \
  hipLaunchKernelGGL((msda_bwd_samples<T, P, HP, LL>), dim3(pl.k1_blocks), dim3(256), 0, s, (const T*)value,     \
                     (const float*)loc, (const float*)attn, (const T*)grad_out, (float*)grad_loc, (float*)grad_attn, \
                     cur, ids, pl.G, S, Lq, M, units, kpriv ? (const int*)stat : nullptr)
      // heads in pairs (M even; GD_MSDA_SORTED_HP=1: one head per wave, A/B)
      const bool hp = M % 2 == 0 && env_int("GD_MSDA_SORTED_HP", 2) == 2;
      // coarse-level slots through the LDS histogram (2 or 4 (n, m) slots)
      const int kc23 = (pl.G.H[2] + 1) * (pl.G.W[2] + 1) + (pl.G.H[3] + 1) * (pl.G.W[3] + 1);
      // (the per-sample pass decides on the device from the count pass's run
      // statistics; GD_MSDA_COUNT_PRIV=0 disables both histograms, =2
      // forces K1's regardless of run length -- A/B)
      const int kenv = env_int("GD_MSDA_COUNT_PRIV", 1);
      const int kpriv = (Lq >= 64 && (hp && !pipe ? 4 : 2) * kc23 <= kCountBins && kenv != 0) ? 1 : 0;
      if (kpriv && kenv == 2) GD_HIP_CHECK(fill_u32_async(stat, 0x10101010u, sizeof(int), s));  // runs >> samples
      // locations loaded level by level (default; 146 instead of 192 VGPRs:
      // 3 waves per SIMD): 345 -> 315 us at the init geometry, 510 -> 475 us
      // on a 2-px spread (profiles/r03g); GD_MSDA_SORTED_LL=0: all 48
      // location / weight floats held from the start
      const bool ll = env_int("GD_MSDA_SORTED_LL", 1) == 1;
      // bf16, heads in pairs: the geometry-shared kernel (round 5;
      // GD_MSDA_SORTED_GS=0: msda_bwd_samples<.., 2, true>, A/B)
      const bool gs = dt == GD_BF16 && hp && !pipe && ll && env_int("GD_MSDA_SORTED_GS", 1) == 1;
      if (gs) {
        hipLaunchKernelGGL(msda_bwd_samples_gs, dim3(pl.k1_blocks), dim3(256), 0, s, (const uint16_t*)value,
                           (const float*)loc, (const float*)attn, (const uint16_t*)grad_out, (float*)grad_loc,
                           (float*)grad_attn, cur, ids, pl.G, S, Lq, M, units, kpriv ? (const int*)stat : nullptr);
      } else if (dt == GD_BF16) {
        if (pipe) GD_K1(uint16_t, true, 1, false);
        else if (hp && ll) GD_K1(uint16_t, false, 2, true);
        else if (hp) GD_K1(uint16_t, false, 2, false);
        else GD_K1(uint16_t, false, 1, false);
      } else {
        if (pipe) GD_K1(float, true, 1, false);
        else if (hp && ll) GD_K1(float, false, 2, true);
        else if (hp) GD_K1(float, false, 2, false);
        else GD_K1(float, false, 1, false);
      }
#undef GD_K1
    }
    GD_LAUNCH_CHECK("msda_bwd_samples");
    if (flags & GD_MSDA_DETERMINISTIC) {
      int bits = 1;
      while (bits < 31 && (int64_t(1) << bits) < pl.nsamples) ++bits;
      hipLaunchKernelGGL(msda_bwd_sort_cells, dim3((pl.ncells + 3) / 4), dim3(256), 0, s, (const int*)off, ids, scr,
                         pl.ncells, bits);
      GD_LAUNCH_CHECK("msda_bwd_sort_cells");
    }
  }
  if (env_int("GD_MSDA_SORTED_K4", 0) != 1) {
    // K4 column sweep (+ chunk combine for the coarse levels)
    float* sw = reinterpret_cast<float*>(w + pl.o_sweep);
    const int sblocks = (pl.W.ntasks + 3) / 4;
    const int lpu = dt == GD_BF16 ? 4 : 8;
    const int cblocks = (pl.W.cstart[4] + 256 / lpu - 1) / (256 / lpu);
    // GD_MSDA_SWEEP_PF=1: next row's first records loaded during this row's
    // exchange (one dependent load less per row; 132 VGPRs)
    const bool pf = env_int("GD_MSDA_SWEEP_PF", 0) == 1;
#define GD_SW(T, TO)                                                                                          \
  do {                                                                                                        \
    if (sblocks > 0 && pf)                                                                                    \
      hipLaunchKernelGGL((msda_bwd_sweep<T, TO, true>), dim3(sblocks), dim3(256), 0, s, (const T*)grad_out,     \
                         (const int*)off, (const int4*)ids, (TO*)grad_value, sw, pl.G, pl.W, S, M);           \
    else if (sblocks > 0)                                                                                     \
      hipLaunchKernelGGL((msda_bwd_sweep<T, TO, false>), dim3(sblocks), dim3(256), 0, s, (const T*)grad_out,    \
                         (const int*)off, (const int4*)ids, (TO*)grad_value, sw, pl.G, pl.W, S, M);           \
    GD_LAUNCH_CHECK("msda_bwd_sweep");                                                                        \
    if (cblocks > 0)                                                                                          \
      hipLaunchKernelGGL((msda_bwd_sweep_combine<T, TO>), dim3(cblocks), dim3(256), 0, s, (const float*)sw,   \
                         (TO*)grad_value, pl.G, pl.W, S, M);                                                  \
    GD_LAUNCH_CHECK("msda_bwd_sweep_combine");                                                                \
  } while (0)
    if (dt == GD_BF16 && gv_dt == GD_BF16) GD_SW(uint16_t, uint16_t);
    else if (dt == GD_BF16) GD_SW(uint16_t, float);
    else GD_SW(float, float);
#undef GD_SW
    return GD_OK;
  }
  // GD_MSDA_SORTED_K4=1: the per-cell partial + per-pixel sum pair (A/B)
  if (dt == GD_BF16)
    hipLaunchKernelGGL((msda_bwd_cellsum<uint16_t>), dim3(pl.G.cstart[4]), dim3(256), 0, s,
                       (const uint16_t*)grad_out, (const int*)off, (const int4*)ids, part, pl.G, M);
  else
    hipLaunchKernelGGL((msda_bwd_cellsum<float>), dim3(pl.G.cstart[4]), dim3(256), 0, s, (const float*)grad_out,
                       (const int*)off, (const int4*)ids, part, pl.G, M);
  GD_LAUNCH_CHECK("msda_bwd_cellsum");
  const int items = N * M * S;
  const int lpu = dt == GD_BF16 ? 4 : 8;
  const int pblocks = (items + 256 / lpu - 1) / (256 / lpu);
#define GD_K4B(T, TO)                                                                                        \
  hipLaunchKernelGGL((msda_bwd_pixsum<T, TO>), dim3(pblocks), dim3(256), 0, s, (const int*)off,              \
                     (const float*)part, (TO*)grad_value, pl.G, S, M, items)
  if (dt == GD_BF16 && gv_dt == GD_BF16) GD_K4B(uint16_t, uint16_t);
  else if (dt == GD_BF16) GD_K4B(uint16_t, float);
  else GD_K4B(float, float);
#undef GD_K4B
  GD_LAUNCH_CHECK("msda_bwd_pixsum");
  return GD_OK;
}

extern "C" gd_status gd_device_status(gd_stream_t stream) {
  GD_HIP_CHECK(hipStreamSynchronize(as_hip(stream)));
  int v = 0;
  GD_HIP_CHECK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(gd::g_device_err), sizeof(int), 0, hipMemcpyDeviceToHost));
  if (v == 0) return GD_OK;
  const int zero = 0;
  GD_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(gd::g_device_err), &zero, sizeof(int), 0, hipMemcpyHostToDevice));
  gd::set_error("device-side check failed (bits 0x%x): %s", v,
            (v & gd::kErrMsdaSlot) ? "msda sorted backward: a record slot past the record buffer (stale or "
                                     "corrupt cell counts); the record was not stored" : "unknown check");
  return GD_ERR_DEVICE;
}
