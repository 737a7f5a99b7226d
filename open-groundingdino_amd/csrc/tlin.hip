// Token-linear forward GEMM for gfx950:  y[M, N] = x[M, K] . W[N, K]^T (+ b)
// (+ ReLU), bf16 operands, fp32 accumulation, bf16 output -- the forward of
// the encoder / fusion / Swin Linear layers (TokenLinear, gdino_amd/wgrad.py)
// over M = tens of thousands of tokens with K, N = 96..2048.
//
// Why a kernel of our own: on these tall-skinny shapes the library GEMM
// runs at 1.5-3.2 TB/s, 2.5-5x its HBM floor (tools/probes/gemm_shapes.py,
// profiles/r05m_gemm_shapes.jsonl: [44 446 x 256] x [256 x 384] 24 us for
// 7 us of bytes, Swin-T stage 0's K = 96 at 5.4x).  With K <= 2048 the whole
// reduction of a 128 x 128 output tile is a short loop, so the tile is
// memory-fed: W (<= 8 MB) stays in L2, x is streamed once per N tile.
//
// Tile 128 (tokens) x 128 (outputs), 256 threads = 4 waves of 64 x 64, each
// 4 x 4 v_mfma_f32_16x16x32_bf16 blocks.  K in chunks of 64: a chunk of x
// and of W is loaded with 16-B vector loads (8 lanes per 128-B row: whole
// cache lines) into registers, stored to an LDS stage (row pitch 72
// elements: 16 consecutive rows' 16-B fragment reads hit 64 distinct banks),
// and the next chunk's loads are in flight while this one is multiplied
// (two stages; deeper register prefetch and a transposed accumulator layout
// with 8-B epilogue writes were both measured slower).  Fragments are natural-order rows (mfma_frag.inc: lane
// (c, g) holds k = 8g..8g+7 of row c), no transposes: both operands are
// K-contiguous.  Epilogue: + bias, ReLU, bf16, staged through LDS so that
// each output row leaves as 16-B stores.  Rows >= M, outputs >= N and
// k >= K are zero-filled on load and masked on store (M, N, K multiples of
// nothing but 8 -- N and K for the 16-B vectors).
//
// Grid: one workgroup per tile, tiles ordered (m, n) with n fastest and
// remapped so that each XCD runs a contiguous range (the N tiles of an M
// block share the XCD's L2 copy of its x rows).
#include "gd_common.h"

namespace gd {
namespace {
#include "mfma_frag.inc"

constexpr int kTlM = 128, kTlN = 128, kTlK = 64;
constexpr int kTlPitch = kTlK + 8;                  // LDS row pitch (elements)
constexpr int kTlStage = (kTlM + kTlN) * kTlPitch;  // one stage: x rows, then W rows
constexpr int kTlOutPitch = kTlN + 8;               // epilogue staging pitch (bf16 elements)
static_assert(kTlM * kTlOutPitch <= 2 * kTlStage, "epilogue staging fits the stages");

__device__ __forceinline__ int tl_xcd_logical(int h, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = h % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + h / 8;
}

// the two bf16 halves of o where the matching half of m is > 0 (else +0):
// threshold_backward(o, m, 0) on a pair
__device__ __forceinline__ uint32_t tl_keep2(uint32_t o, uint32_t m) {
  const uint32_t lo = __uint_as_float(m << 16) > 0.f ? 0x0000ffffu : 0u;
  const uint32_t hi = __uint_as_float(m & 0xffff0000u) > 0.f ? 0xffff0000u : 0u;
  return o & (lo | hi);
}

// MASK: y = (x . w^T) where mask > 0, else 0 -- the input gradient of a
// Linear whose input was a ReLU output (mask), with the ReLU's backward folded
// into the store (applied after the bf16 rounding, as threshold_backward on
// the bf16 product would)
template <bool RELU, bool BIAS, bool MASK>
__global__ void __launch_bounds__(256)
tlin_fwd_kernel(const uint16_t* __restrict__ x, int64_t ldx, const uint16_t* __restrict__ w,
                const uint16_t* __restrict__ bias, int M, int K, int N, uint16_t* __restrict__ y, int64_t ldy,
                int tiles_n, const uint16_t* __restrict__ mask, int64_t ldm) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * kTlStage];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  const int L = tl_xcd_logical(int(blockIdx.x), int(gridDim.x));
  const int m0 = (L / tiles_n) * kTlM, n0 = (L % tiles_n) * kTlN;

  // loader: vector v = tid + 256 h (h < 4) of a [128 rows][8 x 16 B] chunk
  // (one chunk in registers: a second set -- 148 VGPRs -- measured slower)
  const int lpart = tid & 7, lrow = tid >> 3;  // rows lrow + 32 h
  uint4 rx[4], rw[4];
  auto load = [&](int k0) {
    const int k = k0 + 8 * lpart;
    const bool kok = k < K;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int r = lrow + 32 * h;
      const int mr = m0 + r, nr = n0 + r;
      rx[h] = (kok && mr < M) ? *reinterpret_cast<const uint4*>(x + int64_t(mr) * ldx + k) : make_uint4(0, 0, 0, 0);
      rw[h] = (kok && nr < N) ? *reinterpret_cast<const uint4*>(w + int64_t(nr) * K + k) : make_uint4(0, 0, 0, 0);
    }
  };
  auto stash = [&](int buf) {
    uint16_t* xs = lds + buf * kTlStage;
    uint16_t* ws = xs + kTlM * kTlPitch;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int r = lrow + 32 * h;
      *reinterpret_cast<uint4*>(xs + r * kTlPitch + 8 * lpart) = rx[h];
      *reinterpret_cast<uint4*>(ws + r * kTlPitch + 8 * lpart) = rw[h];
    }
  };

  // MASK: this thread's 8 mask vectors (the epilogue's store mapping) are
  // loaded up front, their latency hidden behind the K loop (the VGPRs are
  // free: LDS already limits the CU to two workgroups; loaded after the
  // loop they cost 70 us of the 165 at the encoder FFN shape)
  uint4 mreg[MASK ? 8 : 1];
  if (MASK) {
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      const int v = tid + 256 * h;
      const int mr = m0 + (v >> 4), col = n0 + 8 * (v & 15);
      mreg[h] = (mr < M && col < N) ? *reinterpret_cast<const uint4*>(mask + int64_t(mr) * ldm + col)
                                    : make_uint4(0, 0, 0, 0);
    }
  }

  gd_f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero4();

  const int nchunks = (K + kTlK - 1) / kTlK;
  load(0);
  for (int kc = 0, buf = 0; kc < nchunks; ++kc, buf ^= 1) {
    stash(buf);
    if (kc + 1 < nchunks) load((kc + 1) * kTlK);  // next chunk in flight during the MFMAs
    __syncthreads();
    const uint16_t* xs = lds + buf * kTlStage;
    const uint16_t* ws = xs + kTlM * kTlPitch;
#pragma unroll
    for (int s = 0; s < kTlK / 32; ++s) {
      WFrag<uint16_t> af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i].v = *reinterpret_cast<const gd_bf16x8*>(xs + (64 * wm + 16 * i + c) * kTlPitch + 32 * s + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bf[j].v = *reinterpret_cast<const gd_bf16x8*>(ws + (64 * wn + 16 * j + c) * kTlPitch + 32 * s + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = wmma(bf[j], af[i], acc[i][j]);
    }
  }

  // epilogue: the product is accumulated transposed (W rows as the MFMA's A
  // operand), acc[i][j][r] = y[m0 + 64 wm + 16 i + c][n0 + 64 wn + 16 j + 4 g + r]:
  // a lane's 4 values are consecutive outputs of one token, packed to one
  // 8-B ds_write (16 per lane instead of 64 2-B writes, whose bank conflicts
  // were 30 % of the LDS cycles at the encoder FFN shape; a 16-lane group
  // of one write covers 16 rows at dword offset 4c: conflict-free)
  __syncthreads();  // every wave's last fragment reads are done
  uint16_t* ot = lds;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 64 * wn + 16 * j + 4 * g;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (BIAS && n0 + col < N) {
      const uint2 b2 = *reinterpret_cast<const uint2*>(bias + n0 + col);
      bv[0] = __uint_as_float(b2.x << 16);
      bv[1] = __uint_as_float(b2.x & 0xffff0000u);
      bv[2] = __uint_as_float(b2.y << 16);
      bv[3] = __uint_as_float(b2.y & 0xffff0000u);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] + bv[r];
        if (RELU) v[r] = v[r] > 0.f ? v[r] : 0.f;
      }
      *reinterpret_cast<uint2*>(ot + (64 * wm + 16 * i + c) * kTlOutPitch + col) =
          make_uint2(uint32_t(f32_to_bf16(v[0])) | (uint32_t(f32_to_bf16(v[1])) << 16),
                     uint32_t(f32_to_bf16(v[2])) | (uint32_t(f32_to_bf16(v[3])) << 16));
    }
  }
  __syncthreads();
  // 128 rows x 16 vectors of 8 outputs; 16 lanes per row
#pragma unroll
  for (int h = 0; h < 8; ++h) {
    const int v = tid + 256 * h;
    const int row = v >> 4, part = v & 15;
    const int mr = m0 + row, col = n0 + 8 * part;
    if (mr < M && col < N) {
      uint4 o = *reinterpret_cast<const uint4*>(ot + row * kTlOutPitch + 8 * part);
      if (MASK) {
        const uint4 mv = mreg[h];
        o.x = tl_keep2(o.x, mv.x);
        o.y = tl_keep2(o.y, mv.y);
        o.z = tl_keep2(o.z, mv.z);
        o.w = tl_keep2(o.w, mv.w);
      }
      *reinterpret_cast<uint4*>(y + int64_t(mr) * ldy + col) = o;
    }
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" gd_status gd_token_linear_forward(const void* x, int64_t ldx, const void* weight, const void* bias,
                                            int M, int K, int N, int relu, void* y, int64_t ldy,
                                            gd_stream_t stream) {
  GD_REQUIRE(M >= 0 && K > 0 && N > 0 && K % 8 == 0 && N % 8 == 0,
             "token_linear: M=%d K=%d N=%d (K, N multiples of 8)", M, K, N);
  if (M == 0) return GD_OK;
  GD_REQUIRE(x && weight && y, "token_linear: null pointer");
  GD_REQUIRE(!bias || (reinterpret_cast<uintptr_t>(bias) & 7) == 0, "token_linear: bias must be 8-byte aligned");
  GD_REQUIRE(aligned16(x) && aligned16(weight) && aligned16(y) && ldx % 8 == 0 && ldy % 8 == 0 && ldx >= K &&
                 ldy >= N,
             "token_linear: 16-byte aligned rows required (ldx=%lld ldy=%lld)", (long long)ldx, (long long)ldy);
  const int tiles_m = (M + kTlM - 1) / kTlM, tiles_n = (N + kTlN - 1) / kTlN;
  GD_REQUIRE(int64_t(tiles_m) * tiles_n < (int64_t(1) << 31), "token_linear: grid too large");
  const dim3 grid(unsigned(tiles_m * tiles_n));
  hipStream_t s = as_hip(stream);
  const uint16_t* xp = static_cast<const uint16_t*>(x);
  const uint16_t* wp = static_cast<const uint16_t*>(weight);
  const uint16_t* bp = static_cast<const uint16_t*>(bias);
  uint16_t* yp = static_cast<uint16_t*>(y);
  if (relu) {
    if (bias)
      hipLaunchKernelGGL((tlin_fwd_kernel<true, true, false>), grid, dim3(256), 0, s, xp, ldx, wp, bp, M, K, N, yp,
                         ldy, tiles_n, nullptr, 0);
    else
      hipLaunchKernelGGL((tlin_fwd_kernel<true, false, false>), grid, dim3(256), 0, s, xp, ldx, wp, bp, M, K, N, yp,
                         ldy, tiles_n, nullptr, 0);
  } else {
    if (bias)
      hipLaunchKernelGGL((tlin_fwd_kernel<false, true, false>), grid, dim3(256), 0, s, xp, ldx, wp, bp, M, K, N, yp,
                         ldy, tiles_n, nullptr, 0);
    else
      hipLaunchKernelGGL((tlin_fwd_kernel<false, false, false>), grid, dim3(256), 0, s, xp, ldx, wp, bp, M, K, N, yp,
                         ldy, tiles_n, nullptr, 0);
  }
  GD_LAUNCH_CHECK("token_linear_forward");
  return GD_OK;
}

extern "C" gd_status gd_token_linear_forward_masked(const void* x, int64_t ldx, const void* weight, int M, int K,
                                                   int N, const void* mask, int64_t ldm, void* y, int64_t ldy,
                                                   gd_stream_t stream) {
  GD_REQUIRE(M >= 0 && K > 0 && N > 0 && K % 8 == 0 && N % 8 == 0,
             "token_linear_masked: M=%d K=%d N=%d (K, N multiples of 8)", M, K, N);
  if (M == 0) return GD_OK;
  GD_REQUIRE(x && weight && mask && y, "token_linear_masked: null pointer");
  GD_REQUIRE(aligned16(x) && aligned16(weight) && aligned16(mask) && aligned16(y) && ldx % 8 == 0 && ldm % 8 == 0 &&
                 ldy % 8 == 0 && ldx >= K && ldm >= N && ldy >= N,
             "token_linear_masked: 16-byte aligned rows required (ldx=%lld ldm=%lld ldy=%lld)", (long long)ldx,
             (long long)ldm, (long long)ldy);
  const int tiles_m = (M + kTlM - 1) / kTlM, tiles_n = (N + kTlN - 1) / kTlN;
  GD_REQUIRE(int64_t(tiles_m) * tiles_n < (int64_t(1) << 31), "token_linear_masked: grid too large");
  hipLaunchKernelGGL((tlin_fwd_kernel<false, false, true>), dim3(unsigned(tiles_m * tiles_n)), dim3(256), 0,
                     as_hip(stream), static_cast<const uint16_t*>(x), ldx, static_cast<const uint16_t*>(weight),
                     nullptr, M, K, N, static_cast<uint16_t*>(y), ldy, tiles_n, static_cast<const uint16_t*>(mask),
                     ldm);
  GD_LAUNCH_CHECK("token_linear_forward_masked");
  return GD_OK;
}
