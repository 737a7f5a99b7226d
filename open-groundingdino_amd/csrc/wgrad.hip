// Weight / bias gradients of the token-heavy Linear layers for gfx950:
//   dW[o][i] = sum_t dY[t][o] X[t][i]     db[o] = sum_t dY[t][o]
// over T = 44 446 tokens (800x1333 encoder, bs=2) with small outputs
// (O, I = 128..1024).  The library GEMM the autograd path runs here tiles
// only the O x I output (a 256 x 256 weight is 16 tiles of 64 x 64: 16 of
// 256 CUs busy for 158 us, round-1 profile "MT64x64x256"), so this kernel
// splits the token (K) dimension instead: grid (I/64, O/64, splits), each
// workgroup reduces its token range for one 64 x 64 tile into an fp32
// partial, and wgrad_reduce sums the partials -- deterministic, and dW / db
// come out in fp32 (the fp32 master parameters' gradient dtype) with no bf16
// rounding of the product.
//
// MFMA: contraction over t, the ROW index of both operands, so each 32-token
// chunk of dY and X is staged transposed in LDS ([feature][token], a 16-B
// ds_read per fragment; mfma_frag.inc's stage_t pattern) and every wave
// computes a 32 x 32 quarter of the tile with 2 x 2 v_mfma_f32_16x16x32_bf16
// (fp32 inputs: eight v_mfma_f32_16x16x4_f32 each) per chunk.
#include "gd_common.h"

#include <cmath>
#include <cstdlib>

namespace gd {
namespace {
#include "mfma_frag.inc"

__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void st4(uint16_t* p, float4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(uint32_t(f32_to_bf16(v.x)) | (uint32_t(f32_to_bf16(v.y)) << 16),
                                            uint32_t(f32_to_bf16(v.z)) | (uint32_t(f32_to_bf16(v.w)) << 16));
}

template <typename T> __device__ __forceinline__ float to_float(T v);
template <> __device__ __forceinline__ float to_float<float>(float v) { return v; }

constexpr int kWgChunk = 32;             // tokens per staged chunk
constexpr int kWgRow = kWgChunk + 8;     // LDS row pitch (elements): 16-B aligned rows

template <typename T>
__device__ __forceinline__ WFrag<T> lds_row8(const T* p);
template <>
__device__ __forceinline__ WFrag<float> lds_row8<float>(const float* p) {
  WFrag<float> f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f.v[j] = p[j];
  return f;
}

// Stage rows [t0, t0+32) x features [f0, f0+64) of a row-major [T, ld]
// matrix into xt[64][kWgRow] (transposed), zero past T.  256 threads.
template <typename T>
__device__ __forceinline__ void stage_chunk(T* xt, const T* src, int64_t ld, int t0, int T_, int f0) {
  constexpr int VE = 16 / int(sizeof(T));  // elements per 16-B load
  constexpr int NV = 64 / VE;              // vectors per 64-feature row slice
  for (int i = threadIdx.x; i < kWgChunk * NV; i += 256) {
    const int tt = i / NV, f = (i % NV) * VE;
    const int t = t0 + tt;
    union {
      uint4 u;
      T e[VE];
    } buf;
    if (t < T_) {
      buf.u = *reinterpret_cast<const uint4*>(src + int64_t(t) * ld + f0 + f);
    } else {
      buf.u = make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int e = 0; e < VE; ++e) xt[(f + e) * kWgRow + tt] = buf.e[e];
  }
}

// grid (I/64, O/64, batch * splits); batch b reads dy + b*bsy, x + b*bsx
template <typename T>
__global__ void __launch_bounds__(256)
wgrad_kernel(const T* __restrict__ dy, int64_t ldy, int64_t bsy, const T* __restrict__ x, int64_t ldx, int64_t bsx,
             int T_, int O, int I, int splits, int tokens_per_split, float* __restrict__ part_w,
             float* __restrict__ part_b) {
  __shared__ __attribute__((aligned(16))) T ys[64 * kWgRow];  // dY^T chunk: [o][t]
  __shared__ __attribute__((aligned(16))) T xs[64 * kWgRow];  // X^T chunk:  [i][t]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int wo = wave >> 1, wi = wave & 1;  // the wave's 32 x 32 quarter
  const int i0 = blockIdx.x * 64, o0 = blockIdx.y * 64;
  const int bz = blockIdx.z / splits, split = blockIdx.z - bz * splits;
  dy += bz * bsy;
  x += bz * bsx;
  const int64_t part = int64_t(bz) * splits + split;  // partial slot
  const int tb = split * tokens_per_split;
  const int te = min(T_, tb + tokens_per_split);
  const bool do_bias = part_b != nullptr && blockIdx.x == 0;
  gd_f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = zero4();
  float bsum = 0.f;  // threads 0..63: column o0 + tid of dY

  for (int t0 = tb; t0 < te; t0 += kWgChunk) {
    __syncthreads();  // previous chunk consumed
    stage_chunk<T>(ys, dy, ldy, t0, te, o0);
    stage_chunk<T>(xs, x, ldx, t0, te, i0);
    __syncthreads();
    if (do_bias && threadIdx.x < 64) {
      const T* r = ys + threadIdx.x * kWgRow;
#pragma unroll 8
      for (int k = 0; k < kWgChunk; ++k) bsum += to_float(r[k]);
    }
    WFrag<T> af[2], bf[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) af[m] = lds_row8<T>(ys + (32 * wo + 16 * m + c) * kWgRow + 8 * g);
#pragma unroll
    for (int n = 0; n < 2; ++n) bf[n] = lds_row8<T>(xs + (32 * wi + 16 * n + c) * kWgRow + 8 * g);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) acc[m][n] = wmma(af[m], bf[n], acc[m][n]);
  }
  // partial tile: (o0 + 32wo + 16m + 4g + r, i0 + 32wi + 16n + c)
  float* pw = part_w + part * O * I;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + 32 * wo + 16 * m + 4 * g + r, i = i0 + 32 * wi + 16 * n + c;
        pw[int64_t(o) * I + i] = acc[m][n][r];
      }
  if (do_bias && threadIdx.x < 64) part_b[part * O + o0 + threadIdx.x] = bsum;
}

// ---------------------------------------------------------------------------
// bf16, any O, I multiple of 16: 128 x 128 output tile per workgroup (each
// wave a 64 x 64 quarter: 4 x 4 MFMA 16x16x32 tiles, 64 accumulators), token
// chunks of 32 staged ROW-major (16-B global loads, one ds_write_b128 each)
// into a double-buffered LDS image and read TRANSPOSED into the MFMA operand
// layout with ds_read_b64_tr_b16 (cdna_hip_programming.md T10): lane c of
// 16-lane group g gets tokens 8g..8g+3 (+4) of feature c -- the k-slots of
// the A (dY^T) and B (X) operands.  One barrier per chunk; the next chunk's
// global loads are in flight during the current chunk's MFMAs.
// LDS image of a [32 token][128 feature] chunk: 256-B rows, 16-B chunk ch of
// row r at chunk ch ^ swz(r): a half-wave's transposed read (rows 8g+q and
// 8g+8+q, one 32-B column pair) then covers 8 distinct pairs = all 64 banks,
// and 8 consecutive lanes' ds_write_b128 (one row, chunks 0-7) 32 banks.
constexpr int kTrChunk = 32;
constexpr int kTrTile = 128;

__device__ __forceinline__ int tr_elem(int r, int ch) {  // element offset of (row r, 16-B chunk ch)
  return r * kTrTile + ((ch ^ (2 * (r & 3) + 8 * ((r >> 3) & 1))) << 3);
}

typedef short gd_i16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ gd_i16x4 lds_tr16(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) gd_i16x4*)(p));
}

// operand fragment (8 tokens 8g..8g+7 of feature fbase + c) from an image
__device__ __forceinline__ WFrag<uint16_t> tr_frag(const uint16_t* img, int fbase, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ch = (fbase >> 3) + (p >> 1), sub = 4 * (p & 1);
  const gd_i16x4 lo = lds_tr16(img + tr_elem(8 * g + q, ch) + sub);
  const gd_i16x4 hi = lds_tr16(img + tr_elem(8 * g + 4 + q, ch) + sub);
  WFrag<uint16_t> f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint16_t l16 = uint16_t(lo[j]), h16 = uint16_t(hi[j]);
    f.v[j] = __builtin_bit_cast(__bf16, l16);
    f.v[4 + j] = __builtin_bit_cast(__bf16, h16);
  }
  return f;
}

// grid (ceil(I/128), ceil(O/128), batch * splits); batch b reads dy + b*bsy, x + b*bsx.
// CH tokens per staged chunk (32 or 64): a 64-token chunk is two 32-row
// images per operand (the swizzle depends on r & 3 and (r >> 3) & 1 only, so
// rows 32..63 continue the same pattern), 4 x 16 B of each operand in flight
// per thread instead of 2 and half the barriers per token.
//
// The grid is 1-D: workgroup h is logical tile L = xcd_remap ? remap(h) : h,
// L = ((batch * splits + split) * gy + tile_o) * gx + tile_i.  The hardware
// deals consecutive workgroups round-robin over the 8 XCDs (each with its own
// L2), so with L = h every split's output tiles -- which all read the same
// token rows of X (and of dY across tile_i) -- land on 8 different L2s and
// each fetches those rows again from the fabric.  remap(h) gives XCD h % 8 a
// contiguous range of L (bijective for any count: cdna_hip_programming.md
// §5, "XCD swizzle must be bijective"), so a split's tiles share one L2.
__device__ __forceinline__ int xcd_logical(int h, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = h % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + h / 8;
}

template <bool BIAS, int CH>
__global__ void __launch_bounds__(256)
wgrad_tr_kernel(const uint16_t* __restrict__ dy, int64_t ldy, int64_t bsy, const uint16_t* __restrict__ x,
                int64_t ldx, int64_t bsx, int T_, int O, int I, int splits, int tokens_per_split,
                float* __restrict__ part_w, float* __restrict__ part_b, int gx, int gy, int xcd_remap) {
  static_assert(CH == 32 || CH == 64, "chunk of 32 or 64 tokens");
  constexpr int NH = CH / 16;  // 16-B vectors per thread per operand per chunk
  __shared__ __attribute__((aligned(16))) uint16_t ys[2][CH * kTrTile];
  __shared__ __attribute__((aligned(16))) uint16_t xs[2][CH * kTrTile];
  __shared__ float bsum_s[BIAS ? 16 : 1][kTrTile];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int wo = wave >> 1, wi = wave & 1;  // the wave's 64 x 64 quarter
  const int h = blockIdx.x;
  const int L = xcd_remap ? xcd_logical(h, int(gridDim.x)) : h;
  const int tile_i = L % gx, tile_o = (L / gx) % gy, zz = L / (gx * gy);
  const int i0 = tile_i * kTrTile, o0 = tile_o * kTrTile;
  const int bz = zz / splits, split = zz - bz * splits;
  dy += bz * bsy;
  x += bz * bsx;
  const int64_t part = int64_t(bz) * splits + split;
  const int tb = split * tokens_per_split;
  const int te = min(T_, tb + tokens_per_split);
  const bool do_bias = BIAS && tile_i == 0;

  // loader: vectors tid + 256 h of the chunk's CH rows x 16 chunks
  const int lrow = tid >> 4, lch = tid & 15;
  const bool yok = o0 + 8 * lch < O, xok = i0 + 8 * lch < I;
  const uint16_t* yp = dy + o0 + 8 * lch;
  const uint16_t* xp = x + i0 + 8 * lch;
  uint4 ry[NH], rx[NH];
  auto load = [&](int t0) {
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int t = t0 + lrow + 16 * h;
      const bool in = t < te;
      ry[h] = (in && yok) ? *reinterpret_cast<const uint4*>(yp + int64_t(t) * ldy) : make_uint4(0u, 0u, 0u, 0u);
      rx[h] = (in && xok) ? *reinterpret_cast<const uint4*>(xp + int64_t(t) * ldx) : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  float bacc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bacc[e] = 0.f;

  gd_f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = zero4();

  if (tb < te) load(tb);
  int buf = 0;
  for (int t0 = tb; t0 < te; t0 += CH, buf ^= 1) {
    uint16_t* yb = ys[buf];
    uint16_t* xb = xs[buf];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      *reinterpret_cast<uint4*>(yb + tr_elem(lrow + 16 * h, lch)) = ry[h];
      *reinterpret_cast<uint4*>(xb + tr_elem(lrow + 16 * h, lch)) = rx[h];
    }
    if (do_bias) {
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        bacc[0] += bf16_lo(ry[h].x); bacc[1] += bf16_hi(ry[h].x);
        bacc[2] += bf16_lo(ry[h].y); bacc[3] += bf16_hi(ry[h].y);
        bacc[4] += bf16_lo(ry[h].z); bacc[5] += bf16_hi(ry[h].z);
        bacc[6] += bf16_lo(ry[h].w); bacc[7] += bf16_hi(ry[h].w);
      }
    }
    if (t0 + CH < te) load(t0 + CH);  // next chunk in flight during the MFMAs
    __syncthreads();  // image `buf` complete (and `buf ^ 1` consumed one iteration ago)
#pragma unroll
    for (int k = 0; k < CH / 32; ++k) {  // 32-token sub-images
      WFrag<uint16_t> af[4], bfr[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) af[m] = tr_frag(yb + k * kTrChunk * kTrTile, 64 * wo + 16 * m, lane);
#pragma unroll
      for (int n = 0; n < 4; ++n) bfr[n] = tr_frag(xb + k * kTrChunk * kTrTile, 64 * wi + 16 * n, lane);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = wmma(af[m], bfr[n], acc[m][n]);
    }
  }
  // partial tile: (o0 + 64wo + 16m + 4g + r, i0 + 64wi + 16n + c)
  float* pw = part_w + part * O * I;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = o0 + 64 * wo + 16 * m + 4 * g + r;
      if (o < O) {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int i = i0 + 64 * wi + 16 * n + c;
          if (i < I) pw[int64_t(o) * I + i] = acc[m][n][r];
        }
      }
    }
  if (do_bias) {
#pragma unroll
    for (int e = 0; e < 8; ++e) bsum_s[lrow][8 * lch + e] = bacc[e];
    __syncthreads();
    if (tid < kTrTile && o0 + tid < O) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) sum += bsum_s[k][tid];
      part_b[part * O + o0 + tid] = sum;
    }
  }
}

// ---------------------------------------------------------------------------
// The same tile and MFMA schedule, staged by LDS-DMA (global_load_lds_dwordx4)
// through a 4-slot ring: chunk k+3 is issued while chunk k is computed, so
// three chunks (48 KB per workgroup) are in flight instead of one held in
// registers.  rocprofv3 counters on the register-staged kernel (enc FFN
// shape, 103 us): HBM bytes = the algorithmic 205 MB, LDS bank conflicts ~0,
// waves waiting on memory 45 % of their cycles -- one chunk in flight per
// workgroup does not cover the load latency.
// A DMA wave-instruction writes 64 lanes x 16 B contiguously: rows
// 8 wave + 4 j + lane / 16 of the [32][128] image, position lane % 16; the
// XOR swizzle of tr_elem goes on the SOURCE column (chunk p ^ swz(r)).
// Columns past O / I read column 0 of the tile instead (their products land
// only in accumulator rows / columns the epilogue does not store).  Only
// whole 32-token chunks go through the ring; a split's token tail is staged
// through registers with zero fill after the ring has drained.
// Sync: counted vmcnt + raw s_barrier (a __syncthreads() would wait vmcnt(0)
// and drain the ring; cdna_hip_programming.md §5, "Pipelining across
// barriers"); the DMA is gd_common.h's asm GD_LDS_DMA16, which hipcc does not
// track, so nothing else waits on it either.
constexpr int kGlStages = 4;
constexpr int kGlImg = kTrChunk * kTrTile;  // elements of one operand image (8 KB)
constexpr int kGlStage = 2 * kGlImg;        // dY image, then X image

__device__ __forceinline__ int tr_swz(int r) { return 2 * (r & 3) + 8 * ((r >> 3) & 1); }

template <bool BIAS>
__global__ void __launch_bounds__(256)
wgrad_glds_kernel(const uint16_t* __restrict__ dy, int64_t ldy, int64_t bsy, const uint16_t* __restrict__ x,
                  int64_t ldx, int64_t bsx, int T_, int O, int I, int splits, int tokens_per_split,
                  float* __restrict__ part_w, float* __restrict__ part_b, int gx, int gy, int xcd_remap) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kGlStages * kGlStage];  // the only LDS object
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int wo = wave >> 1, wi = wave & 1;  // the wave's 64 x 64 quarter
  const int h = blockIdx.x;
  const int L = xcd_remap ? xcd_logical(h, int(gridDim.x)) : h;
  const int tile_i = L % gx, tile_o = (L / gx) % gy, zz = L / (gx * gy);
  const int i0 = tile_i * kTrTile, o0 = tile_o * kTrTile;
  const int bz = zz / splits, split = zz - bz * splits;
  dy += bz * bsy;
  x += bz * bsx;
  const int64_t part = int64_t(bz) * splits + split;
  const int tb = split * tokens_per_split;
  const int te = min(T_, tb + tokens_per_split);
  const bool do_bias = BIAS && tile_i == 0;
  const int nfull = te > tb ? (te - tb) / kTrChunk : 0;
  const int tail = te > tb ? (te - tb) - nfull * kTrChunk : 0;

  // this lane's DMA sources: rows ra = 8 wave + lane / 16 and ra + 4 (same swizzle)
  const int ra = 8 * wave + (lane >> 4);
  const int pc = 8 * ((lane & 15) ^ tr_swz(ra));
  const int ycol = o0 + pc < O ? o0 + pc : o0;
  const int xcol = i0 + pc < I ? i0 + pc : i0;
  const uint16_t* ysrc = dy + int64_t(tb + ra) * ldy + ycol;
  const uint16_t* xsrc = x + int64_t(tb + ra) * ldx + xcol;
  uint16_t* const wdst = lds + 8 * wave * kTrTile;  // + slot * kGlStage (+ kGlImg for X)
  auto issue = [&](int k) {
    uint16_t* d = wdst + (k % kGlStages) * kGlStage;
    const int64_t ry = int64_t(k) * kTrChunk * ldy, rx = int64_t(k) * kTrChunk * ldx;
    GD_LDS_DMA16(ysrc + ry, d);
    GD_LDS_DMA16(ysrc + ry + 4 * ldy, d + 4 * kTrTile);
    GD_LDS_DMA16(xsrc + rx, d + kGlImg);
    GD_LDS_DMA16(xsrc + rx + 4 * ldx, d + kGlImg + 4 * kTrTile);
  };

  gd_f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = zero4();
  // db on the matrix cores: waves wi == 0 multiply their dY^T fragments by an
  // all-ones B operand (4 MFMAs per chunk instead of 64 VALU conversions and
  // adds, which made the bias workgroups the stragglers); every column of
  // accb[m] holds the row sums of rows 64 wo + 16 m + 4 g + r
  gd_f32x4 accb[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) accb[m] = zero4();
  WFrag<uint16_t> ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones.v[j] = __builtin_bit_cast(__bf16, uint16_t(0x3F80));

  auto compute = [&](int slot) {
    const uint16_t* yb = lds + slot * kGlStage;
    const uint16_t* xb = yb + kGlImg;
    WFrag<uint16_t> af[4], bfr[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) af[m] = tr_frag(yb, 64 * wo + 16 * m, lane);
#pragma unroll
    for (int n = 0; n < 4; ++n) bfr[n] = tr_frag(xb, 64 * wi + 16 * n, lane);
    if (do_bias && wi == 0) {
#pragma unroll
      for (int m = 0; m < 4; ++m) accb[m] = wmma(af[m], ones, accb[m]);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = wmma(af[m], bfr[n], acc[m][n]);
  };

  for (int k = 0; k < 3 && k < nfull; ++k) issue(k);
  for (int k = 0; k < nfull; ++k) {
    const int ahead = min(nfull - 1 - k, 2);  // chunks issued after k, still allowed in flight
    if (ahead == 2)
      gd_wait_vmcnt(8);
    else if (ahead == 1)
      gd_wait_vmcnt(4);
    else
      gd_wait_vmcnt(0);
    gd_raw_barrier();  // every wave's chunk-k DMA landed; every wave done with chunk k - 1
    if (k + 3 < nfull) issue(k + 3);  // slot (k + 3) % 4 held chunk k - 1
    compute(k % kGlStages);
  }
  if (tail > 0) {  // ring drained (vmcnt(0) at its last chunk); stage the tail through registers
    gd_wait_vmcnt(0);
    gd_raw_barrier();
    const int slot = nfull % kGlStages;
    uint16_t* yb = lds + slot * kGlStage;
    uint16_t* xb = yb + kGlImg;
    const int t0 = tb + nfull * kTrChunk;
    const int lrow = tid >> 4, lch = tid & 15;
    const bool yok = o0 + 8 * lch < O, xok = i0 + 8 * lch < I;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int t = t0 + lrow + 16 * hh;
      const bool in = t < te;
      const uint4 vy = (in && yok) ? *reinterpret_cast<const uint4*>(dy + int64_t(t) * ldy + o0 + 8 * lch)
                                   : make_uint4(0u, 0u, 0u, 0u);
      const uint4 vx = (in && xok) ? *reinterpret_cast<const uint4*>(x + int64_t(t) * ldx + i0 + 8 * lch)
                                   : make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(yb + tr_elem(lrow + 16 * hh, lch)) = vy;
      *reinterpret_cast<uint4*>(xb + tr_elem(lrow + 16 * hh, lch)) = vx;
    }
    __syncthreads();
    compute(slot);
  }
  // partial tile (o0 + 64wo + 16m + 4g + r, i0 + 64wi + 16n + c), through LDS
  // in two 64-row halves so that it leaves as 16-B row stores (512 B per
  // row) rather than 4-B stores in 64-B pieces: a 128 x 128 partial is 64 KB
  // per workgroup, written by every split.  Pitch 132 floats: the 16 lanes
  // c and 4 groups g of one ds_write hit 64 distinct banks.
  constexpr int kEpPitch = kTrTile + 4;
  float* ep = reinterpret_cast<float*>(lds);
  float* pw = part_w + part * O * I;
  gd_wait_vmcnt(0);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    __syncthreads();  // the ring's last reads / the previous half's row reads are done
    if (wo == half) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int n = 0; n < 4; ++n) ep[(16 * m + 4 * g + r) * kEpPitch + 64 * wi + 16 * n + c] = acc[m][n][r];
    }
    __syncthreads();
    for (int v = tid; v < 64 * (kTrTile / 4); v += 256) {
      const int rr = v / (kTrTile / 4), q = v % (kTrTile / 4);
      const int o = o0 + 64 * half + rr, i = i0 + 4 * q;
      if (o < O && i < I)
        *reinterpret_cast<float4*>(pw + int64_t(o) * I + i) = *reinterpret_cast<const float4*>(ep + rr * kEpPitch + 4 * q);
    }
  }
  if (do_bias && wi == 0 && c == 0) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + 64 * wo + 16 * m + 4 * g + r;
        if (o < O) part_b[part * O + o] = accb[m][r];
      }
  }
}

// out[b] = sum over splits of the partials, written in fp32 or bf16 with
// batch stride ob; db (batch 1) likewise.  A workgroup owns 32 float4
// column groups; its 8 thread groups each sum every 8th split (split k to
// group k % 8) and the 8 group sums are added in LDS in group order: a fixed
// order (deterministic) and 8x the threads of one thread per float4, whose
// 65-workgroup grid for a 256 x 256 weight left most CUs idle on the serial
// split loop (11 us for ~25 MB of L2 / MALL-resident partials).
constexpr int kRedCols = 32, kRedGroups = 8;

template <typename TO>
__global__ void __launch_bounds__(256)
wgrad_reduce_kernel(const float* __restrict__ part_w, const float* __restrict__ part_b, int splits, int batch,
                    int O, int I, TO* __restrict__ out, int64_t ob, float* __restrict__ db) {
  __shared__ float4 red[kRedGroups][kRedCols];
  const int col = threadIdx.x % kRedCols, grp = threadIdx.x / kRedCols;
  const int64_t t = int64_t(blockIdx.x) * kRedCols + col;
  const int64_t nw4 = int64_t(O) * I / 4;  // float4 groups per batch item
  const int64_t nb4 = db ? O / 4 : 0;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* src = nullptr;
  int64_t stride = 0;
  if (t < nw4 * batch) {
    const int64_t b = t / nw4, e = t - b * nw4;
    src = reinterpret_cast<const float4*>(part_w) + b * splits * nw4 + e;
    stride = nw4;
  } else if (t < nw4 * batch + nb4) {
    src = reinterpret_cast<const float4*>(part_b) + (t - nw4 * batch);
    stride = nb4;
  }
  if (src) {
    // four independent loads in flight per step (hipcc otherwise issued one
    // load and waited for it per split: 12 serial round trips at 96 splits);
    // the adds keep the split order, so the sums are unchanged bit for bit
    auto acc4 = [&](float4 v) {
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    };
    int k = grp;
    for (; k + 3 * kRedGroups < splits; k += 4 * kRedGroups) {
      const float4 v0 = src[int64_t(k) * stride];
      const float4 v1 = src[int64_t(k + kRedGroups) * stride];
      const float4 v2 = src[int64_t(k + 2 * kRedGroups) * stride];
      const float4 v3 = src[int64_t(k + 3 * kRedGroups) * stride];
      acc4(v0);
      acc4(v1);
      acc4(v2);
      acc4(v3);
    }
    for (; k < splits; k += kRedGroups) acc4(src[int64_t(k) * stride]);
  }
  red[grp][col] = s;
  __syncthreads();
  if (grp != 0 || !src) return;
#pragma unroll
  for (int g = 1; g < kRedGroups; ++g) {
    const float4 v = red[g][col];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  if (t < nw4 * batch) {
    const int64_t b = t / nw4, e = t - b * nw4;
    st4(out + b * ob + e * 4, s);
  } else {
    st4(db + (t - nw4 * batch) * 4, s);
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// A/B knobs, read once: GD_WGRAD_GLDS=0 (the register-staged kernel instead
// of the LDS-DMA ring), GD_WGRAD_CHUNK (its tokens per chunk, 32 | 64),
// GD_WGRAD_XCD=0 (no XCD remap), GD_WGRAD_WGS (the workgroup count the split
// choice aims for)
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}
int tr_chunk() {
  static const int v = env_int("GD_WGRAD_CHUNK", 32) == 64 ? 64 : 32;
  return v;
}
int xcd_remap() {
  static const int v = env_int("GD_WGRAD_XCD", 1) != 0;
  return v;
}
int target_wgs() {  // 0: the per-shape default
  static const int v = env_int("GD_WGRAD_WGS", 0) > 0 ? env_int("GD_WGRAD_WGS", 0) : 0;
  return v;
}

int glds_on() {
  static const int v = env_int("GD_WGRAD_GLDS", 1) != 0;
  return v;
}

template <bool BIAS>
void launch_tr(int gx, int gy, int gz, hipStream_t s, const uint16_t* dy, int64_t ldy, int64_t bsy, const uint16_t* x,
               int64_t ldx, int64_t bsx, int T, int O, int I, int splits, int tps, float* pw, float* pb) {
  const dim3 grid(unsigned(gx * gy * gz));
  const int remap = xcd_remap();
  if (glds_on())
    hipLaunchKernelGGL((wgrad_glds_kernel<BIAS>), grid, dim3(256), 0, s, dy, ldy, bsy, x, ldx, bsx, T, O, I, splits,
                       tps, pw, pb, gx, gy, remap);
  else if (tr_chunk() == 64)
    hipLaunchKernelGGL((wgrad_tr_kernel<BIAS, 64>), grid, dim3(256), 0, s, dy, ldy, bsy, x, ldx, bsx, T, O, I, splits,
                       tps, pw, pb, gx, gy, remap);
  else
    hipLaunchKernelGGL((wgrad_tr_kernel<BIAS, 32>), grid, dim3(256), 0, s, dy, ldy, bsy, x, ldx, bsx, T, O, I, splits,
                       tps, pw, pb, gx, gy, remap);
}

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" size_t gd_wgrad_workspace_bytes(int O, int I, int splits) {
  return sizeof(float) * (size_t(splits) * O * I + size_t(splits) * O);
}

extern "C" int gd_wgrad_splits_batched(int T, int O, int I, int batch) {
  // about 384 workgroups of 128 x 128 output tiles (1.5 per CU), at least
  // 128 tokens each: the fp32 partials (splits x O x I) stay a fraction of
  // the token-major inputs the kernel streams
  const int tiles = ((O + kTrTile - 1) / kTrTile) * ((I + kTrTile - 1) / kTrTile) * (batch > 0 ? batch : 1);
  // 256 workgroups (one per CU).  Round 4 picked 384 / 512 (512 for
  // FFN-sized weights) from kernels timed alone (profiles/r04c_wgrad_ab.jsonl:
  // enc FFN 88 -> 75 us); in the round-6 train step fewer splits -- less
  // fp32 partial traffic and reduce work next to the other kernels -- won:
  // 46.04 vs 45.76 images/s over three interleaved pairs and a separate run
  // (profiles/r06i_knobs.txt; GD_WGRAD_WGS=384 / 512 / 768 / 1024 / 192 for A/B)
  const int wgs = target_wgs() > 0 ? target_wgs() : 256;
  int s = tiles > 0 ? (wgs + tiles - 1) / tiles : 1;
  const int cap = T / 128 > 1 ? T / 128 : 1;
  return s < 1 ? 1 : (s > cap ? cap : s);
}

extern "C" int gd_wgrad_splits(int T, int O, int I) { return gd_wgrad_splits_batched(T, O, I, 1); }

extern "C" gd_status gd_wgrad_batched(gd_dtype dt, const void* grad_y, int64_t ldy, int64_t batch_stride_y,
                                      const void* x, int64_t ldx, int64_t batch_stride_x, int T, int O, int I,
                                      int batch, int splits, void* workspace, gd_dtype out_dtype, void* out,
                                      int64_t batch_stride_out, float* grad_b, gd_stream_t stream) {
  GD_REQUIRE(dt == GD_F32 || dt == GD_BF16, "wgrad: dtype %d not supported (F32, BF16)", int(dt));
  GD_REQUIRE(out_dtype == GD_F32 || out_dtype == GD_BF16, "wgrad: out dtype %d not supported", int(out_dtype));
  // bf16: O, I multiples of 16 (the 128 x 128 transposed-read kernel);
  // fp32: multiples of 64 (the 64 x 64 kernel)
  const int gran = dt == GD_BF16 ? 16 : 64;
  GD_REQUIRE(T >= 0 && O > 0 && I > 0 && O % gran == 0 && I % gran == 0 && splits >= 1 && batch >= 1 &&
                 int64_t(batch) * splits < 65536 && O / 64 < 65536,
             "wgrad: bad sizes T=%d O=%d I=%d (multiples of %d) batch=%d splits=%d", T, O, I, gran, batch, splits);
  GD_REQUIRE(!grad_b || batch == 1, "wgrad: bias gradient only for batch 1");
  GD_REQUIRE(grad_y && x && workspace && out, "wgrad: null pointer");
  const int64_t align = 16 / (dt == GD_BF16 ? 2 : 4);
  GD_REQUIRE(aligned16(grad_y) && aligned16(x) && ldy % align == 0 && ldx % align == 0 && ldy >= O && ldx >= I &&
                 batch_stride_y % align == 0 && batch_stride_x % align == 0,
             "wgrad: rows must be 16-byte aligned (ldy=%lld ldx=%lld)", (long long)ldy, (long long)ldx);
  GD_REQUIRE(aligned16(out) && aligned16(workspace) && batch_stride_out % 8 == 0 &&
                 (batch == 1 || batch_stride_out >= int64_t(O) * I),
             "wgrad: out / workspace must be 16-byte aligned, batch_stride_out >= O*I");
  hipStream_t s = as_hip(stream);
  float* part_w = static_cast<float*>(workspace);
  float* part_b = part_w + int64_t(batch) * splits * O * I;
  if (dt == GD_BF16) {
    const int ch = tr_chunk();
    const int tps = ((T + splits - 1) / splits + ch - 1) / ch * ch;
    const int gx = (I + kTrTile - 1) / kTrTile, gy = (O + kTrTile - 1) / kTrTile;
    GD_REQUIRE(int64_t(gx) * gy * batch * splits < (int64_t(1) << 31), "wgrad: grid too large");
    if (grad_b)
      launch_tr<true>(gx, gy, batch * splits, s, (const uint16_t*)grad_y, ldy, batch_stride_y, (const uint16_t*)x,
                      ldx, batch_stride_x, T, O, I, splits, tps, part_w, part_b);
    else
      launch_tr<false>(gx, gy, batch * splits, s, (const uint16_t*)grad_y, ldy, batch_stride_y, (const uint16_t*)x,
                       ldx, batch_stride_x, T, O, I, splits, tps, part_w, nullptr);
  } else {
    const int tps = ((T + splits - 1) / splits + kWgChunk - 1) / kWgChunk * kWgChunk;
    const dim3 grid(unsigned(I / 64), unsigned(O / 64), unsigned(batch * splits));
    hipLaunchKernelGGL((wgrad_kernel<float>), grid, dim3(256), 0, s, (const float*)grad_y, ldy, batch_stride_y,
                       (const float*)x, ldx, batch_stride_x, T, O, I, splits, tps, part_w,
                       grad_b ? part_b : nullptr);
  }
  GD_LAUNCH_CHECK("wgrad");
  const int64_t n = int64_t(O) * I / 4 * batch + (grad_b ? O / 4 : 0);  // float4 groups (O % 16 == 0)
  const dim3 rg(unsigned((n + kRedCols - 1) / kRedCols));
  if (out_dtype == GD_F32)
    hipLaunchKernelGGL((wgrad_reduce_kernel<float>), rg, dim3(256), 0, s, part_w, part_b, splits, batch, O, I,
                       (float*)out, batch_stride_out, grad_b);
  else
    hipLaunchKernelGGL((wgrad_reduce_kernel<uint16_t>), rg, dim3(256), 0, s, part_w, part_b, splits, batch, O, I,
                       (uint16_t*)out, batch_stride_out, grad_b);
  GD_LAUNCH_CHECK("wgrad_reduce");
  return GD_OK;
}

extern "C" gd_status gd_wgrad(gd_dtype dt, const void* grad_y, int64_t ldy, const void* x, int64_t ldx, int T,
                              int O, int I, int splits, void* workspace, float* grad_w, float* grad_b,
                              gd_stream_t stream) {
  return gd_wgrad_batched(dt, grad_y, ldy, 0, x, ldx, 0, T, O, I, 1, splits, workspace, GD_F32, grad_w,
                          int64_t(O) * I, grad_b, stream);
}
