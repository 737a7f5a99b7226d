/*
 * oracle/msda_ref.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (fp64, scalar C) of the reference's multi-scale deformable
 * attention, used as the parity checker for the HIP kernels.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product path never does.
 *
 * Follows, line for line in meaning (not in code):
 *   forward  : ms_deformable_im2col_gpu_kernel
 *              /root/reference/models/GroundingDINO/ops/src/cuda/ms_deform_im2col_cuda.cuh:238-299
 *              with ms_deform_attn_im2col_bilinear  (.cuh:34-84)
 *   backward : ms_deform_attn_col2im_bilinear       (.cuh:88-159)
 *              summed over channels as ..._shm_blocksize_aware_reduce_v1 (.cuh:302-403)
 * and the pure-PyTorch semantics ms_deform_attn_core_pytorch
 *   /root/reference/models/GroundingDINO/ops/functions/ms_deform_attn_func.py:41-61
 * (grid_sample, align_corners=False, zero padding).
 *
 * Pinned against golden vectors generated from that pure-PyTorch function
 * (tests/golden/make_golden.py); see tests/test_oracle.py.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* value[n][pos][m][c] at flat (pos, m, c) inside batch n */
static inline double vget(const double* v, int S, int M, int D, int n, int pos, int m, int c) {
  return v[(((size_t)n * S + pos) * M + m) * D + c];
}

typedef struct {
  int valid;
  int hl, wl, hh, wh;   /* corner coordinates */
  double w[4];          /* bilinear weights of corners (ll, lh, hl, hh) */
  double lh, lw;        /* fractional parts */
  int ok[4];            /* corner inside the map */
} bilin_t;

/* Sample point in pixel space: (loc * size) - 0.5, .cuh:285-286 */
static bilin_t bilinear_setup(double loc_w, double loc_h, int H, int W) {
  bilin_t b;
  memset(&b, 0, sizeof(b));
  const double h = loc_h * H - 0.5;
  const double w = loc_w * W - 0.5;
  /* strict band: -1 < h < H and -1 < w < W, .cuh:288 */
  if (!(h > -1.0 && w > -1.0 && h < (double)H && w < (double)W)) return b;
  b.valid = 1;
  b.hl = (int)floor(h);
  b.wl = (int)floor(w);
  b.hh = b.hl + 1;
  b.wh = b.wl + 1;
  b.lh = h - b.hl;
  b.lw = w - b.wl;
  const double hh = 1.0 - b.lh, hw = 1.0 - b.lw;
  b.w[0] = hh * hw;       /* (hl, wl) */
  b.w[1] = hh * b.lw;     /* (hl, wh) */
  b.w[2] = b.lh * hw;     /* (hh, wl) */
  b.w[3] = b.lh * b.lw;   /* (hh, wh) */
  b.ok[0] = b.hl >= 0 && b.wl >= 0;
  b.ok[1] = b.hl >= 0 && b.wh <= W - 1;
  b.ok[2] = b.hh <= H - 1 && b.wl >= 0;
  b.ok[3] = b.hh <= H - 1 && b.wh <= W - 1;
  return b;
}

static inline int corner_pos(const bilin_t* b, int k, int W) {
  const int y = (k < 2) ? b->hl : b->hh;
  const int x = (k & 1) ? b->wh : b->wl;
  return y * W + x;
}

void oracle_msda_forward(const double* value, const int64_t* shapes, const int64_t* lsi,
                         const double* loc, const double* attn, int N, int S, int M, int D,
                         int L, int Lq, int P, double* out) {
  for (int n = 0; n < N; ++n)
    for (int q = 0; q < Lq; ++q)
      for (int m = 0; m < M; ++m) {
        const size_t u = ((size_t)n * Lq + q) * M + m;
        double* o = out + u * D;
        for (int c = 0; c < D; ++c) o[c] = 0.0;
        for (int l = 0; l < L; ++l) {
          const int H = (int)shapes[2 * l], W = (int)shapes[2 * l + 1];
          const int start = (int)lsi[l];
          for (int p = 0; p < P; ++p) {
            const size_t s = (u * L + l) * P + p;
            const bilin_t b = bilinear_setup(loc[2 * s], loc[2 * s + 1], H, W);
            if (!b.valid) continue;
            const double a = attn[s];
            for (int c = 0; c < D; ++c) {
              double val = 0.0;
              for (int k = 0; k < 4; ++k)
                if (b.ok[k]) val += b.w[k] * vget(value, S, M, D, n, start + corner_pos(&b, k, W), m, c);
              o[c] += val * a;
            }
          }
        }
      }
}

void oracle_msda_backward(const double* value, const int64_t* shapes, const int64_t* lsi,
                          const double* loc, const double* attn, const double* grad_out, int N,
                          int S, int M, int D, int L, int Lq, int P, double* grad_value,
                          double* grad_loc, double* grad_attn) {
  memset(grad_value, 0, sizeof(double) * (size_t)N * S * M * D);
  for (int n = 0; n < N; ++n)
    for (int q = 0; q < Lq; ++q)
      for (int m = 0; m < M; ++m) {
        const size_t u = ((size_t)n * Lq + q) * M + m;
        const double* g = grad_out + u * D;
        for (int l = 0; l < L; ++l) {
          const int H = (int)shapes[2 * l], W = (int)shapes[2 * l + 1];
          const int start = (int)lsi[l];
          for (int p = 0; p < P; ++p) {
            const size_t s = (u * L + l) * P + p;
            grad_attn[s] = 0.0;
            grad_loc[2 * s] = 0.0;
            grad_loc[2 * s + 1] = 0.0;
            const bilin_t b = bilinear_setup(loc[2 * s], loc[2 * s + 1], H, W);
            if (!b.valid) continue;
            const double a = attn[s];
            /* d(corner weight)/dh and /dw, .cuh:121-151 */
            const double dwdh[4] = {-(1.0 - b.lw), -b.lw, 1.0 - b.lw, b.lw};
            const double dwdw[4] = {-(1.0 - b.lh), 1.0 - b.lh, -b.lh, b.lh};
            double sa = 0.0, sw = 0.0, sh = 0.0;
            for (int c = 0; c < D; ++c) {
              double val = 0.0, gh = 0.0, gw = 0.0;
              for (int k = 0; k < 4; ++k) {
                if (!b.ok[k]) continue;
                const int pos = start + corner_pos(&b, k, W);
                const double v = vget(value, S, M, D, n, pos, m, c);
                val += b.w[k] * v;
                gh += dwdh[k] * v;
                gw += dwdw[k] * v;
                grad_value[(((size_t)n * S + pos) * M + m) * D + c] += b.w[k] * g[c] * a;
              }
              sa += g[c] * val;
              sw += gw * g[c] * a;
              sh += gh * g[c] * a;
            }
            grad_attn[s] = sa;
            grad_loc[2 * s] = W * sw;
            grad_loc[2 * s + 1] = H * sh;
          }
        }
      }
}
