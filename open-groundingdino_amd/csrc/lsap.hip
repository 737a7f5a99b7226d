// Rectangular linear sum assignment (Hungarian matching) on the device.
//
// Reference call site: models/GroundingDINO/matcher.py:104-110 (the matcher
// copies every cost matrix to the host, C.cpu(), and calls
// scipy.optimize.linear_sum_assignment per image).  This kernel restates the
// algorithm scipy runs there -- scipy 1.15 scipy/optimize/rectangular_lsap
// (Crouse's shortest-augmenting-path variant of Jonker-Volgenant, float64
// arithmetic on the float32 costs) -- with the SAME operation order and the
// SAME tie-breaking, so its assignment equals scipy's bit for bit, ties
// included:
//   * a tall matrix (more rows than columns) is solved transposed;
//   * per row, Dijkstra over the remaining columns, kept in scipy's
//     `remaining` array (initial order nc-1 .. 0, removal by swapping in the
//     last entry): the next column is the first position of minimal
//     reduced cost, except that among equal minima an unassigned column wins,
//     the LAST such position in scan order -- exactly what scipy's sequential
//     `if (spc[j] < lowest || (spc[j] == lowest && row4col[j] == -1))` picks;
//   * r = ((minVal + cost) - u[i]) - v[j], the dual updates and the
//     augmentation in scipy's order, all in float64;
//   * the transposed result is returned sorted by its (original) row index.
// Nothing leaves the device: the matching step no longer needs the
// device -> host copy and host wait that serialised the train step.
//
// One problem per 64-lane workgroup (one wave).  The column state (v, the
// shortest-path costs, path, row4col, the remaining list) lives in LDS; a
// scan step gives each lane every 64th remaining position and picks the
// winner with a butterfly reduction over (cost, tie key) that every lane ends
// with, so the wave-uniform control state stays in registers.
#include "gd_common.h"

#include <math.h>

namespace gd {
namespace {

constexpr int kLsapMaxCols = 2048;  // columns after the transpose: max(Q, n)
constexpr int kLsapMaxRows = 1024;  // rows after the transpose: min(Q, n)

// better(a, b): a is picked over b (smaller cost, then smaller tie key)
__device__ __forceinline__ bool lsap_better(double sa, int ka, double sb, int kb) {
  return sa < sb || (sa == sb && ka < kb);
}

__global__ __launch_bounds__(64) void lsap_kernel(const float* __restrict__ cost, int64_t problem_stride, int Q,
                                                  int K, const int* __restrict__ sizes, int64_t* __restrict__ out_row,
                                                  int64_t* __restrict__ out_col, int* __restrict__ status) {
  __shared__ double v[kLsapMaxCols];
  __shared__ double spc[kLsapMaxCols];
  __shared__ int path[kLsapMaxCols];
  __shared__ int row4col[kLsapMaxCols];
  __shared__ int remaining[kLsapMaxCols];
  __shared__ unsigned char sc[kLsapMaxCols];
  __shared__ double u[kLsapMaxRows];
  __shared__ int col4row[kLsapMaxRows];
  __shared__ unsigned char sr[kLsapMaxRows];

  const int p = blockIdx.x;
  const int lane = threadIdx.x;
  int n = sizes[p];
  n = n < 0 ? 0 : (n > K ? K : n);
  const float* C = cost + int64_t(p) * problem_stride;  // [Q, K] row-major; columns >= n unused
  int64_t* orow = out_row + int64_t(p) * K;
  int64_t* ocol = out_col + int64_t(p) * K;
  const bool transpose = n < Q;
  const int nr = transpose ? n : Q;
  const int nc = transpose ? Q : n;
  const int npairs = nr;  // min(Q, n)
  for (int r = npairs + lane; r < K; r += 64) {
    orow[r] = -1;
    ocol[r] = -1;
  }
  if (nr == 0) {
    if (lane == 0 && status) status[p] = 0;
    return;
  }
  // cost of (row i, column j) of the matrix scipy solves (after its transpose)
  auto cost_rc = [&](int i, int j) -> double {
    return double(transpose ? C[int64_t(j) * K + i] : C[int64_t(i) * K + j]);
  };

  for (int j = lane; j < nc; j += 64) {
    v[j] = 0.0;
    row4col[j] = -1;
    path[j] = -1;
  }
  for (int i = lane; i < nr; i += 64) {
    u[i] = 0.0;
    col4row[i] = -1;
  }
  __syncthreads();

  bool feasible = true;
  for (int cur = 0; cur < nr && feasible; ++cur) {
    // ---- augmenting_path(cur) ---------------------------------------------
    for (int it = lane; it < nc; it += 64) {
      remaining[it] = nc - it - 1;
      spc[it] = INFINITY;
      sc[it] = 0;
    }
    for (int i = lane; i < nr; i += 64) sr[i] = 0;
    __syncthreads();
    double min_val = 0.0;
    int i = cur, sink = -1, num_rem = nc;
    while (sink == -1) {
      if (lane == 0) sr[i] = 1;
      const double ui = u[i];
      double best_s = INFINITY;
      int best_k = 0x7fffffff, best_it = -1;
      for (int it = lane; it < num_rem; it += 64) {
        const int j = remaining[it];
        const double r = min_val + cost_rc(i, j) - ui - v[j];
        double s = spc[j];
        if (r < s) {
          path[j] = i;
          spc[j] = r;
          s = r;
        }
        // tie key: an unassigned column beats an assigned one; among
        // unassigned the later scan position wins, among assigned the earlier
        const int key = row4col[j] == -1 ? -1 - it : it;
        if (lsap_better(s, key, best_s, best_k)) {
          best_s = s;
          best_k = key;
          best_it = it;
        }
      }
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) {
        const double os = __shfl_xor(best_s, m, 64);
        const int ok = __shfl_xor(best_k, m, 64);
        const int oi = __shfl_xor(best_it, m, 64);
        if (lsap_better(os, ok, best_s, best_k)) {
          best_s = os;
          best_k = ok;
          best_it = oi;
        }
      }
      min_val = best_s;
      if (!(min_val < INFINITY) || best_it < 0) {  // infeasible (only with +inf costs)
        feasible = false;
        break;
      }
      const int j = remaining[best_it];
      const int rj = row4col[j];
      if (rj == -1)
        sink = j;
      else
        i = rj;
      __syncthreads();  // every lane has read remaining[] / spc[] of this step
      if (lane == 0) {
        sc[j] = 1;
        remaining[best_it] = remaining[num_rem - 1];
      }
      --num_rem;
      __syncthreads();
    }
    if (!feasible) break;
    // ---- dual update (scipy order: u[cur] first, then the other SR rows,
    // then the SC columns; spc / col4row still those of this search) -------
    for (int r = lane; r < nr; r += 64)
      if (sr[r] && r != cur) u[r] += min_val - spc[col4row[r]];
    for (int j = lane; j < nc; j += 64)
      if (sc[j]) v[j] -= min_val - spc[j];
    __syncthreads();
    if (lane == 0) {
      u[cur] += min_val;
      // ---- augment along the path back to cur --------------------------
      int j = sink;
      for (;;) {
        const int pi = path[j];
        row4col[j] = pi;
        const int t = col4row[pi];
        col4row[pi] = j;
        j = t;
        if (pi == cur) break;
      }
    }
    __syncthreads();
  }

  if (!feasible) {
    // scipy raises ValueError here; the reference then matches every target
    // to its argmin query (matcher.py:111-119).  Unreachable for finite
    // costs (the matcher zeroes NaN / inf entries first).
    for (int t = lane; t < n; t += 64) {
      int best = 0;
      float bv = C[t];
      for (int q = 1; q < Q; ++q) {
        const float c = C[int64_t(q) * K + t];
        if (c < bv) {
          bv = c;
          best = q;
        }
      }
      orow[t] = best;
      ocol[t] = t;
    }
    for (int r = n + lane; r < K; r += 64) {
      orow[r] = -1;
      ocol[r] = -1;
    }
    if (lane == 0 && status) status[p] = 1;
    return;
  }
  if (transpose) {
    // pairs (query col4row[t], target t) in ascending query order: the
    // queries are distinct, so a target's rank is the count of smaller ones
    for (int t = lane; t < nr; t += 64) {
      const int q = col4row[t];
      int rank = 0;
      for (int t2 = 0; t2 < nr; ++t2) rank += col4row[t2] < q;
      orow[rank] = q;
      ocol[rank] = t;
    }
  } else {
    for (int q = lane; q < nr; q += 64) {
      orow[q] = q;
      ocol[q] = col4row[q];
    }
  }
  if (lane == 0 && status) status[p] = 0;
}

}  // namespace
}  // namespace gd

using namespace gd;

extern "C" gd_status gd_linear_sum_assignment(const float* cost, int problems, int Q, int K,
                                              int64_t problem_stride, const int* sizes, int64_t* out_row,
                                              int64_t* out_col, int* status, gd_stream_t stream) {
  GD_REQUIRE(problems >= 0 && Q >= 0 && K >= 0, "lsa: bad sizes problems=%d Q=%d K=%d", problems, Q, K);
  if (problems == 0 || K == 0) return GD_OK;
  GD_REQUIRE(Q <= kLsapMaxCols && (Q <= kLsapMaxRows || K <= kLsapMaxRows) && K <= kLsapMaxCols,
             "lsa: Q=%d K=%d exceed the device solver (max(Q, n) <= %d, min(Q, n) <= %d)", Q, K, kLsapMaxCols,
             kLsapMaxRows);
  GD_REQUIRE(cost && sizes && out_row && out_col, "lsa: null pointer");
  GD_REQUIRE(problem_stride >= int64_t(Q) * K, "lsa: problem_stride %lld < Q*K", (long long)problem_stride);
  hipLaunchKernelGGL(lsap_kernel, dim3(problems), dim3(64), 0, as_hip(stream), cost, problem_stride, Q, K, sizes,
                     out_row, out_col, status);
  GD_LAUNCH_CHECK("lsap_kernel");
  return GD_OK;
}
