// Deterministic (fixed-order) reductions of per-block partial sums.
//
// Every cross-block reduction of the training step (LayerNorm / FiLM parameter gradients,
// variance-head gradients, bias column sums, embedding-row gradients, loss sums, the global
// gradient norm) writes one partial per block and is finished here in a fixed order -- no
// float atomics anywhere, so two runs with the same seed are bitwise identical (SURVEY §5,
// §7.8 item 5).  The partial buffers were written by the previous kernel on the same stream,
// so the kernel boundary orders them; no cross-XCD L2 coherence tricks are needed.
//
//   seg_colsum:  out[s, c] (+)= sum_{r < rows} P[s*rows + r, c]      (c < ncols, s < nseg)
//     64-column tiles x 4 row lanes per 256-thread block; each lane walks its rows in
//     order, the 4 lanes combine in order.  More than 256 rows per segment: a first level
//     splits the rows into contiguous chunks (parallelism), a second level sums the chunks.
//   small_sum:   out[k] = sum_{r < rows} P[r, k]   (k < 4, one block, fixed thread->row map
//     and a fixed LDS tree) -- the loss / grad-norm scalars.
#include "common.h"

namespace {

constexpr int SC_COLS = 64, SC_LANES = 4;

__global__ void __launch_bounds__(256) seg_colsum_kernel(const float* __restrict__ P, long ld, int rows_per_seg,
                                                         int r_per_split, int ncols, float* __restrict__ out,
                                                         long out_ld, int accumulate, int ncols1,
                                                         float* __restrict__ out2) {
  __shared__ float red[SC_LANES][SC_COLS];
  const int tx = threadIdx.x & (SC_COLS - 1), ty = threadIdx.x / SC_COLS;
  const int c = blockIdx.x * SC_COLS + tx;
  const int seg = blockIdx.y, split = blockIdx.z;
  const int r0 = split * r_per_split;
  const int r1 = min(rows_per_seg, r0 + r_per_split);
  float s = 0.f;
  if (c < ncols) {
    const float* base = P + (long)seg * rows_per_seg * ld + c;
    int r = r0 + ty;
    // 4 independent chains per lane keep loads in flight; combined in a fixed order
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (; r + 3 * SC_LANES < r1; r += 4 * SC_LANES) {
      a0 += base[(long)r * ld];
      a1 += base[(long)(r + SC_LANES) * ld];
      a2 += base[(long)(r + 2 * SC_LANES) * ld];
      a3 += base[(long)(r + 3 * SC_LANES) * ld];
    }
    for (; r < r1; r += SC_LANES) a0 += base[(long)r * ld];
    s = (a0 + a1) + (a2 + a3);
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < ncols) {
    const float v = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
    const long orow = ((long)seg * gridDim.z + split) * out_ld;
    float* o = (out2 && c >= ncols1) ? out2 + orow + (c - ncols1) : out + orow + c;
    *o = accumulate ? *o + v : v;
  }
}

__global__ void __launch_bounds__(1024) small_sum_kernel(const float* __restrict__ P, int rows, int k,
                                                         float* __restrict__ out) {
  __shared__ float red[4][1024];
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = threadIdx.x; r < rows; r += 1024)
    for (int j = 0; j < k; ++j) a[j] += P[(long)r * k + j];
  for (int j = 0; j < 4; ++j) red[j][threadIdx.x] = a[j];
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int j = 0; j < k; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < k) out[threadIdx.x] = red[threadIdx.x][0];
}

}  // namespace

// out[s*out_ld + c] (+)= sum_r P[(s*rows + r)*ld + c].  With out2: columns c >= ncols1 go to
// out2[s*out_ld + c - ncols1] instead (e.g. a weight and a bias gradient in one pass).
// ws: >= nseg * splits * ncols floats scratch for the two-level form (splits = min(16, rows / 256));
// pass ws_floats = 0 to force one level.
SSAMD_API int ssamd_seg_colsum(const float* P, long ld, int nseg, int rows, int ncols, float* out, long out_ld,
                               int accumulate, int ncols1, float* out2, float* ws, long ws_floats, hipStream_t s) {
  if (nseg <= 0 || ncols <= 0) return 0;
  if (rows <= 0) return -2;  // callers always have >= 1 partial row
  int splits = rows / 256;
  if (splits > 16) splits = 16;
  if (splits < 2 || ws == nullptr || ws_floats < (long)nseg * splits * ncols) splits = 1;
  const int tiles = cdiv(ncols, SC_COLS);
  if (splits == 1) {
    hipLaunchKernelGGL(seg_colsum_kernel, dim3(tiles, nseg, 1), dim3(256), 0, s, P, ld, rows, rows, ncols, out,
                       out_ld, accumulate, ncols1, out2);
    return (int)hipGetLastError();
  }
  const int rps = cdiv(rows, splits);
  // level 1: ws[(seg*splits + split), c]; level 2: sum the splits of each segment in order
  hipLaunchKernelGGL(seg_colsum_kernel, dim3(tiles, nseg, splits), dim3(256), 0, s, P, ld, rows, rps, ncols, ws,
                     (long)ncols, 0, ncols, (float*)nullptr);
  hipLaunchKernelGGL(seg_colsum_kernel, dim3(tiles, nseg, 1), dim3(256), 0, s, ws, (long)ncols, splits, splits, ncols,
                     out, out_ld, accumulate, ncols1, out2);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_small_sum(const float* P, int rows, int k, float* out, hipStream_t s) {
  if (k < 1 || k > 4) return -1;
  hipLaunchKernelGGL(small_sum_kernel, dim3(1), dim3(1024), 0, s, P, rows, k, out);
  return (int)hipGetLastError();
}
