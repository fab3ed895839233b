// BatchNorm1d (channel-last, training batch statistics over all B*L rows incl. padding,
// the reference PostNet semantics -- transformer/Layers.py:78-148) fused with tanh (or ReLU:
// the GST Conv2d + BatchNorm2d stack on NHWC rows) and dropout, forward and backward.
// The int argument `act_tanh` is an activation code: 0 none, 1 tanh, 2 ReLU.
//
//   stats:    per-block partial (sum, sum of squares) per channel  -> [nblk][C] fp32
//   finalize: combine partials (fp64), mean / biased var -> rstd, scale = g*rstd,
//             shift = b - mean*scale, running stats update (momentum, unbiased var);
//             eval mode: scale/shift from the running stats
//   apply:    y = drop( act( h*scale + shift ) )        bf16 or fp32 out
//   bwd:      dz = dy * keep * act'(z);  partial sums of dz and dz*xhat;
//             finalize dgamma / dbeta;  dh = g*rstd*(dz - dbeta/R - xhat*dgamma/R)
// Row-major [R, C] with C % 8 == 0; one 16-B (8-channel) chunk per lane.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int BN_U = 4;  // rows per thread and load batch in the streaming kernels

__device__ __forceinline__ float act_fwd(int act, float z) { return bn_act_fwd(act, z); }
__device__ __forceinline__ float act_grad(int act, float z) { return bn_act_grad(act, z); }

struct RowMap {
  int chunks;      // C / 8
  int rows_iter;   // rows covered by one pass of the block
};

__device__ __forceinline__ RowMap rowmap(int C) {
  RowMap m;
  m.chunks = C / 8;
  m.rows_iter = NT / m.chunks;
  if (m.rows_iter < 1) m.rows_iter = 1;
  return m;
}

__device__ __forceinline__ void load8(const bf16_t* p, float* v) {
  short8 x = *reinterpret_cast<const short8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = bf2f((bf16_t)x[i]);
}

// grid: nblk blocks, each a contiguous slice of rows; requires C/8 <= 256 (C <= 2048)
__global__ void __launch_bounds__(NT) bn_stats_kernel(const bf16_t* __restrict__ h, long R, int C, long rows_per_blk,
                                                      float* __restrict__ psum, float* __restrict__ psq) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2][rows_iter][C]
  const RowMap m = rowmap(C);
  const int tid = threadIdx.x;
  const int c8 = tid % m.chunks, ro = tid / m.chunks;
  const bool active = ro < m.rows_iter;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long r0 = blockIdx.x * rows_per_blk, r1 = min(R, r0 + rows_per_blk);
  if (active) {
    for (long rb = r0 + ro; rb < r1; rb += BN_U * m.rows_iter) {
      short8 x[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long r = rb + u * m.rows_iter;
        if (r < r1) x[u] = *reinterpret_cast<const short8*>(h + r * C + c8 * 8);
      }
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        if (rb + u * m.rows_iter >= r1) break;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float v = bf2f((bf16_t)x[u][i]);
          s[i] += v;
          q[i] += v * v;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[ro * C + c8 * 8 + i] = s[i];
      red[(m.rows_iter + ro) * C + c8 * 8 + i] = q[i];
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float a = 0.f, b = 0.f;
    for (int j = 0; j < m.rows_iter; ++j) { a += red[j * C + c]; b += red[(m.rows_iter + j) * C + c]; }
    psum[(long)blockIdx.x * C + c] = a;
    psq[(long)blockIdx.x * C + c] = b;
  }
}

__global__ void __launch_bounds__(NT) bn_finalize_kernel(const float* __restrict__ psum, const float* __restrict__ psq,
                                                         int nblk, long R, int C, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* __restrict__ rmean,
                                                         float* __restrict__ rvar, float momentum, float eps, int training,
                                                         float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                         float* __restrict__ scale, float* __restrict__ shift) {
  // one wave per channel: lanes stride over the per-block partials, shuffle reduction
  const int c = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  float mean, var;
  if (training) {
    double s = 0.0, q = 0.0;
    for (int b = lane; b < nblk; b += 64) { s += psum[(long)b * C + c]; q += psq[(long)b * C + c]; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
    const double mu = s / (double)R;
    double vb = q / (double)R - mu * mu;
    if (vb < 0.0) vb = 0.0;
    mean = (float)mu;
    var = (float)vb;
    if (rmean && lane == 0) {
      const double unb = R > 1 ? vb * (double)R / (double)(R - 1) : vb;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
    }
  } else {
    mean = rmean[c];
    var = rvar[c];
  }
  if (lane != 0) return;
  const float rs = rsqrtf(var + eps);
  const float sc = gamma[c] * rs;
  mean_out[c] = mean;
  rstd_out[c] = rs;
  scale[c] = sc;
  shift[c] = beta[c] - mean * sc;
}

template <bool OUT_F32>
__global__ void __launch_bounds__(NT) bn_apply_kernel(const bf16_t* __restrict__ h, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, void* __restrict__ out, long R,
                                                      int C, int act_tanh, float p, uint64_t seed) {
  const RowMap m = rowmap(C);
  const int c8 = threadIdx.x % m.chunks, ro = threadIdx.x / m.chunks;
  if (ro >= m.rows_iter) return;
  const int c0 = c8 * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { sc[i] = scale[c0 + i]; sh[i] = shift[c0 + i]; }
  // BN_U rows per thread and batch, every load of a batch issued before any use (memory-level
  // parallelism: the per-row loop kept ~2 loads in flight per thread)
  const long stride = (long)gridDim.x * m.rows_iter;
  for (long r0 = (long)blockIdx.x * m.rows_iter + ro; r0 < R; r0 += BN_U * stride) {
    short8 x[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long r = r0 + u * stride;
      if (r < R) x[u] = *reinterpret_cast<const short8*>(h + r * C + c0);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long r = r0 + u * stride;
      if (r >= R) break;
      float v[8], ks[8];
      drop_scales<8>(seed, (uint64_t)(r * C + c0), p, ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float z = bf2f((bf16_t)x[u][i]) * sc[i] + sh[i];
        z = act_fwd(act_tanh, z);
        v[i] = z * ks[i];
      }
      if constexpr (OUT_F32) {
        float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + r * C + c0);
        o[0] = make_float4(v[0], v[1], v[2], v[3]);
        o[1] = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        short8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (short)f2bf(v[i]);
        *reinterpret_cast<short8*>(reinterpret_cast<bf16_t*>(out) + r * C + c0) = o;
      }
    }
  }
}

template <bool DY_F32>
__device__ __forceinline__ void load_dy(const void* dy, long off, float* v) {
  if constexpr (DY_F32) {
    const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dy) + off);
    float4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    load8(reinterpret_cast<const bf16_t*>(dy) + off, v);
  }
}

// dz = dy * keep * act'(z); partial sums of dz and dz*xhat
template <bool DY_F32>
__global__ void __launch_bounds__(NT) bn_bwd_reduce_kernel(const void* __restrict__ dy, const bf16_t* __restrict__ h,
                                                           const float* __restrict__ scale, const float* __restrict__ shift,
                                                           const float* __restrict__ mean, const float* __restrict__ rstd,
                                                           long R, int C, long rows_per_blk, int act_tanh, float p,
                                                           uint64_t seed, float* __restrict__ pdb, float* __restrict__ pdg) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const RowMap m = rowmap(C);
  const int tid = threadIdx.x;
  const int c8 = tid % m.chunks, ro = tid / m.chunks;
  const bool active = ro < m.rows_iter;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long r0 = blockIdx.x * rows_per_blk, r1 = min(R, r0 + rows_per_blk);
  if (active) {
    float sc[8], sh[8], mu[8], rs[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = scale[c8 * 8 + i]; sh[i] = shift[c8 * 8 + i]; mu[i] = mean[c8 * 8 + i]; rs[i] = rstd[c8 * 8 + i];
    }
    for (long rb = r0 + ro; rb < r1; rb += BN_U * m.rows_iter) {
      float hv[BN_U][8], g[BN_U][8];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long r = rb + u * m.rows_iter;
        if (r < r1) {
          load8(h + r * C + c8 * 8, hv[u]);
          load_dy<DY_F32>(dy, r * C + c8 * 8, g[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long r = rb + u * m.rows_iter;
        if (r >= r1) break;
        const long off = r * C + c8 * 8;
        float ks[8];
        drop_scales<8>(seed, (uint64_t)off, p, ks);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float dz = g[u][i] * ks[i];
          if (act_tanh) dz *= act_grad(act_tanh, hv[u][i] * sc[i] + sh[i]);
          a[i] += dz;
          b[i] += dz * (hv[u][i] - mu[i]) * rs[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[ro * C + c8 * 8 + i] = a[i];
      red[(m.rows_iter + ro) * C + c8 * 8 + i] = b[i];
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float x = 0.f, y = 0.f;
    for (int j = 0; j < m.rows_iter; ++j) { x += red[j * C + c]; y += red[(m.rows_iter + j) * C + c]; }
    pdb[(long)blockIdx.x * C + c] = x;
    pdg[(long)blockIdx.x * C + c] = y;
  }
}

__global__ void __launch_bounds__(NT) bn_bwd_finalize_kernel(const float* __restrict__ pdb, const float* __restrict__ pdg,
                                                             int nblk, int C, float* __restrict__ dbeta,
                                                             float* __restrict__ dgamma,
                                                             const float* __restrict__ gscale = nullptr) {
  const int c = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  double x = 0.0, y = 0.0;
  for (int b = lane; b < nblk; b += 64) { x += pdb[(long)b * C + c]; y += pdg[(long)b * C + c]; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { x += __shfl_xor(x, o, 64); y += __shfl_xor(y, o, 64); }
  if (lane == 0) {
    dbeta[c] = (float)x;
    dgamma[c] = gscale ? (float)(y * (double)gscale[c]) : (float)y;  // gscale: per-column rstd (GEMM partials)
  }
}

template <bool DY_F32>
__global__ void __launch_bounds__(NT) bn_bwd_apply_kernel(const void* __restrict__ dy, const bf16_t* __restrict__ h,
                                                          const float* __restrict__ gamma, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, const float* __restrict__ dbeta,
                                                          const float* __restrict__ dgamma, bf16_t* __restrict__ dh, long R,
                                                          int C, int act_tanh, float p, uint64_t seed, int training) {
  const RowMap m = rowmap(C);
  const int c8 = threadIdx.x % m.chunks, ro = threadIdx.x / m.chunks;
  if (ro >= m.rows_iter) return;
  const int c0 = c8 * 8;
  const float invR = 1.f / (float)R;
  // dh = k1 * dz + k2 * h + k3   (training);   dh = scale * dz (eval)
  float sc[8], sh[8], k1[8], k2[8], k3[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = c0 + i;
    sc[i] = scale[c];
    sh[i] = shift[c];
    if (training) {
      const float gr = gamma[c] * rstd[c];
      k1[i] = gr;
      k2[i] = -gr * rstd[c] * dgamma[c] * invR;
      k3[i] = -gr * dbeta[c] * invR - k2[i] * mean[c];
    } else {
      k1[i] = sc[i];
      k2[i] = 0.f;
      k3[i] = 0.f;
    }
  }
  const long stride = (long)gridDim.x * m.rows_iter;
  for (long r0 = (long)blockIdx.x * m.rows_iter + ro; r0 < R; r0 += BN_U * stride) {
    float hv[BN_U][8], g[BN_U][8];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long r = r0 + u * stride;
      if (r < R) {
        load8(h + r * C + c0, hv[u]);
        load_dy<DY_F32>(dy, r * C + c0, g[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long r = r0 + u * stride;
      if (r >= R) break;
      const long off = r * C + c0;
      short8 o;
      float ks[8];
      drop_scales<8>(seed, (uint64_t)off, p, ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float dz = g[u][i] * ks[i];
        if (act_tanh) dz *= act_grad(act_tanh, hv[u][i] * sc[i] + sh[i]);
        o[i] = (short)f2bf(k1[i] * dz + k2[i] * hv[u][i] + k3[i]);
      }
      *reinterpret_cast<short8*>(dh + off) = o;
    }
  }
}

// dh = k1 * dz + k2 * h + k3 from dz that the producing data-gradient GEMM already formed (dy * keep *
// act'), k_gemm.hip EpiX.bn_*: a pure two-read / one-write stream (no dropout hash, no tanh here)
template <int U>
__global__ void __launch_bounds__(NT) bn_bwd_apply_dz_kernel(const bf16_t* __restrict__ dz, const bf16_t* __restrict__ h,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ stats,
                                                             const float* __restrict__ dbeta,
                                                             const float* __restrict__ dgamma, bf16_t* __restrict__ dh,
                                                             long R, int C, int training) {
  const RowMap m = rowmap(C);
  const int c8 = threadIdx.x % m.chunks, ro = threadIdx.x / m.chunks;
  if (ro >= m.rows_iter) return;
  const int c0 = c8 * 8;
  const float invR = 1.f / (float)R;
  float k1[8], k2[8], k3[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = c0 + i;
    const float mean = stats[c], rs = stats[C + c];
    if (training) {
      const float gr = gamma[c] * rs;
      k1[i] = gr;
      k2[i] = -gr * rs * dgamma[c] * invR;
      k3[i] = -gr * dbeta[c] * invR - k2[i] * mean;
    } else {
      k1[i] = stats[2 * C + c];
      k2[i] = 0.f;
      k3[i] = 0.f;
    }
  }
  // U rows per thread and load batch: 2U loads of 16 B in flight per lane
  const long stride = (long)gridDim.x * m.rows_iter;
  for (long r0 = (long)blockIdx.x * m.rows_iter + ro; r0 < R; r0 += U * stride) {
    short8 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = r0 + u * stride;
      if (r < R) {
        a[u] = __builtin_nontemporal_load(reinterpret_cast<const short8*>(dz + r * C + c0));
        b[u] = *reinterpret_cast<const short8*>(h + r * C + c0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = r0 + u * stride;
      if (r >= R) break;
      short8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        o[i] = (short)f2bf(k1[i] * bf2f((bf16_t)a[u][i]) + k2[i] * bf2f((bf16_t)b[u][i]) + k3[i]);
      *reinterpret_cast<short8*>(dh + r * C + c0) = o;
    }
  }
}

}  // namespace

static int blocks_for(long R) {
  long b = (R + 255) / 256;
  if (b > 512) b = 512;
  return (int)(b < 1 ? 1 : b);
}

// ws: 2 * nblk * C floats (nblk = blocks_for(R) <= 1024)
SSAMD_API int ssamd_bn_fwd(const bf16_t* h, const float* gamma, const float* beta, float* rmean, float* rvar,
                           float* mean, float* rstd, float* scale, float* shift, void* out, int out_f32, long R, int C,
                           int training, float momentum, float eps, int act_tanh, float p, unsigned long long seed,
                           float* ws, hipStream_t s) {
  if (C % 8 || C / 8 > NT) return -2;
  const int nblk = blocks_for(R);
  const long rpb = (R + nblk - 1) / nblk;
  const RowMap m = {C / 8, NT / (C / 8)};
  if (training && R > 0) {
    hipLaunchKernelGGL(bn_stats_kernel, dim3(nblk), dim3(NT), (size_t)2 * m.rows_iter * C * 4, s, h, R, C, rpb, ws,
                       ws + (long)nblk * C);
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 3) / 4), dim3(NT), 0, s, ws, ws + (long)nblk * C, nblk, R, C,
                     gamma, beta, rmean, rvar, momentum, eps, training, mean, rstd, scale, shift);
  if (R > 0) {
    const int g = (int)min((R + m.rows_iter - 1) / m.rows_iter, 4096L);
    if (out_f32)
      hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(g), dim3(NT), 0, s, h, scale, shift, out, R, C, act_tanh, p,
                         (uint64_t)seed);
    else
      hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(g), dim3(NT), 0, s, h, scale, shift, out, R, C, act_tanh, p,
                         (uint64_t)seed);
  }
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_bn_bwd(const void* dy, int dy_f32, const bf16_t* h, const float* gamma, const float* scale,
                           const float* shift, const float* mean, const float* rstd, bf16_t* dh, float* dgamma,
                           float* dbeta, long R, int C, int training, int act_tanh, float p, unsigned long long seed,
                           float* ws, hipStream_t s) {
  if (C % 8 || C / 8 > NT) return -2;
  if (R == 0) {
    hipMemsetAsync(dgamma, 0, C * 4, s);
    hipMemsetAsync(dbeta, 0, C * 4, s);
    return (int)hipGetLastError();
  }
  const int nblk = blocks_for(R);
  const long rpb = (R + nblk - 1) / nblk;
  const RowMap m = {C / 8, NT / (C / 8)};
  const size_t lds = (size_t)2 * m.rows_iter * C * 4;
  if (dy_f32)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, dim3(nblk), dim3(NT), lds, s, dy, h, scale, shift, mean, rstd, R, C,
                       rpb, act_tanh, p, (uint64_t)seed, ws, ws + (long)nblk * C);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, dim3(nblk), dim3(NT), lds, s, dy, h, scale, shift, mean, rstd, R, C,
                       rpb, act_tanh, p, (uint64_t)seed, ws, ws + (long)nblk * C);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 3) / 4), dim3(NT), 0, s, ws, ws + (long)nblk * C, nblk, C,
                     dbeta, dgamma);
  const int g = (int)min((R + m.rows_iter - 1) / m.rows_iter, 4096L);
  if (dy_f32)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(g), dim3(NT), 0, s, dy, h, gamma, scale, shift, mean, rstd, dbeta,
                       dgamma, dh, R, C, act_tanh, p, (uint64_t)seed, training);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, dim3(g), dim3(NT), 0, s, dy, h, gamma, scale, shift, mean, rstd,
                       dbeta, dgamma, dh, R, C, act_tanh, p, (uint64_t)seed, training);
  return (int)hipGetLastError();
}

// apply-dz geometry: 8 rows per thread, <= 1024 blocks (4 per CU) looping -- 4.8 TB/s at the PostNet shape vs
// 3.3 with one pass per block over 4250 blocks (tools/exp_bnh.py sweep, profiles/r4_exp_bn_apply_dz.jsonl)
static int g_bn_dz_u = 8, g_bn_dz_grid = 1024;
SSAMD_API void ssamd_bn_set_dz_cfg(int u, int grid) {
  g_bn_dz_u = u;
  g_bn_dz_grid = grid;
}

// Second half of the BatchNorm backward when the data-gradient GEMM produced dz and the column partials
// (ssamd_conv_gemm_bnbwd): fixed-order combine of the nparts per-tile partials -> dbeta / dgamma, then
// dh = k1 * dz + k2 * h + k3.  stats = [mean | rstd | scale | shift] x C (the forward's).
SSAMD_API int ssamd_bn_bwd_dz(const bf16_t* dz, const bf16_t* h, const float* gamma, const float* stats,
                              const float* part, int nparts, bf16_t* dh, float* dgamma, float* dbeta, long R, int C,
                              int training, hipStream_t s) {
  if (C % 8 || C / 8 > NT) return -2;
  if (R == 0) {
    hipMemsetAsync(dgamma, 0, C * 4, s);
    hipMemsetAsync(dbeta, 0, C * 4, s);
    return (int)hipGetLastError();
  }
  // the GEMM head's second partial is sum dz * (h - mean): rstd is applied here, once per column
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 3) / 4), dim3(NT), 0, s, part, part + (long)nparts * C, nparts,
                     C, dbeta, dgamma, stats + C);
  const RowMap m = {C / 8, NT / (C / 8)};
  // one row batch (U rows per thread) per block and pass: >= 2048 blocks keep every CU streaming
  const int U = g_bn_dz_u;
  const long per = (long)m.rows_iter * U;
  const int g = (int)max(1L, min((R + per - 1) / per, (long)g_bn_dz_grid));
  if (U == 4)
    hipLaunchKernelGGL(bn_bwd_apply_dz_kernel<4>, dim3(g), dim3(NT), 0, s, dz, h, gamma, stats, dbeta, dgamma, dh, R,
                       C, training);
  else if (U == 16)
    hipLaunchKernelGGL(bn_bwd_apply_dz_kernel<16>, dim3(g), dim3(NT), 0, s, dz, h, gamma, stats, dbeta, dgamma, dh, R,
                       C, training);
  else
    hipLaunchKernelGGL(bn_bwd_apply_dz_kernel<8>, dim3(g), dim3(NT), 0, s, dz, h, gamma, stats, dbeta, dgamma, dh, R,
                       C, training);
  return (int)hipGetLastError();
}

SSAMD_DROP_SALT_LOADER(bn)
