// Memory-bound glue kernels: length regulator, embeddings, fused loss, clip + Adam.
#include "common.h"

namespace {

// ----------------------------------------------------------------------------
// LengthRegulator (reference model/modules.py:168-201): sync-free.
//   cum[b, i] = sum_{j<=i} d[b, j]   (inclusive prefix sum, computed in-kernel per block)
//   frame f of item b copies phoneme p = #{i : cum[b,i] <= f} (f < mel_len[b]) else zeros,
//   then optionally adds a positional row pe[f] (decoder input, Models.py:154-162).
// Grid (ceil(M / 64), B), 256 threads; each half-wave moves one 512-B row (C=256)
// with 16-B vector loads; cum is staged once per block in LDS.
// ----------------------------------------------------------------------------
constexpr int LR_ROWS = 64;

__device__ int block_prefix_durations(const int64_t* d, int T, int* cum) {
  // serial-per-thread chunks + wave scan; T is small (<= a few hundred)
  for (int i = threadIdx.x; i < T; i += blockDim.x) cum[i] = (int)max((int64_t)0, d[i]);
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int i = 0; i < T; ++i) { s += cum[i]; cum[i] = s; }
  }
  __syncthreads();
  return T > 0 ? cum[T - 1] : 0;
}

// packed mode (cu != nullptr): frame f of sequence b is row cu[b] + f, frames f >= plen[b] do not exist
__global__ void __launch_bounds__(256) lr_fwd_kernel(const bf16_t* __restrict__ x, const int64_t* __restrict__ dur,
                                                     const bf16_t* __restrict__ pe, bf16_t* __restrict__ out,
                                                     const int64_t* __restrict__ cu, const int64_t* __restrict__ plen,
                                                     int T, int M, int C) {
  extern __shared__ int cum[];
  const int b = blockIdx.y;
  const int Mb = cu ? min(M, (int)plen[b]) : M;
  if (blockIdx.x * LR_ROWS >= Mb) return;  // block-uniform
  const long obase = cu ? (long)cu[b] : (long)b * M;
  const int total = block_prefix_durations(dur + (long)b * T, T, cum);
  const int vec = C / 8;  // 16-B chunks per row
  for (int e = threadIdx.x; e < LR_ROWS * vec; e += blockDim.x) {
    const int r = e / vec, c8 = e % vec;
    const int f = blockIdx.x * LR_ROWS + r;
    if (f >= Mb) break;
    short8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (f < total) {
      int lo = 0, hi = T;  // first i with cum[i] > f
      while (lo < hi) { int mid = (lo + hi) >> 1; if (cum[mid] <= f) lo = mid + 1; else hi = mid; }
      v = *reinterpret_cast<const short8*>(x + ((long)b * T + lo) * C + c8 * 8);
    }
    if (pe) {
      short8 p = *reinterpret_cast<const short8*>(pe + (long)f * C + c8 * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (short)f2bf(bf2f((bf16_t)v[i]) + bf2f((bf16_t)p[i]));
    }
    *reinterpret_cast<short8*>(out + (obase + f) * C + c8 * 8) = v;
  }
}

// dx[b, p] = sum over the frames f in [cum[p-1], cum[p]) with f < M of dout[b, f]
// LRB_ROWS phonemes per block (a thread per 16-B chunk of one phoneme at C = 256): the per-phoneme frame
// sums are short dependent chains, so the grid is made wide (64 phonemes per block left 200-400 blocks
// each walking 8 chunks x ~8 frames serially: 70 us for the LJSpeech batch) and each thread issues four
// frames' loads before adding them in frame order (the same sums, bit for bit).
constexpr int LRB_ROWS = 8;
__global__ void __launch_bounds__(256) lr_bwd_kernel(const bf16_t* __restrict__ dout, const int64_t* __restrict__ dur,
                                                     bf16_t* __restrict__ dx, const int64_t* __restrict__ cu,
                                                     const int64_t* __restrict__ plen, int T, int M, int C) {
  extern __shared__ int cum[];
  const int b = blockIdx.y;
  const int Mb = cu ? min(M, (int)plen[b]) : M;
  const long obase = cu ? (long)cu[b] : (long)b * M;
  block_prefix_durations(dur + (long)b * T, T, cum);
  const int vec = C / 8;
  for (int e = threadIdx.x; e < LRB_ROWS * vec; e += blockDim.x) {
    const int r = e / vec, c8 = e % vec;
    const int p = blockIdx.x * LRB_ROWS + r;
    if (p >= T) break;
    const int f0 = p ? cum[p - 1] : 0;
    const int f1 = min(cum[p], Mb);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16_t* src = dout + obase * C + c8 * 8;
    int f = f0;
    for (; f + 4 <= f1; f += 4) {
      short8 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const short8*>(src + (long)(f + j) * C);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += bf2f((bf16_t)v[j][i]);
    }
    for (; f < f1; ++f) {
      short8 v = *reinterpret_cast<const short8*>(src + (long)f * C);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += bf2f((bf16_t)v[i]);
    }
    short8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (short)f2bf(acc[i]);
    *reinterpret_cast<short8*>(dx + ((long)b * T + p) * C + c8 * 8) = o;
  }
}

// ----------------------------------------------------------------------------
// Embedding gather + add (phoneme embedding + PE, Models.py:56-62,89-91; pitch /
// energy bucketized embeddings, modules.py:83-101).
//   mode 0: out[r] = table[ids[r]] + pe[r % L]            (ids int64)
//   mode 1: out[r] = x[r] + table[bucketize(vals[r], bins)]  (torch.bucketize, right=False)
// Backward: dtable[v] = sum of dout rows with id v, deterministic (one block per table row).
// ----------------------------------------------------------------------------
__device__ __forceinline__ int bucketize_lower(float v, const float* bins, int nb) {
  int lo = 0, hi = nb;  // number of bins strictly less than v
  while (lo < hi) { int mid = (lo + hi) >> 1; if (bins[mid] < v) lo = mid + 1; else hi = mid; }
  return lo;
}

__global__ void __launch_bounds__(256) embed_fwd_kernel(int mode, const int64_t* __restrict__ ids,
                                                        const float* __restrict__ vals, const float* __restrict__ bins,
                                                        int nbins, const bf16_t* __restrict__ table,
                                                        const bf16_t* __restrict__ addend, int L,
                                                        bf16_t* __restrict__ out, int* __restrict__ idx_out, long rows,
                                                        int C) {
  const int vec = C / 8;
  const long total = rows * vec;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long r = e / vec;
    const int c8 = (int)(e % vec);
    int id;
    if (mode == 0) id = (int)ids[r];
    else id = bucketize_lower(vals[r], bins, nbins);
    if (idx_out && c8 == 0) idx_out[r] = id;
    short8 t = *reinterpret_cast<const short8*>(table + (long)id * C + c8 * 8);
    const bf16_t* ad = mode == 0 ? addend + (long)(r % L) * C : addend + r * C;
    short8 p = *reinterpret_cast<const short8*>(ad + c8 * 8);
    short8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (short)f2bf(bf2f((bf16_t)t[i]) + bf2f((bf16_t)p[i]));
    *reinterpret_cast<short8*>(out + r * C + c8 * 8) = o;
  }
}

// Deterministic backward: block v owns table row v.  It scans the saved bucket ids in row order
// (wave ballots, order-preserving compaction into an LDS hit list) and sums the dout rows of its
// hits in that order -- every dtable element is produced by one thread in a fixed order, no atomics.
constexpr int EB_UNROLL = 4, EB_HITS = 2048;

__global__ void __launch_bounds__(256) embed_bwd_kernel(const int* __restrict__ idx, const bf16_t* __restrict__ dout,
                                                        float* __restrict__ dtable, long rows, int C) {
  __shared__ int hits[EB_HITS + 256 * EB_UNROLL];
  __shared__ int wcnt[4 * EB_UNROLL];
  const int v = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int MAXC = 4;  // channels per thread: C <= 1024
  float acc[MAXC] = {0.f, 0.f, 0.f, 0.f};
  int nh = 0;
  auto flush = [&](int n) {
    int k = 0;
    for (; k + 4 <= n; k += 4) {  // 4 independent row loads in flight, added in row order
#pragma unroll
      for (int j = 0; j < MAXC; ++j) {
        const int c = tid + j * 256;
        if (c < C) {
          const float x0 = bf2f(dout[(long)hits[k] * C + c]), x1 = bf2f(dout[(long)hits[k + 1] * C + c]);
          const float x2 = bf2f(dout[(long)hits[k + 2] * C + c]), x3 = bf2f(dout[(long)hits[k + 3] * C + c]);
          acc[j] = (((acc[j] + x0) + x1) + x2) + x3;
        }
      }
    }
    for (; k < n; ++k)
#pragma unroll
      for (int j = 0; j < MAXC; ++j) {
        const int c = tid + j * 256;
        if (c < C) acc[j] += bf2f(dout[(long)hits[k] * C + c]);
      }
  };
  for (long base = 0; base < rows; base += 256 * EB_UNROLL) {
    int id[EB_UNROLL];
#pragma unroll
    for (int u = 0; u < EB_UNROLL; ++u) {
      const long r = base + u * 256 + tid;
      id[u] = r < rows ? idx[r] : -1;
    }
    unsigned long long m[EB_UNROLL];
#pragma unroll
    for (int u = 0; u < EB_UNROLL; ++u) {
      m[u] = __ballot(id[u] == v);
      if (lane == 0) wcnt[u * 4 + wave] = __popcll(m[u]);
    }
    __syncthreads();
    int off = nh;
#pragma unroll
    for (int u = 0; u < EB_UNROLL; ++u) {
      int before = 0, tot = 0;
      for (int w = 0; w < 4; ++w) {
        const int cw = wcnt[u * 4 + w];
        if (w < wave) before += cw;
        tot += cw;
      }
      if (id[u] == v) {
        const int pos = __popcll(m[u] & ((1ull << lane) - 1ull));
        hits[off + before + pos] = (int)(base + u * 256 + tid);
      }
      off += tot;
    }
    __syncthreads();
    nh = off;
    if (nh >= EB_HITS) {
      flush(nh);
      nh = 0;
      __syncthreads();
    }
  }
  flush(nh);
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = tid + j * 256;
    if (c < C) dtable[(long)v * C + c] = acc[j];
  }
}

// ----------------------------------------------------------------------------
// Fused masked L1 pair (model/loss.py:74-75): sums |p1-t| and |p2-t| over valid
// frames (f < mel_len[b]) without masked_select compaction.
// ----------------------------------------------------------------------------
__global__ void __launch_bounds__(256) l1pair_fwd_kernel(const float* __restrict__ p1, const float* __restrict__ p2,
                                                         const float* __restrict__ tgt, const int64_t* __restrict__ lens,
                                                         int M, int Mt, int C, float* __restrict__ part, long rows) {
  float s1 = 0.f, s2 = 0.f;
  const long total = rows * C;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long r = e / C;
    const int c = (int)(e % C);
    const int b = (int)(r / M), f = (int)(r % M);
    if (f >= lens[b]) continue;
    const float t = tgt[((long)b * Mt + f) * C + c];
    s1 += fabsf(p1[e] - t);
    s2 += fabsf(p2[e] - t);
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  __shared__ float red[2][4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][wave] = s1; red[1][wave] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {  // per-block partial; finished by a fixed-order sum (k_reduce.hip)
    part[2 * blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    part[2 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

__global__ void __launch_bounds__(256) l1pair_bwd_kernel(const float* __restrict__ p1, const float* __restrict__ p2,
                                                         const float* __restrict__ tgt, const int64_t* __restrict__ lens,
                                                         int M, int Mt, int C, const float* __restrict__ gscale,
                                                         const float* __restrict__ count, float* __restrict__ g1,
                                                         float* __restrict__ g2, long rows) {
  const float inv = 1.f / fmaxf(*count, 1.f);
  const float s1 = gscale[0] * inv, s2 = gscale[1] * inv;
  const long total = rows * C;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long r = e / C;
    const int c = (int)(e % C);
    const int b = (int)(r / M), f = (int)(r % M);
    float a = 0.f, bb = 0.f;
    if (f < lens[b]) {
      const float t = tgt[((long)b * Mt + f) * C + c];
      const float d1 = p1[e] - t, d2 = p2[e] - t;
      a = d1 > 0.f ? s1 : (d1 < 0.f ? -s1 : 0.f);
      bb = d2 > 0.f ? s2 : (d2 < 0.f ? -s2 : 0.f);
    }
    g1[e] = a;
    g2[e] = bb;
  }
}

// ----------------------------------------------------------------------------
// Global-norm clip + Adam over the flat fp32 arena (model/optimizer.py:10-15,
// train.py:97).  Pass 1: sum of squares -> per-block partials ws[1..], summed in a fixed order
// into ws[0] (deterministic).  Pass 2: coef = min(1, clip / (sqrt(ss) + 1e-6)); a non-finite norm
// skips the update (and counts it) -- no host synchronisation anywhere.
// ----------------------------------------------------------------------------
__global__ void __launch_bounds__(256) sumsq_kernel(const float* __restrict__ g, long n, float* __restrict__ out) {
  float s = 0.f;
  const long n4 = n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 v = g4[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += g[i] * g[i];
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// one Adam element update (shared by adam_kernel and adam_img_kernel: same expression tree, so the
// same FMA contraction and bitwise-identical results on either path)
__device__ __forceinline__ float adam_upd(float pk, float gk, float& mk, float& vk, float coef, float wd, float b1,
                                          float b2, float step, float bc2_sqrt, float eps) {
#pragma clang fp contract(off)  // explicit fmaf only: no context-dependent contraction between the kernels
  gk = fmaf(gk, coef, wd * pk);
  mk = fmaf(b1, mk, (1.f - b1) * gk);
  vk = fmaf(b2, vk, ((1.f - b2) * gk) * gk);
  return fmaf(-step, mk / (sqrtf(vk) / bc2_sqrt + eps), pk);
}

__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n,
                                                   const float* __restrict__ ss, float clip, float lr, float b1,
                                                   float b2, float eps, float wd, float bc1, float bc2_sqrt,
                                                   float* __restrict__ norm_out, long long* __restrict__ skipped) {
  const float norm = sqrtf(*ss);
  if (!isfinite(norm)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) { *norm_out = norm; *skipped += 1; }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *norm_out = norm;
  const float coef = clip > 0.f ? fminf(1.f, clip / (norm + 1e-6f)) : 1.f;
  const float step = lr / bc1;
  const long n4 = n / 4;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = p4[i], gg = g4[i], mm = m4[i], vv = v4[i];
    float* pa = &pp.x; float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) pa[k] = adam_upd(pa[k], ga[k], ma[k], va[k], coef, wd, b1, b2, step, bc2_sqrt, eps);
    p4[i] = pp; m4[i] = mm; v4[i] = vv;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float mk = m[i], vk = v[i];
    p[i] = adam_upd(p[i], g[i], mk, vk, coef, wd, b1, b2, step, bc2_sqrt, eps);
    m[i] = mk;
    v[i] = vk;
  }
}

}  // namespace

static int grid_for(long work, int per_thread = 1) {
  long blocks = (work / per_thread + 255) / 256;
  if (blocks < 1) blocks = 1;
  return (int)(blocks > 4096 ? 4096 : blocks);
}

SSAMD_API int ssamd_lr_fwd(const bf16_t* x, const int64_t* dur, const bf16_t* pe, bf16_t* out, const int64_t* cu,
                           const int64_t* plen, int B, int T, int M, int C, hipStream_t s) {
  if (C % 8) return -1;
  if (B == 0 || M == 0) return 0;
  hipLaunchKernelGGL(lr_fwd_kernel, dim3(cdiv(M, LR_ROWS), B), dim3(256), (size_t)T * 4 + 16, s, x, dur, pe, out, cu,
                     plen, T, M, C);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_lr_bwd(const bf16_t* dout, const int64_t* dur, bf16_t* dx, const int64_t* cu, const int64_t* plen,
                           int B, int T, int M, int C, hipStream_t s) {
  if (C % 8) return -1;
  if (B == 0 || T == 0) return 0;
  hipLaunchKernelGGL(lr_bwd_kernel, dim3(cdiv(T, LRB_ROWS), B), dim3(256), (size_t)T * 4 + 16, s, dout, dur, dx, cu,
                     plen, T, M, C);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------
// Packed-sequence bookkeeping, one launch: grid = B blocks.
//   cu[b] = sum_{i<b} len[i] (cu[B] = total), rinfo[cu[b]+t] = {t, len[b]}, dst[cu[b]+t] = b*M + t
// ----------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(256) pack_info_kernel(const int64_t* __restrict__ lens, int B, int M,
                                                        int64_t* __restrict__ cu, int2* __restrict__ rinfo,
                                                        int64_t* __restrict__ dst) {
  __shared__ long part[256];
  const int b = blockIdx.x;
  long sacc = 0;
  for (int i = threadIdx.x; i < b; i += 256) sacc += min((long)lens[i], (long)M);
  part[threadIdx.x] = sacc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  const long base = part[0];
  const int len = (int)min((long)lens[b], (long)M);
  if (threadIdx.x == 0) {
    cu[b] = base;
    if (b == B - 1) cu[B] = base + len;
  }
  for (int t = threadIdx.x; t < len; t += 256) {
    rinfo[base + t] = make_int2(t, len);
    dst[base + t] = (long)b * M + t;
  }
}
}  // namespace

SSAMD_API int ssamd_pack_info(const int64_t* lens, int B, int M, int64_t* cu, int* rinfo, int64_t* dst, hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(pack_info_kernel, dim3(B), dim3(256), 0, s, lens, B, M, cu, reinterpret_cast<int2*>(rinfo), dst);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_embed_fwd(int mode, const int64_t* ids, const float* vals, const float* bins, int nbins,
                              const bf16_t* table, const bf16_t* addend, int L, bf16_t* out, int* idx_out, long rows,
                              int C, hipStream_t s) {
  if (C % 8) return -1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_for(rows * (C / 8))), dim3(256), 0, s, mode, ids, vals, bins, nbins,
                     table, addend, L, out, idx_out, rows, C);
  return (int)hipGetLastError();
}

// One-hot expansion of the saved ids: oh[r, v] = (idx[r] == v) in bf16, [rows, Vpad] -- the
// embedding backward then is the weight-gradient GEMM dtable = oh^T @ dout on the MFMA wgrad
// kernel (exact: the one-hot factors are 0 / 1), deterministic through its fixed-order slab reduce,
// and insensitive to skewed id distributions (pitch / energy buckets).
namespace {
__global__ void __launch_bounds__(256) onehot_kernel(const int* __restrict__ idx, long rows, int Vpad,
                                                     bf16_t* __restrict__ oh) {
  const int v8 = Vpad / 8;
  const long total = rows * v8;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long r = e / v8;
    const int c0 = (int)(e - r * v8) * 8;
    const int id = idx[r];
    short8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (c0 + i == id) ? (short)0x3F80 : (short)0;  // bf16 1.0
    *reinterpret_cast<short8*>(oh + r * Vpad + c0) = o;
  }
}
}  // namespace

SSAMD_API int ssamd_onehot(const int* idx, long rows, int Vpad, bf16_t* oh, hipStream_t s) {
  if (Vpad % 8) return -1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(onehot_kernel, dim3(grid_for(rows * (Vpad / 8))), dim3(256), 0, s, idx, rows, Vpad, oh);
  return (int)hipGetLastError();
}

// dtable [V, C] is overwritten (rows of unused ids become 0).  C <= 1024.
SSAMD_API int ssamd_embed_bwd(const int* idx, const bf16_t* dout, float* dtable, long rows, int C, int V,
                              hipStream_t s) {
  if (C > 1024 || V <= 0) return -1;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(V), dim3(256), 0, s, idx, dout, dtable, rows, C);
  return (int)hipGetLastError();
}

SSAMD_API long ssamd_l1pair_ws(int B, int M, int C) { return 2L * grid_for((long)B * M * C, 4); }

// sums[0..1] = (sum |p1 - t|, sum |p2 - t|) over valid frames; ws: ssamd_l1pair_ws floats of partials.
SSAMD_API int ssamd_l1pair_fwd(const float* p1, const float* p2, const float* tgt, const int64_t* lens, int B, int M,
                               int Mt, int C, float* sums, float* ws, long ws_floats, hipStream_t s) {
  long rows = (long)B * M;
  if (rows == 0) return (int)hipMemsetAsync(sums, 0, 2 * sizeof(float), s);
  const int nblk = grid_for(rows * C, 4);
  if (ws_floats < 2L * nblk) return -3;
  hipLaunchKernelGGL(l1pair_fwd_kernel, dim3(nblk), dim3(256), 0, s, p1, p2, tgt, lens, M, Mt, C, ws, rows);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  return ssamd_small_sum(ws, nblk, 2, sums, s);
}

SSAMD_API int ssamd_l1pair_bwd(const float* p1, const float* p2, const float* tgt, const int64_t* lens, int B, int M,
                               int Mt, int C, const float* gscale, const float* count, float* g1, float* g2,
                               hipStream_t s) {
  long rows = (long)B * M;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(l1pair_bwd_kernel, dim3(grid_for(rows * C, 4)), dim3(256), 0, s, p1, p2, tgt, lens, M, Mt, C,
                     gscale, count, g1, g2, rows);
  return (int)hipGetLastError();
}

namespace {
// FastSpeech2 loss finalize (one block): the mel valid-element count (fixed-order sum of
// min(len, M) x C, or the external global count), the five loss terms and their total in the
// reference order mel + post + dur + pitch + energy (model/loss.py:91-93).
// out: [total, mel, post, pitch, energy, dur];  cnt_out[0] = the mel count (backward divisor)
__global__ void __launch_bounds__(256) fs2_loss_final_kernel(const float* __restrict__ l1sums,
                                                             const float* __restrict__ var3,
                                                             const int64_t* __restrict__ lens, int B, int M, int C,
                                                             const float* __restrict__ ext, float* __restrict__ out,
                                                             float* __restrict__ cnt_out) {
  __shared__ float red[256];
  float c = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) c += (float)(lens[b] < M ? lens[b] : M);
  red[threadIdx.x] = c;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float cnt = ext ? ext[0] : red[0] * (float)C;
    const float inv = 1.f / fmaxf(cnt, 1.f);
    const float mel = l1sums[0] * inv, post = l1sums[1] * inv;
    out[1] = mel;
    out[2] = post;
    out[3] = var3[0];
    out[4] = var3[1];
    out[5] = var3[2];
    out[0] = (((mel + post) + var3[2]) + var3[0]) + var3[1];
    cnt_out[0] = cnt;
  }
}
}  // namespace

SSAMD_API int ssamd_fs2_loss_final(const float* l1sums, const float* var3, const int64_t* lens, int B, int M, int C,
                                   const float* ext, float* out, float* cnt_out, hipStream_t s) {
  hipLaunchKernelGGL(fs2_loss_final_kernel, dim3(1), dim3(256), 0, s, l1sums, var3, lens, B, M, C, ext, out, cnt_out);
  return (int)hipGetLastError();
}

SSAMD_API long ssamd_clip_adam_ws(long n) { return 1L + grid_for(n, 16); }

// ws: ssamd_clip_adam_ws(n) floats (ws[0] = global sum of squares, ws[1..] = block partials)
SSAMD_API int ssamd_clip_adam(float* p, const float* g, float* m, float* v, long n, float* ws, float clip, float lr,
                              float b1, float b2, float eps, float wd, int step, float* norm_out, long long* skipped,
                              hipStream_t s) {
  const int nblk = grid_for(n, 16);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, s, g, n, ws + 1);
  ssamd_small_sum(ws + 1, nblk, 1, ws, s);
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = 1.f - powf(b2, (float)step);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, 8)), dim3(256), 0, s, p, g, m, v, n, ws, clip, lr, b1, b2, eps, wd,
                     bc1, sqrtf(bc2), norm_out, skipped);
  return (int)hipGetLastError();
}

namespace {
__global__ void __launch_bounds__(256) relu_mask_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                        bf16_t* __restrict__ out, long n) {
  const long n8 = n / 8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    short8 a = reinterpret_cast<const short8*>(dy)[i];
    short8 b = reinterpret_cast<const short8*>(y)[i];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = bf2f((bf16_t)b[k]) > 0.f ? a[k] : (short)0;
    reinterpret_cast<short8*>(out)[i] = a;
  }
  for (long i = n8 * 8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = bf2f(y[i]) > 0.f ? dy[i] : (bf16_t)0;
}
}  // namespace

SSAMD_API int ssamd_relu_mask(const bf16_t* dy, const bf16_t* y, bf16_t* out, long n, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(relu_mask_kernel, dim3(grid_for(n, 8)), dim3(256), 0, s, dy, y, out, n);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------
// Batched weight-image refresh: ONE launch re-derives every bf16 operand image of
// every weight after an optimizer step (instead of one cast/permute kernel per weight).
//   mode 0: conv fwd   [Cout][ks][Cin]  <- fp32 [Cout][Cin][ks]   (Linear: ks = 1, plain cast)
//   mode 1: conv dgrad [Cin][ks][Cout]  <- fp32 [Cout][Cin][ks], taps flipped (Linear: transpose)
// ----------------------------------------------------------------------------
struct WDesc {
  const float* src;
  bf16_t* dst;
  int cout, cin, ks, mode;
};

namespace {
__global__ void __launch_bounds__(256) weight_prep_kernel(const WDesc* __restrict__ tab, const long* __restrict__ cum,
                                                          int n, long total) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    int lo = 0, hi = n;  // last d with cum[d] <= e
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (cum[mid] <= e) lo = mid; else hi = mid; }
    const WDesc d = tab[lo];
    const long i = e - cum[lo];
    long src;
    if (d.mode == 0) {  // dst [co][tap][ci]
      const int ci = (int)(i % d.cin);
      const long r = i / d.cin;
      const int tap = (int)(r % d.ks);
      const int co = (int)(r / d.ks);
      src = ((long)co * d.cin + ci) * d.ks + tap;
    } else {  // dst [ci][tap'][co], tap = ks-1-tap'
      const int co = (int)(i % d.cout);
      const long r = i / d.cout;
      const int tp = (int)(r % d.ks);
      const int ci = (int)(r / d.ks);
      src = ((long)co * d.cin + ci) * d.ks + (d.ks - 1 - tp);
    }
    d.dst[i] = f2bf(d.src[src]);
  }
}
}  // namespace

namespace {
// Tiled variant: one block per 64 (cout) x 64 (j = cin*ks + tap) tile of one weight, staged in LDS, so
// both the fp32 reads (along j) and the transposed dgrad-image writes (along cout) are coalesced.
__global__ void __launch_bounds__(256) weight_prep_tiled_kernel(const WDesc* __restrict__ tab,
                                                                const int4* __restrict__ tiles) {
  __shared__ float t[64][65];
  const int4 tl = tiles[blockIdx.x];
  const WDesc d = tab[tl.x];
  const int co0 = tl.y, j0 = tl.z;
  const int K = d.cin * d.ks;
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int r = e >> 6, c = e & 63;
    const int co = co0 + r, j = j0 + c;
    t[r][c] = (co < d.cout && j < K) ? d.src[(long)co * K + j] : 0.f;
  }
  __syncthreads();
  if (d.mode == 1) {  // dgrad image [cin][ks - 1 - tap][cout]: consecutive threads -> consecutive cout
    for (int e = threadIdx.x; e < 4096; e += 256) {
      const int jr = e >> 6, c = e & 63;
      const int co = co0 + c, j = j0 + jr;
      if (co >= d.cout || j >= K) continue;
      const int ci = j / d.ks, tap = j - ci * d.ks;
      d.dst[((long)ci * d.ks + (d.ks - 1 - tap)) * d.cout + co] = f2bf(t[c][jr]);
    }
  } else {  // forward image [cout][tap][cin]
    for (int e = threadIdx.x; e < 4096; e += 256) {
      const int r = e >> 6, c = e & 63;
      const int co = co0 + r, j = j0 + c;
      if (co >= d.cout || j >= K) continue;
      const int ci = j / d.ks, tap = j - ci * d.ks;
      d.dst[(long)co * K + (long)tap * d.cin + ci] = f2bf(t[r][c]);
    }
  }
}
}  // namespace

// ----------------------------------------------------------------------------
// Clip + Adam that also writes the bf16 operand images (replaces adam_kernel + weight_prep after
// every step).  Blocks [0, ntiles): one 64 (cout) x 64 (j = cin*ks + tap) tile of an image-bearing
// weight -- p / g / m / v read coalesced along j, updated exactly as adam_kernel, the new fp32 tile
// staged in LDS and written as the forward image [cout][tap][cin] and/or the dgrad image
// [cin][ks-1-tap][cout] (same layouts and rounding as weight_prep_tiled_kernel).  Blocks past
// ntiles: the remaining arena elements (biases, norms, embeddings), listed as ranges.
// ----------------------------------------------------------------------------
struct AdamImg {
  long off;       // arena element offset of the weight [cout][cin][ks]
  bf16_t* fwd;    // forward image or null
  bf16_t* dgrad;  // dgrad image or null
  int cout, cin, ks, pad_;
};

namespace {

__global__ void __launch_bounds__(256) adam_img_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       const float* __restrict__ ss, float clip, float lr, float b1,
                                                       float b2, float eps, float wd, float bc1, float bc2_sqrt,
                                                       float* __restrict__ norm_out, long long* __restrict__ skipped,
                                                       const AdamImg* __restrict__ wt, const int4* __restrict__ tiles,
                                                       int ntiles, const long* __restrict__ rcum,
                                                       const long* __restrict__ rstart, int nr, long rtotal) {
  const float norm = sqrtf(*ss);
  if (!isfinite(norm)) {  // skipped step: parameters and their images stay as they are
    if (blockIdx.x == 0 && threadIdx.x == 0) { *norm_out = norm; *skipped += 1; }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *norm_out = norm;
  const float coef = clip > 0.f ? fminf(1.f, clip / (norm + 1e-6f)) : 1.f;
  const float step = lr / bc1;
  if ((int)blockIdx.x < ntiles) {
    __shared__ float t[64][65];
    const int4 tl = tiles[blockIdx.x];
    const AdamImg d = wt[tl.x];
    const int co0 = tl.y, j0 = tl.z;
    const int K = d.cin * d.ks;
    for (int e = threadIdx.x; e < 4096; e += 256) {
      const int r = e >> 6, c = e & 63;
      const int co = co0 + r, j = j0 + c;
      float nv = 0.f;
      if (co < d.cout && j < K) {
        const long i = d.off + (long)co * K + j;
        float mk = m[i], vk = v[i];
        nv = adam_upd(p[i], g[i], mk, vk, coef, wd, b1, b2, step, bc2_sqrt, eps);
        p[i] = nv;
        m[i] = mk;
        v[i] = vk;
      }
      t[r][c] = nv;
    }
    __syncthreads();
    if (d.dgrad) {  // [cin][ks - 1 - tap][cout]: consecutive threads -> consecutive cout
      for (int e = threadIdx.x; e < 4096; e += 256) {
        const int jr = e >> 6, c = e & 63;
        const int co = co0 + c, j = j0 + jr;
        if (co >= d.cout || j >= K) continue;
        const int ci = j / d.ks, tap = j - ci * d.ks;
        d.dgrad[((long)ci * d.ks + (d.ks - 1 - tap)) * d.cout + co] = f2bf(t[c][jr]);
      }
    }
    if (d.fwd) {  // [cout][tap][cin]
      for (int e = threadIdx.x; e < 4096; e += 256) {
        const int r = e >> 6, c = e & 63;
        const int co = co0 + r, j = j0 + c;
        if (co >= d.cout || j >= K) continue;
        const int ci = j / d.ks, tap = j - ci * d.ks;
        d.fwd[(long)co * K + (long)tap * d.cin + ci] = f2bf(t[r][c]);
      }
    }
    return;
  }
  // remaining elements: rest index e -> range r (rcum[r] <= e < rcum[r+1]) -> arena rstart[r] + e - rcum[r]
  const long nthr = (long)(gridDim.x - ntiles) * blockDim.x;
  for (long e = (long)(blockIdx.x - ntiles) * blockDim.x + threadIdx.x; e < rtotal; e += nthr) {
    int lo = 0, hi = nr;
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (rcum[mid] <= e) lo = mid; else hi = mid; }
    const long i = rstart[lo] + (e - rcum[lo]);
    float mk = m[i], vk = v[i];
    p[i] = adam_upd(p[i], g[i], mk, vk, coef, wd, b1, b2, step, bc2_sqrt, eps);
    m[i] = mk;
    v[i] = vk;
  }
}
}  // namespace

// clip + Adam + image refresh (see adam_img_kernel); ws as ssamd_clip_adam
SSAMD_API int ssamd_clip_adam_img(float* p, const float* g, float* m, float* v, long n, float* ws, float clip, float lr,
                                  float b1, float b2, float eps, float wd, int step, float* norm_out,
                                  long long* skipped, const void* wtab, const void* tiles, int ntiles,
                                  const long* rcum, const long* rstart, int nr, long rtotal, hipStream_t s) {
  const int nblk = grid_for(n, 16);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, s, g, n, ws + 1);
  ssamd_small_sum(ws + 1, nblk, 1, ws, s);
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = 1.f - powf(b2, (float)step);
  const int rblocks = rtotal > 0 ? (int)std::min<long>((long)cdiv(rtotal, 256L * 4), 2048L) : 0;
  if (ntiles + rblocks == 0) return 0;
  hipLaunchKernelGGL(adam_img_kernel, dim3(ntiles + rblocks), dim3(256), 0, s, p, g, m, v, ws, clip, lr, b1, b2, eps,
                     wd, bc1, sqrtf(bc2), norm_out, skipped, reinterpret_cast<const AdamImg*>(wtab),
                     reinterpret_cast<const int4*>(tiles), ntiles, rcum, rstart, nr, rtotal);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_weight_prep_tiled(const void* table, const void* tiles, int ntiles, hipStream_t s) {
  if (ntiles == 0) return 0;
  hipLaunchKernelGGL(weight_prep_tiled_kernel, dim3(ntiles), dim3(256), 0, s, reinterpret_cast<const WDesc*>(table),
                     reinterpret_cast<const int4*>(tiles));
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_weight_prep(const void* table, const long* cum, int n, long total, hipStream_t s) {
  if (n == 0 || total == 0) return 0;
  hipLaunchKernelGGL(weight_prep_kernel, dim3(grid_for(total, 4)), dim3(256), 0, s,
                     reinterpret_cast<const WDesc*>(table), cum, n, total);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------
// Fused variance losses (reference model/loss.py:76-89): the masked MSE of pitch, energy
// and log-duration in one pass.  Each term k reads pred_k [B, L_k] (row stride ldp_k), its target
// (fp32, or int64 durations -> log(d + 1), row stride ldt_k) and its pad mask (bool [B, L_k],
// true = padded).  Pass 1: per-block partial (sum, count) for the 3 terms; pass 2 (one block):
// fixed-order sums, loss_k = sum_k / max(count_k, 1) with count_k from the masks or given
// (the all-reduced global counts under data parallelism).  Backward: d pred_k = 2 g_k (pred - t)
// * valid / count_k.  Deterministic, no atomics.
// ----------------------------------------------------------------------------
struct VTerm {
  const float* pred;
  const void* tgt;
  const bool* mask;
  float* grad;
  int L, ldp, ldt, dur;
};

namespace {
__device__ __forceinline__ float vterm_diff(const VTerm& t, int b, int j, bool& valid) {
  valid = !t.mask[(long)b * t.L + j];
  if (!valid) return 0.f;
  const float p = t.pred[(long)b * t.ldp + j];
  const float y = t.dur ? logf((float)reinterpret_cast<const int64_t*>(t.tgt)[(long)b * t.ldt + j] + 1.f)
                        : reinterpret_cast<const float*>(t.tgt)[(long)b * t.ldt + j];
  return p - y;
}

__global__ void __launch_bounds__(256) var_loss_fwd_kernel(VTerm t0, VTerm t1, VTerm t2, int B,
                                                           float* __restrict__ part) {
  const VTerm ts[3] = {t0, t1, t2};
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const long n0 = (long)B * t0.L, n1 = n0 + (long)B * t1.L, n2 = n1 + (long)B * t2.L;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n2; e += (long)gridDim.x * 256) {
    const int k = e < n0 ? 0 : (e < n1 ? 1 : 2);
    const long o = e - (k == 0 ? 0 : (k == 1 ? n0 : n1));
    const int L = ts[k].L;
    const int b = (int)(o / L), j = (int)(o - (long)b * L);
    bool valid;
    const float d = vterm_diff(ts[k], b, j, valid);
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q == k) {
        acc[q] += d * d;
        acc[3 + q] += valid ? 1.f : 0.f;
      }
  }
  __shared__ float red[6][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const float v = wave_sum(acc[q]);
    if (lane == 0) red[q][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = (red[threadIdx.x][0] + red[threadIdx.x][1]) +
                                                             (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

__global__ void __launch_bounds__(256) var_loss_final_kernel(const float* __restrict__ part, int nblk,
                                                             const float* __restrict__ ext_counts,
                                                             float* __restrict__ loss, float* __restrict__ counts) {
  __shared__ float red[6][256];
  float a[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int r = threadIdx.x; r < nblk; r += 256)
#pragma unroll
    for (int q = 0; q < 6; ++q) a[q] += part[r * 6 + q];
#pragma unroll
  for (int q = 0; q < 6; ++q) red[q][threadIdx.x] = a[q];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
#pragma unroll
      for (int q = 0; q < 6; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 3) {
    const float c = ext_counts ? ext_counts[threadIdx.x] : red[3 + threadIdx.x][0];
    counts[threadIdx.x] = c;
    loss[threadIdx.x] = red[threadIdx.x][0] / fmaxf(c, 1.f);
  }
}

__global__ void __launch_bounds__(256) var_loss_bwd_kernel(VTerm t0, VTerm t1, VTerm t2, int B,
                                                           const float* __restrict__ g,
                                                           const float* __restrict__ counts) {
  const VTerm ts[3] = {t0, t1, t2};
  float sc[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) sc[q] = 2.f * g[q] / fmaxf(counts[q], 1.f);
  const long n0 = (long)B * t0.L, n1 = n0 + (long)B * t1.L, n2 = n1 + (long)B * t2.L;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n2; e += (long)gridDim.x * 256) {
    const int k = e < n0 ? 0 : (e < n1 ? 1 : 2);
    const long o = e - (k == 0 ? 0 : (k == 1 ? n0 : n1));
    const int L = ts[k].L;
    const int b = (int)(o / L), j = (int)(o - (long)b * L);
    bool valid;
    const float d = vterm_diff(ts[k], b, j, valid);
    const float s = k == 0 ? sc[0] : (k == 1 ? sc[1] : sc[2]);
    ts[k].grad[(long)b * ts[k].ldp + j] = valid ? s * d : 0.f;
  }
}
}  // namespace

SSAMD_API long ssamd_var_loss_ws() { return 6L * 1024; }

// loss[3] = masked MSE of the 3 terms; counts[3] = the divisors used (ext_counts or mask counts)
SSAMD_API int ssamd_var_loss_fwd(VTerm t0, VTerm t1, VTerm t2, int B, const float* ext_counts, float* loss,
                                 float* counts, float* ws, hipStream_t s) {
  const long n = (long)B * (t0.L + t1.L + t2.L);
  const int nblk = n ? (grid_for(n, 4) > 1024 ? 1024 : grid_for(n, 4)) : 1;
  hipLaunchKernelGGL(var_loss_fwd_kernel, dim3(nblk), dim3(256), 0, s, t0, t1, t2, B, ws);
  hipLaunchKernelGGL(var_loss_final_kernel, dim3(1), dim3(256), 0, s, ws, nblk, ext_counts, loss, counts);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_var_loss_bwd(VTerm t0, VTerm t1, VTerm t2, int B, const float* g, const float* counts,
                                 hipStream_t s) {
  const long n = (long)B * (t0.L + t1.L + t2.L);
  if (n == 0) return 0;
  hipLaunchKernelGGL(var_loss_bwd_kernel, dim3(grid_for(n, 4)), dim3(256), 0, s, t0, t1, t2, B, g, counts);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------
// Inference duration rounding (reference model/modules.py:132-137):
//   d = max(round(exp(log_d) - 1), 0);  d = max(round(d * control), 0);  d = 0 at t >= len[b]
// and mel_len[b] = sum_t d -- one block per utterance, the row sum in a fixed order.
// control: null (1.0), one scalar (ctl_stride 0) or a [B, T] per-phoneme factor (word-level control).
// torch.round / rintf both round half to even.
// ----------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(256) duration_round_kernel(const float* __restrict__ log_d,
                                                             const float* __restrict__ ctl, int ctl_per_elem,
                                                             const int64_t* __restrict__ lens, int T,
                                                             int64_t* __restrict__ d_out, int64_t* __restrict__ mel_len) {
  __shared__ long long red[256];
  const int b = blockIdx.x;
  const int len = lens ? (int)lens[b] : T;
  long long s = 0;
  for (int t = threadIdx.x; t < T; t += 256) {
    long long d = 0;
    if (t < len) {
      float v = fmaxf(rintf(expf(log_d[(long)b * T + t]) - 1.f), 0.f);
      if (ctl) v = fmaxf(rintf(v * (ctl_per_elem ? ctl[(long)b * T + t] : ctl[0])), 0.f);
      d = (long long)v;
    }
    d_out[(long)b * T + t] = d;
    s += d;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) mel_len[b] = red[0];
}

// Sequence mean pool (reference model/modules.py:396: enc_seq.mean(dim=1) over the padded length; SURVEY
// K16): out[b, c] = sum_{t < rows_b} x[row(b, t), c] / div.  Padded layout (cu null): rows_b = L, row =
// b*L + t.  Packed layout: sequence b owns rows cu[b] .. cu[b+1]-1.  One block per (b, 64-column tile),
// 4 row lanes summed in order then combined in order: deterministic.
__global__ void __launch_bounds__(256) seq_mean_kernel(const bf16_t* __restrict__ x, const int64_t* __restrict__ cu,
                                                       int L, int C, float div, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int b = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), lane_r = threadIdx.x >> 6;
  const long r0 = cu ? cu[b] : (long)b * L;
  const long r1 = cu ? cu[b + 1] : r0 + L;
  float s = 0.f;
  if (c < C)
    for (long r = r0 + lane_r; r < r1; r += 4) s += bf2f(x[r * C + c]);
  red[lane_r][threadIdx.x & 63] = s;
  __syncthreads();
  if (lane_r == 0 && c < C) out[(long)b * C + c] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) +
                                                    (red[2][threadIdx.x] + red[3][threadIdx.x])) / div;
}

// backward: dx[row(b, t), c] = g[b, c] / div for every row of sequence b (padded: all L rows).
__global__ void __launch_bounds__(256) seq_mean_bwd_kernel(const float* __restrict__ g, const int64_t* __restrict__ cu,
                                                           int B, int L, int C, float div, bf16_t* __restrict__ dx,
                                                           long rows) {
  const int c8n = C / 8;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < rows * c8n; e += (long)gridDim.x * 256) {
    const long r = e / c8n;
    const int c0 = (int)(e - r * c8n) * 8;
    int b;
    if (cu) {  // sequence of packed row r (B is small: binary search over the offsets)
      int lo = 0, hi = B;
      while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (cu[mid] <= r) lo = mid; else hi = mid; }
      b = lo;
    } else {
      b = (int)(r / L);
    }
    short8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (short)f2bf(g[(long)b * C + c0 + i] / div);
    *reinterpret_cast<short8*>(dx + r * C + c0) = o;
  }
}

// Per-utterance row vector add (the speaker embedding, reference model/fastspeech2.py:74-77):
//   out[b, t, :] = x[b, t, :] + table[ids[b], :]      (bf16 out, fp32 table)
__global__ void __launch_bounds__(256) add_rowvec_kernel(const bf16_t* __restrict__ x, const float* __restrict__ table,
                                                         const int64_t* __restrict__ ids, int L, int C,
                                                         bf16_t* __restrict__ out, long rows) {
  const int c8n = C / 8;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < rows * c8n; e += (long)gridDim.x * 256) {
    const long r = e / c8n;
    const int c0 = (int)(e - r * c8n) * 8;
    const float* tv = table + (ids ? ids[r / L] : r / L) * (long)C + c0;  // ids null: row b of table
    const short8 v = *reinterpret_cast<const short8*>(x + r * C + c0);
    short8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (short)f2bf(bf2f((bf16_t)v[i]) + tv[i]);
    *reinterpret_cast<short8*>(out + r * C + c0) = o;
  }
}

// dtable[v, c] = sum over utterances b with ids[b] == v (in b order) of S[b, c] (S = per-utterance row sums)
__global__ void __launch_bounds__(256) rowvec_grad_kernel(const float* __restrict__ S, const int64_t* __restrict__ ids,
                                                          int B, int C, float* __restrict__ dtable) {
  const int v = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b)
    if (ids[b] == v) s += S[(long)b * C + c];
  dtable[(long)v * C + c] = s;
}
}  // namespace

SSAMD_API int ssamd_duration_round(const float* log_d, const float* ctl, int ctl_per_elem, const int64_t* lens, int B,
                                   int T, int64_t* d_out, int64_t* mel_len, hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(duration_round_kernel, dim3(B), dim3(256), 0, s, log_d, ctl, ctl_per_elem, lens, T, d_out,
                     mel_len);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_seq_mean(const bf16_t* x, const int64_t* cu, int B, int L, int C, float div, float* out,
                             hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(seq_mean_kernel, dim3(cdiv(C, 64), B), dim3(256), 0, s, x, cu, L, C, div, out);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_seq_mean_bwd(const float* g, const int64_t* cu, int B, int L, int C, float div, bf16_t* dx,
                                 long rows, hipStream_t s) {
  if (C % 8) return -1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(seq_mean_bwd_kernel, dim3(grid_for(rows * (C / 8))), dim3(256), 0, s, g, cu, B, L, C, div, dx,
                     rows);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_add_rowvec(const bf16_t* x, const float* table, const int64_t* ids, int B, int L, int C,
                               bf16_t* out, hipStream_t s) {
  if (C % 8) return -1;
  const long rows = (long)B * L;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(add_rowvec_kernel, dim3(grid_for(rows * (C / 8))), dim3(256), 0, s, x, table, ids, L, C, out,
                     rows);
  return (int)hipGetLastError();
}

// dtable [V, C] (overwritten) from dout [B, L, C]: per-utterance fixed-order row sums, then per-row gather
SSAMD_API int ssamd_rowvec_grad(const bf16_t* dout, const int64_t* ids, int B, int L, int C, int V, float* dtable,
                                float* ws, long ws_floats, hipStream_t s) {
  if ((long)B * C > ws_floats) return -3;
  int rc = ssamd_seq_mean(dout, nullptr, B, L, C, 1.f, ws, s);  // S[b] = sum_t dout[b, t]
  if (rc) return rc;
  hipLaunchKernelGGL(rowvec_grad_kernel, dim3(cdiv(C, 256), V), dim3(256), 0, s, ws, ids, B, C, dtable);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------
// Packed <-> padded row layouts (ops/packing.py) without torch gather / scatter:
//   pack:    out[r] = x[dst[r]] (+ pe[dst[r] % M])                bf16 [R, C]
//   unpack:  out[b*M + t] = t < lens[b] ? src[cu[b] + t] : fill   bf16 or fp32 [B*M, C]
//   pad_colsum: per-block partial column sums of dout over the padded rows only (the gradient
//   of the fill row), finished by a fixed-order column sum.
// ----------------------------------------------------------------------------
namespace {
template <typename T>
__device__ __forceinline__ float ld_as_f(const T* p);
template <>
__device__ __forceinline__ float ld_as_f<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld_as_f<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T>
__device__ __forceinline__ void st_from_f(T* p, float v);
template <>
__device__ __forceinline__ void st_from_f<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void st_from_f<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// 8 consecutive channels as fp32: one 16-B access for bf16 rows, two for fp32 rows (16/32-B aligned: C % 8 == 0)
__device__ __forceinline__ void ld8f(const bf16_t* p, float* v) {
  const short8 x = *reinterpret_cast<const short8*>(p);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = bf2f((bf16_t)x[q]);
}
__device__ __forceinline__ void ld8f(const float* p, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8f(bf16_t* p, const float* v) {
  short8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = (short)f2bf(v[q]);
  *reinterpret_cast<short8*>(p) = o;
}
__device__ __forceinline__ void st8f(float* p, const float* v) {
  reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}

template <typename T>
__global__ void __launch_bounds__(256) pack_rows_kernel(const T* __restrict__ x, const int64_t* __restrict__ dst,
                                                        const bf16_t* __restrict__ pe, int M, long R, int C,
                                                        T* __restrict__ out) {
  const int c8n = C / 8;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < R * c8n; e += (long)gridDim.x * 256) {
    const long r = e / c8n;
    const int c0 = (int)(e - r * c8n) * 8;
    const long s = dst[r];
    const T* xs = x + s * C + c0;
    T* o = out + r * C + c0;
    float v[8];
    ld8f(xs, v);
    if (pe) {
      float pv[8];
      ld8f(pe + (s % M) * C + c0, pv);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += pv[i];
    }
    st8f(o, v);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) unpack_rows_kernel(const T* __restrict__ src, const int64_t* __restrict__ cu,
                                                          const int64_t* __restrict__ lens, const float* __restrict__ fill,
                                                          int M, int C, long rows, T* __restrict__ out) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < rows * C; e += (long)gridDim.x * 256) {
    const long row = e / C;
    const int c = (int)(e - row * C);
    const int b = (int)(row / M), t = (int)(row - (long)b * M);
    float v = fill ? fill[c] : 0.f;
    if (t < lens[b]) v = ld_as_f<T>(src + (cu[b] + t) * C + c);
    st_from_f<T>(out + e, v);
  }
}

// Between two packed layouts of the same sequences: output row i is (b, t) = divmod(dst_out[i], M_out);
// it takes source row cu_src[b] + t when t < lens_src[b] (else 0), plus pe[t] when given.  8 channels
// per thread (16-B bf16 / 2x16-B fp32 accesses).
template <typename T>
__global__ void __launch_bounds__(256) repack_rows_kernel(const T* __restrict__ src, const int64_t* __restrict__ cu_src,
                                                          const int64_t* __restrict__ lens_src,
                                                          const int64_t* __restrict__ dst_out, int M_out, long rows,
                                                          int C, const bf16_t* __restrict__ pe, T* __restrict__ out) {
  const int c8n = C / 8;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < rows * c8n; e += (long)gridDim.x * 256) {
    const long i = e / c8n;
    const int c0 = (int)(e - i * c8n) * 8;
    const long d = dst_out[i];
    const int b = (int)(d / M_out), t = (int)(d - (long)b * M_out);
    const bool ok = t < lens_src[b];
    T* o = out + i * C + c0;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (ok) ld8f(src + (cu_src[b] + t) * C + c0, v);
    if (pe) {
      float pv[8];
      ld8f(pe + (long)t * C + c0, pv);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += pv[q];
    }
    st8f(o, v);
  }
}

// block = 64 columns x 4 row lanes over a 256-row chunk: coalesced 64-column row pieces, 64 rows
// per thread, lanes combined in LDS in a fixed order
template <typename T>
__global__ void __launch_bounds__(256) pad_colsum_kernel(const T* __restrict__ dout, const int64_t* __restrict__ lens,
                                                         int M, int C, long rows, int rows_per_blk,
                                                         float* __restrict__ part) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const long r0 = (long)blockIdx.y * rows_per_blk, r1 = min(rows, r0 + rows_per_blk);
  float s = 0.f;
  if (c < C && r0 + rl < r1) {
    // (sequence, position) of the first row once, then stepped: no 64-bit division per row
    long row = r0 + rl;
    int b = (int)(row / M), t = (int)(row - (long)b * M);
    int lb = (int)lens[b];
    for (; row < r1; row += 4) {
      if (t >= lb) s += ld_as_f<T>(dout + row * C + c);
      t += 4;
      while (t >= M) {
        t -= M;
        ++b;
        if (row + 4 < r1) lb = (int)lens[b];
      }
    }
  }
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && c < C) part[(long)blockIdx.y * C + c] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}
}  // namespace

// f32: 1 = fp32 rows, 0 = bf16 rows; pe (bf16 [>=M, C]) optional
SSAMD_API int ssamd_pack_rows(const void* x, const int64_t* dst, const bf16_t* pe, int M, long R, int C, int f32,
                              void* out, hipStream_t s) {
  if (C % 8) return -1;
  if (R == 0) return 0;
  const int g = grid_for(R * (C / 8));
  if (f32)
    hipLaunchKernelGGL(pack_rows_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)x, dst, pe, M, R, C,
                       (float*)out);
  else
    hipLaunchKernelGGL(pack_rows_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)x, dst, pe, M, R, C,
                       (bf16_t*)out);
  return (int)hipGetLastError();
}

// f32: 1 = fp32 rows, 0 = bf16 rows; pe (bf16 [>= max t + 1, C]) optional
SSAMD_API int ssamd_repack_rows(const void* src, const int64_t* cu_src, const int64_t* lens_src, const int64_t* dst_out,
                                int M_out, long rows, int C, const bf16_t* pe, int f32, void* out, hipStream_t s) {
  if (C % 8) return -1;
  if (rows == 0) return 0;
  const int g = grid_for(rows * (C / 8));
  if (f32)
    hipLaunchKernelGGL(repack_rows_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)src, cu_src, lens_src, dst_out,
                       M_out, rows, C, pe, (float*)out);
  else
    hipLaunchKernelGGL(repack_rows_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)src, cu_src, lens_src,
                       dst_out, M_out, rows, C, pe, (bf16_t*)out);
  return (int)hipGetLastError();
}

// f32: 1 = fp32 rows, 0 = bf16 rows
SSAMD_API int ssamd_unpack_rows(const void* src, const int64_t* cu, const int64_t* lens, const float* fill, int B, int M,
                                int C, int f32, void* out, hipStream_t s) {
  const long rows = (long)B * M;
  if (rows == 0) return 0;
  const int g = grid_for(rows * C);
  if (f32)
    hipLaunchKernelGGL(unpack_rows_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)src, cu, lens, fill, M, C,
                       rows, (float*)out);
  else
    hipLaunchKernelGGL(unpack_rows_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)src, cu, lens, fill, M, C,
                       rows, (bf16_t*)out);
  return (int)hipGetLastError();
}

SSAMD_API long ssamd_pad_colsum_ws(int B, int M, int C) { return (long)cdiv((long)B * M, 256) * C + seg_colsum_ws(1, C); }

// dfill[c] = sum over padded rows (t >= lens[b]) of dout[b*M + t, c]; fixed order
SSAMD_API int ssamd_pad_colsum(const void* dout, int f32, const int64_t* lens, int B, int M, int C, float* dfill,
                               float* ws, long ws_floats, hipStream_t s) {
  const long rows = (long)B * M;
  if (rows == 0) return (int)hipMemsetAsync(dfill, 0, C * sizeof(float), s);
  const int chunks = cdiv(rows, 256);
  if (ws_floats < ssamd_pad_colsum_ws(B, M, C)) return -3;
  dim3 grid(cdiv(C, 64), chunks);
  if (f32)
    hipLaunchKernelGGL(pad_colsum_kernel<float>, grid, dim3(256), 0, s, (const float*)dout, lens, M, C, rows, 256, ws);
  else
    hipLaunchKernelGGL(pad_colsum_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)dout, lens, M, C, rows, 256,
                       ws);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  return ssamd_seg_colsum(ws, C, 1, chunks, C, dfill, 0, 0, C, nullptr, ws + (long)chunks * C, seg_colsum_ws(1, C), s);
}

// ----------------------------------------------------------------------------
// FiLM parameter gradients of one LayerNorm site (reference model/blocks.py:43-62):
//   d gamma = S1 * s_g,  d beta = S2 * s_b            (bf16 or fp32 [n])
//   d s_g = sum(S1 * gamma),  d s_b = sum(S2 * beta)   (scalars, fixed-order block reduction)
// S1 / S2 = per-(b, c) sums from the LayerNorm backward.  accum != 0: d gamma / d beta
// are added to (running sums over the sites that share gamma / beta, in backward order on one
// stream: deterministic) instead of one gradient per site summed by autograd.  l2_sg / l2_sb (optional):
// this site's entries of the FiLM L2 term's gradient (ops/hip.py film_scalars_cat), folded into the
// scalar gradients so each scalar gets ONE gradient, written straight into its arena slot.
// ----------------------------------------------------------------------------
namespace {
// Many 256-thread blocks, one float4 group per thread (one 1024-thread block looping over n was
// ~24 us per site, latency-bound on one CU); each block writes its two partial sums, a one-block
// finish adds them in a fixed order (deterministic) and folds in the L2 term.
constexpr int FG_T = 256;
__global__ void __launch_bounds__(FG_T) film_grads_kernel(const float* __restrict__ S1, const float* __restrict__ S2,
                                                          const float* __restrict__ g, const float* __restrict__ bt,
                                                          const float* __restrict__ sg, const float* __restrict__ sb,
                                                          int n, int out_f32, void* __restrict__ dg,
                                                          void* __restrict__ dbt, float* __restrict__ part, int accum) {
  __shared__ float red[2][FG_T / 64];
  const float a = *sg, c = *sb;
  const int tid = threadIdx.x;
  const int i = 4 * (blockIdx.x * FG_T + tid);
  float s1 = 0.f, s2 = 0.f;
  if (i < n) {  // n % 4 == 0 (host check)
    const float4 x1 = *reinterpret_cast<const float4*>(S1 + i);
    const float4 x2 = *reinterpret_cast<const float4*>(S2 + i);
    const float4 gg = *reinterpret_cast<const float4*>(g + i);
    const float4 bb = *reinterpret_cast<const float4*>(bt + i);
    float4 o1 = make_float4(0.f, 0.f, 0.f, 0.f), o2 = o1;
    if (accum) {
      if (out_f32) {
        o1 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dg) + i);
        o2 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dbt) + i);
      } else {
        const short4v p1 = *reinterpret_cast<const short4v*>(reinterpret_cast<const bf16_t*>(dg) + i);
        const short4v p2 = *reinterpret_cast<const short4v*>(reinterpret_cast<const bf16_t*>(dbt) + i);
        o1 = make_float4(bf2f((bf16_t)p1[0]), bf2f((bf16_t)p1[1]), bf2f((bf16_t)p1[2]), bf2f((bf16_t)p1[3]));
        o2 = make_float4(bf2f((bf16_t)p2[0]), bf2f((bf16_t)p2[1]), bf2f((bf16_t)p2[2]), bf2f((bf16_t)p2[3]));
      }
    }
    // accumulate rounds like autograd's add of per-site gradients (fp32 add, one rounding)
    const float4 r1 = make_float4(o1.x + x1.x * a, o1.y + x1.y * a, o1.z + x1.z * a, o1.w + x1.w * a);
    const float4 r2 = make_float4(o2.x + x2.x * c, o2.y + x2.y * c, o2.z + x2.z * c, o2.w + x2.w * c);
    if (out_f32) {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(dg) + i) = r1;
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(dbt) + i) = r2;
    } else {
      const short4v q1 = {(short)f2bf(r1.x), (short)f2bf(r1.y), (short)f2bf(r1.z), (short)f2bf(r1.w)};
      const short4v q2 = {(short)f2bf(r2.x), (short)f2bf(r2.y), (short)f2bf(r2.z), (short)f2bf(r2.w)};
      *reinterpret_cast<short4v*>(reinterpret_cast<bf16_t*>(dg) + i) = q1;
      *reinterpret_cast<short4v*>(reinterpret_cast<bf16_t*>(dbt) + i) = q2;
    }
    s1 = x1.x * gg.x + x1.y * gg.y + x1.z * gg.z + x1.w * gg.w;
    s2 = x2.x * bb.x + x2.y * bb.y + x2.z * bb.z + x2.w * bb.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = s1;
    red[1][tid >> 6] = s2;
  }
  __syncthreads();
  if (tid == 0) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int w = 0; w < FG_T / 64; ++w) {
      t1 += red[0][w];
      t2 += red[1][w];
    }
    part[2 * blockIdx.x] = t1;
    part[2 * blockIdx.x + 1] = t2;
  }
}

__global__ void __launch_bounds__(256) film_grads_finish_kernel(const float* __restrict__ part, int nblk,
                                                                float* __restrict__ dsg, float* __restrict__ dsb,
                                                                const float* __restrict__ l2_sg,
                                                                const float* __restrict__ l2_sb) {
  __shared__ float red[2][256];
  const int tid = threadIdx.x;
  float t1 = 0.f, t2 = 0.f;
  for (int b = tid; b < nblk; b += 256) {
    t1 += part[2 * b];
    t2 += part[2 * b + 1];
  }
  red[0][tid] = t1;
  red[1][tid] = t2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) {
      red[0][tid] += red[0][tid + w];
      red[1][tid] += red[1][tid + w];
    }
    __syncthreads();
  }
  if (tid == 0) {  // + the FiLM L2 term's gradient of this site's scalars, when folded in
    dsg[0] = l2_sg ? red[0][0] + l2_sg[0] : red[0][0];
    dsb[0] = l2_sb ? red[1][0] + l2_sb[0] : red[1][0];
  }
}
}  // namespace

// per-device partial-sum buffer of the film_grads blocks (2 floats per block; stream-ordered reuse)
// partials buffer (caller-allocated, stream-ordered like every other workspace): 2 floats per block
SSAMD_API long ssamd_film_grads_ws(int n) { return n > 0 ? 2L * cdiv(n / 4, FG_T) : 0; }
SSAMD_API int ssamd_film_grads(const float* S1, const float* S2, const float* g, const float* bt, const float* sg,
                               const float* sb, int n, int out_f32, void* dg, void* dbt, float* dsg, float* dsb,
                               const float* l2_sg, const float* l2_sb, int accum, float* part, long part_floats,
                               hipStream_t s) {
  if (n % 4) return -2;
  const int nblk = n > 0 ? cdiv(n / 4, FG_T) : 0;
  if (part_floats < 2L * nblk || (nblk > 0 && !part)) return -3;
  if (nblk > 0)
    hipLaunchKernelGGL(film_grads_kernel, dim3(nblk), dim3(FG_T), 0, s, S1, S2, g, bt, sg, sb, n, out_f32, dg, dbt,
                       part, accum);
  hipLaunchKernelGGL(film_grads_finish_kernel, dim3(1), dim3(256), 0, s, part, nblk, dsg, dsb, l2_sg, l2_sb);
  return (int)hipGetLastError();
}

// Cross-stream ordering for the weight-gradient side stream: `waiter` waits for everything queued on
// `signaler` so far.  One event record + one stream wait from a per-device ring of pre-created
// timing-free events (a wait is bound to the record current at the time of the wait call, so a ring
// slot can be re-recorded while earlier waits are pending); replaces torch's Stream.wait_stream (a
// fresh Python Event object per call) on the per-layer backward path.
#include <mutex>
namespace {
constexpr int SW_DEV = 16, SW_RING = 64;
hipEvent_t g_sw_ev[SW_DEV][SW_RING];
int g_sw_next[SW_DEV];
bool g_sw_init[SW_DEV];
std::mutex g_sw_mu;
}  // namespace

SSAMD_API int ssamd_stream_wait(hipStream_t waiter, hipStream_t signaler) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= SW_DEV) return -2;
  std::lock_guard<std::mutex> lk(g_sw_mu);
  if (!g_sw_init[dev]) {
    for (int i = 0; i < SW_RING; ++i)
      if (hipEventCreateWithFlags(&g_sw_ev[dev][i], hipEventDisableTiming) != hipSuccess) return -3;
    g_sw_init[dev] = true;
  }
  hipEvent_t e = g_sw_ev[dev][g_sw_next[dev]];
  g_sw_next[dev] = (g_sw_next[dev] + 1) % SW_RING;
  if (hipEventRecord(e, signaler) != hipSuccess) return -4;
  return hipStreamWaitEvent(waiter, e, 0) == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------- multi-tensor device copy
// Up to 6 independent device-to-device copies in ONE launch (the static-input refresh of a HIP-graph replay:
// a batch-1 synthesis is launch-bound, each torch copy_ is a launch of its own).  blockIdx.y = copy index;
// 16-B vectors when source, destination and size are 16-B aligned, bytes otherwise.
struct MCopy {
  const unsigned char* s[6];
  unsigned char* d[6];
  long b[6];
};

__global__ void __launch_bounds__(256) multi_copy_kernel(MCopy m, int n) {
  const int t = blockIdx.y;
  if (t >= n) return;
  const unsigned char* s = m.s[t];
  unsigned char* d = m.d[t];
  const long nb = m.b[t];
  const long i0 = blockIdx.x * 256L + threadIdx.x, st = gridDim.x * 256L;
  if ((((uintptr_t)s | (uintptr_t)d | (uintptr_t)nb) & 15) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    uint4* d4 = reinterpret_cast<uint4*>(d);
    for (long i = i0; i < nb / 16; i += st) d4[i] = s4[i];
  } else {
    for (long i = i0; i < nb; i += st) d[i] = s[i];
  }
}

SSAMD_API int ssamd_multi_copy(int n, const void* s0, void* d0, long b0, const void* s1, void* d1, long b1,
                               const void* s2, void* d2, long b2, const void* s3, void* d3, long b3, const void* s4,
                               void* d4, long b4, const void* s5, void* d5, long b5, hipStream_t s) {
  if (n < 0 || n > 6) return -2;
  if (n == 0) return 0;
  MCopy m;
  const void* ss[6] = {s0, s1, s2, s3, s4, s5};
  void* dd[6] = {d0, d1, d2, d3, d4, d5};
  const long bb[6] = {b0, b1, b2, b3, b4, b5};
  long mx = 0;
  for (int i = 0; i < 6; ++i) {
    m.s[i] = static_cast<const unsigned char*>(ss[i]);
    m.d[i] = static_cast<unsigned char*>(dd[i]);
    m.b[i] = i < n ? bb[i] : 0;
    if (i < n && (bb[i] < 0 || (bb[i] > 0 && (!ss[i] || !dd[i])))) return -2;
    if (i < n) mx = std::max(mx, bb[i]);
  }
  const int gx = (int)std::max<long>(1L, std::min<long>((long)cdiv(mx, 256L * 16), 64L));
  hipLaunchKernelGGL(multi_copy_kernel, dim3(gx, n), dim3(256), 0, s, m, n);
  return (int)hipGetLastError();
}
