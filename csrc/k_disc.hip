// HiFi-GAN training kernels (reference hifigan/models.py:176-264 MPD / MSD / losses,
// hifigan/meldataset.py:49-72 mel_spectrogram, hifigan/train.py:113-160 the G / D steps).
//
// 1. sconv: conv1d with stride, dilation, groups and zero padding on channel-last bf16 activations
//    [B, T, C] -- every discriminator layer (MPD's (k, 1) Conv2d over [B, C, T/p, p] is a conv1d over T/p
//    for each of the p columns: sequences [B*p, T/p, C]), the generator's conv_post, and the STFT of the
//    mel loss (a stride-hop conv whose weights are the windowed DFT basis).  MFMA v_mfma_f32_16x16x32_bf16
//    on 64 x 64 x 64 tiles, 4 waves in a 2 x 2 grid of 32 x 32 sub-tiles, register-staged double-buffered
//    LDS (XOR-swizzled 128-B rows: conflict-free ds_read_b128 fragments and 16-B writes):
//      * forward:  y[b, t, g*Ng + n] = act(bias + sum_{j, c} W[g*Ng + n, c, j] x[b, t*s + j*d - p, g*Cg + c])
//        as an implicit GEMM over (b, t) x n with k = j*Cg + c gathered from x (im2col on the fly);
//      * data gradient (polyphase): for stride s the input rows of one residue r = (t_in + p) mod s see
//        only the taps j = r + s*u -- one block column per (group, residue), k = u*Ng + n, so a stride-256
//        STFT backward does 4 taps per row instead of 1024 mostly-zero ones;
//      * weight gradient: dW[g*Ng + n, c, j] = sum_{b, t} dz[b, t, g*Ng + n] x[b, t*s + j*d - p, g*Cg + c],
//        split over row ranges into fp32 slabs (no atomics) + a fixed-order reduce into the torch layout.
//        Both operands are row-major in the reduction dimension: the LDS tiles are read with
//        ds_read_b64_tr_b16 (hardware transpose) through an 8-B-chunk swizzle.
// 2. elementwise / loss kernels of the G and D steps: activation backward fused with the feature-matching
//    gradient, LSGAN losses with their gradients, L1 partial sums, AvgPool1d(4, 2, 2) fwd / bwd, the MPD
//    reflect-pad + period fold, the STFT input prep (reflect pad + fp32 -> bf16 hi/lo split) and its
//    backward, and the per-frame mel-L1 kernel (|X|, mel projection, log-clamp, L1 and the whole gradient
//    d loss / d (re, im) in one pass).
// All reductions are fixed-order (per-block partials, one finalising block): bitwise reproducible.
#include "common.h"

#include <algorithm>

namespace {

constexpr int SC_NT = 256;

struct SConvGeom {
  int B, Tin, Tout, Cin, Cout, G, Cg, Ng, ks, s, d, p;
  int K;    // ks * Cg: forward / weight-gradient reduction width per group (k = j * Cg + c)
  int Kp;   // forward weight-image row length (K rounded up to 8)
  int U;    // ceil(ks / s): taps per residue class (data gradient)
  int UNp;  // U * Ng rounded up to 8: one residue slice of the data-gradient image row
  int NQ;   // data-gradient rows per sequence and residue class
};

// [64][64] bf16 tile, 128-B rows, 16-B chunk c of row r stored at chunk c ^ ((r >> 1) & 7): the
// ds_read_b128 fragment reads (lane -> row lane & 15, chunk 4 * kk + (lane >> 4)) hit 16 distinct bank
// quads in every 16-lane group, and 8 lanes writing one row's 8 chunks cover 128 B
__device__ __forceinline__ int sw16(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// the same tile for ds_read_b64_tr_b16 reads (4 rows x 16 columns per 16-lane group): 8-B chunk c8 of row r
// at c8 ^ 4 * h(r), h = bits 1 and 3 of r -> rows {0..3, 8..11} (+4) x 4 chunks of a half-wave are distinct banks
__device__ __forceinline__ int sw8(int r, int c8) {
  return r * 128 + ((c8 ^ ((((r >> 1) & 1) | ((r >> 2) & 2)) << 2)) << 3);
}

__device__ __forceinline__ short4v ds_tr(const char* p) {
  typedef __attribute__((address_space(3))) short4v lds_s4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(__attribute__((address_space(3))) char*)(p));
}

__device__ __forceinline__ float lrelu_f(float v, float s) { return v >= 0.f ? v : v * s; }

// im2col element block: 8 consecutive k = j * Cg + c of output row (b, t) -> x[b, t*s + j*d - p, g*Cg + c]
// (xrow0 = b * Tin, tpos = t * s - p; zero outside [0, Tin) and past K)
template <bool VEC>
__device__ __forceinline__ short8 load_xcol(const bf16_t* __restrict__ x, const SConvGeom& q, int g, bool ok,
                                            int xrow0, int tpos, int k) {
  short8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!ok) return v;
  if constexpr (VEC) {
    if (k < q.K) {
      const int j = k / q.Cg, c = k - j * q.Cg;
      const int ti = tpos + j * q.d;
      if ((unsigned)ti < (unsigned)q.Tin) v = *reinterpret_cast<const short8*>(x + (long)(xrow0 + ti) * q.Cin + g * q.Cg + c);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = k + e;
      if (kk < q.K) {
        const int j = kk / q.Cg, c = kk - j * q.Cg;
        const int ti = tpos + j * q.d;
        if ((unsigned)ti < (unsigned)q.Tin) v[e] = (short)x[(long)(xrow0 + ti) * q.Cin + g * q.Cg + c];
      }
    }
  }
  return v;
}

// data-gradient A block: 8 consecutive k = u * Ng + n of input row (b, qi) of residue r -> dz[b, qi - u*d, g*Ng + n]
// (tap j = r + s*u reads output (t_in + p - j*d) / s = qi - u*d: s == 1 or d == 1)
template <bool VEC>
__device__ __forceinline__ short8 load_dzcol(const bf16_t* __restrict__ dz, const SConvGeom& q, int g, bool ok,
                                             int zrow0, int qi, int k) {
  short8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!ok) return v;
  const int KR = q.U * q.Ng;
  if constexpr (VEC) {
    if (k < KR) {
      const int u = k / q.Ng, n = k - u * q.Ng;
      const int to = qi - u * q.d;  // j = r + s*u; s > 1 only with d = 1
      if ((unsigned)to < (unsigned)q.Tout) v = *reinterpret_cast<const short8*>(dz + (long)(zrow0 + to) * q.Cout + g * q.Ng + n);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = k + e;
      if (kk < KR) {
        const int u = kk / q.Ng, n = kk - u * q.Ng;
        const int to = qi - u * q.d;  // j = r + s*u; s > 1 only with d = 1
        if ((unsigned)to < (unsigned)q.Tout) v[e] = (short)dz[(long)(zrow0 + to) * q.Cout + g * q.Ng + n];
      }
    }
  }
  return v;
}

__device__ __forceinline__ int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
__device__ __forceinline__ int ceildiv_s(int a, int b) { return -floordiv(-a, b); }

constexpr int SC_FWD = 0, SC_DGRAD = 1;
constexpr int ACT_NONE = 0, ACT_LRELU = 1, ACT_TANH = 2;

// forward (MODE 0) / polyphase data gradient (MODE 1).  grid (m tiles, column tiles, G [* s for MODE 1])
template <int MODE, bool VEC, int ACT, bool OUTF32, bool ACCUM>
__global__ void __launch_bounds__(SC_NT) sconv_kernel(const bf16_t* __restrict__ src, const bf16_t* __restrict__ wimg,
                                                     const float* __restrict__ bias, void* __restrict__ out,
                                                     SConvGeom q, float slope) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 8192];  // A[2], B[2]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int col = lane & 15, quad = lane >> 4;
  int g, r = 0;
  if constexpr (MODE == SC_FWD) {
    g = blockIdx.z;
  } else {
    g = blockIdx.z / q.s;
    r = blockIdx.z - g * q.s;
  }
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int NCOL = MODE == SC_FWD ? q.Ng : q.Cg;
  const int KRED = MODE == SC_FWD ? q.K : q.U * q.Ng;
  const int WLEN = MODE == SC_FWD ? q.Kp : q.UNp;     // valid (zero-padded) columns of one image row slice
  const long WROW = MODE == SC_FWD ? q.Kp : (long)q.s * q.UNp;
  const bf16_t* wb = MODE == SC_FWD ? wimg + (long)g * q.Ng * WROW : wimg + (long)g * q.Cg * WROW + (long)r * q.UNp;
  const int qmin = MODE == SC_FWD ? 0 : ceildiv_s(q.p - r, q.s);
  const int MROWS = MODE == SC_FWD ? q.B * q.Tout : q.B * q.NQ;

  // this thread's two A rows (fixed over the k loop) and two B rows
  bool aok[2];
  int ar0[2], ar1[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + i * SC_NT, rr = v >> 3;
    const int m = m0 + rr;
    bool ok = m < MROWS;
    const int mm = ok ? m : 0;
    if constexpr (MODE == SC_FWD) {
      const int b = mm / q.Tout, t = mm - b * q.Tout;
      ar0[i] = b * q.Tin;
      ar1[i] = t * q.s - q.p;
    } else {
      const int b = mm / q.NQ, iq = mm - b * q.NQ;
      const int qi = qmin + iq;
      const int ti = qi * q.s + r - q.p;
      ok = ok && ti >= 0 && ti < q.Tin;
      ar0[i] = b * q.Tout;
      ar1[i] = qi;
    }
    aok[i] = ok;
  }
  const int nk = (KRED + 63) / 64;
  short8 ra[2], rb[2];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + i * SC_NT, ch = v & 7;
      const int k = kt * 64 + ch * 8;
      if constexpr (MODE == SC_FWD) ra[i] = load_xcol<VEC>(src, q, g, aok[i], ar0[i], ar1[i], k);
      else ra[i] = load_dzcol<VEC>(src, q, g, aok[i], ar0[i], ar1[i], k);
      const int nr = v >> 3;
      short8 bv = {0, 0, 0, 0, 0, 0, 0, 0};
      if (n0 + nr < NCOL && k < WLEN) bv = *reinterpret_cast<const short8*>(wb + (long)(n0 + nr) * WROW + k);
      rb[i] = bv;
    }
  };
  auto lstore = [&](int buf) {
    char* As = lds + buf * 8192;
    char* Bs = lds + 16384 + buf * 8192;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + i * SC_NT, rr = v >> 3, ch = v & 7;
      *reinterpret_cast<short8*>(As + sw16(rr, ch)) = ra[i];
      *reinterpret_cast<short8*>(Bs + sw16(rr, ch)) = rb[i];
    }
  };
  float4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const char* As = lds + buf * 8192;
    const char* Bs = lds + 16384 + buf * 8192;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      short8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const short8*>(As + sw16(wm * 32 + i * 16 + col, kk * 4 + quad));
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const short8*>(Bs + sw16(wn * 32 + j * 16 + col, kk * 4 + quad));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }
  // epilogue: lane holds rows 4*quad + e of column col of each 16 x 16 sub-tile
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + col;
      if (n >= NCOL) continue;
      float bv = 0.f;
      if constexpr (MODE == SC_FWD) bv = bias ? bias[g * q.Ng + n] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 32 + i * 16 + 4 * quad + e;
        if (m >= MROWS) continue;
        long o;
        if constexpr (MODE == SC_FWD) {
          o = (long)m * q.Cout + g * q.Ng + n;
        } else {
          const int b = m / q.NQ, iq = m - b * q.NQ;
          const int ti = (qmin + iq) * q.s + r - q.p;
          if (ti < 0 || ti >= q.Tin) continue;
          o = ((long)b * q.Tin + ti) * q.Cin + g * q.Cg + n;
        }
        float v = acc[i][j][e] + bv;
        if constexpr (ACT == ACT_LRELU) v = lrelu_f(v, slope);
        else if constexpr (ACT == ACT_TANH) v = tanhf(v);
        if constexpr (OUTF32) {
          float* op = reinterpret_cast<float*>(out) + o;
          if constexpr (ACCUM) *op += v;
          else *op = v;
        } else {
          reinterpret_cast<bf16_t*>(out)[o] = f2bf(v);
        }
      }
    }
}

// weight gradient.  grid (n tiles * k tiles, G, splits); slabs [split][Cout][K] fp32
// bslabs (nullable): [split][Cout] column sums of dz (the bias gradient), from the blocks of k tile 0
template <bool VZ, bool VX>
__global__ void __launch_bounds__(SC_NT) sconv_wgrad_kernel(const bf16_t* __restrict__ dz, const bf16_t* __restrict__ x,
                                                           float* __restrict__ slabs, float* __restrict__ bslabs,
                                                           SConvGeom q, int rows_per_split, int ktiles) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 8192];  // Z[2], X[2]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = blockIdx.y, split = blockIdx.z;
  const int n0 = (blockIdx.x / ktiles) * 64, k0 = (blockIdx.x % ktiles) * 64;
  const int M = q.B * q.Tout;
  const int r_begin = split * rows_per_split;
  const int r_end = min(M, r_begin + rows_per_split);
  const int nsteps = r_end > r_begin ? (r_end - r_begin + 63) / 64 : 0;
  const bool dobias = bslabs != nullptr && k0 == 0;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // n = n0 + (tid & 7) * 8 + e, over this thread's rows
  short8 rz[2], rx[2];
  auto gload = [&](int st) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + i * SC_NT, rr = v >> 3, ch = v & 7;
      const int m = r_begin + st * 64 + rr;
      const bool ok = m < r_end;
      short8 zv = {0, 0, 0, 0, 0, 0, 0, 0};
      const int n = n0 + ch * 8;
      if (ok) {
        if constexpr (VZ) {
          if (n < q.Ng) zv = *reinterpret_cast<const short8*>(dz + (long)m * q.Cout + g * q.Ng + n);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (n + e < q.Ng) zv[e] = (short)dz[(long)m * q.Cout + g * q.Ng + n + e];
        }
      }
      rz[i] = zv;
      if (dobias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[e] += bf2f((bf16_t)zv[e]);
      }
      const int mm = ok ? m : 0;
      const int b = mm / q.Tout, t = mm - b * q.Tout;
      rx[i] = load_xcol<VX>(x, q, g, ok, b * q.Tin, t * q.s - q.p, k0 + ch * 8);
    }
  };
  auto lstore = [&](int buf) {
    char* Zs = lds + buf * 8192;
    char* Xs = lds + 16384 + buf * 8192;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + i * SC_NT, rr = v >> 3, ch = v & 7;
      *reinterpret_cast<short8*>(Zs + sw8(rr, 2 * ch)) = rz[i];
      *reinterpret_cast<short8*>(Xs + sw8(rr, 2 * ch)) = rx[i];
    }
  };
  float4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  const int g16 = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  if (nsteps > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    if (st + 1 < nsteps) gload(st + 1);
    const char* Zs = lds + buf * 8192;
    const char* Xs = lds + 16384 + buf * 8192;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rbase = h * 32 + 8 * g16 + qq;
      short8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c8 = (wm * 32 + i * 16) / 4 + pp;
        const short4v v0 = ds_tr(Zs + sw8(rbase, c8)), v1 = ds_tr(Zs + sw8(rbase + 4, c8));
        a[i] = (short8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c8 = (wn * 32 + j * 16) / 4 + pp;
        const short4v v0 = ds_tr(Xs + sw8(rbase, c8)), v1 = ds_tr(Xs + sw8(rbase + 4, c8));
        b[j] = (short8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nsteps) lstore(buf ^ 1);
    __syncthreads();
  }
  if (dobias) {  // 32 threads share each 8-column chunk: LDS reduce (the loop's last barrier freed the tiles)
    float* red = reinterpret_cast<float*>(lds);  // [32][64]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(tid >> 3) * 64 + (tid & 7) * 8 + e] = bsum[e];
    __syncthreads();
    if (tid < 64 && n0 + tid < q.Ng) {
      float t = 0.f;
      for (int j = 0; j < 32; ++j) t += red[j * 64 + tid];
      bslabs[(long)split * q.Cout + g * q.Ng + n0 + tid] = t;
    }
  }
  float* S = slabs + (long)split * q.Cout * q.K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + wm * 32 + i * 16 + 4 * (lane >> 4) + e;
        const int k = k0 + wn * 32 + j * 16 + (lane & 15);
        if (n < q.Ng && k < q.K) S[(long)(g * q.Ng + n) * q.K + k] = acc[i][j][e];
      }
}

// dW[o][c][j] (torch layout [Cout][Cg][ks]) = sum over splits (fixed order) of slab[s][o][j * Cg + c]
__global__ void __launch_bounds__(256) sconv_wreduce_kernel(const float* __restrict__ slabs, float* __restrict__ dW,
                                                            const float* __restrict__ bslabs, float* __restrict__ db,
                                                            int splits, int Cout, int Cg, int ks) {
  const long K = (long)ks * Cg, tot = (long)Cout * K;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot + (db ? Cout : 0); i += (long)gridDim.x * 256) {
    if (i >= tot) {  // bias: db[o] = sum over splits (fixed order)
      const int o = (int)(i - tot);
      float t = 0.f;
      for (int sp = 0; sp < splits; ++sp) t += bslabs[(long)sp * Cout + o];
      db[o] = t;
      continue;
    }
    const int o = (int)(i / K);
    const int rem = (int)(i - (long)o * K);
    const int c = rem / ks, j = rem - c * ks;  // torch order
    const long src = (long)o * K + (long)j * Cg + c;
    float t = 0.f;
    for (int sp = 0; sp < splits; ++sp) t += slabs[(long)sp * tot + src];
    dW[i] = t;
  }
}

// ------------------------------------------------------------------------------------------ elementwise
// dz = ((dy or 0) + fm_scale * sign(y - r)) * act'(y); act' from the activation OUTPUT y (lrelu: y >= 0 -> 1
// else slope -- the same sign as its input; tanh: 1 - y^2; none: 1).  r (nullable): the real-input feature map
// of the feature-matching loss (reference hifigan/models.py:234-240, L1 -> sign).
template <int ACT>
__global__ void __launch_bounds__(256) act_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                      const bf16_t* __restrict__ rr, float fm_scale,
                                                      bf16_t* __restrict__ dz, long n, float slope) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float yv = bf2f(y[i]);
    float g = dy ? bf2f(dy[i]) : 0.f;
    if (rr) {
      const float dv = yv - bf2f(rr[i]);
      g += dv > 0.f ? fm_scale : (dv < 0.f ? -fm_scale : 0.f);
    }
    float dd = 1.f;
    if constexpr (ACT == ACT_LRELU) dd = yv >= 0.f ? 1.f : slope;
    else if constexpr (ACT == ACT_TANH) dd = 1.f - yv * yv;
    dz[i] = f2bf(g * dd);
  }
}

// dz = dy (fp32) * (1 - y^2) (tanh output y fp32) -> bf16: the generator's conv_post backward
__global__ void __launch_bounds__(256) tanh_bwd_f32_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                           bf16_t* __restrict__ dz, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float yv = y[i];
    dz[i] = f2bf(dy[i] * (1.f - yv * yv));
  }
}

// bf16 elementwise, 8 per thread (n % 8 == 0 checked on the host)
// op 0: y = lrelu(a);  1: y = a + b;  2: y = (a + b + c) * s;  3: y = a * s;  4: y = a * lrelu'(b) (b: the input)
template <int OP>
__global__ void __launch_bounds__(256) ew8_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                                  const bf16_t* __restrict__ c, bf16_t* __restrict__ y, long n8,
                                                  float s) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const short8 va = reinterpret_cast<const short8*>(a)[i];
    short8 vb = va, vc = va, o;
    if constexpr (OP == 1 || OP == 2 || OP == 4) vb = reinterpret_cast<const short8*>(b)[i];
    if constexpr (OP == 2) vc = reinterpret_cast<const short8*>(c)[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xa = bf2f((bf16_t)va[e]);
      float v;
      if constexpr (OP == 0) v = lrelu_f(xa, s);
      else if constexpr (OP == 1) v = xa + bf2f((bf16_t)vb[e]);
      else if constexpr (OP == 2) v = (xa + bf2f((bf16_t)vb[e]) + bf2f((bf16_t)vc[e])) * s;
      else if constexpr (OP == 3) v = xa * s;
      else v = bf2f((bf16_t)vb[e]) >= 0.f ? xa : xa * s;
      o[e] = (short)f2bf(v);
    }
    reinterpret_cast<short8*>(y)[i] = o;
  }
}

// per-block partial sums of |a - b| (bf16 or fp32 operands) -> part[blockIdx.x] (fixed grid)
template <bool F32>
__global__ void __launch_bounds__(256) l1_part_kernel(const void* __restrict__ a, const void* __restrict__ b, long n,
                                                      float* __restrict__ part) {
  float t = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float va, vb;
    if constexpr (F32) {
      va = reinterpret_cast<const float*>(a)[i];
      vb = reinterpret_cast<const float*>(b)[i];
    } else {
      va = bf2f(reinterpret_cast<const bf16_t*>(a)[i]);
      vb = bf2f(reinterpret_cast<const bf16_t*>(b)[i]);
    }
    t += fabsf(va - vb);
  }
  __shared__ float red[4];
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out[slot] (+)= scale * sum(part[0..n)) in a fixed order (one block)
__global__ void __launch_bounds__(256) sum_parts_kernel(const float* __restrict__ part, int n, float scale,
                                                        float* __restrict__ out, int accumulate) {
  float t = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) t += part[i];
  __shared__ float red[4];
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
    out[0] = accumulate ? out[0] + v : v;
  }
}

// LSGAN on discriminator scores s (fp32, n): loss[0] (+)= mean((t - s)^2); ds = -2 (t - s) / n * gscale (bf16,
// nullable) -- reference hifigan/models.py:243-264 (real: t = 1, fake in the D step: t = 0, G step: t = 1)
// loss[0] += mean((target - s)^2) [+ fm_scale * sum |s - r|: the feature-matching term of the score map, the
// discriminator's conv_post output, which the reference's feature_loss includes (hifigan/models.py:193-198)];
// ds = d loss / ds * gscale
__global__ void __launch_bounds__(256) lsgan_kernel(const float* __restrict__ s, int n, float target, float gscale,
                                                    const float* __restrict__ r, float fm_scale,
                                                    bf16_t* __restrict__ ds, float* __restrict__ loss) {
  float t = 0.f, a = 0.f;
  const float inv = 1.f / (float)n;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float e = target - s[i];
    t += e * e;
    float g = -2.f * e * inv;
    if (r) {
      const float dv = s[i] - r[i];
      a += fabsf(dv);
      g += dv > 0.f ? fm_scale : (dv < 0.f ? -fm_scale : 0.f);
    }
    if (ds) ds[i] = f2bf(g * gscale);
  }
  __shared__ float red[8];
  t = wave_sum(t);
  a = wave_sum(a);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = t;
    red[4 + (threadIdx.x >> 6)] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    loss[0] += ((red[0] + red[1]) + (red[2] + red[3])) * inv + ((red[4] + red[5]) + (red[6] + red[7])) * fm_scale;
}

// AvgPool1d(4, 2, padding=2), count_include_pad (reference MultiScaleDiscriminator meanpools) over [R, T]
// rows: y[r, t] = (x[2t-2] + x[2t-1] + x[2t] + x[2t+1]) / 4, T_out = T / 2 + 1
__global__ void __launch_bounds__(256) avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int R,
                                                          int T, int To) {
  const long tot = (long)R * To;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    const int r = (int)(i / To), t = (int)(i - (long)r * To);
    float v = 0.f;
#pragma unroll
    for (int e = -2; e < 2; ++e) {
      const int u = 2 * t + e;
      if (u >= 0 && u < T) v += bf2f(x[(long)r * T + u]);
    }
    y[i] = f2bf(v * 0.25f);
  }
}

// dx[r, u] (+)= sum over the (<= 2) windows covering u of dy / 4  (fp32)
__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const float* __restrict__ dy, float* __restrict__ dx, int R,
                                                          int T, int To, int accumulate) {
  const long tot = (long)R * T;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    const int r = (int)(i / T), u = (int)(i - (long)r * T);
    // windows t with 2t - 2 <= u <= 2t + 1: t in {u/2 - 1 .. u/2 + 1}
    float v = 0.f;
    for (int t = u / 2 - 1; t <= u / 2 + 1; ++t)
      if (t >= 0 && t < To && 2 * t - 2 <= u && u <= 2 * t + 1) v += dy[(long)r * To + t];
    v *= 0.25f;
    dx[i] = accumulate ? dx[i] + v : v;
  }
}

// MPD input: y [R, T] -> reflect-pad to Tp = ceil(T / P) * P -> fold [R, Tp / P, P] -> [R * P, Tp / P]
// (sequence r * P + w holds column w), reference hifigan DiscriminatorP.forward
__global__ void __launch_bounds__(256) mpd_fold_kernel(const bf16_t* __restrict__ y, bf16_t* __restrict__ out, int R,
                                                       int T, int P, int H) {
  const long tot = (long)R * P * H;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    const int seq = (int)(i / H), h = (int)(i - (long)seq * H);
    const int r = seq / P, w = seq - r * P;
    int t = h * P + w;
    if (t >= T) t = 2 * (T - 1) - t;  // reflect (no edge repeat)
    out[i] = y[(long)r * T + t];
  }
}

// backward of mpd_fold: dy[r, t] (+)= d at every folded position that reads t
__global__ void __launch_bounds__(256) mpd_unfold_kernel(const float* __restrict__ d, float* __restrict__ dy, int R,
                                                         int T, int P, int H) {
  const long tot = (long)R * T;
  const int Tp = H * P;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    const int r = (int)(i / T), t = (int)(i - (long)r * T);
    float v = d[((long)r * P + t % P) * H + t / P];
    const int tr = 2 * (T - 1) - t;  // padded position reflecting onto t
    if (tr >= T && tr < Tp) v += d[((long)r * P + tr % P) * H + tr / P];
    dy[i] += v;
  }
}

// STFT input: y fp32 [R, N] -> reflect pad Pd each side -> bf16 [R, N + 2 Pd, 8] = (hi, lo, hi, 0, 0, 0, 0, 0),
// hi = bf16(y), lo = bf16(y - hi): with the DFT image (W_hi, W_hi, W_lo, 0...) the bf16 MFMA accumulates
// W_hi y_hi + W_hi y_lo + W_lo y_hi -- the fp32 transform to ~2^-16 relative (the reference STFT is fp32)
__global__ void __launch_bounds__(256) stft_prep_kernel(const float* __restrict__ y, short8* __restrict__ out, int R,
                                                        int N, int Pd) {
  const int Np = N + 2 * Pd;
  const long tot = (long)R * Np;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    const int r = (int)(i / Np);
    int t = (int)(i - (long)r * Np) - Pd;
    if (t < 0) t = -t;
    if (t >= N) t = 2 * (N - 1) - t;
    const float v = y[(long)r * N + t];
    const bf16_t hi = f2bf(v);
    const bf16_t lo = f2bf(v - bf2f(hi));
    out[i] = (short8){(short)hi, (short)lo, (short)hi, 0, 0, 0, 0, 0};
  }
}

// backward of the reflect pad: dy[r, t] (+)= d[r, t + Pd] + the mirrored padded positions
__global__ void __launch_bounds__(256) stft_unpad_kernel(const float* __restrict__ d, float* __restrict__ dy, int R,
                                                         int N, int Pd, int accumulate) {
  const int Np = N + 2 * Pd;
  const long tot = (long)R * N;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    const int r = (int)(i / N), t = (int)(i - (long)r * N);
    const float* dr = d + (long)r * Np;
    float v = dr[t + Pd];
    if (t >= 1 && t <= Pd) v += dr[Pd - t];                   // left pad index Pd - t reflects t
    if (t <= N - 2 && t >= N - 1 - Pd) v += dr[Pd + 2 * (N - 1) - t];  // right pad index reflects t
    dy[i] = accumulate ? dy[i] + v : v;
  }
}

// One frame per block: spec row [re 0..NB) [im NB..2NB) (fp32, row stride lds) -> |X| = sqrt(re^2 + im^2 + 1e-9)
// -> mel = basis [NM][NB] |X| -> log(max(mel, 1e-5)) vs target [R][NM][F] at (r, :, f) -> |diff| summed into
// part[frame]; gradient of scale * L1: dmel = scale * sign(diff) / mel (0 where clamped), d|X| = basis^T dmel,
// d re = d|X| re / |X|, d im likewise -> dspec (bf16, row stride ldd; frames f >= Fv get zeros)
// (reference hifigan/meldataset.py:49-72 + train.py:135 F.l1_loss(y_mel, y_g_hat_mel) * 45)
__global__ void __launch_bounds__(256) mel_l1_kernel(const float* __restrict__ spec, int ldspec,
                                                     const float* __restrict__ basis, int NB, int NM,
                                                     const float* __restrict__ target, int Ft, int F, int Fv,
                                                     float scale, float* __restrict__ part, bf16_t* __restrict__ dspec,
                                                     int ldd) {
  extern __shared__ float sh[];
  float* mag = sh;             // [NB]
  float* dm = sh + NB;         // [NM]
  const int fr = blockIdx.x, r = fr / F, f = fr - r * F;
  const float* srow = spec + (long)fr * ldspec;
  bf16_t* drow = dspec + (long)fr * ldd;
  if (f >= Fv) {
    for (int k = threadIdx.x; k < ldd; k += 256) drow[k] = 0;
    if (threadIdx.x == 0) part[fr] = 0.f;
    return;
  }
  for (int k = threadIdx.x; k < NB; k += 256) {
    const float re = srow[k], im = srow[NB + k];
    mag[k] = sqrtf(re * re + im * im + 1e-9f);
  }
  __syncthreads();
  float l1 = 0.f;
  for (int m = threadIdx.x; m < NM; m += 256) {
    const float* br = basis + (long)m * NB;
    float acc = 0.f;
    for (int k = 0; k < NB; ++k) acc += br[k] * mag[k];
    const float cl = fmaxf(acc, 1e-5f);
    const float diff = logf(cl) - target[((long)r * NM + m) * Ft + f];
    l1 += fabsf(diff);
    const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
    dm[m] = acc > 1e-5f ? scale * sg / acc : 0.f;
  }
  __shared__ float red[4];
  l1 = wave_sum(l1);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l1;
  __syncthreads();
  if (threadIdx.x == 0) part[fr] = (red[0] + red[1]) + (red[2] + red[3]);
  for (int k = threadIdx.x; k < NB; k += 256) {
    float gm = 0.f;
    for (int m = 0; m < NM; ++m) gm += basis[(long)m * NB + k] * dm[m];
    const float re = srow[k], im = srow[NB + k], a = mag[k];
    drow[k] = f2bf(gm * re / a);
    drow[NB + k] = f2bf(gm * im / a);
  }
  for (int k = 2 * NB + threadIdx.x; k < ldd; k += 256) drow[k] = 0;
}

// forward image [Cout][Kp] (column j*Cg + c = W[o][c][j], zero past K) and data-gradient image [G*Cg][s][UNp]
// (column u*Ng + n of residue r = W[g*Ng + n][c][r + s*u], zero past ks / U*Ng) from the fp32 weight [Cout][Cg][ks]
__global__ void __launch_bounds__(256) sconv_fimg_kernel(const float* __restrict__ w, bf16_t* __restrict__ img, int Cout,
                                                         int Cg, int ks, int Kp) {
  const long tot = (long)Cout * Kp;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    const int o = (int)(i / Kp), k = (int)(i - (long)o * Kp);
    float v = 0.f;
    if (k < ks * Cg) {
      const int j = k / Cg, c = k - j * Cg;
      v = w[((long)o * Cg + c) * ks + j];
    }
    img[i] = f2bf(v);
  }
}

__global__ void __launch_bounds__(256) sconv_dimg_kernel(const float* __restrict__ w, bf16_t* __restrict__ img, int G,
                                                         int Cg, int Ng, int ks, int s, int U, int UNp) {
  const long tot = (long)G * Cg * s * UNp;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < tot; i += (long)gridDim.x * 256) {
    const int col = (int)(i % UNp);
    const long rowr = i / UNp;
    const int r = (int)(rowr % s);
    const int gc = (int)(rowr / s);
    const int g = gc / Cg, c = gc - g * Cg;
    float v = 0.f;
    if (col < U * Ng) {
      const int u = col / Ng, n = col - u * Ng;
      const int j = r + s * u;
      if (j < ks) v = w[((long)(g * Ng + n) * Cg + c) * ks + j];
    }
    img[i] = f2bf(v);
  }
}

int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

bool make_geom(SConvGeom& q, int B, int Tin, int Cin, int Cout, int G, int ks, int s, int d, int p) {
  if (B <= 0 || Tin <= 0 || G <= 0 || Cin % G || Cout % G || ks <= 0 || s <= 0 || d <= 0 || p < 0) return false;
  q.B = B; q.Tin = Tin; q.Cin = Cin; q.Cout = Cout; q.G = G; q.ks = ks; q.s = s; q.d = d; q.p = p;
  q.Cg = Cin / G;
  q.Ng = Cout / G;
  const int span = Tin + 2 * p - d * (ks - 1) - 1;
  if (span < 0) return false;
  q.Tout = span / s + 1;
  q.K = ks * q.Cg;
  q.Kp = (q.K + 7) / 8 * 8;
  q.U = (ks + s - 1) / s;
  q.UNp = (q.U * q.Ng + 7) / 8 * 8;
  int nq = 0;
  for (int r = 0; r < s; ++r) {
    // rows t_in = qi * s + r - p in [0, Tin)
    const int lo = (p - r) >= 0 ? (p - r + s - 1) / s : -((r - p) / s);
    const int hi_num = Tin - 1 - r + p;
    const int hi = hi_num >= 0 ? hi_num / s : -((-hi_num + s - 1) / s);
    nq = std::max(nq, hi - lo + 1);
  }
  q.NQ = nq;
  return q.Tout > 0 && (long)B * Tin * Cin < (1L << 31) && (long)B * q.Tout * Cout < (1L << 31);
}

int wgrad_splits(const SConvGeom& q) {
  const int M = q.B * q.Tout;
  const int chunks = (M + 63) / 64;
  const int tiles = ((q.Ng + 63) / 64) * ((q.K + 63) / 64) * q.G;
  int sp = (1024 + tiles - 1) / tiles;
  const int maxsp = std::max(1, chunks / 4);
  if (sp > maxsp) sp = maxsp;
  return sp < 1 ? 1 : sp;
}

}  // namespace

// Forward: x [B, Tin, Cin] bf16 -> y [B, Tout, Cout] (bf16, or fp32 when out_f32); wimg bf16 [Cout][Kp] with
// row o = [j][c] (j-major, Kp = round8(ks * Cin / G), zero tail); act 0 none, 1 lrelu(slope), 2 tanh.
SSAMD_API int ssamd_sconv_fwd(const bf16_t* x, const bf16_t* wimg, const float* bias, void* y, int B, int Tin, int Cin,
                              int Cout, int G, int ks, int s, int d, int p, int act, float slope, int out_f32,
                              hipStream_t st) {
  SConvGeom q;
  if (!make_geom(q, B, Tin, Cin, Cout, G, ks, s, d, p) || act < 0 || act > 2) return -2;
  const bool vec = q.Cg % 8 == 0;
  dim3 grid((B * q.Tout + 63) / 64, (q.Ng + 63) / 64, G);
#define SC_L(V, A, O) hipLaunchKernelGGL((sconv_kernel<SC_FWD, V, A, O, false>), grid, dim3(SC_NT), 0, st, x, wimg, bias, y, q, slope)
#define SC_A(V, O) \
  if (act == 0) SC_L(V, ACT_NONE, O); else if (act == 1) SC_L(V, ACT_LRELU, O); else SC_L(V, ACT_TANH, O);
  if (vec) {
    if (out_f32) { SC_A(true, true) } else { SC_A(true, false) }
  } else {
    if (out_f32) { SC_A(false, true) } else { SC_A(false, false) }
  }
#undef SC_A
#undef SC_L
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_sconv_tout(int Tin, int ks, int s, int d, int p) {
  const int span = Tin + 2 * p - d * (ks - 1) - 1;
  return span < 0 ? 0 : span / s + 1;
}

// Data gradient: dz [B, Tout, Cout] bf16 -> dx [B, Tin, Cin] (bf16, or fp32 with optional accumulate);
// wdimg bf16 [Cin][s][UNp]: row g*Cg + c, residue r, column u * Ng + n = W[g*Ng + n][c][r + s*u] (0 past ks),
// UNp = round8(ceil(ks / s) * Cout / G).  Requires s == 1 or d == 1.
SSAMD_API int ssamd_sconv_dgrad(const bf16_t* dz, const bf16_t* wdimg, void* dx, int B, int Tin, int Cin, int Cout,
                                int G, int ks, int s, int d, int p, int out_f32, int accum, hipStream_t st) {
  SConvGeom q;
  if (!make_geom(q, B, Tin, Cin, Cout, G, ks, s, d, p) || (s != 1 && d != 1)) return -2;
  if (accum && !out_f32) return -2;
  const bool vec = q.Ng % 8 == 0;
  dim3 grid((B * q.NQ + 63) / 64, (q.Cg + 63) / 64, G * s);
#define SD_L(V, O, A) hipLaunchKernelGGL((sconv_kernel<SC_DGRAD, V, ACT_NONE, O, A>), grid, dim3(SC_NT), 0, st, dz, wdimg, nullptr, dx, q, 0.f)
  if (vec) {
    if (!out_f32) SD_L(true, false, false);
    else if (accum) SD_L(true, true, true);
    else SD_L(true, true, false);
  } else {
    if (!out_f32) SD_L(false, false, false);
    else if (accum) SD_L(false, true, true);
    else SD_L(false, true, false);
  }
#undef SD_L
  return (int)hipGetLastError();
}

SSAMD_API long ssamd_sconv_wgrad_ws(int B, int Tin, int Cin, int Cout, int G, int ks, int s, int d, int p) {
  SConvGeom q;
  if (!make_geom(q, B, Tin, Cin, Cout, G, ks, s, d, p)) return -1;
  return (long)wgrad_splits(q) * Cout * (q.K + 1);  // weight slabs + bias slabs
}

// Weight gradient: dz [B, Tout, Cout], x [B, Tin, Cin] -> dW fp32 [Cout][Cin / G][ks] (torch layout) and (db non-null)
// the bias gradient db [Cout] = column sums of dz, through ws (>= ssamd_sconv_wgrad_ws floats).
SSAMD_API int ssamd_sconv_wgrad(const bf16_t* dz, const bf16_t* x, float* ws, long ws_floats, float* dW, float* db,
                                int B, int Tin, int Cin, int Cout, int G, int ks, int s, int d, int p, hipStream_t st) {
  SConvGeom q;
  if (!make_geom(q, B, Tin, Cin, Cout, G, ks, s, d, p)) return -2;
  const int sp = wgrad_splits(q);
  if ((long)sp * Cout * (q.K + 1) > ws_floats) return -3;
  float* bws = db ? ws + (long)sp * Cout * q.K : nullptr;
  const int M = B * q.Tout;
  int rps = (M + sp - 1) / sp;
  rps = (rps + 63) / 64 * 64;
  const int ktiles = (q.K + 63) / 64;
  dim3 grid(((q.Ng + 63) / 64) * ktiles, G, sp);
  const bool vz = q.Ng % 8 == 0, vx = q.Cg % 8 == 0;
#define SW_L(A, Bv) hipLaunchKernelGGL((sconv_wgrad_kernel<A, Bv>), grid, dim3(SC_NT), 0, st, dz, x, ws, bws, q, rps, ktiles)
  if (vz && vx) SW_L(true, true);
  else if (vz) SW_L(true, false);
  else if (vx) SW_L(false, true);
  else SW_L(false, false);
#undef SW_L
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  hipLaunchKernelGGL(sconv_wreduce_kernel, dim3(grid_for((long)Cout * q.K + Cout)), dim3(256), 0, st, ws, dW, bws, db, sp,
                     Cout, q.Cg, ks);
  return (int)hipGetLastError();
}

// act 0 none, 1 lrelu(slope), 2 tanh: dz = ((dy or 0) + fm_scale * sign(y - r)) * act'(y)
SSAMD_API int ssamd_act_bwd(const bf16_t* dy, const bf16_t* y, const bf16_t* r, float fm_scale, bf16_t* dz, long n,
                            int act, float slope, hipStream_t st) {
  if (n <= 0) return 0;
  const dim3 g(grid_for(n));
  if (act == 0) hipLaunchKernelGGL(act_bwd_kernel<ACT_NONE>, g, dim3(256), 0, st, dy, y, r, fm_scale, dz, n, slope);
  else if (act == 1) hipLaunchKernelGGL(act_bwd_kernel<ACT_LRELU>, g, dim3(256), 0, st, dy, y, r, fm_scale, dz, n, slope);
  else if (act == 2) hipLaunchKernelGGL(act_bwd_kernel<ACT_TANH>, g, dim3(256), 0, st, dy, y, r, fm_scale, dz, n, slope);
  else return -2;
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_tanh_bwd_f32(const float* dy, const float* y, bf16_t* dz, long n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(tanh_bwd_f32_kernel, dim3(grid_for(n)), dim3(256), 0, st, dy, y, dz, n);
  return (int)hipGetLastError();
}

// op 0: lrelu(a, s);  1: a + b;  2: (a + b + c) * s;  3: a * s;  4: a * lrelu'(b, s)   (bf16, n % 8 == 0)
SSAMD_API int ssamd_ew(int op, const bf16_t* a, const bf16_t* b, const bf16_t* c, bf16_t* y, long n, float s,
                       hipStream_t st) {
  if (n % 8) return -2;
  if (n == 0) return 0;
  const long n8 = n / 8;
  const dim3 g(grid_for(n8));
  switch (op) {
    case 0: hipLaunchKernelGGL(ew8_kernel<0>, g, dim3(256), 0, st, a, b, c, y, n8, s); break;
    case 1: hipLaunchKernelGGL(ew8_kernel<1>, g, dim3(256), 0, st, a, b, c, y, n8, s); break;
    case 2: hipLaunchKernelGGL(ew8_kernel<2>, g, dim3(256), 0, st, a, b, c, y, n8, s); break;
    case 3: hipLaunchKernelGGL(ew8_kernel<3>, g, dim3(256), 0, st, a, b, c, y, n8, s); break;
    case 4: hipLaunchKernelGGL(ew8_kernel<4>, g, dim3(256), 0, st, a, b, c, y, n8, s); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

// out[0] (+)= scale * sum |a - b| (a, b bf16 or fp32); part: >= 256 floats of scratch
SSAMD_API int ssamd_l1_sum(const void* a, const void* b, long n, int f32, float scale, float* part, float* out,
                           int accumulate, hipStream_t st) {
  if (n <= 0) return 0;
  const int nb = (int)std::min<long>(256, (n + 255) / 256);
  if (f32) hipLaunchKernelGGL(l1_part_kernel<true>, dim3(nb), dim3(256), 0, st, a, b, n, part);
  else hipLaunchKernelGGL(l1_part_kernel<false>, dim3(nb), dim3(256), 0, st, a, b, n, part);
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(256), 0, st, part, nb, scale, out, accumulate);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_sum_parts(const float* part, int n, float scale, float* out, int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(256), 0, st, part, n, scale, out, accumulate);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_lsgan(const float* s, int n, float target, float gscale, const float* r, float fm_scale, bf16_t* ds,
                          float* loss, hipStream_t st) {
  if (n <= 0) return -2;
  hipLaunchKernelGGL(lsgan_kernel, dim3(1), dim3(256), 0, st, s, n, target, gscale, r, r ? fm_scale : 0.f, ds, loss);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_avgpool4(const bf16_t* x, bf16_t* y, int R, int T, hipStream_t st) {
  const int To = T / 2 + 1;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(grid_for((long)R * To)), dim3(256), 0, st, x, y, R, T, To);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_avgpool4_bwd(const float* dy, float* dx, int R, int T, int accumulate, hipStream_t st) {
  const int To = T / 2 + 1;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for((long)R * T)), dim3(256), 0, st, dy, dx, R, T, To, accumulate);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_mpd_fold(const bf16_t* y, bf16_t* out, int R, int T, int P, hipStream_t st) {
  const int H = (T + P - 1) / P;
  if (H * P - T >= T) return -2;  // reflect pad needs n_pad < T
  hipLaunchKernelGGL(mpd_fold_kernel, dim3(grid_for((long)R * P * H)), dim3(256), 0, st, y, out, R, T, P, H);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_mpd_unfold(const float* d, float* dy, int R, int T, int P, hipStream_t st) {
  const int H = (T + P - 1) / P;
  hipLaunchKernelGGL(mpd_unfold_kernel, dim3(grid_for((long)R * T)), dim3(256), 0, st, d, dy, R, T, P, H);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_stft_prep(const float* y, bf16_t* out, int R, int N, int Pd, hipStream_t st) {
  if (Pd >= N) return -2;
  hipLaunchKernelGGL(stft_prep_kernel, dim3(grid_for((long)R * (N + 2 * Pd))), dim3(256), 0, st, y,
                     reinterpret_cast<short8*>(out), R, N, Pd);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_stft_unpad(const float* d, float* dy, int R, int N, int Pd, int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(stft_unpad_kernel, dim3(grid_for((long)R * N)), dim3(256), 0, st, d, dy, R, N, Pd, accumulate);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_mel_l1(const float* spec, int ldspec, const float* basis, int NB, int NM, const float* target, int Ft,
                           int R, int F, int Fv, float scale, float* part, bf16_t* dspec, int ldd, hipStream_t st) {
  if (ldspec < 2 * NB || ldd < 2 * NB || R * F <= 0) return -2;
  const size_t sh = (size_t)(NB + NM) * sizeof(float);
  hipLaunchKernelGGL(mel_l1_kernel, dim3(R * F), dim3(256), sh, st, spec, ldspec, basis, NB, NM, target, Ft, F, Fv, scale,
                     part, dspec, ldd);
  return (int)hipGetLastError();
}

// bf16 images of an fp32 weight [Cout][Cin / G][ks] (either pointer nullable): forward [Cout][round8(ks * Cg)] and
// data gradient [Cin][s][round8(ceil(ks / s) * Cout / G)]
SSAMD_API int ssamd_sconv_images(const float* w, bf16_t* fimg, bf16_t* dimg, int Cout, int Cin, int G, int ks, int s,
                                 hipStream_t st) {
  if (G <= 0 || Cin % G || Cout % G || ks <= 0 || s <= 0) return -2;
  const int Cg = Cin / G, Ng = Cout / G;
  if (fimg) {
    const int Kp = (ks * Cg + 7) / 8 * 8;
    hipLaunchKernelGGL(sconv_fimg_kernel, dim3(grid_for((long)Cout * Kp)), dim3(256), 0, st, w, fimg, Cout, Cg, ks, Kp);
  }
  if (dimg) {
    const int U = (ks + s - 1) / s, UNp = (U * Ng + 7) / 8 * 8;
    hipLaunchKernelGGL(sconv_dimg_kernel, dim3(grid_for((long)Cin * s * UNp)), dim3(256), 0, st, w, dimg, G, Cg, Ng, ks, s,
                       U, UNp);
  }
  return (int)hipGetLastError();
}
