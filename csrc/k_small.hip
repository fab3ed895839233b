// Small-N kernels that are not MFMA-shaped (N = 1 output channel):
//
//  * variance-predictor head (reference model/modules.py:247,253-257):
//    out[r] = (h[r,:] . w + b) masked to 0 at padded rows; one wave per row, fused mask.
//    Backward: dh = g (x) w (masked), dw = sum_r g h, db = sum_r g -- block-reduced into one
//    partial row per block, finished by a fixed-order column sum (deterministic, no atomics).
//  * HiFi-GAN conv_post (K V4/V6, reference hifigan/models.py:145,161-163 +
//    utils/model.py:105-113): LeakyReLU(0.01) -> Conv1d(C -> 1, k=7, pad 3) -> tanh, and
//    optionally * max_wav_value -> clamp -> int16, channel-last input read once through an
//    LDS tile (each input row feeds 7 outputs).
#include "common.h"

namespace {

constexpr int HEAD_ROWS = 64;  // rows per 256-thread block (16 per wave)

template <int EPL>  // elements per lane: C = 64 * EPL
__global__ void __launch_bounds__(256) head_fwd_kernel(const bf16_t* __restrict__ h, const float* __restrict__ w,
                                                       const float* __restrict__ b, const int64_t* __restrict__ lens,
                                                       long R, int L, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float wv[EPL];
#pragma unroll
  for (int i = 0; i < EPL; ++i) wv[i] = w[lane * EPL + i];
  const float bias = b ? *b : 0.f;
  for (int rr = 0; rr < HEAD_ROWS / 4; ++rr) {
    const long r = (long)blockIdx.x * HEAD_ROWS + rr * 4 + wave;
    if (r >= R) break;
    float s = 0.f;
    const bf16_t* hp = h + r * (64 * EPL) + lane * EPL;
#pragma unroll
    for (int i = 0; i < EPL; ++i) s += bf2f(hp[i]) * wv[i];
    s = wave_sum(s);
    if (lane == 0) {
      bool valid = true;
      if (lens) {
        const long bb = r / L;
        valid = (r - bb * L) < lens[bb];
      }
      out[r] = valid ? s + bias : 0.f;
    }
  }
}

template <int EPL>
__global__ void __launch_bounds__(256) head_bwd_kernel(const float* __restrict__ g, const bf16_t* __restrict__ h,
                                                       const float* __restrict__ w, const int64_t* __restrict__ lens,
                                                       long R, int L, bf16_t* __restrict__ dh,
                                                       float* __restrict__ part) {
  __shared__ float red[4][64 * EPL + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float wv[EPL], acc[EPL];
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    wv[i] = w[lane * EPL + i];
    acc[i] = 0.f;
  }
  float gsum = 0.f;
  for (int rr = 0; rr < HEAD_ROWS / 4; ++rr) {
    const long r = (long)blockIdx.x * HEAD_ROWS + rr * 4 + wave;
    if (r >= R) break;
    float gv = g[r];
    if (lens) {
      const long bb = r / L;
      if ((r - bb * L) >= lens[bb]) gv = 0.f;
    }
    const bf16_t* hp = h + r * (64 * EPL) + lane * EPL;
    bf16_t* dp = dh + r * (64 * EPL) + lane * EPL;
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      acc[i] += gv * bf2f(hp[i]);
      dp[i] = f2bf(gv * wv[i]);
    }
    gsum += gv;
  }
#pragma unroll
  for (int i = 0; i < EPL; ++i) red[wave][lane * EPL + i] = acc[i];
  if (lane == 0) red[wave][64 * EPL] = gsum;
  __syncthreads();
  float* pb = part + (long)blockIdx.x * (64 * EPL + 1);
  for (int c = threadIdx.x; c <= 64 * EPL; c += 256) pb[c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

// conv_post: block = 256 output samples of one utterance; LDS tile of (256 + 6) input rows x C
constexpr int CP_T = 256;

template <int C>
__global__ void __launch_bounds__(CP_T) conv_post_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, int Tp, float slope,
                                                         float scale, float* __restrict__ outf,
                                                         int16_t* __restrict__ outi, const int4* __restrict__ tt,
                                                         long ostride) {
  // rows staged with 16-B loads (8 channels per lane) into fp32 rows of RS = C + 4 floats (16-B aligned; the
  // 36-dword pitch at C = 32 spreads a 16-lane group's ds_read_b128 over all 64 banks), the 7 x C dot
  // product read back 4 channels per ds_read_b128 in the same tap / channel order as a scalar loop
  constexpr int RS = C + 4;
  constexpr int CH = C / 8;  // 16-B chunks per input row
  __shared__ __attribute__((aligned(16))) float xs[(CP_T + 6) * RS];
  __shared__ __attribute__((aligned(16))) float ws[7 * C];
  // padded: block (x, y) = samples [x * CP_T, ...) of row y of [B, Tp]; packed (tt: the length-exact vocoder,
  // k_vocoder.hip TileGeo): tt[block] = {first row of the sequence in x, its length, t0, sequence}, the output
  // row of sequence u at out + u * ostride
  int T, t0;
  long xo, oo;
  if (tt) {
    const int4 e = tt[blockIdx.x];
    xo = e.x;
    T = e.y;
    t0 = e.z;
    oo = (long)e.w * ostride;
  } else {
    T = Tp;
    t0 = blockIdx.x * CP_T;
    xo = (long)blockIdx.y * Tp;
    oo = xo;
  }
  const bf16_t* xb = x + xo * C;
  for (int e = threadIdx.x; e < 7 * C; e += CP_T) {  // w[0][c][tap] -> ws[tap][c]
    const int c = e / 7, tap = e % 7;
    ws[tap * C + c] = w[e];
  }
  for (int e = threadIdx.x; e < (CP_T + 6) * CH; e += CP_T) {
    const int rr = e / CH, q = e % CH;
    const int t = t0 - 3 + rr;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (t >= 0 && t < T) {
      const short8 raw = *reinterpret_cast<const short8*>(xb + (long)t * C + q * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float f = bf2f((bf16_t)raw[i]);
        v[i] = f > 0.f ? f : slope * f;  // fused pre-activation
      }
    }
    float4* dst = reinterpret_cast<float4*>(xs + rr * RS + q * 8);
    dst[0] = make_float4(v[0], v[1], v[2], v[3]);
    dst[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  float s = b ? *b : 0.f;
#pragma unroll
  for (int tap = 0; tap < 7; ++tap) {
    const float4* xr = reinterpret_cast<const float4*>(xs + (threadIdx.x + tap) * RS);
    const float4* wr = reinterpret_cast<const float4*>(ws + tap * C);
#pragma unroll
    for (int c4 = 0; c4 < C / 4; ++c4) {
      const float4 xv = xr[c4], wv = wr[c4];
      s += xv.x * wv.x;
      s += xv.y * wv.y;
      s += xv.z * wv.z;
      s += xv.w * wv.w;
    }
  }
  const float y = tanhf(s);
  const long o = oo + t;
  if (outi) {
    float v = y * scale;
    v = fminf(fmaxf(v, -32768.f), 32767.f);
    outi[o] = (int16_t)v;
  } else {
    outf[o] = y;
  }
}

}  // namespace

#define HEAD_DISPATCH(C, ...)                                                     \
  switch (C) {                                                                    \
    case 64: { constexpr int EPL = 1; __VA_ARGS__; break; }                      \
    case 128: { constexpr int EPL = 2; __VA_ARGS__; break; }                     \
    case 256: { constexpr int EPL = 4; __VA_ARGS__; break; }                     \
    case 512: { constexpr int EPL = 8; __VA_ARGS__; break; }                     \
    default: return -1;                                                           \
  }

SSAMD_API int ssamd_head_fwd(const bf16_t* h, const float* w, const float* b, const int64_t* lens, long R, int L,
                             int C, float* out, hipStream_t s) {
  if (R == 0) return 0;
  HEAD_DISPATCH(C, hipLaunchKernelGGL(head_fwd_kernel<EPL>, dim3(cdiv(R, HEAD_ROWS)), dim3(256), 0, s, h, w, b, lens,
                                      R, L, out));
  return (int)hipGetLastError();
}

SSAMD_API long ssamd_head_bwd_ws(long R, int C) { return (long)cdiv(R, HEAD_ROWS) * (C + 1) + seg_colsum_ws(1, C + 1); }

// dw / db (db may be null) are overwritten with fixed-order sums of the per-block partials.
SSAMD_API int ssamd_head_bwd(const float* g, const bf16_t* h, const float* w, const int64_t* lens, long R, int L,
                             int C, bf16_t* dh, float* dw, float* db, float* ws, long ws_floats, hipStream_t s) {
  if (R == 0) return 0;
  const int nblk = cdiv(R, HEAD_ROWS);
  if (ws_floats < ssamd_head_bwd_ws(R, C)) return -3;
  HEAD_DISPATCH(C, hipLaunchKernelGGL(head_bwd_kernel<EPL>, dim3(nblk), dim3(256), 0, s, g, h, w, lens, R, L, dh, ws));
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  return ssamd_seg_colsum(ws, C + 1, 1, nblk, db ? C + 1 : C, dw, 0, 0, C, db, ws + (long)nblk * (C + 1),
                          seg_colsum_ws(1, C + 1), s);
}

SSAMD_API int ssamd_conv_post(const bf16_t* x, const float* w, const float* b, int B, int T, int C, float slope,
                              float scale, float* outf, int16_t* outi, hipStream_t s) {
  if ((long)B * T == 0) return 0;
  dim3 grid(cdiv(T, CP_T), B);
  switch (C) {
    case 32: hipLaunchKernelGGL(conv_post_kernel<32>, grid, dim3(CP_T), 0, s, x, w, b, T, slope, scale, outf, outi,
                                (const int4*)nullptr, 0L); break;
    case 8: hipLaunchKernelGGL(conv_post_kernel<8>, grid, dim3(CP_T), 0, s, x, w, b, T, slope, scale, outf, outi,
                               (const int4*)nullptr, 0L); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// Packed rows (length-exact vocoder): x [R, C], tt = ntt tiles of CP_T rows (k_vocoder.hip TileGeo layout), sample t
// of sequence u written to out[u * ostride + t] (the caller zero-fills the samples past each length).
SSAMD_API int ssamd_conv_post_pk(const bf16_t* x, const float* w, const float* b, const int* tt, int ntt, int C,
                                 float slope, float scale, float* outf, int16_t* outi, long ostride, hipStream_t s) {
  if (ntt <= 0) return 0;
  if (!tt) return -2;
  const int4* t4 = reinterpret_cast<const int4*>(tt);
  switch (C) {
    case 32: hipLaunchKernelGGL(conv_post_kernel<32>, dim3(ntt), dim3(CP_T), 0, s, x, w, b, 0, slope, scale, outf, outi,
                                t4, ostride); break;
    case 8: hipLaunchKernelGGL(conv_post_kernel<8>, dim3(ntt), dim3(CP_T), 0, s, x, w, b, 0, slope, scale, outf, outi,
                               t4, ostride); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_conv_post_tile_rows() { return CP_T; }
