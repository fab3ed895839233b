// HiFi-GAN MRF residual layer, fused (reference hifigan/models.py:20-103 ResBlock1):
//
//     y = x + conv2( lrelu( conv1_d( lrelu(x) ) + b1 ) ) + b2          [channel-last, C channels]
//     out = (acc_in + y) * out_scale   (optional: the MRF branch sum / mean, in place)
//
// for the narrow high-rate stages (C = 32 / 64 at 128-256x the mel rate), where a generic GEMM
// tile wastes most of its N width and every separate lrelu / add pass re-streams GBs of
// activations.  One workgroup owns BM = 128 output rows of one utterance:
//   1. stage lrelu(x) for the rows both convs need (halo d*(K-1)/2 + (K-1)/2 each side, zero
//      outside [0, T)) into LDS;
//   2. conv1 (dilation d) for BM + K-1 rows on v_mfma_f32_16x16x32_bf16: A fragments from the
//      LDS tile at row offset tap*d, B fragments (weights [C][K][C], L2-resident, shared by all
//      blocks) streamed per tap; + b1, lrelu, zero outside [0, T) -> t1 tile in LDS (bf16);
//   3. conv2 (dilation 1) over the t1 tile, + b2 -> fp32 tile in LDS (aliases the x tile);
//   4. coalesced 16-B epilogue: + x (residual), + acc_in, * out_scale -> out.
// Each activation byte is read once (plus the halo) and written once per layer: the unfused
// path (lrelu, conv, lrelu-epilogue conv, add) moves ~4x more.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int BM = 128;
constexpr int MAXD = 5;

template <int C, int K>
struct RB {
  static constexpr int H2 = (K - 1) / 2;
  static constexpr int R1 = BM + 2 * H2;           // t1 rows the second conv needs
  static constexpr int R1P = (R1 + 15) / 16 * 16;  // padded to whole 16-row MFMA blocks
  static constexpr int NRB1 = R1P / 16, NRB2 = BM / 16;
  static constexpr int LDC = C + 8;                // LDS pitch (bf16): 16-B rows, conflict-free row reads
  static constexpr int RX = R1P + (K - 1) * MAXD;  // staged x rows at the largest dilation
  static constexpr int NS = C / 16;                // 16-wide output sub-tiles
  static constexpr int KC = C / 32;                // 32-deep K chunks per tap
  static constexpr int XS_BYTES = RX * LDC * 2;
  static constexpr int OUT_BYTES = BM * C * 4;
  static constexpr int R0_BYTES = ((XS_BYTES > OUT_BYTES ? XS_BYTES : OUT_BYTES) + 15) / 16 * 16;
  static constexpr int LDS = R0_BYTES + R1P * LDC * 2;
  static constexpr int MAXRB = (NRB1 + 3) / 4;     // row blocks per wave (4 waves)
};

__device__ __forceinline__ float lrelu(float v, float s) { return v >= 0.f ? v : v * s; }

// acc[r][s] += A(rows of `src` at offset row_off + rb*16, K-chunk) * W[:, tap, chunk]
template <int C, int K>
__device__ __forceinline__ void conv_tile(const bf16_t* __restrict__ src, int row_step, const bf16_t* __restrict__ w,
                                          int nrb, int wave, int lane, float4v (&acc)[RB<C, K>::MAXRB][RB<C, K>::NS]) {
  using R = RB<C, K>;
  const int col = lane & 15, quad = lane >> 4;
#pragma unroll
  for (int r = 0; r < R::MAXRB; ++r)
#pragma unroll
    for (int s = 0; s < R::NS; ++s) acc[r][s] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int tap = 0; tap < K; ++tap) {
#pragma unroll
    for (int kc = 0; kc < R::KC; ++kc) {
      short8 bf[R::NS];
#pragma unroll
      for (int s = 0; s < R::NS; ++s)
        bf[s] = *reinterpret_cast<const short8*>(w + ((long)(s * 16 + col) * K + tap) * C + kc * 32 + 8 * quad);
#pragma unroll
      for (int r = 0; r < R::MAXRB; ++r) {
        const int rb = wave + 4 * r;
        if (rb < nrb) {
          const short8 a = *reinterpret_cast<const short8*>(
              src + (long)(rb * 16 + col + tap * row_step) * R::LDC + kc * 32 + 8 * quad);
#pragma unroll
          for (int s = 0; s < R::NS; ++s) acc[r][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bf[s], acc[r][s], 0, 0, 0);
        }
      }
    }
  }
}

template <int C, int K>
__global__ void __launch_bounds__(NT) resblock_layer_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w1,
                                                            const float* __restrict__ b1, const bf16_t* __restrict__ w2,
                                                            const float* __restrict__ b2, const bf16_t* acc_in,
                                                            bf16_t* out, int T, int tiles, int d, float slope,
                                                            float out_scale) {
  using R = RB<C, K>;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(lds);               // [RX][LDC]  lrelu(x) tile
  float* os = reinterpret_cast<float*>(lds);                 // [BM][C]    conv2 + b2 (after conv1)
  bf16_t* t1 = reinterpret_cast<bf16_t*>(lds + R::R0_BYTES);  // [R1P][LDC] lrelu(conv1 + b1)
  const int b = blockIdx.x / tiles, t0 = (blockIdx.x - b * tiles) * BM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int h1 = d * (K - 1) / 2;
  const bf16_t* xb = x + (long)b * T * C;

  // 1. lrelu(x) rows [t0 - h1 - H2, ...): only the rows this dilation reads
  const int rows_x = R::R1P + (K - 1) * d;
  for (int q = tid; q < rows_x * (C / 8); q += NT) {
    const int r = q / (C / 8), c0 = (q - r * (C / 8)) * 8;
    const int t = t0 - h1 - R::H2 + r;
    short8 v;
    if (t >= 0 && t < T) {
      v = *reinterpret_cast<const short8*>(xb + (long)t * C + c0);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (short)f2bf(lrelu(bf2f((bf16_t)v[i]), slope));
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = 0;
    }
    *reinterpret_cast<short8*>(xs + r * R::LDC + c0) = v;
  }
  __syncthreads();

  // 2. conv1 (dilation d): t1 row i <- x rows i + tap*d
  float4v acc[R::MAXRB][R::NS];
  conv_tile<C, K>(xs, d, w1, R::NRB1, wave, lane, acc);
#pragma unroll
  for (int r = 0; r < R::MAXRB; ++r) {
    const int rb = wave + 4 * r;
    if (rb < R::NRB1) {
#pragma unroll
      for (int s = 0; s < R::NS; ++s) {
        const int ch = s * 16 + col;
        const float bias = b1[ch];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = rb * 16 + 4 * quad + i;
          const int t = t0 - R::H2 + row;
          const float v = (row < R::R1 && t >= 0 && t < T) ? lrelu(acc[r][s][i] + bias, slope) : 0.f;
          t1[row * R::LDC + ch] = f2bf(v);
        }
      }
    }
  }
  __syncthreads();  // t1 complete; the x tile is dead from here on (os aliases it)

  // 3. conv2 (dilation 1): out row j <- t1 rows j + tap
  conv_tile<C, K>(t1, 1, w2, R::NRB2, wave, lane, acc);
#pragma unroll
  for (int r = 0; r < R::MAXRB; ++r) {
    const int rb = wave + 4 * r;
    if (rb < R::NRB2) {
#pragma unroll
      for (int s = 0; s < R::NS; ++s) {
        const int ch = s * 16 + col;
        const float bias = b2[ch];
#pragma unroll
        for (int i = 0; i < 4; ++i) os[(rb * 16 + 4 * quad + i) * C + ch] = acc[r][s][i] + bias;
      }
    }
  }
  __syncthreads();

  // 4. + residual (+ MRF accumulator), scale, coalesced 16-B stores
  bf16_t* ob = out + (long)b * T * C;
  const bf16_t* ab = acc_in ? acc_in + (long)b * T * C : nullptr;
  for (int q = tid; q < BM * (C / 8); q += NT) {
    const int j = q / (C / 8), c0 = (q - j * (C / 8)) * 8;
    const int t = t0 + j;
    if (t >= T) continue;
    const short8 xr = *reinterpret_cast<const short8*>(xb + (long)t * C + c0);
    short8 ar;
    if (ab) ar = *reinterpret_cast<const short8*>(ab + (long)t * C + c0);
    short8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = os[j * C + c0 + i] + bf2f((bf16_t)xr[i]);
      if (ab) v += bf2f((bf16_t)ar[i]);
      o[i] = (short)f2bf(v * out_scale);
    }
    *reinterpret_cast<short8*>(ob + (long)t * C + c0) = o;
  }
}

template <int C, int K>
int launch_rb(const bf16_t* x, const bf16_t* w1, const float* b1, const bf16_t* w2, const float* b2,
              const bf16_t* acc_in, bf16_t* out, int B, int T, int d, float slope, float out_scale, hipStream_t s) {
  using R = RB<C, K>;
  static bool lds_set = false;
  if (!lds_set) {
    allow_lds(resblock_layer_kernel<C, K>, R::LDS);
    lds_set = true;
  }
  const int tiles = (T + BM - 1) / BM;
  hipLaunchKernelGGL((resblock_layer_kernel<C, K>), dim3((long)B * tiles), dim3(NT), R::LDS, s, x, w1, b1, w2, b2,
                     acc_in, out, T, tiles, d, slope, out_scale);
  return (int)hipGetLastError();
}

}  // namespace

// x / out / acc_in [B, T, C] bf16 (acc_in may alias out, or be null); w1 / w2 bf16 [C][K][C] (the
// implicit-GEMM forward image); b1 / b2 fp32 [C].  C in {32, 64}, K in {3, 7, 11}, 1 <= d <= 5.
SSAMD_API int ssamd_resblock_layer(const bf16_t* x, const bf16_t* w1, const float* b1, const bf16_t* w2,
                                   const float* b2, const bf16_t* acc_in, bf16_t* out, int B, int T, int C, int K,
                                   int d, float slope, float out_scale, hipStream_t s) {
  if (d < 1 || d > MAXD) return -2;
  if ((long)B * T == 0) return 0;
#define RB_CASE(CC, KK) \
  if (C == CC && K == KK) return launch_rb<CC, KK>(x, w1, b1, w2, b2, acc_in, out, B, T, d, slope, out_scale, s);
  RB_CASE(32, 3) RB_CASE(32, 7) RB_CASE(32, 11)
  RB_CASE(64, 3) RB_CASE(64, 7) RB_CASE(64, 11)
#undef RB_CASE
  return -2;
}
