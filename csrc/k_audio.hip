// Log-mel front-end (reference audio/stft.py:130-178 TacotronSTFT.mel_spectrogram; SURVEY §2.3
// A1/A2): reflect-padded framing, Hann window, real DFT magnitude, mel projection, log(clamp),
// and energy = ||X||_2 over frequency -- one fused kernel, one workgroup per (utterance, frame).
//
// The DFT is a radix-2 decimation-in-time FFT on the frame in LDS (fp32: the log-mel feeds a
// log, so bf16 MFMA products would cost ~1e-2 in log space); twiddles are a per-block LDS table.
// The mel projection reads the [n_mel, n_fft/2+1] basis from L2 (164 KB, shared by all blocks):
// wave w computes mel rows w, w+4, ... with lanes striding over frequency + a wave reduction.
// Inference / preprocessing only (no backward): the reference-audio style path and offline
// features.  Used by speakingstyle_amd/audio/stft.py on GPU tensors.
#include "common.h"

namespace {

constexpr int NT = 256;

template <int NFFT>
__global__ void __launch_bounds__(NT) logmel_kernel(const float* __restrict__ wav, long N, int hop, int frames,
                                                    const float* __restrict__ window, const float* __restrict__ basis,
                                                    int n_mel, float clip, float* __restrict__ mel,
                                                    float* __restrict__ energy) {
  constexpr int NB = NFFT / 2 + 1;
  constexpr int LOG2 = __builtin_ctz(NFFT);
  __shared__ float re[NFFT], im[NFFT], cs[NFFT / 2], sn[NFFT / 2], mag[NB];
  __shared__ float red[NT / 64];
  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const float* x = wav + (long)b * N;
  for (int t = tid; t < NFFT / 2; t += NT) {
    float s, c;
    sincospif(2.f * (float)t / (float)NFFT, &s, &c);
    cs[t] = c;
    sn[t] = -s;  // forward transform: exp(-2 pi i t / NFFT)
  }
  // centre-padded frame f starts at sample f*hop - NFFT/2 (reflect padding, no edge repeat)
  const long start = (long)f * hop - NFFT / 2;
  for (int i = tid; i < NFFT; i += NT) {
    long s = start + i;
    if (s < 0) s = -s;
    if (s >= N) s = 2 * (N - 1) - s;
    const float v = (s >= 0 && s < N) ? x[s] * window[i] : 0.f;
    const int r = (int)(__brev((unsigned)i) >> (32 - LOG2));
    re[r] = v;
    im[r] = 0.f;
  }
  __syncthreads();
#pragma unroll 1
  for (int lh = 0; lh < LOG2; ++lh) {
    const int half = 1 << lh;
    const int tstep = NFFT >> (lh + 1);  // twiddle index stride for span 2*half
    for (int k = tid; k < NFFT / 2; k += NT) {
      const int j = k & (half - 1);
      const int i0 = ((k >> lh) << (lh + 1)) + j, i1 = i0 + half;
      const float wr = cs[j * tstep], wi = sn[j * tstep];
      const float xr = re[i1] * wr - im[i1] * wi;
      const float xi = re[i1] * wi + im[i1] * wr;
      re[i1] = re[i0] - xr;
      im[i1] = im[i0] - xi;
      re[i0] += xr;
      im[i0] += xi;
    }
    __syncthreads();
  }
  float e = 0.f;
  for (int k = tid; k < NB; k += NT) {
    const float m2 = re[k] * re[k] + im[k] * im[k];
    mag[k] = sqrtf(m2);
    e += m2;
  }
  e = wave_sum(e);
  if ((tid & 63) == 0) red[tid >> 6] = e;
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += red[w];
    energy[(long)b * frames + f] = sqrtf(s);
  }
  const int lane = tid & 63;
  for (int m = tid >> 6; m < n_mel; m += NT / 64) {
    const float* row = basis + (long)m * NB;
    float acc = 0.f;
    for (int k = lane; k < NB; k += 64) acc += row[k] * mag[k];
    acc = wave_sum(acc);
    if (lane == 0) mel[((long)b * n_mel + m) * frames + f] = logf(fmaxf(acc, clip));
  }
}

}  // namespace

// wav [B, N] fp32; window [n_fft] (win_length window centred, zero padded); basis [n_mel, n_fft/2+1]
// -> mel [B, n_mel, frames] (log, clamp at `clip`), energy [B, frames];  frames = N / hop + 1
SSAMD_API int ssamd_logmel(const float* wav, int B, long N, int n_fft, int hop, const float* window, const float* basis,
                           int n_mel, float clip, float* mel, float* energy, hipStream_t s) {
  if (N < n_fft / 2 + 1 || hop <= 0) return -2;  // reflect padding needs N > n_fft / 2
  const int frames = (int)(N / hop + 1);
  if (B == 0) return 0;
  dim3 grid(frames, B);
  switch (n_fft) {
    case 512:
      hipLaunchKernelGGL(logmel_kernel<512>, grid, dim3(NT), 0, s, wav, N, hop, frames, window, basis, n_mel, clip, mel, energy);
      break;
    case 1024:
      hipLaunchKernelGGL(logmel_kernel<1024>, grid, dim3(NT), 0, s, wav, N, hop, frames, window, basis, n_mel, clip, mel, energy);
      break;
    case 2048:
      hipLaunchKernelGGL(logmel_kernel<2048>, grid, dim3(NT), 0, s, wav, N, hop, frames, window, basis, n_mel, clip, mel, energy);
      break;
    default:
      return -2;
  }
  return (int)hipGetLastError();
}
