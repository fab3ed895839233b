// Native host runtime: F0 estimation for the offline preprocessor.
//
// The reference extracts pitch with pyworld (the WORLD vocoder's C++ library):
// `pw.dio` followed by `pw.stonemask` (preprocessor/preprocessor.py:182-187, frame
// period = hop / sr).  pyworld is not installable in this image, so both algorithms
// are implemented here from their published descriptions (M. Morise, "DIO: a fast
// and reliable F0 estimator", and the StoneMask instantaneous-frequency refinement):
//
// DIO: the DC-free, 50 Hz low-cut spectrum of the whole utterance is low-passed once
// per candidate band (Nuttall window whose length follows the band's upper F0); the
// four zero-crossing event families of each filtered signal (negative- and positive-
// going crossings, peaks, dips) give interval-based F0 tracks that are interpolated to
// the frame grid.  Their mean is the band's candidate, their relative spread its score;
// a candidate outside [band/2, band] or [floor, ceil] is rejected.  Per frame the best
// scoring candidate wins, then the contour is cleaned: frame-to-frame jumps beyond
// `allowed_range` removed, voiced runs shorter than the minimum voice length removed,
// and voiced runs extended forward / backward through continuous candidates.
//
// StoneMask: per voiced frame, a 3-period Blackman window and its derivative window
// give the instantaneous frequency at the first <= 6 harmonics; the refined F0 is the
// amplitude-weighted mean of IF / harmonic number (kept only within 20 % of the input).
//
// Same API contract as pyworld (frame grid t_i = i * frame_period, 0 = unvoiced).
// Exact numerical parity with pyworld is unpinned (no pyworld in the image); the CPU
// tests check the estimator on signals with a known F0 (tests/test_f0_world.py).
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdint>
#include <vector>

namespace {

using cplx = std::complex<double>;
constexpr double kPi = 3.14159265358979323846;
constexpr double kSafe = 1e-12;
constexpr double kMaxScore = 100000.0;

int round_half_away(double x) { return x >= 0 ? (int)(x + 0.5) : (int)(x - 0.5); }

// in-place iterative radix-2 FFT (sign -1: forward, +1: inverse without 1/N)
void fft(std::vector<cplx>& a, int sign) {
  const size_t n = a.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    const double ang = sign * 2.0 * kPi / (double)len;
    const size_t half = len >> 1;
    std::vector<cplx> w(half);
    for (size_t k = 0; k < half; ++k) w[k] = cplx(std::cos(ang * k), std::sin(ang * k));
    for (size_t i = 0; i < n; i += len)
      for (size_t k = 0; k < half; ++k) {
        const cplx u = a[i + k], v = a[i + k + half] * w[k];
        a[i + k] = u + v;
        a[i + k + half] = u - v;
      }
  }
}

size_t pow2_at_least(size_t n) {
  size_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

// linear interpolation with end-segment extrapolation (x ascending)
void interp_linear(const std::vector<double>& x, const std::vector<double>& y, const double* xi, int n,
                   double* yi) {
  const size_t m = x.size();
  size_t k = 0;
  for (int i = 0; i < n; ++i) {
    while (k + 2 < m && xi[i] >= x[k + 1]) ++k;
    const double dx = x[k + 1] - x[k];
    const double s = dx != 0.0 ? (y[k + 1] - y[k]) / dx : 0.0;
    yi[i] = y[k] + s * (xi[i] - x[k]);
  }
}

// negative-going zero crossings of s -> (interval locations [s], F0 = 1 / interval [Hz])
void zero_crossings(const std::vector<double>& s, double fs, std::vector<double>& loc, std::vector<double>& f0) {
  std::vector<double> edges;
  for (size_t i = 0; i + 1 < s.size(); ++i)
    if (s[i] > 0.0 && s[i + 1] <= 0.0) edges.push_back((double)i + s[i] / (s[i] - s[i + 1]));
  loc.clear();
  f0.clear();
  for (size_t i = 0; i + 1 < edges.size(); ++i) {
    loc.push_back((edges[i] + edges[i + 1]) * 0.5 / fs);
    f0.push_back(fs / (edges[i + 1] - edges[i]));
  }
}

struct DioParams {
  double fs, frame_period, f0_floor, f0_ceil, channels_in_octave, allowed_range;
};

// one band's candidate / score tracks
void band_candidate(const std::vector<cplx>& spec, size_t fft_size, int y_length, double fs, double boundary_f0,
                    const DioParams& p, const std::vector<double>& tpos, double* cand, double* score) {
  const int n_frames = (int)tpos.size();
  const int half_avg = round_half_away(fs / boundary_f0 / 2.0);
  const int wl = half_avg * 4;
  std::vector<cplx> lp(fft_size, cplx(0, 0));
  for (int i = 0; i < wl; ++i) {  // Nuttall low-pass
    const double x = wl > 1 ? (double)i / (double)(wl - 1) : 0.0;
    lp[i] = 0.355768 - 0.487396 * std::cos(2 * kPi * x) + 0.144232 * std::cos(4 * kPi * x) -
            0.012604 * std::cos(6 * kPi * x);
  }
  fft(lp, -1);
  for (size_t i = 0; i < fft_size; ++i) lp[i] *= spec[i];
  fft(lp, +1);
  std::vector<double> filt(y_length);
  const int bias = half_avg * 2;  // group delay of the symmetric window
  for (int i = 0; i < y_length; ++i) filt[i] = (size_t)(i + bias) < fft_size ? lp[i + bias].real() / fft_size : 0.0;

  std::vector<double> neg = filt, pos(y_length), peak(y_length), dip(y_length);
  for (int i = 0; i < y_length; ++i) pos[i] = -filt[i];
  for (int i = 0; i + 1 < y_length; ++i) peak[i] = filt[i] - filt[i + 1];
  if (y_length > 0) peak[y_length - 1] = 0.0;
  for (int i = 0; i < y_length; ++i) dip[i] = -peak[i];
  std::vector<double> loc[4], f0[4];
  zero_crossings(neg, fs, loc[0], f0[0]);
  zero_crossings(pos, fs, loc[1], f0[1]);
  zero_crossings(peak, fs, loc[2], f0[2]);
  zero_crossings(dip, fs, loc[3], f0[3]);
  for (int k = 0; k < 4; ++k)
    if (loc[k].size() < 2) {
      for (int i = 0; i < n_frames; ++i) {
        cand[i] = 0.0;
        score[i] = kMaxScore;
      }
      return;
    }
  std::vector<double> tr[4];
  for (int k = 0; k < 4; ++k) {
    tr[k].resize(n_frames);
    interp_linear(loc[k], f0[k], tpos.data(), n_frames, tr[k].data());
  }
  for (int i = 0; i < n_frames; ++i) {
    const double mean = (tr[0][i] + tr[1][i] + tr[2][i] + tr[3][i]) * 0.25;
    double var = 0.0;
    for (int k = 0; k < 4; ++k) var += (tr[k][i] - mean) * (tr[k][i] - mean);
    const double sd = std::sqrt(var / 3.0);
    if (mean > boundary_f0 || mean < boundary_f0 * 0.5 || mean > p.f0_ceil || mean < p.f0_floor) {
      cand[i] = 0.0;
      score[i] = kMaxScore;
    } else {
      cand[i] = mean;
      score[i] = sd / (mean + kSafe);  // relative dispersion of the four event families
    }
  }
}

double select_best(double ref, const std::vector<std::vector<double>>& cands, int j, double allowed) {
  double best = 0.0, err = allowed;
  for (const auto& c : cands) {
    const double e = std::fabs(ref - c[j]) / (ref + kSafe);
    if (e > err) continue;
    best = c[j];
    err = e;
  }
  return best;
}

void fix_contour(const DioParams& p, const std::vector<std::vector<double>>& cands, std::vector<double>& f0) {
  const int n = (int)f0.size();
  const int vmin = (int)(0.5 + 1000.0 / p.frame_period / p.f0_floor) * 2 + 1;
  if (n <= vmin) return;
  // step 1: drop the edges and frame-to-frame jumps beyond allowed_range
  std::vector<double> base = f0, s1(n, 0.0);
  for (int i = 0; i < vmin && i < n; ++i) base[i] = 0.0;
  for (int i = std::max(0, n - vmin); i < n; ++i) base[i] = 0.0;
  for (int i = vmin; i < n; ++i)
    s1[i] = std::fabs((base[i] - base[i - 1]) / (kSafe + base[i])) < p.allowed_range ? base[i] : 0.0;
  // step 2: drop voiced runs shorter than the minimum voice length
  std::vector<double> s2 = s1;
  const int c = (vmin - 1) / 2;
  for (int i = c; i < n - c; ++i)
    for (int j = -c; j <= c; ++j)
      if (s1[i + j] == 0.0) {
        s2[i] = 0.0;
        break;
      }
  // voiced run boundaries of s2
  std::vector<int> starts, ends;  // first voiced frame / last voiced frame of each run
  for (int i = 0; i < n; ++i) {
    const bool v = s2[i] != 0.0, pv = i > 0 && s2[i - 1] != 0.0;
    if (v && !pv) starts.push_back(i);
    if (pv && !v) ends.push_back(i - 1);
  }
  if (!s2.empty() && s2[n - 1] != 0.0) ends.push_back(n - 1);
  const int runs = (int)starts.size();
  // step 3: extend every run forward through continuous candidates
  std::vector<double> s3 = s2;
  for (int r = 0; r < runs; ++r) {
    const int limit = r == runs - 1 ? n - 1 : starts[r + 1] - 1;
    for (int j = ends[r]; j < limit; ++j) {
      s3[j + 1] = select_best(s3[j], cands, j + 1, p.allowed_range);
      if (s3[j + 1] == 0.0) break;
    }
  }
  // step 4: extend backward
  std::vector<double> s4 = s3;
  for (int r = runs - 1; r >= 0; --r) {
    const int limit = r == 0 ? 1 : ends[r - 1] + 1;
    for (int j = starts[r]; j > limit; --j) {
      s4[j - 1] = select_best(s4[j], cands, j - 1, p.allowed_range);
      if (s4[j - 1] == 0.0) break;
    }
  }
  f0.swap(s4);
}

double refine_one(const double* x, int64_t n, double fs, double t, double f0) {
  if (f0 <= 40.0 || f0 > fs / 12.0) return 0.0;
  const int hw = (int)(1.5 * fs / f0 + 1.0);
  const int len = 2 * hw + 1;
  const double win_t = (double)len / fs;
  const size_t nfft = (size_t)1 << (1 + (int)(std::log((double)len) / std::log(2.0)));
  std::vector<double> w(len), dw(len);
  std::vector<int64_t> idx(len);
  const int c0 = round_half_away(t * fs);
  for (int i = 0; i < len; ++i) {
    idx[i] = (int64_t)c0 + i - hw - 1;  // WORLD samples index_raw - 1 (one sample before the frame time)
    const double u = (double)idx[i] / fs - t;
    w[i] = 0.42 + 0.5 * std::cos(2 * kPi * u / win_t) + 0.08 * std::cos(4 * kPi * u / win_t);  // Blackman
  }
  dw[0] = -w[1] * 0.5;
  for (int i = 1; i + 1 < len; ++i) dw[i] = -(w[i + 1] - w[i - 1]) * 0.5;
  dw[len - 1] = w[len - 2] * 0.5;
  std::vector<cplx> A(nfft, cplx(0, 0)), D(nfft, cplx(0, 0));
  for (int i = 0; i < len; ++i) {
    const double s = x[std::max<int64_t>(0, std::min<int64_t>(n - 1, idx[i]))];
    A[i] = s * w[i];
    D[i] = s * dw[i];
  }
  fft(A, -1);
  fft(D, -1);
  const int nh = std::min((int)(fs / 2.0 / f0), 6);
  double num = 0.0, den = 0.0;
  for (int h = 0; h < nh; ++h) {
    const int k = round_half_away(f0 * (double)nfft / fs * (h + 1));
    if (k < 0 || (size_t)k > nfft / 2) break;
    const double pw = std::norm(A[k]);
    // instantaneous frequency of bin k: k fs / N + Im(conj(A) D) / |A|^2 * fs / (2 pi)
    const double cross = A[k].real() * D[k].imag() - A[k].imag() * D[k].real();
    const double ifreq = (double)k * fs / (double)nfft + cross / (pw + kSafe) * fs / (2.0 * kPi);
    const double amp = std::sqrt(pw);
    num += amp * ifreq;
    den += amp * (h + 1);
  }
  const double m = num / (den + kSafe);
  return std::fabs(m - f0) > f0 * 0.2 ? f0 : m;
}

}  // namespace

extern "C" {

// Number of frames of the DIO grid for n samples (t_i = i * frame_period ms).
int64_t ssamd_dio_frames(int64_t n, double fs, double frame_period) {
  return (int64_t)(1000.0 * (double)n / fs / frame_period) + 1;
}

// DIO F0 candidates + contour.  f0 / tpos: ssamd_dio_frames(n, fs, frame_period) entries.
// Returns 0, or -1 on bad arguments.
int ssamd_dio(const double* x, int64_t n, double fs, double frame_period, double f0_floor, double f0_ceil,
              double channels_in_octave, double allowed_range, double* f0, double* tpos) {
  if (!x || n <= 0 || fs <= 0 || frame_period <= 0 || f0_floor <= 0 || f0_ceil <= f0_floor || channels_in_octave <= 0)
    return -1;
  const DioParams p{fs, frame_period, f0_floor, f0_ceil, channels_in_octave, allowed_range};
  const int64_t nf = ssamd_dio_frames(n, fs, frame_period);
  std::vector<double> t(nf);
  for (int64_t i = 0; i < nf; ++i) t[i] = (double)i * frame_period / 1000.0;
  const int bands = 1 + (int)(std::log(f0_ceil / f0_floor) / std::log(2.0) * channels_in_octave);
  std::vector<double> bf(bands);
  for (int i = 0; i < bands; ++i) bf[i] = f0_floor * std::pow(2.0, (i + 1) / channels_in_octave);
  const int y_length = (int)n;
  const size_t fft_size = pow2_at_least((size_t)y_length + 4 * (size_t)(1.0 + fs / bf[0] / 2.0));

  // DC-free spectrum with the 50 Hz low-cut (zero-phase: delta - normalised Hann low-pass)
  double mean = 0.0;
  for (int64_t i = 0; i < n; ++i) mean += x[i];
  mean /= (double)n;
  std::vector<cplx> spec(fft_size, cplx(0, 0));
  for (int64_t i = 0; i < n; ++i) spec[i] = x[i] - mean;
  fft(spec, -1);
  const int N = round_half_away(fs / 50.0) * 2 + 1;
  std::vector<double> h(N);
  double hs = 0.0;
  for (int i = 1; i <= N; ++i) {
    h[i - 1] = 0.5 - 0.5 * std::cos(i * 2.0 * kPi / (N + 1));
    hs += h[i - 1];
  }
  std::vector<cplx> lc(fft_size, cplx(0, 0));
  const int half = (N - 1) / 2;
  for (int i = 0; i < N; ++i) {
    const int64_t pos = ((int64_t)i - half + (int64_t)fft_size) % (int64_t)fft_size;  // centred at 0
    lc[pos] += -h[i] / hs;
  }
  lc[0] += 1.0;
  fft(lc, -1);
  for (size_t i = 0; i < fft_size; ++i) spec[i] *= lc[i];

  std::vector<std::vector<double>> cand(bands, std::vector<double>(nf)), score(bands, std::vector<double>(nf));
  for (int b = 0; b < bands; ++b) band_candidate(spec, fft_size, y_length, fs, bf[b], p, t, cand[b].data(), score[b].data());
  std::vector<double> best(nf);
  for (int64_t i = 0; i < nf; ++i) {
    double s = score[0][i];
    best[i] = cand[0][i];
    for (int b = 1; b < bands; ++b)
      if (s > score[b][i]) {
        s = score[b][i];
        best[i] = cand[b][i];
      }
  }
  fix_contour(p, cand, best);
  for (int64_t i = 0; i < nf; ++i) {
    f0[i] = best[i];
    if (tpos) tpos[i] = t[i];
  }
  return 0;
}

// StoneMask refinement of f0 (nf frames at times tpos [s]) -> out (may alias f0).
int ssamd_stonemask(const double* x, int64_t n, double fs, const double* tpos, const double* f0, int64_t nf,
                    double* out) {
  if (!x || n <= 0 || fs <= 0 || !tpos || !f0 || !out) return -1;
  for (int64_t i = 0; i < nf; ++i) out[i] = refine_one(x, n, fs, tpos[i], f0[i]);
  return 0;
}

}  // extern "C"
