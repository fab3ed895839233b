// Sanitizer self-test of the native host runtime (csrc/host_collate.cpp, csrc/host_f0.cpp).
//
// Built by `python csrc/build.py --sanitize` twice -- once with
// -fsanitize=address,undefined and once with -fsanitize=thread -- and run by
// tests/test_native_host.py.  It drives ssamd_pad_rows through the shapes the
// data loader produces (empty items, items exactly max_rows long, the single-
// thread small-batch path and the threaded path, more threads than items) and
// checks every output byte against a scalar reference, so an out-of-bounds
// copy, a use of uninitialised padding or a data race between the thread team's
// item ranges is reported by the sanitizer runtime (non-zero exit).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

extern "C" int ssamd_pad_rows(const void* const* srcs, const int64_t* rows, int n, int64_t row_bytes,
                              int64_t max_rows, void* out, int nthreads);
extern "C" int64_t ssamd_dio_frames(int64_t n, double fs, double frame_period);
extern "C" int ssamd_dio(const double* x, int64_t n, double fs, double frame_period, double f0_floor,
                         double f0_ceil, double channels_in_octave, double allowed_range, double* f0, double* tpos);
extern "C" int ssamd_stonemask(const double* x, int64_t n, double fs, const double* tpos, const double* f0,
                               int64_t nf, double* out);

// F0 estimator (csrc/host_f0.cpp) on exact-size buffers: a 150 Hz tone, very short inputs
static int check_f0() {
  int bad = 0;
  const double fs = 22050.0, fp = 256.0 / 22050.0 * 1000.0;
  for (int64_t n : {int64_t(1), int64_t(300), int64_t(22050)}) {
    std::vector<double> x((size_t)n);
    for (int64_t i = 0; i < n; ++i) x[(size_t)i] = 0.3 * std::sin(2.0 * 3.141592653589793 * 150.0 * i / fs);
    const int64_t nf = ssamd_dio_frames(n, fs, fp);
    std::vector<double> f0((size_t)nf), t((size_t)nf), r((size_t)nf);
    bad += ssamd_dio(x.data(), n, fs, fp, 71.0, 800.0, 2.0, 0.1, f0.data(), t.data()) != 0;
    bad += ssamd_stonemask(x.data(), n, fs, t.data(), f0.data(), nf, r.data()) != 0;
    if (n == 22050) {
      const double mid = r[(size_t)nf / 2];
      bad += !(mid > 148.0 && mid < 152.0);
    }
  }
  return bad;
}

static int check_case(std::mt19937& rng, int n, int64_t row_bytes, int64_t max_rows, int nthreads) {
  std::vector<std::vector<unsigned char>> items(n);
  std::vector<const void*> ptrs(n);
  std::vector<int64_t> rows(n);
  std::uniform_int_distribution<int64_t> len(0, max_rows);
  for (int i = 0; i < n; ++i) {
    rows[i] = (i == 0) ? max_rows : (i == 1 ? 0 : len(rng));
    // exact-size heap blocks: any read past rows[i]*row_bytes is an ASan report
    items[i].resize((size_t)(rows[i] * row_bytes));
    for (auto& b : items[i]) b = (unsigned char)(rng() & 0xff);
    ptrs[i] = items[i].empty() ? nullptr : items[i].data();
  }
  std::vector<unsigned char> out((size_t)(n * max_rows * row_bytes));
  if (ssamd_pad_rows(ptrs.data(), rows.data(), n, row_bytes, max_rows, out.data(), nthreads) != 0) {
    std::fprintf(stderr, "unexpected error return (n=%d)\n", n);
    return 1;
  }
  for (int i = 0; i < n; ++i) {
    const unsigned char* o = out.data() + (size_t)i * max_rows * row_bytes;
    const int64_t used = rows[i] * row_bytes;
    for (int64_t b = 0; b < max_rows * row_bytes; ++b) {
      const unsigned char want = b < used ? items[i][(size_t)b] : 0;
      if (o[b] != want) {
        std::fprintf(stderr, "mismatch item %d byte %lld\n", i, (long long)b);
        return 1;
      }
    }
  }
  return 0;
}

int main() {
  std::mt19937 rng(1234);
  int bad = 0;
  bad += check_case(rng, 3, 4, 5, 8);            // tiny: single-thread path
  bad += check_case(rng, 64, 320, 900, 8);       // mel-like rows, threaded (> 1 MiB)
  bad += check_case(rng, 5, 320, 1000, 16);      // fewer items than threads
  bad += check_case(rng, 300, 8, 200, 8);        // int64 scalars
  // too-long item: must refuse without writing
  {
    unsigned char src[16] = {0};
    const void* p = src;
    int64_t r = 4;
    unsigned char out[12];
    std::memset(out, 0xab, sizeof(out));
    if (ssamd_pad_rows(&p, &r, 1, 4, 3, out, 4) != -1) bad += 1;
    for (unsigned char c : out) bad += (c != 0xab);
  }
  bad += check_f0();
  if (bad) {
    std::fprintf(stderr, "selftest_host_collate: %d failures\n", bad);
    return 1;
  }
  std::printf("selftest_host_collate ok\n");
  return 0;
}
