// Native host runtime: batch collation for the data loader.
//
// The reference pads every batch in Python loops (utils/tools.py:285-337: pad_1d /
// pad_2d, one numpy slice assignment per utterance).  For the large MI355X batches
// (hundreds of utterances x ~800 frames x 80 mel channels per rank) this copy is done
// here by a small thread team straight into the destination buffer (which the loader
// pins and ships to the GPU with a non-blocking copy): each item's rows are memcpy'd
// and its tail zero-filled, items are split statically over the threads.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

extern "C" {

// out[i] = [srcs[i][0 .. rows[i]) | zeros up to max_rows], each row row_bytes wide.
// Returns 0, or -1 if some item is longer than max_rows (nothing is written then).
int ssamd_pad_rows(const void* const* srcs, const int64_t* rows, int n, int64_t row_bytes, int64_t max_rows,
                   void* out, int nthreads) {
  for (int i = 0; i < n; ++i)
    if (rows[i] < 0 || rows[i] > max_rows) return -1;
  const int64_t item_bytes = max_rows * row_bytes;
  auto work = [&](int lo, int hi) {
    for (int i = lo; i < hi; ++i) {
      char* dst = static_cast<char*>(out) + (int64_t)i * item_bytes;
      const int64_t used = rows[i] * row_bytes;
      if (used) std::memcpy(dst, srcs[i], (size_t)used);
      if (used < item_bytes) std::memset(dst + used, 0, (size_t)(item_bytes - used));
    }
  };
  const int64_t total = (int64_t)n * item_bytes;
  int t = std::max(1, std::min(nthreads, n));
  if (total < (1 << 20)) t = 1;  // small batches: threads cost more than they save
  if (t == 1) {
    work(0, n);
    return 0;
  }
  std::vector<std::thread> team;
  team.reserve(t);
  for (int k = 0; k < t; ++k) {
    const int lo = (int)((int64_t)n * k / t), hi = (int)((int64_t)n * (k + 1) / t);
    team.emplace_back(work, lo, hi);
  }
  for (auto& th : team) th.join();
  return 0;
}

}  // extern "C"
