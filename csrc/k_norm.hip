// Fused residual + LayerNorm + dropout + FiLM + pad-mask (forward / backward).
//
//   out = rowmask( FiLM( post_drop( LN( pre_drop(a) + res ) ) ) )
//   FiLM(y) = (s_g * gamma[b,:] + 1) * y + s_b * beta[b,:]
//
// Covers every LayerNorm site of the model: MHA tail (SubLayers.py:54-55 +
// Layers.py:27-28), FFN tail + FiLM + mask (SubLayers.py:89-91, Layers.py:31-35),
// variance-predictor ReLU->LN->Dropout (model/modules.py:216-245) and the
// reference-encoder conv stack.  One wave per row, C/64 contiguous channels per
// lane (C in {256, 512, 768, 1024}), fp32 statistics, bf16 I/O.  Dropout masks come
// from a counter hash so the backward regenerates them (no mask tensor).
// Grid: (ceil(L / 64), B) -> every block works on ONE batch item, which makes
// the per-(b, c) FiLM gradient sums a block-local reduction.
// Row stride ``lda`` (elements) of the LayerNorm input a and of its gradient dh: a may be a column slice
// of a wider GEMM output (the duration and pitch predictors' first convs run as ONE N = 512 GEMM whose
// halves feed two LayerNorms); every other operand is dense [rows][C].  The dropout hash indexes the
// logical element (row * C + c) either way.
#include "common.h"

namespace {

constexpr int WAVES = 4;
constexpr int ROWS_PER_WAVE = 16;
constexpr int ROWS_PER_BLOCK = WAVES * ROWS_PER_WAVE;

template <int EPL>
__device__ __forceinline__ void load_row(const bf16_t* p, float* v) {
  if constexpr (EPL == 4) {
    short4v x = *reinterpret_cast<const short4v*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = bf2f((bf16_t)x[i]);
  } else {
#pragma unroll
    for (int j = 0; j < EPL / 8; ++j) {
      short8 x = *reinterpret_cast<const short8*>(p + 8 * j);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[8 * j + i] = bf2f((bf16_t)x[i]);
    }
  }
}

template <int EPL>
__device__ __forceinline__ void store_row(bf16_t* p, const float* v) {
  if constexpr (EPL == 4) {
    short4v x;
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = (short)f2bf(v[i]);
    *reinterpret_cast<short4v*>(p) = x;
  } else {
#pragma unroll
    for (int j = 0; j < EPL / 8; ++j) {
      short8 x;
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = (short)f2bf(v[8 * j + i]);
      *reinterpret_cast<short8*>(p + 8 * j) = x;
    }
  }
}

// LPR = lanes per row: 64 (one wave per row), or 32 for C = 256 (two rows per wave, 16-B accesses)
template <int EPL, int LPR>
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// A row piece kept as raw bf16 (EPL / 8 x 16 B) so its load can be issued an iteration ahead: converting at
// the load site would make the wait (and, vmcnt counting stores too, the drain of the previous row's stores)
// happen right there.
template <int EPL>
struct RawRow {
  short8 x[EPL / 8];
};
template <int EPL>
__device__ __forceinline__ void load_raw(const bf16_t* p, RawRow<EPL>& r) {
#pragma unroll
  for (int j = 0; j < EPL / 8; ++j) r.x[j] = *reinterpret_cast<const short8*>(p + 8 * j);
}
template <int EPL>
__device__ __forceinline__ void raw_to_f(const RawRow<EPL>& r, float* v) {
#pragma unroll
  for (int j = 0; j < EPL / 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) v[8 * j + i] = bf2f((bf16_t)r.x[j][i]);
}

template <int EPL, int LPR, bool RES, int RPWV = ROWS_PER_WAVE>
__global__ void __launch_bounds__(256) addln_fwd_kernel(
    const bf16_t* __restrict__ a, const bf16_t* __restrict__ res, const float* __restrict__ w,
    const float* __restrict__ bias, const float* __restrict__ fg, const float* __restrict__ fb,
    const float* __restrict__ s_g, const float* __restrict__ s_b, const int64_t* __restrict__ lens,
    const int64_t* __restrict__ cu, bf16_t* __restrict__ out, float* __restrict__ mean_out, float* __restrict__ rstd_out, int L, int C,
    float pre_p, float post_p, uint64_t seed, float eps, int lda) {
  constexpr int RPW = 64 / LPR;  // rows a wave covers per iteration
  const int b = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sub = lane / LPR, rl = lane % LPR;
  const int c0 = rl * EPL;
  const int len = lens ? (int)lens[b] : L;
  // packed variable-length rows (cu = row offsets): sequence b owns rows cu[b] .. cu[b]+len-1
  const long rowb = cu ? (long)cu[b] : (long)b * L;
  const int Lb = cu ? len : L;
  if (blockIdx.x * (WAVES * RPWV) >= Lb) return;
  float wv[EPL], bv[EPL], G[EPL], Bt[EPL];
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    wv[i] = w[c0 + i];
    bv[i] = bias[c0 + i];
    G[i] = 1.f;
    Bt[i] = 0.f;
  }
  if (fg) {
    const float sg = *s_g, sb = *s_b;
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      G[i] = sg * fg[(long)b * C + c0 + i] + 1.f;
      Bt[i] = sb * fb[(long)b * C + c0 + i];
    }
  }
  const float invC = 1.f / C;
  // Rows are software-pipelined one ahead (row r+1's a / res loads are issued before row r's store) in
  // straight-line code: a half-wave past the sequence end recomputes and rewrites the last row (identical
  // bytes) instead of branching, and the per-row statistics are stored after the loop, so the waitcnt pass
  // never merges paths with different outstanding stores (which turns every wait into a full drain).
  constexpr int NR = RPWV / RPW;
  RawRow<EPL> ra[2], rr[2];
  float mus[NR], rss[NR];
  auto t_of = [&](int r) { return min(blockIdx.x * (WAVES * RPWV) + (r * WAVES + wave) * RPW + sub, Lb - 1); };
  auto fetch = [&](int r, int q) {
    const long row = rowb + t_of(r);
    load_raw<EPL>(a + row * lda + c0, ra[q]);
    if constexpr (RES) load_raw<EPL>(res + row * C + c0, rr[q]);
  };
  fetch(0, 0);
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int cur = r & 1;
    if (r + 1 < NR) fetch(r + 1, cur ^ 1);
    const int t = t_of(r);
    const long row = rowb + t;
    float h[EPL];
    raw_to_f<EPL>(ra[cur], h);
    if (pre_p > 0.f) {
      float ks[EPL];
      drop_scales<EPL>(seed, (uint64_t)row * C + c0, pre_p, ks);
#pragma unroll
      for (int i = 0; i < EPL; ++i) h[i] *= ks[i];
    }
    if constexpr (RES) {
      float rv[EPL];
      raw_to_f<EPL>(rr[cur], rv);
#pragma unroll
      for (int i = 0; i < EPL; ++i) h[i] += rv[i];
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < EPL; ++i) s += h[i];
    const float mu = row_sum<EPL, LPR>(s) * invC;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      const float d = h[i] - mu;
      q += d * d;
    }
    const float rs = rsqrtf(row_sum<EPL, LPR>(q) * invC + eps);
    float y[EPL], k2[EPL];
    const bool valid = t < len;
    drop_scales<EPL>(seed ^ 0x5bd1e9955bd1e995ULL, (uint64_t)row * C + c0, post_p, k2);
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      float v = (h[i] - mu) * rs * wv[i] + bv[i];
      v *= k2[i];
      v = G[i] * v + Bt[i];
      y[i] = valid ? v : 0.f;
    }
    store_row<EPL>(out + row * C + c0, y);
    mus[r] = mu;
    rss[r] = rs;
  }
  if (rl == 0 && mean_out) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const long row = rowb + t_of(r);
      mean_out[row] = mus[r];
      rstd_out[row] = rss[r];
    }
  }
}

// Backward.  dh = d(pre_drop(a) + res); da = dh * pre_mask; dres = dh.
// Parameter gradients, deterministic: every block writes its (in-block LDS-reduced) partials
//   part[blk][0..C)   dw        part[blk][C..2C)  db          (LayerNorm affine)
//   part[blk][2C..3C) S1[b]     part[blk][3C..4C) S2[b]       (FiLM: S1 = sum_t dout*yd, S2 = sum_t dout)
// (blk = b * gridDim.x + blockIdx.x) and the host finishes them with fixed-order column sums
// (k_reduce.hip) -- no float atomics.
template <int EPL, int LPR, bool RELU, bool RES, bool DA>
__global__ void __launch_bounds__(256) addln_bwd_kernel(
    const bf16_t* __restrict__ dout, const bf16_t* __restrict__ a, const bf16_t* __restrict__ res,
    const float* __restrict__ w, const float* __restrict__ bias, const float* __restrict__ fg,
    const float* __restrict__ s_g, const int64_t* __restrict__ lens, const int64_t* __restrict__ cu,
    const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, bf16_t* __restrict__ dh_out, bf16_t* __restrict__ da_out,
    float* __restrict__ part, int film, int L, int C, float pre_p, float post_p, uint64_t seed, int lda) {
  // [WAVES * RPW][CP] partials, CP = C + C / 32: channel c at c + c / 32, so the dword stores of a 32-lane
  // half (lane rl: channels EPL*rl + i) hit 32 distinct banks (unpadded, EPL*rl mod 32 took only 32/EPL
  // values: a 4- / 2-way conflict on every partial store, SQ_LDS_BANK_CONFLICT / IDX_ACTIVE = 0.38), and
  // the column reads stay consecutive dwords
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int CP = C + C / 32;
  constexpr int RPW = 64 / LPR;
  const int b = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sub = lane / LPR, rl = lane % LPR;
  const int c0 = rl * EPL;
  const int len = lens ? (int)lens[b] : L;
  const long rowb = cu ? (long)cu[b] : (long)b * L;
  const int Lb = cu ? len : L;
  const int nk = film ? 4 : 2;
  float* pb = part + ((long)b * gridDim.x + blockIdx.x) * nk * C;
  if (blockIdx.x * ROWS_PER_BLOCK >= Lb) {  // block-uniform, before any barrier: a zero partial
    for (int c = threadIdx.x; c < nk * C; c += 256) pb[c] = 0.f;
    return;
  }
  float wv[EPL], bv[EPL], G[EPL];
  float acc_w[EPL], acc_b[EPL], acc_s1[EPL], acc_s2[EPL];
  const float sg = fg ? *s_g : 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    wv[i] = w[c0 + i];
    bv[i] = bias[c0 + i];
    G[i] = fg ? sg * fg[(long)b * C + c0 + i] + 1.f : 1.f;
    acc_w[i] = acc_b[i] = acc_s1[i] = acc_s2[i] = 0.f;
  }
  const float invC = 1.f / C;
  // Rows software-pipelined one ahead, as in the forward: row r+1's a / res / dout / statistics loads are
  // issued before row r's math and stores, in straight-line code (a half-wave past the block's rows
  // recomputes and rewrites the last row -- identical bytes -- and adds nothing to the partial sums), so
  // each row no longer waits out a full memory round trip (the kernel was 70 % s_waitcnt).
  constexpr int NR = ROWS_PER_WAVE / RPW;
  RawRow<EPL> ra[2], rr[2], rg[2];
  float mun[2], rsn[2];
  auto t_raw = [&](int r) { return blockIdx.x * ROWS_PER_BLOCK + (r * WAVES + wave) * RPW + sub; };
  auto fetch = [&](int r, int q) {
    const long row = rowb + min(t_raw(r), Lb - 1);
    load_raw<EPL>(a + row * lda + c0, ra[q]);
    if constexpr (RES) load_raw<EPL>(res + row * C + c0, rr[q]);
    load_raw<EPL>(dout + row * C + c0, rg[q]);
    mun[q] = mean_in[row];
    rsn[q] = rstd_in[row];
  };
  fetch(0, 0);
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int cur = r & 1;
    if (r + 1 < NR) fetch(r + 1, cur ^ 1);
    const int tr = t_raw(r);
    const int t = min(tr, Lb - 1);
    const long row = rowb + t;
    const bool valid = t < len;     // masked (padding) row: zero gradient flows back
    const bool count = tr < len;    // contributes to the parameter sums (the clamped repeats do not)
    float h[EPL], m1[EPL];
    raw_to_f<EPL>(ra[cur], h);
    // RELU: a is a ReLU output and its producer's backward leaves the ReLU mask to this kernel (it
    // reads a anyway): d a = dh * (a > 0) -- no residual, no pre-dropout (host check).  Its own
    // instantiation, the mask as bits: the common kernel keeps its register count (occupancy).
    uint32_t pos = 0;
    if constexpr (RELU) {
#pragma unroll
      for (int i = 0; i < EPL; ++i) pos |= (h[i] > 0.f ? 1u : 0u) << i;
    }
    drop_scales<EPL>(seed, (uint64_t)row * C + c0, pre_p, m1);
#pragma unroll
    for (int i = 0; i < EPL; ++i) h[i] *= m1[i];
    if constexpr (RES) {
      float rv[EPL];
      raw_to_f<EPL>(rr[cur], rv);
#pragma unroll
      for (int i = 0; i < EPL; ++i) h[i] += rv[i];
    }
    float go[EPL];
    raw_to_f<EPL>(rg[cur], go);
    const float mu = mun[cur], rs = rsn[cur];
    float xh[EPL], dx[EPL], m2v[EPL];
    float sum1 = 0.f, sum2 = 0.f;
    drop_scales<EPL>(seed ^ 0x5bd1e9955bd1e995ULL, (uint64_t)row * C + c0, post_p, m2v);
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      xh[i] = (h[i] - mu) * rs;
      const float m2 = m2v[i];
      const float y = xh[i] * wv[i] + bv[i];
      const float dy = go[i] * G[i] * m2;
      if (count) {
        acc_s1[i] += go[i] * y * m2;
        acc_s2[i] += go[i];
        acc_w[i] += dy * xh[i];
        acc_b[i] += dy;
      }
      dx[i] = dy * wv[i];
      sum1 += dx[i];
      sum2 += dx[i] * xh[i];
    }
    sum1 = row_sum<EPL, LPR>(sum1) * invC;
    sum2 = row_sum<EPL, LPR>(sum2) * invC;
    float dh[EPL];
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      float v = rs * (dx[i] - sum1 - xh[i] * sum2);
      if constexpr (RELU) v = (pos >> i) & 1u ? v : 0.f;
      dh[i] = valid ? v : 0.f;
    }
    store_row<EPL>(dh_out + row * lda + c0, dh);
    if constexpr (DA) {
#pragma unroll
      for (int i = 0; i < EPL; ++i) dh[i] *= m1[i];
      store_row<EPL>(da_out + row * C + c0, dh);
    }
  }
  // block reduction of the accumulators in a fixed order -> this block's partial row
  float* accs[4] = {acc_w, acc_b, acc_s1, acc_s2};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k >= nk) break;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < EPL; ++i) red[(wave * RPW + sub) * CP + c0 + (c0 >> 5) + i] = accs[k][i];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      float t = 0.f;
      const int cp = c + (c >> 5);
#pragma unroll
      for (int w = 0; w < WAVES * RPW; ++w) t += red[w * CP + cp];  // fixed order
      pb[k * C + c] = t;
    }
  }
}

}  // namespace

// C = 256: half a wave per row with 8 channels (16 B) per lane; wider rows: one wave per row
#define DISPATCH_EPL(C, ...)                                                       \
  switch ((C) / 64) {                                                              \
    case 4: { constexpr int EPL = 8, LPR = 32; __VA_ARGS__; break; }               \
    case 8: { constexpr int EPL = 8, LPR = 64; __VA_ARGS__; break; }               \
    case 16: { constexpr int EPL = 16, LPR = 64; __VA_ARGS__; break; }             \
    default: return -1;                                                            \
  }

static int g_addln_small_rows = 1024;  // B * L at or below which the forward runs one row iteration per wave
SSAMD_API void ssamd_addln_set_small_rows(int v) { g_addln_small_rows = v; }

SSAMD_API int ssamd_addln_fwd(const bf16_t* a, const bf16_t* res, const float* w, const float* bias, const float* fg,
                              const float* fb, const float* s_g, const float* s_b, const int64_t* lens,
                              const int64_t* cu, bf16_t* out,
                              float* mean, float* rstd, int B, int L, int C, float pre_p, float post_p,
                              unsigned long long seed, float eps, int lda, hipStream_t stream) {
  if (C % 256 != 0 && C != 256 && C != 512 && C != 1024) return -1;
  if (lda == 0) lda = C;
  if (lda < C || lda % 8) return -2;
  if (B == 0 || L == 0) return 0;
  if ((long)B * L <= g_addln_small_rows) {
    // few rows (batch-1 serving): one row iteration per wave, more blocks -- the 16-row loop of a wave would
    // mostly recompute the sequence's last row (t_of clamps) and serialise its loads
    DISPATCH_EPL(C, {
      constexpr int RW = 64 / LPR;
      dim3 grid_s(cdiv(L, WAVES * RW), B);
      if (res)
        hipLaunchKernelGGL((addln_fwd_kernel<EPL, LPR, true, RW>), grid_s, dim3(256), 0, stream, a, res, w, bias, fg,
                           fb, s_g, s_b, lens, cu, out, mean, rstd, L, C, pre_p, post_p, (uint64_t)seed, eps, lda);
      else
        hipLaunchKernelGGL((addln_fwd_kernel<EPL, LPR, false, RW>), grid_s, dim3(256), 0, stream, a, res, w, bias, fg,
                           fb, s_g, s_b, lens, cu, out, mean, rstd, L, C, pre_p, post_p, (uint64_t)seed, eps, lda);
    });
    return (int)hipGetLastError();
  }
  dim3 grid(cdiv(L, ROWS_PER_BLOCK), B);
  if (res) {
    DISPATCH_EPL(C, hipLaunchKernelGGL((addln_fwd_kernel<EPL, LPR, true>), grid, dim3(256), 0, stream, a, res, w, bias, fg, fb, s_g,
                                     s_b, lens, cu, out, mean, rstd, L, C, pre_p, post_p, (uint64_t)seed, eps, lda));
  } else {
    DISPATCH_EPL(C, hipLaunchKernelGGL((addln_fwd_kernel<EPL, LPR, false>), grid, dim3(256), 0, stream, a, res, w, bias, fg, fb, s_g,
                                     s_b, lens, cu, out, mean, rstd, L, C, pre_p, post_p, (uint64_t)seed, eps, lda));
  }
  return (int)hipGetLastError();
}

// Workspace floats ssamd_addln_bwd needs (partials + the two-level column-sum scratch).
SSAMD_API long ssamd_addln_bwd_ws(int B, int L, int C, int film) {
  return (long)cdiv(L, ROWS_PER_BLOCK) * B * (film ? 4 : 2) * C + seg_colsum_ws(1, 2 * C);
}

// dw / db / S1 / S2 are overwritten (not accumulated).  S1 / S2 may be null (no FiLM).
SSAMD_API int ssamd_addln_bwd(const bf16_t* dout, const bf16_t* a, const bf16_t* res, const float* w,
                              const float* bias, const float* fg, const float* s_g, const int64_t* lens,
                              const int64_t* cu, const float* mean, const float* rstd, bf16_t* dh, bf16_t* da, float* dw, float* db,
                              float* S1, float* S2, int B, int L, int C, float pre_p, float post_p,
                              unsigned long long seed, int relu_in, int lda, float* ws, long ws_floats,
                              hipStream_t stream) {
  if (lda == 0) lda = C;
  if (lda < C || lda % 8) return -2;
  if (B == 0 || L == 0) return 0;
  if (relu_in && (res || da || pre_p > 0.f)) return -2;
  const int film = S1 != nullptr && S2 != nullptr;
  const int gx = cdiv(L, ROWS_PER_BLOCK);
  const long nblk = (long)gx * B;
  const int nk = film ? 4 : 2;
  if (ws_floats < ssamd_addln_bwd_ws(B, L, C, film)) return -3;
  dim3 grid(gx, B);
  size_t lds = (size_t)WAVES * 2 * (C + C / 32) * sizeof(float);  // [WAVES * rows per wave][C padded]
#define ADDLN_BWD(RELU_, RES_, DA_)                                                                          \
  DISPATCH_EPL(C, hipLaunchKernelGGL((addln_bwd_kernel<EPL, LPR, RELU_, RES_, DA_>), grid, dim3(256), lds, stream, \
                                     dout, a, res, w, bias, fg, s_g, lens, cu, mean, rstd, dh, da, ws, film, L, C,  \
                                     pre_p, post_p, (uint64_t)seed, lda))
  if (relu_in) {
    ADDLN_BWD(true, false, false);
  } else if (res && da) {
    ADDLN_BWD(false, true, true);
  } else if (res) {
    ADDLN_BWD(false, true, false);
  } else if (da) {
    ADDLN_BWD(false, false, true);
  } else {
    ADDLN_BWD(false, false, false);
  }
#undef ADDLN_BWD
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  float* scratch = ws + nblk * nk * C;
  // dw | db over every block, in block order (dw == null: the caller reduces them later from ws with
  // ssamd_addln_wb_reduce -- on the weight-gradient side stream, off the data-gradient chain)
  if (dw) {
    rc = ssamd_seg_colsum(ws, (long)nk * C, 1, (int)nblk, 2 * C, dw, 0, 0, C, db, scratch, seg_colsum_ws(1, 2 * C),
                          stream);
    if (rc) return rc;
  }
  if (!film) return 0;
  // S1[b] | S2[b] over the gx blocks of sequence b
  return ssamd_seg_colsum(ws + 2 * C, (long)nk * C, B, gx, 2 * C, S1, C, 0, C, S2, nullptr, 0, stream);
}

// LayerNorm weight / bias gradients from the partials ssamd_addln_bwd left in ws (called with dw = null).
SSAMD_API int ssamd_addln_wb_reduce(const float* ws, int B, int L, int C, int film, float* dw, float* db,
                                    float* scratch, hipStream_t stream) {
  if (B == 0 || L == 0) return 0;
  const long nblk = (long)cdiv(L, ROWS_PER_BLOCK) * B;
  const int nk = film ? 4 : 2;
  return ssamd_seg_colsum(ws, (long)nk * C, 1, (int)nblk, 2 * C, dw, 0, 0, C, db, scratch, seg_colsum_ws(1, 2 * C),
                          stream);
}

SSAMD_DROP_SALT_LOADER(norm)

// ---------------------------------------------------------------- inference: skinny GEMM + residual + LayerNorm
// out = FiLM(LN(X W^T + bias + res)) with the pad mask, C = 256, for <= 1024 rows (batch-1 serving: the FFT
// blocks' output projection / second FFN conv followed by their post-LN are two tiny launches each).  A block owns
// 16 complete rows (below); MFMA fragments straight from global memory.  No dropout (inference), no statistics.
constexpr int GLN_C = 256;
constexpr int GLN_P = GLN_C + 4;  // LDS row pitch (floats)

// the wave's k-steps st = kq + 4 i: every operand load issued before the first MFMA when the count is a
// compile-time SPW (one memory round trip per wave), a 2-deep loop otherwise
template <int SPW>
__device__ __forceinline__ void gln_mma(const bf16_t* xrow, const bf16_t* wrow, bool rv, int K, int kq, int nk,
                                        float4v (&acc)[4]) {
  if constexpr (SPW > 0) {
    constexpr int CH = SPW < 4 ? SPW : 4;  // steps per load round (4 x 5 fragments: 80 VGPRs at 128 per lane)
#pragma unroll
    for (int c = 0; c < SPW; c += CH) {
      short8 a[CH], b[CH][4];
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int k0 = (kq + 4 * (c + i)) * 32;
        a[i] = rv ? *reinterpret_cast<const short8*>(xrow + k0) : short8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; ++j) b[i][j] = *reinterpret_cast<const short8*>(wrow + (long)j * 16 * K + k0);
      }
#pragma unroll
      for (int i = 0; i < CH; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[i][j], acc[j], 0, 0, 0);
    }
  } else {
#pragma unroll 2
    for (int st = kq; st < nk; st += 4) {
      const short8 a = rv ? *reinterpret_cast<const short8*>(xrow + st * 32) : short8{0, 0, 0, 0, 0, 0, 0, 0};
      short8 b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const short8*>(wrow + (long)j * 16 * K + st * 32);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[j], 0, 0, 0);
    }
  }
}

// 16 waves own 16 complete rows: wave w computes columns 64 (w & 3) .. +64 over a quarter of the k-steps (w >> 2);
// the quarters meet in LDS in a fixed order ((2 + 0) and (3 + 1), then the two sums), then wave w normalises row w.
__global__ void __launch_bounds__(1024) gemm_addln_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                          const float* __restrict__ bias, const bf16_t* __restrict__ res,
                                                          const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                          const float* __restrict__ fg, const float* __restrict__ fb,
                                                          const float* __restrict__ s_g, const float* __restrict__ s_b,
                                                          const int64_t* __restrict__ lens,
                                                          const int64_t* __restrict__ cu, int B, int L, long M, int K,
                                                          bf16_t* __restrict__ out, float eps) {
  __shared__ float part[2][16][GLN_P];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cg = wave & 3, kq = wave >> 2;
  const long m0 = (long)blockIdx.x * 16;
  const long r = m0 + (lane & 15);
  const int ks8 = 8 * (lane >> 4);
  const bf16_t* xrow = X + (r < M ? r : 0) * K + ks8;
  const bf16_t* wrow = W + (long)(cg * 64 + (lane & 15)) * K + ks8;
  float4v acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  const int nk = K / 32;
  if (nk == 8) gln_mma<2>(xrow, wrow, r < M, K, kq, nk, acc);
  else if (nk == 32) gln_mma<8>(xrow, wrow, r < M, K, kq, nk, acc);
  else gln_mma<0>(xrow, wrow, r < M, K, kq, nk, acc);
  auto put = [&](int slot, bool add) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float& d = part[slot][4 * (lane >> 4) + i][cg * 64 + j * 16 + (lane & 15)];
        d = add ? d + acc[j][i] : acc[j][i];
      }
  };
  if (kq >= 2) put(kq - 2, false);
  __syncthreads();
  if (kq < 2) put(kq, true);
  __syncthreads();
  const int c0 = lane * 4;
  const int row = wave;
  const long m = m0 + row;
  if (m >= M) return;
  // sequence / position of row m: padded rows b = m / L; packed rows search cu (B is small at these sizes)
  int b = 0;
  bool valid = true;
  if (cu) {
    valid = false;
    for (int bb = 0; bb < B; ++bb)
      if (m >= cu[bb] && m < cu[bb] + lens[bb]) {
        b = bb;
        valid = true;
      }
  } else {
    b = (int)(m / L);
    if (lens) valid = m - (long)b * L < lens[b];
  }
  float h[4];
  const short4v rv = *reinterpret_cast<const short4v*>(res + m * GLN_C + c0);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    h[q] = part[0][row][c0 + q] + part[1][row][c0 + q] + (bias ? bias[c0 + q] : 0.f) + bf2f((bf16_t)rv[q]);
  float s = h[0] + h[1] + h[2] + h[3];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mu = s * (1.f / GLN_C);
  float v2 = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) v2 += (h[q] - mu) * (h[q] - mu);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v2 += __shfl_xor(v2, o, 64);
  const float rs = rsqrtf(v2 * (1.f / GLN_C) + eps);
  short4v o4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float y = (h[q] - mu) * rs * lnw[c0 + q] + lnb[c0 + q];
    if (fg) y = (*s_g * fg[(long)b * GLN_C + c0 + q] + 1.f) * y + *s_b * fb[(long)b * GLN_C + c0 + q];
    o4[q] = (short)f2bf(valid ? y : 0.f);
  }
  *reinterpret_cast<short4v*>(out + m * GLN_C + c0) = o4;
}

// X [M][K] bf16 (K % 32 == 0), W [256][K] bf16 image, res / out [M][256] bf16; lens / cu as ssamd_addln_fwd
// (padded rows of B sequences of L, or packed rows with offsets cu).  M <= 1024.
SSAMD_API int ssamd_gemm_addln(const bf16_t* X, const bf16_t* W, const float* bias, const bf16_t* res, const float* lnw,
                               const float* lnb, const float* fg, const float* fb, const float* s_g, const float* s_b,
                               const int64_t* lens, const int64_t* cu, int B, int L, long M, int K, bf16_t* out,
                               float eps, hipStream_t s) {
  if (K % 32 || K <= 0 || M > 1024 || !res || !lnw || !lnb || (cu && !lens) || (fg && (!fb || !s_g || !s_b)))
    return -2;
  if (M == 0) return 0;
  hipLaunchKernelGGL(gemm_addln_kernel, dim3(cdiv(M, 16L)), dim3(1024), 0, s, X, W, bias, res, lnw, lnb, fg, fb, s_g,
                     s_b, lens, cu, B, L, M, K, out, eps);
  return (int)hipGetLastError();
}
