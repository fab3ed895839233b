// Implicit-GEMM Conv1d / Linear on CDNA4 MFMA (bf16 in, fp32 accumulate), channel-last.
//
// Forward / data-gradient ("TN" form, both operands K-contiguous):
//   Y[m, n] = epi( sum_k A[m, k] * Bt[n, k] )
//   m = (b, t) over B*L rows;  k = tap * Cin + cin;
//   A[m, k] = X[b, t + tap*dil - pad, cin]   (zero outside [0, L): per-sequence padding)
// A Linear layer is the ks = 1, pad = 0 case.  The data gradient of a conv is the
// same kernel on dY with the flipped/transposed weight and pad' = (ks-1)*dil - pad.
// Epilogue (fused, coalesced through LDS): + bias[n] -> activation (relu / lrelu 0.1
// / tanh) -> * (aux > 0) (ReLU backward) -> + residual -> zero rows t >= len[b]
// -> bf16 or fp32 store.
//
// Weight gradient ("rows-reduction" form):
//   G[n, k] = sum_m dY[m, n] * Acol[m, k]      (split over m into fp32 slabs)
// both operands are read with the reduction index m on the row axis, so the MFMA
// fragments come from LDS through ds_read_b64_tr_b16 (hardware transpose read).
// A reduce kernel sums the slabs and writes dW in the PyTorch [Cout, Cin, ks] layout.
//
// Tiling: 128x128 output tile per 256-thread block (4 waves as 2x2, 64x64 per wave =
// 4x4 v_mfma_f32_16x16x32_bf16 accumulators), BK = 64, LDS double buffer with
// register staging (one barrier per K-step), XOR-swizzled LDS images (conflict-free
// ds_read_b128 / tr reads), XCD-aware bijective block remap so that the 8 blocks
// that share an A panel run on one XCD's L2.
#include <mutex>
#include "common.h"
#include <type_traits>

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int NT = 256;
constexpr int CSTRIDE = 132;  // fp32 epilogue staging row stride (conflict-free writes)

struct ConvGeom {
  int B, L, Cin, ks, dil, pad;  // A operand geometry
  int M, N, K;                  // GEMM sizes (M = B*L, K = ks*Cin)
  // packed variable-length rows (optional): rinfo[m] = {position in its sequence, sequence length};
  // sequences are contiguous, so tap shifts stay row offsets.  nullptr: fixed L per sequence.
  const int2* rinfo;
  // packed rows, sequence offsets (cu[0..nseq]) -- used by the ring wgrad kernel (LDS copy)
  const int64_t* cu;
  int nseq;
  int prio;  // 1: the second half of an 8-wave block runs at s_setprio 1 (experiment knob)
  // 256x256 tile order: ngrp > 1 splits the N tiles into ngrp groups, group-major, so that each
  // XCD's contiguous range of remapped ids covers nN / ngrp N tiles of more M tiles (its B slice
  // stays L2-resident instead of the whole weight image streaming through every XCD's L2)
  int ngrp;
  // 3-tap ConvTranspose form (convT_as_conv3 with K = 2s, pad = s/2; 0 = off): output columns below ksplit are
  // the phases r < s/2, which read taps {0, 1} only, the rest taps {1, 2} -- a 256-column big64 tile (never
  // straddling ksplit) skips the k slabs of its all-zero tap: 2/3 of the MFMA work, bitwise the same result
  int ksplit;
};

// (tm, tn) of remapped block id T (bijective over nM * nN; ngrp must divide nN)
__device__ __forceinline__ int2 tile_of(int T, int nM, int nN, int ngrp) {
  if (ngrp > 1) {
    const int per = nN / ngrp, gs = nM * per;
    const int grp = T / gs, r = T - grp * gs;
    return make_int2(r / per, grp * per + r % per);
  }
  return make_int2(T / nN, T % nN);
}

// (position, bound) of row m for the conv zero-padding test
__device__ __forceinline__ int2 row_pos(const ConvGeom& g, int m) {
  if (g.rinfo) return g.rinfo[m];
  const int b = m / g.L;
  return make_int2(m - b * g.L, g.L);
}

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_TANH = 3 };

// Extended epilogue (bf16 output; 256x256 "big64" and 256x128 "ring" kernels), applied after
// bias -> act -> aux -> residual -> row mask:  v = (v + acc) * scale;  y2 = lrelu_0.1(v);
// Y = post_act(v).  acc may alias Y (in-place MRF branch sum: every element is read before it
// is written, by the same thread).  Used by the HiFi-GAN inference path so that no activation
// or accumulation pass runs outside a GEMM (models/hifigan.py).
struct EpiX {
  const bf16_t* acc;
  bf16_t* y2;
  float scale;
  int post_act;
  // BatchNorm-backward head operands (EPI_BNH only, see below): bn_stats = the forward's
  // [mean | rstd | scale | shift] x N, bn_part = the per-M-tile column partials, bn_p / bn_seed = the
  // dropout that followed the BatchNorm (bn_h = acc, bn_act = post_act)
  const float* bn_stats;
  float* bn_part;
  float bn_p;
  unsigned long long bn_seed;
  // ReLU bitmask (big64 LDS-staged epilogue, N % 8 == 0): mask_out[m][n/8] bit q = (y[m][n+q] > 0)
  // written by a ReLU GEMM; mask_in multiplies the output by the stored bits instead of reading a
  // bf16 aux operand (16x fewer bytes for the FFN hidden layer's dgrad)
  unsigned char* mask_out;
  const unsigned char* mask_in;
  // BatchNorm backward head (PostNet; the BNH instantiation of the big64 LDS-staged epilogue, bf16 out,
  // ldy == N): the GEMM output is dy = dL/d(BN-act-dropout output) of the layer whose pre-BN input is
  // bn_h [M][N]; the epilogue stores  dz = dy * keep(seed, p) * act'(bn_h * scale + shift)  instead of dy
  // and writes the tile's column partials  sum_rows dz  and  sum_rows dz * (bn_h - mean)  to
  // bn_part[tm][N] and bn_part[nM + tm][N] (tm = M tile; fixed order, no atomics).  bn_stats = the
  // forward's [mean | rstd | scale | shift] x N.  The partial sums replace k_bn.hip's bn_bwd_reduce pass
  // (a full re-read of dy and bn_h); the dropout mask and act' are bit-identical to it.
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: consecutive remapped ids land on the same XCD (round-robin dispatch)
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, k = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

// swizzled byte offset of 16-B chunk `c` (0..7) of row `row` in a [rows][64 bf16] image
__device__ __forceinline__ int swz128(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ short8 load_a_chunk(const bf16_t* __restrict__ X, const ConvGeom& g, int m, int tt, int lim,
                                               int k, float invCin) {
  short8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (m < g.M && k < g.K) {
    const int tap = (int)(((float)k + 0.5f) * invCin);
    const int cin = k - tap * g.Cin;
    const int sh = tap * g.dil - g.pad;
    const int ts = tt + sh;
    if (ts >= 0 && ts < lim) v = *reinterpret_cast<const short8*>(X + ((long)m + sh) * g.Cin + cin);
  }
  return v;
}

// Register epilogue of a 4 x 4 grid of 16x16 accumulator fragments (the 128x128 kernels): every global
// operand (bias columns, row validity, aux / residual segments) is loaded before the first store -- one
// load per fragment between stores made each wait drain the stores before it (vmcnt counts both).
template <bool OUT_F32>
__device__ __forceinline__ void epi4x4_prefetch(const float4v (&acc)[4][4], int mb, int nb, int lane, const ConvGeom& g,
                                                const float* __restrict__ bias, const bf16_t* __restrict__ aux,
                                                const bf16_t* __restrict__ resid, const int64_t* __restrict__ lens,
                                                int act, int ldy, void* __restrict__ Yv) {
  float4 bvj[4];
  short4v xa[4][4], xr[4][4];
  bool vrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = nb + j * 16 + 4 * (lane >> 4);
    bvj[j] = (bias && n < g.N) ? *reinterpret_cast<const float4*>(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mb + i * 16 + (lane & 15);
    const int mm = m < g.M ? m : 0;
    const int bb = mm / g.L, tt = mm - bb * g.L;
    vrow[i] = lens == nullptr || tt < (int)lens[bb];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nb + j * 16 + 4 * (lane >> 4);
      const bool in = m < g.M && n < g.N;
      const long off = (long)m * ldy + n;
      if (in && aux) xa[i][j] = *reinterpret_cast<const short4v*>(aux + off);
      if (in && resid) xr[i][j] = *reinterpret_cast<const short4v*>(resid + off);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mb + i * 16 + (lane & 15);
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nb + j * 16 + 4 * (lane >> 4);
      if (n >= g.N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
        v[0] += bvj[j].x; v[1] += bvj[j].y; v[2] += bvj[j].z; v[3] += bvj[j].w;
      }
      if (act == ACT_RELU) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
      } else if (act == ACT_LRELU) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = v[q] > 0.f ? v[q] : 0.1f * v[q];
      } else if (act == ACT_TANH) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = tanhf(v[q]);
      }
      const long off = (long)m * ldy + n;
      if (aux) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = bf2f((bf16_t)xa[i][j][q]) > 0.f ? v[q] : 0.f;
      }
      if (resid) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += bf2f((bf16_t)xr[i][j][q]);
      }
      if (!vrow[i]) v[0] = v[1] = v[2] = v[3] = 0.f;
      if constexpr (OUT_F32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(Yv) + off) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        short4v o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (short)f2bf(v[q]);
        *reinterpret_cast<short4v*>(reinterpret_cast<bf16_t*>(Yv) + off) = o;
      }
    }
  }
}

template <bool OUT_F32, bool REG_EPI>
__global__ void __launch_bounds__(NT, 2) conv_gemm_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                          const float* __restrict__ bias, const bf16_t* __restrict__ aux,
                                                          const bf16_t* __restrict__ resid,
                                                          const int64_t* __restrict__ lens, void* __restrict__ Yv,
                                                          ConvGeom g, int act, int ldy) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nN = (g.N + BN - 1) / BN;
  const int nM = (g.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nN * nM);
  const int tn = wg % nN, tm = wg / nN;
  const int m0 = tm * BM, n0 = tn * BN;
  // wave index as a scalar: LDS-DMA destinations (M0) and per-wave offsets stay in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const float invCin = 1.f / (float)g.Cin;

  // staging assignment: chunk e = tid + 256*i, row = e/8, c = e%8 (i = 0..3)
  int a_lim[4], a_t[4], a_m[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (tid >> 3) + 32 * i;
    a_m[i] = m0 + row;
    const int2 rp = row_pos(g, a_m[i] < g.M ? a_m[i] : 0);
    a_t[i] = rp.x;
    a_lim[i] = rp.y;
  }
  const int cchunk = tid & 7;

  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};

  short8 ra[4], rb[4];
  auto gload = [&](int kt) {
    const int k = kt * BK + cchunk * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) ra[i] = load_a_chunk(X, g, a_m[i], a_t[i], a_lim[i], k, invCin);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + (tid >> 3) + 32 * i;
      short8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (n < g.N && k < g.K) v = *reinterpret_cast<const short8*>(W + (long)n * g.K + k);
      rb[i] = v;
    }
  };
  auto lstore = [&](int buf) {
    char* As = smem + buf * (2 * BM * BK * 2);
    char* Bs = As + BM * BK * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 3) + 32 * i;
      *reinterpret_cast<short8*>(As + swz128(row, cchunk)) = ra[i];
      *reinterpret_cast<short8*>(Bs + swz128(row, cchunk)) = rb[i];
    }
  };

  const int nk = (g.K + BK - 1) / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const char* As = smem + buf * (2 * BM * BK * 2);
    const char* Bs = As + BM * BK * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      short8 fa[4], fb[4];
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[i] = *reinterpret_cast<const short8*>(As + swz128(wm * 64 + i * 16 + (lane & 15), c));
        fb[i] = *reinterpret_cast<const short8*>(Bs + swz128(wn * 64 + i * 16 + (lane & 15), c));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (REG_EPI)  // transposed accumulator: lane holds 4 consecutive columns of one row
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
    }
    if (kt + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  if constexpr (REG_EPI) {
    // ---- register epilogue (no LDS round trip): fragment (i, j) -> row m, columns n..n+3
    epi4x4_prefetch<OUT_F32>(acc, m0 + wm * 64, n0 + wn * 64, lane, g, bias, aux, resid, lens, act, ldy, Yv);
    return;
  }

  // ---- epilogue: stage fp32 tile in LDS, then coalesced 8-wide row segments
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int col = wn * 64 + j * 16 + (lane & 15);
        Cs[row * CSTRIDE + col] = acc[i][j][r];
      }
  __syncthreads();
  const int seg = tid & 15;  // 8 columns each
  for (int rr = tid >> 4; rr < BM; rr += NT / 16) {
    const int m = m0 + rr;
    if (m >= g.M) break;
    const int nb = n0 + seg * 8;
    if (nb >= g.N) continue;
    const int bb = m / g.L, tt = m - bb * g.L;
    const bool valid = lens == nullptr || tt < (int)lens[bb];
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = Cs[rr * CSTRIDE + seg * 8 + q];
    const bool full = nb + 8 <= g.N;
    if (bias) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += (full || nb + q < g.N) ? bias[nb + q] : 0.f;
    }
    if (act == ACT_RELU) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
    } else if (act == ACT_LRELU) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = v[q] > 0.f ? v[q] : 0.1f * v[q];
    } else if (act == ACT_TANH) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = tanhf(v[q]);
    }
    const long off = (long)m * ldy + nb;
    if (full && (ldy % 8) == 0) {
      if (aux) {
        short8 x = *reinterpret_cast<const short8*>(aux + off);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = bf2f((bf16_t)x[q]) > 0.f ? v[q] : 0.f;
      }
      if (resid) {
        short8 x = *reinterpret_cast<const short8*>(resid + off);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += bf2f((bf16_t)x[q]);
      }
      if (!valid) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = 0.f;
      }
      if constexpr (OUT_F32) {
        float4* Y = reinterpret_cast<float4*>(reinterpret_cast<float*>(Yv) + off);
        Y[0] = make_float4(v[0], v[1], v[2], v[3]);
        Y[1] = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        short8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = (short)f2bf(v[q]);
        *reinterpret_cast<short8*>(reinterpret_cast<bf16_t*>(Yv) + off) = o;
      }
    } else {
      for (int q = 0; q < 8; ++q) {
        if (nb + q >= g.N) break;
        float x = v[q];
        if (aux && !(bf2f(aux[off + q]) > 0.f)) x = 0.f;
        if (resid) x += bf2f(resid[off + q]);
        if (!valid) x = 0.f;
        if constexpr (OUT_F32) reinterpret_cast<float*>(Yv)[off + q] = x;
        else reinterpret_cast<bf16_t*>(Yv)[off + q] = f2bf(x);
      }
    }
  }
}

// ----------------------------------------------------------------------------
// Same GEMM with global_load_lds staging (gfx950 LDS-DMA): each lane DMAs one 16-B chunk
// straight into LDS (no VGPR round trip, no ds_write); the XOR swizzle moves to the
// per-lane SOURCE address (the LDS image is lane-linear per wave instruction).  Lanes
// whose chunk is conv padding / out of range read a 16-B zero block instead.
// ----------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) bf16_t g_zero_chunk_mem[8];
// The zero chunk's address, produced by an opaque asm so it stays in an SGPR pair for the whole
// kernel: read directly, the global's GOT entry is reloaded (s_load + lgkmcnt wait) before every
// LDS-DMA issue, because the loops' s_waitcnt asm carries a "memory" clobber.  Each kernel below
// shadows g_zero_chunk with this local.
__device__ __forceinline__ const void* zero_chunk_ptr() {
  const void* p = g_zero_chunk_mem;
  asm volatile("" : "+s"(p));
  return p;
}

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
// buffer-descriptor LDS-DMA (16 B per lane, lane-linear destination): an out-of-range voffset lands zeros
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, soff,
                                           0, 0);
}

template <bool OUT_F32>
__global__ void __launch_bounds__(NT, 2) conv_gemm_glds_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                               const float* __restrict__ bias,
                                                               const bf16_t* __restrict__ aux,
                                                               const bf16_t* __restrict__ resid,
                                                               const int64_t* __restrict__ lens, void* __restrict__ Yv,
                                                               ConvGeom g, int act, int ldy) {
  const void* const g_zero_chunk = zero_chunk_ptr();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nN = (g.N + BN - 1) / BN;
  const int nM = (g.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nN * nM);
  const int tn = wg % nN, tm = wg / nN;
  const int m0 = tm * BM, n0 = tn * BN;
  // wave index as a scalar: LDS-DMA destinations (M0) and per-wave offsets stay in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const float invCin = 1.f / (float)g.Cin;

  // DMA assignment: wave instruction i (0..3) fills rows rb(i) .. rb(i)+7, lane -> (row, phys chunk)
  int a_lim[4], a_t[4], a_m[4], rowi[4], lchunk[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 4 + wave) * 8 + (lane >> 3);
    rowi[i] = row;
    lchunk[i] = (lane & 7) ^ ((row >> 1) & 7);
    a_m[i] = m0 + row;
    const int2 rp = row_pos(g, a_m[i] < g.M ? a_m[i] : 0);
    a_t[i] = rp.x;
    a_lim[i] = rp.y;
  }
  auto stage = [&](int kt, int buf) {
    char* As = smem + buf * (2 * BM * BK * 2);
    char* Bs = As + BM * BK * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kt * BK + lchunk[i] * 8;
      const void* src = g_zero_chunk;
      if (a_m[i] < g.M && k < g.K) {
        const int tap = (int)(((float)k + 0.5f) * invCin);
        const int cin = k - tap * g.Cin;
        const int sh = tap * g.dil - g.pad;
        const int ts = a_t[i] + sh;
        if (ts >= 0 && ts < a_lim[i]) src = X + ((long)a_m[i] + sh) * g.Cin + cin;
      }
      glds16(src, As + (i * 4 + wave) * 8 * 128);
      const int n = n0 + rowi[i];
      const void* srcb = (n < g.N && k < g.K) ? (const void*)(W + (long)n * g.K + k) : (const void*)g_zero_chunk;
      glds16(srcb, Bs + (i * 4 + wave) * 8 * 128);
    }
  };

  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + BK - 1) / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, buf ^ 1);
    const char* As = smem + buf * (2 * BM * BK * 2);
    const char* Bs = As + BM * BK * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      short8 fa[4], fb[4];
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[i] = *reinterpret_cast<const short8*>(As + swz128(wm * 64 + i * 16 + (lane & 15), c));
        fb[i] = *reinterpret_cast<const short8*>(Bs + swz128(wn * 64 + i * 16 + (lane & 15), c));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  epi4x4_prefetch<OUT_F32>(acc, m0 + wm * 64, n0 + wn * 64, lane, g, bias, aux, resid, lens, act, ldy, Yv);
}

// ----------------------------------------------------------------------------
// 256x128 tile, 8 waves (4x2, 64x64 each), 3-stage LDS-DMA ring with a COUNTED vmcnt:
// the DMA for stage k+2 is issued before computing stage k, and only stage k+1 is
// waited for at the end of the iteration (raw s_barrier -- __syncthreads() would drain
// every in-flight LDS-DMA).  144 KiB LDS, 1 block (2 waves/SIMD) per CU.
// ----------------------------------------------------------------------------
constexpr int BM3 = 256, NT3 = 512, NSTAGE = 3;
constexpr int STAGE_BYTES = (BM3 + BN) * BK * 2;  // 48 KiB

template <bool OUT_F32, bool FASTK, bool PACKED, bool BUF = false>
__global__ void __launch_bounds__(NT3, 1) conv_gemm_ring_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                                const float* __restrict__ bias,
                                                                const bf16_t* __restrict__ aux,
                                                                const bf16_t* __restrict__ resid,
                                                                const int64_t* __restrict__ lens, void* __restrict__ Yv,
                                                                ConvGeom g, int act, int ldy, EpiX ex) {
  const void* const g_zero_chunk = zero_chunk_ptr();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nN = (g.N + BN - 1) / BN;
  const int nM = (g.M + BM3 - 1) / BM3;
  const int wg = xcd_remap(blockIdx.x, nN * nM);
  const int tn = wg % nN, tm = wg / nN;
  const int m0 = tm * BM3, n0 = tn * BN;
  // wave index as a scalar: LDS-DMA destinations (M0) and per-wave offsets stay in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const float invCin = 1.f / (float)g.Cin;

  // A: 256 rows = 32 wave-instructions (4 per wave); B: 128 rows = 16 (2 per wave)
  int a_lim[4], a_t[4], a_m[4], achunk[4];
  const bf16_t* arow_ptr[4];
  const bf16_t* brow_ptr[2];
  bool a_ok[4], b_ok[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 8 + wave) * 8 + (lane >> 3);
    achunk[i] = (lane & 7) ^ ((row >> 1) & 7);
    a_m[i] = m0 + row;
    a_ok[i] = a_m[i] < g.M;
    const int mm = a_ok[i] ? a_m[i] : 0;
    if constexpr (PACKED) {
      const int2 rp = g.rinfo[mm];  // unconditional: the four loads issue back to back
      a_t[i] = rp.x;
      a_lim[i] = rp.y;
    } else {
      const int bb = mm / g.L;
      a_t[i] = mm - bb * g.L;
      a_lim[i] = g.L;
    }
    arow_ptr[i] = X + (long)mm * g.Cin + achunk[i] * 8;  // tap-0, cin-0 origin
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (i * 8 + wave) * 8 + (lane >> 3);
    const int bch = (lane & 7) ^ ((row >> 1) & 7);
    const int n = n0 + row;
    b_ok[i] = n < g.N;
    brow_ptr[i] = W + (long)(b_ok[i] ? n : 0) * g.K + bch * 8;
  }
  // BUF (FASTK only): LDS-DMA through buffer descriptors, as in conv_gemm_big64_kernel
  constexpr int kOOB = (int)0x80000000;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(X - (long)g.pad * g.Cin), 0, BUF ? (g.M + g.pad) * g.Cin * 2 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, BUF ? g.N * g.K * 2 : 0,
                                                                      0x00020000);
  int avo[4], bvo[2];
  if constexpr (BUF) {
#pragma unroll
    for (int i = 0; i < 4; ++i) avo[i] = a_ok[i] ? ((a_m[i] + g.pad) * g.Cin + achunk[i] * 8) * 2 : kOOB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (i * 8 + wave) * 8 + (lane >> 3);
      const int bch = (lane & 7) ^ ((row >> 1) & 7);
      bvo[i] = b_ok[i] ? ((n0 + row) * g.K + bch * 8) * 2 : kOOB;
    }
  }
  auto stage = [&](int kt, int buf) {
    char* As = smem + buf * STAGE_BYTES;
    char* Bs = As + BM3 * BK * 2;
    const int k0 = kt * BK;
    if constexpr (BUF) {
      const int tap = k0 / g.Cin;
      const int cin0 = k0 - tap * g.Cin;
      const int shift = tap * g.dil - g.pad;
      const int aoff = (shift * g.Cin + cin0) * 2;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ts = a_t[i] + shift;
        const bool ok = (unsigned)ts < (unsigned)a_lim[i];
        buf_lds16(rA, ok ? avo[i] + aoff : kOOB, 0, As + (i * 8 + wave) * 8 * 128);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) buf_lds16(rB, bvo[i], k0 * 2, Bs + (i * 8 + wave) * 8 * 128);
    } else if constexpr (FASTK) {
      // Cin % 64 == 0: the whole 64-wide k slab sits in one tap -> wave-uniform shift / offset
      const int tap = k0 / g.Cin;
      const int cin0 = k0 - tap * g.Cin;
      const int shift = tap * g.dil - g.pad;
      const long off = (long)shift * g.Cin + cin0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ts = a_t[i] + shift;
        const bool ok = a_ok[i] && (unsigned)ts < (unsigned)a_lim[i];
        glds16(ok ? (const void*)(arow_ptr[i] + off) : (const void*)g_zero_chunk, As + (i * 8 + wave) * 8 * 128);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
        glds16(b_ok[i] ? (const void*)(brow_ptr[i] + k0) : (const void*)g_zero_chunk, Bs + (i * 8 + wave) * 8 * 128);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + achunk[i] * 8;
        const void* src = g_zero_chunk;
        if (a_ok[i] && k < g.K) {
          const int tap = (int)(((float)k + 0.5f) * invCin);
          const int cin = k - tap * g.Cin;
          const int sh = tap * g.dil - g.pad;
          const int ts = a_t[i] + sh;
          if (ts >= 0 && ts < a_lim[i]) src = arow_ptr[i] - achunk[i] * 8 + (long)sh * g.Cin + cin;
        }
        glds16(src, As + (i * 8 + wave) * 8 * 128);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = (i * 8 + wave) * 8 + (lane >> 3);
        const int k = k0 + ((lane & 7) ^ ((row >> 1) & 7)) * 8;
        glds16((b_ok[i] && k < g.K) ? (const void*)(brow_ptr[i] + k0) : (const void*)g_zero_chunk,
               Bs + (i * 8 + wave) * 8 * 128);
      }
    }
  };

  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + BK - 1) / BK;
  stage(0, 0);
  if (nk > 1) {
    stage(1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 2 < nk) stage(kt + 2, (buf + 2) % NSTAGE);
    const char* As = smem + buf * STAGE_BYTES;
    const char* Bs = As + BM3 * BK * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      short8 fa[4], fb[4];
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[i] = *reinterpret_cast<const short8*>(As + swz128(wm * 64 + i * 16 + (lane & 15), c));
        fb[i] = *reinterpret_cast<const short8*>(Bs + swz128(wn * 64 + i * 16 + (lane & 15), c));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    // retire stage kt+1 (leave kt+2 in flight), make it visible, and free buf for re-staging
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    buf = (buf + 1) % NSTAGE;
  }
  // Every global operand of the 16 (i, j) fragments (bias columns, row validity, aux / residual /
  // accumulator segments) is loaded before the first store: one load per fragment between stores made
  // each wait (vmcnt counts stores too) drain the stores before it -- 16 serialised round trips per wave.
  float4 bvj[4];
  short4v xa[4][4], xr[4][4], xc[4][4];
  bool vrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
    bvj[j] = (bias && n < g.N) ? *reinterpret_cast<const float4*>(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    const int mm = m < g.M ? m : 0;
    const int bb = mm / g.L, tt = mm - bb * g.L;
    vrow[i] = lens == nullptr || tt < (int)lens[bb];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      const bool in = m < g.M && n < g.N;
      const long off = (long)m * ldy + n;
      if (in && aux) xa[i][j] = *reinterpret_cast<const short4v*>(aux + off);
      if (in && resid) xr[i][j] = *reinterpret_cast<const short4v*>(resid + off);
      if constexpr (!OUT_F32) {
        if (in && ex.acc) xc[i][j] = *reinterpret_cast<const short4v*>(ex.acc + off);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if (m >= g.M) continue;
    const bool valid = vrow[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= g.N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
        v[0] += bvj[j].x; v[1] += bvj[j].y; v[2] += bvj[j].z; v[3] += bvj[j].w;
      }
      if (act == ACT_RELU) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
      } else if (act == ACT_LRELU) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = v[q] > 0.f ? v[q] : 0.1f * v[q];
      } else if (act == ACT_TANH) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = tanhf(v[q]);
      }
      const long off = (long)m * ldy + n;
      if (aux) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = bf2f((bf16_t)xa[i][j][q]) > 0.f ? v[q] : 0.f;
      }
      if (resid) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += bf2f((bf16_t)xr[i][j][q]);
      }
      if (!valid) v[0] = v[1] = v[2] = v[3] = 0.f;
      if constexpr (OUT_F32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(Yv) + off) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        if (ex.acc) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += bf2f((bf16_t)xc[i][j][q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = valid ? v[q] * ex.scale : 0.f;
        if (ex.y2) {
          short4v o2;
#pragma unroll
          for (int q = 0; q < 4; ++q) o2[q] = (short)f2bf(v[q] > 0.f ? v[q] : 0.1f * v[q]);
          *reinterpret_cast<short4v*>(ex.y2 + off) = o2;
        }
        if (ex.post_act == ACT_LRELU) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = v[q] > 0.f ? v[q] : 0.1f * v[q];
        }
        short4v o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (short)f2bf(v[q]);
        *reinterpret_cast<short4v*>(reinterpret_cast<bf16_t*>(Yv) + off) = o;
      }
    }
  }
}


// 256x256 tiles (big64 forward / data gradient, the weight gradient): 8 waves (2 x 4 of 128 x 64).
// (A BK = 32 4-stage ring and a persistent variant of the forward kernel were measured and lost
// in round 2: profiles/README.md; removed.)
constexpr int BG = 256;


template <bool OUT_F32>
__device__ __forceinline__ void epi_store4(float (&v)[4], int m, int n, const float* __restrict__ bias,
                                           const bf16_t* __restrict__ aux, const bf16_t* __restrict__ resid,
                                           bool valid, int act, int ldy, void* __restrict__ Yv) {
  if (act < 0) return;  // timing experiments only (ssamd_gemm_debug_nostore)
  if (bias) {
    const float4 bv = *reinterpret_cast<const float4*>(bias + n);
    v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
  }
  if (act == ACT_RELU) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
  } else if (act == ACT_LRELU) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = v[q] > 0.f ? v[q] : 0.1f * v[q];
  } else if (act == ACT_TANH) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = tanhf(v[q]);
  }
  const long off = (long)m * ldy + n;
  if (aux) {
    const short4v x = *reinterpret_cast<const short4v*>(aux + off);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = bf2f((bf16_t)x[q]) > 0.f ? v[q] : 0.f;
  }
  if (resid) {
    const short4v x = *reinterpret_cast<const short4v*>(resid + off);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] += bf2f((bf16_t)x[q]);
  }
  if (!valid) v[0] = v[1] = v[2] = v[3] = 0.f;
  if constexpr (OUT_F32) {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(Yv) + off) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    short4v o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = (short)f2bf(v[q]);
    *reinterpret_cast<short4v*>(reinterpret_cast<bf16_t*>(Yv) + off) = o;
  }
}

constexpr int STG64_BYTES = 2 * BG * 64 * 2;  // 64 KiB
constexpr int B64_LDS = 256 * 528;          // 2 stages (128 KiB) or the padded bf16 epilogue tile (132 KiB)

// Scheduling fence for the ping-pong main loop: keeps the compiler from moving LDS reads / DMA issues
// (memory clobber) or MFMAs (sched_barrier) across the block barrier that separates two phases.
__device__ __forceinline__ void pp_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// EPIM: epilogue specialisations, each its own instantiation so the other variants' code / registers are
// untouched (measured: the BatchNorm head folded into every variant as a runtime branch slowed the
// ReLU-mask data gradient ~25 % and the step ~1.5 %):
//   EPI_BNH   the BatchNorm-backward head (EpiX aliases, see EpiX);
//   EPI_MASK  the ReLU-bitmask data gradient (mask_in only): the thread's 16 mask bytes (one per row it
//             stores) are loaded before the prologue's drain, instead of as dependent byte loads inside the
//             epilogue (one exposed memory round trip per 8 rows with nothing else in flight).
// STG (BUF only): the staggered 8-phase main loop -- see the comment at its loop below.
constexpr int EPI_GEN = 0, EPI_BNH = 1, EPI_MASK = 2;

// Epilogue staging tile (bf16, 528-B rows = 132 dwords): the accumulator staging writes 4-column (8-B) pieces with
// ds_write_b64, whose 16-lane groups are 16 consecutive rows of one piece; at a 132-dword pitch rows r and r + 8
// share banks (4 r mod 32), so rows with bit 3 set store the two 8-B halves of each 16-B chunk swapped (their
// pieces land 2 dwords over: 32 distinct banks per group).  The 16-B chunk reads undo the swap in registers.
__device__ __forceinline__ int ct_woff(int ml, int nl) { return ml * 528 + ((nl * 2) ^ (((ml >> 3) & 1) << 3)); }
__device__ __forceinline__ short8 ct_read(const char* Ct, int r, int c16) {
  const short8 v = *reinterpret_cast<const short8*>(Ct + r * 528 + c16 * 16);
  return ((r >> 3) & 1) ? __builtin_shufflevector(v, v, 4, 5, 6, 7, 0, 1, 2, 3) : v;
}
// One 256x256 output tile (block vb) of the big64 GEMM.
template <bool OUT_F32, bool FASTK, bool PACKED, bool BUF, int EPIM, bool STG>
__device__ __forceinline__ void big64_tile(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                           const float* __restrict__ bias, const bf16_t* __restrict__ aux,
                                           const bf16_t* __restrict__ resid, const int64_t* __restrict__ lens,
                                           void* __restrict__ Yv, ConvGeom g, int act, int ldy, EpiX ex, int vb) {
  const void* const g_zero_chunk = zero_chunk_ptr();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nN = (g.N + BG - 1) / BG;
  const int nM = (g.M + BG - 1) / BG;
  const int2 tmn = tile_of(xcd_remap(vb, nN * nM), nM, nN, g.ngrp);
  const int tm = tmn.x, tn = tmn.y;
  const int m0 = tm * BG, n0 = tn * BG;
  // wave index as a scalar: LDS-DMA destinations (M0) and per-wave offsets stay in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // 2 x 4 waves of 128 (m) x 64 (n)
  const float invCin = 1.f / (float)g.Cin;
  if (g.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);

  // DMA: a wave instruction fills 8 rows x 128 B; A and B: 256 rows = 32 instructions = 4 per wave
  int a_lim[4], a_t[4], a_m[4], achunk[4];
  const bf16_t* arow_ptr[4];
  const bf16_t* brow_ptr[4];
  bool a_ok[4], b_ok[4];
  int2 rp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 8 + wave) * 8 + (lane >> 3);
    achunk[i] = (lane & 7) ^ ((row >> 1) & 7);
    a_m[i] = m0 + row;
    a_ok[i] = a_m[i] < g.M;
    if constexpr (PACKED) rp[i] = g.rinfo[a_ok[i] ? a_m[i] : 0];  // both loads issue back to back
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int mm = a_ok[i] ? a_m[i] : 0;
    if constexpr (PACKED) {
      a_t[i] = rp[i].x;
      a_lim[i] = rp[i].y;
    } else {
      const int bb = mm / g.L;
      a_t[i] = mm - bb * g.L;
      a_lim[i] = g.L;
    }
    arow_ptr[i] = X + (long)mm * g.Cin + achunk[i] * 8;
    const int row = (i * 8 + wave) * 8 + (lane >> 3);
    const int n = n0 + row;
    b_ok[i] = n < g.N;
    brow_ptr[i] = W + (long)(b_ok[i] ? n : 0) * g.K + achunk[i] * 8;  // same row -> same chunk swizzle
  }
  // BUF (FASTK only): LDS-DMA through buffer descriptors -- A over X rows [-pad, M), B over the weight
  // image -- with loop-invariant 32-bit per-lane offsets: the k slab's tap shift is one scalar added
  // per A row (plus the validity select), the B slab offset a scalar soffset; out of range = zeros
  constexpr int kOOB = (int)0x80000000;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(X - (long)g.pad * g.Cin), 0, BUF ? (g.M + g.pad) * g.Cin * 2 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, BUF ? g.N * g.K * 2 : 0,
                                                                      0x00020000);
  int avo[4], bvo[4];
  if constexpr (BUF) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      avo[i] = a_ok[i] ? ((a_m[i] + g.pad) * g.Cin + achunk[i] * 8) * 2 : kOOB;
      const int row = (i * 8 + wave) * 8 + (lane >> 3);
      bvo[i] = b_ok[i] ? ((n0 + row) * g.K + achunk[i] * 8) * 2 : kOOB;
    }
  }
  auto stage = [&](int kt, int buf) {
    char* As = smem + buf * STG64_BYTES;
    char* Bs = As + BG * 64 * 2;
    const int k0 = kt * 64;
    if constexpr (BUF) {
      const int tap = k0 / g.Cin;
      const int cin0 = k0 - tap * g.Cin;
      const int shift = tap * g.dil - g.pad;
      const int aoff = (shift * g.Cin + cin0) * 2;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ts = a_t[i] + shift;
        const bool ok = (unsigned)ts < (unsigned)a_lim[i];
        buf_lds16(rA, ok ? avo[i] + aoff : kOOB, 0, As + (i * 8 + wave) * 1024);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) buf_lds16(rB, bvo[i], k0 * 2, Bs + (i * 8 + wave) * 1024);
    } else if constexpr (FASTK) {  // Cin % 64 == 0: the 64-wide k slab sits in one tap
      const int tap = k0 / g.Cin;
      const int cin0 = k0 - tap * g.Cin;
      const int shift = tap * g.dil - g.pad;
      const long off = (long)shift * g.Cin + cin0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ts = a_t[i] + shift;
        const bool ok = a_ok[i] && (unsigned)ts < (unsigned)a_lim[i];
        glds16(ok ? (const void*)(arow_ptr[i] + off) : (const void*)g_zero_chunk, As + (i * 8 + wave) * 1024);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        glds16(b_ok[i] ? (const void*)(brow_ptr[i] + k0) : (const void*)g_zero_chunk, Bs + (i * 8 + wave) * 1024);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + achunk[i] * 8;
        const void* src = g_zero_chunk;
        if (a_ok[i] && k < g.K) {
          const int tap = (int)(((float)k + 0.5f) * invCin);
          const int cin = k - tap * g.Cin;
          const int sh = tap * g.dil - g.pad;
          const int ts = a_t[i] + sh;
          if (ts >= 0 && ts < a_lim[i]) src = arow_ptr[i] - achunk[i] * 8 + (long)sh * g.Cin + cin;
        }
        glds16(src, As + (i * 8 + wave) * 1024);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + achunk[i] * 8;
        glds16((b_ok[i] && k < g.K) ? (const void*)(brow_ptr[i] + k0) : (const void*)g_zero_chunk,
               Bs + (i * 8 + wave) * 1024);
      }
    }
  };

  float4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};

  // EPI_MASK: this thread's epilogue mask bytes (rows r0 + 16 it of column chunk c), loaded now so that
  // they land with the prologue's LDS-DMA instead of as dependent loads in the epilogue
  unsigned char mpre[16];
  if constexpr (EPIM == EPI_MASK) {
    const int c = tid & 31, r0 = tid >> 5;
    const int n = n0 + c * 8;
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int m = m0 + r0 + 16 * it;
      mpre[it] = (n < g.N && m < g.M) ? ex.mask_in[(long)m * (g.N >> 3) + (n >> 3)] : (unsigned char)0;
    }
  }
  // EPI_BNH: the BatchNorm input h of this thread's 16 epilogue rows.  The first BNH_PRE rows (4 VGPRs each)
  // are loaded now and land under the main loop; the rest (register budget: the whole 16 would push the
  // epilogue past 256 VGPRs) are issued right after the accumulator staging, before its barrier
  // (STG: its fragment ring holds 16 more VGPRs -- half the rows prefetched, the rest after the main loop)
  constexpr int BNH_PRE = STG ? 8 : 16;
  short8 hpre[16];
  auto load_h = [&](int it0, int it1) {
    const int c = tid & 31, r0 = tid >> 5;
    const int n = n0 + c * 8;
#pragma unroll
    for (int it = it0; it < it1; ++it) {
      const int m = m0 + r0 + 16 * it;
      hpre[it] = (short8){0, 0, 0, 0, 0, 0, 0, 0};  // rows / columns out of range: h = 0 (their dz is 0 too)
      if (n < g.N && m < g.M) hpre[it] = *reinterpret_cast<const short8*>(ex.acc + (long)m * ldy + n);
    }
  };
  if constexpr (EPIM == EPI_BNH) {
    load_h(0, BNH_PRE);
  }
  // split-K (gridDim.y > 1): block y owns the k slabs [kt0, kt1) and writes its fp32 partial
  // tile to slice y of the workspace (Yv), reduced afterwards in a fixed order (splitk_reduce)
  const int nk_all = (g.K + 63) / 64;
  int kt0 = 0, nk = nk_all;
  if (gridDim.y > 1) {
    const int per = (nk_all + gridDim.y - 1) / gridDim.y;
    kt0 = blockIdx.y * per;
    nk = min(nk_all, kt0 + per);
    Yv = reinterpret_cast<float*>(Yv) + (long)blockIdx.y * g.M * ldy;
  }
  if (g.ksplit > 0 && gridDim.y == 1) {  // ConvTranspose 3-tap form: skip the tile's all-zero tap (see ConvGeom)
    const int kc = g.Cin / 64;
    if (n0 < g.ksplit) nk = 2 * kc;
    else kt0 = kc;
  }
  if constexpr (STG) {
    // Staggered 8-phase main loop (MI355X: one wave of each group per SIMD, so one wave's MFMA cluster runs
    // while its partner issues LDS reads and LDS-DMA; loads stay in flight across barriers).
    // Groups: G0 = waves 0-3 (A rows 0-127), G1 = waves 4-7 (A rows 128-255).  A k-tile is computed in 4
    // phases, each a quadrant (qa, qb) = (0,0) (0,1) (1,1) (1,0) of the wave's 128 x 64 output (16 MFMAs);
    // a phase is  R: [LDS-DMA of one staging unit] [ds_reads of the quadrant] [vmcnt]  barrier
    //             M: setprio(1) [16 MFMAs] setprio(0)  barrier
    // and G1 runs one barrier behind G0 (an extra barrier before the loop), so G0's M segments pair with
    // G1's R segments and vice versa.  Units (16 KiB, 2 DMA instructions per lane): U0 = A rows of qa 0
    // (both groups), U1 = B rows of qb 1, U2 = A rows of qa 1, U3 = B rows of qb 0; the qb 0 B fragments
    // stay in registers from phase 0 to phase 3, so a unit's last read is in phase 0 (U0, U3), 1 (U1) or
    // 2 (U2).  With the stagger a unit is rewritten >= 2 phases after its last read (its reads are
    // retired by both groups' lgkmcnt before the barrier that follows their next segment):
    //   P2(t): U0(t+2)   P3(t): U1(t+2)   P0(t+1): U2(t+2)   P1(t+1): U3(t+2)    (into tile t's buffer)
    // RAW: U3(t+2), the last unit of tile t+2, is waited for in P3(t+1)'s R segment -- vmcnt(4) leaves the
    // 2 units issued after it in flight -- and first read in P0(t+2), a barrier later for both groups.
    int bblk[4], bvo2[4];  // B 8-row blocks of this wave: U3 (qb = 0) -> [0], [1]; U1 (qb = 1) -> [2], [3]
    bblk[0] = 8 * (wave >> 2) + (wave & 3);
    bblk[1] = bblk[0] + 16;
    bblk[2] = bblk[0] + 4;
    bblk[3] = bblk[1] + 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = bblk[u] * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      bvo2[u] = (n0 + row < g.N) ? ((n0 + row) * g.K + ch * 8) * 2 : kOOB;
    }
    // A 8-row blocks: load i covers block i * 8 + wave (rows 64 i + 8 wave ..): U0 = i in {0, 2}, U2 = {1, 3}
    auto stage_a = [&](int kt, int q, int buf) {
      char* As = smem + buf * STG64_BYTES;
      const int k0 = kt * 64;
      const int tap = k0 / g.Cin;
      const int cin0 = k0 - tap * g.Cin;
      const int shift = tap * g.dil - g.pad;
      const int aoff = (shift * g.Cin + cin0) * 2;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int i = q + 2 * jj;
        const int ts = a_t[i] + shift;
        const bool ok = (unsigned)ts < (unsigned)a_lim[i];
        buf_lds16(rA, ok ? avo[i] + aoff : kOOB, 0, As + (i * 8 + wave) * 1024);
      }
    };
    auto stage_b = [&](int kt, int q, int buf) {  // q = 0: U3 (qb = 0 rows), q = 1: U1 (qb = 1 rows)
      char* Bs = smem + buf * STG64_BYTES + BG * 64 * 2;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) buf_lds16(rB, bvo2[q * 2 + jj], kt * 128, Bs + bblk[q * 2 + jj] * 1024);
    };
    short8 fa[2][4], fb0[2][2], fb1[2][2];
    auto read_a = [&](const char* As, int qa) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fa[kk][i] = *reinterpret_cast<const short8*>(As + swz128(wm * 128 + qa * 64 + i * 16 + (lane & 15), c));
      }
    };
    auto read_b = [&](const char* Bs, int qb, short8 (&fb)[2][2]) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[kk][j] = *reinterpret_cast<const short8*>(Bs + swz128(wn * 64 + qb * 32 + j * 16 + (lane & 15), c));
      }
    };
    auto mma = [&](int qa, int qb, const short8 (&fb)[2][2]) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qa * 4 + i][qb * 2 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk][j], fa[kk][i], acc[qa * 4 + i][qb * 2 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    const int nkt = nk - kt0;
    // prologue: tiles kt0 and kt0 + 1 whole; tile kt0 landed (the 8 younger DMA instructions in flight)
    if (nkt > 0) { stage_a(kt0, 0, 0); stage_b(kt0, 1, 0); stage_a(kt0, 1, 0); stage_b(kt0, 0, 0); }
    if (nkt > 1) {
      stage_a(kt0 + 1, 0, 1); stage_b(kt0 + 1, 1, 1); stage_a(kt0 + 1, 1, 1); stage_b(kt0 + 1, 0, 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pp_barrier();
    if (wm == 1) pp_barrier();  // G1 runs one barrier behind G0
    for (int t = 0; t < nkt; ++t) {
      const int buf = t & 1, kt = kt0 + t;
      const char* As = smem + buf * STG64_BYTES;
      const char* Bs = As + BG * 64 * 2;
      const bool s1 = t >= 1 && t + 1 < nkt;  // U2 / U3 of tile t+1 go out in P0 / P1 of tile t
      const bool s2 = t + 2 < nkt;            // U0 / U1 of tile t+2 go out in P2 / P3 of tile t
      // P0
      if (s1) stage_a(kt + 1, 1, buf ^ 1);
      read_a(As, 0);
      read_b(Bs, 0, fb0);
      pp_barrier();
      mma(0, 0, fb0);
      pp_barrier();
      // P1
      if (s1) stage_b(kt + 1, 0, buf ^ 1);
      read_b(Bs, 1, fb1);
      pp_barrier();
      mma(0, 1, fb1);
      pp_barrier();
      // P2
      if (s2) stage_a(kt + 2, 0, buf);
      read_a(As, 1);
      pp_barrier();
      mma(1, 1, fb1);
      pp_barrier();
      // P3: tile t+1 must be complete before P0(t+1): its last unit (U3, issued in P1) retired here
      if (s2) stage_b(kt + 2, 1, buf);
      if (t + 1 < nkt) {
        if (s2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      pp_barrier();
      mma(1, 0, fb0);
      pp_barrier();
    }
    if (wm == 0) pp_barrier();  // equal barrier counts: G0 catches up with G1's extra one
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();
  } else {
  // double buffer: stage kt+1 is DMA'd while stage kt is computed (one stage = 1024 MFMA cycles
  // per wave, far longer than an L2-warm LDS-DMA), one barrier per 64-wide k slab
  if (kt0 < nk) stage(kt0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = kt0; kt < nk; ++kt) {
    const int buf = (kt - kt0) & 1;
    if (kt + 1 < nk) stage(kt + 1, buf ^ 1);
    const char* As = smem + buf * STG64_BYTES;
    const char* Bs = As + BG * 64 * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
      short8 fa[8], fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const short8*>(Bs + swz128(wn * 64 + j * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const short8*>(As + swz128(wm * 128 + i * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  }  // !STG
  if constexpr (!OUT_F32) {
    if (act >= 0 && (g.N & 7) == 0 && (ldy & 7) == 0) {
      // LDS-staged epilogue: the accumulator layout gives each lane 4 columns of one row, i.e.
      // 32-B row pieces per store instruction (16 rows each); staging the bf16 tile through LDS
      // (528-B padded rows: conflict-free both ways) turns that into 16-B-per-lane stores of whole
      // 512-B rows, and the aux / residual operands are read the same coalesced way.
      // (Measured: the direct register stores cost up to 55 % of a K = 256 GEMM.)
      char* Ct = smem;  // [BG][528 B] staging tile (ct_woff / ct_read)
      // bias and activation are compile-time branches of the staging loop: as runtime checks inside the
      // unrolled 8 x 4 loop they cost ~350 scalar branches per tile, and the bias float4 was re-loaded
      // (behind a full vmcnt wait) for every (i, j) -- 32 serialised L2 round trips per tile
      auto stage_tile = [&](auto actc, auto biasc) {
        constexpr int A = decltype(actc)::value;
        constexpr bool HB = decltype(biasc)::value;
        float4 bv[4];
        if constexpr (HB) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
            bv[j] = n < g.N ? *reinterpret_cast<const float4*>(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int ml = wm * 128 + i * 16 + (lane & 15);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int nl = wn * 64 + j * 16 + 4 * (lane >> 4);
            float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            if constexpr (HB) {
              v[0] += bv[j].x; v[1] += bv[j].y; v[2] += bv[j].z; v[3] += bv[j].w;
            }
            if constexpr (A == ACT_RELU) {
#pragma unroll
              for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
            } else if constexpr (A == ACT_LRELU) {
#pragma unroll
              for (int q = 0; q < 4; ++q) v[q] = v[q] > 0.f ? v[q] : 0.1f * v[q];
            } else if constexpr (A == ACT_TANH) {
#pragma unroll
              for (int q = 0; q < 4; ++q) v[q] = tanhf(v[q]);
            }
            short4v o;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = (short)f2bf(v[q]);
            *reinterpret_cast<short4v*>(Ct + ct_woff(ml, nl)) = o;
          }
        }
      };
      auto stage_act = [&](auto biasc) {
        if (act == ACT_RELU) stage_tile(std::integral_constant<int, ACT_RELU>{}, biasc);
        else if (act == ACT_LRELU) stage_tile(std::integral_constant<int, ACT_LRELU>{}, biasc);
        else if (act == ACT_TANH) stage_tile(std::integral_constant<int, ACT_TANH>{}, biasc);
        else stage_tile(std::integral_constant<int, ACT_NONE>{}, biasc);
      };
      if constexpr (EPIM == EPI_BNH) stage_tile(std::integral_constant<int, ACT_NONE>{}, std::false_type{});  // no bias / act
      else if (bias) stage_act(std::true_type{});
      else stage_act(std::false_type{});
      if constexpr (EPIM == EPI_BNH) {
        if constexpr (BNH_PRE < 16) load_h(BNH_PRE, 16);
      }
      __syncthreads();
      // the prefetched mask bytes were retired by the main loop's inline-asm waits, which the waitcnt pass
      // does not see: without this counted wait it drains every earlier row's store before each row
      if constexpr (EPIM == EPI_MASK) __builtin_amdgcn_s_waitcnt(0x0F70);
      bf16_t* Y = reinterpret_cast<bf16_t*>(Yv);
      if constexpr (EPIM == EPI_BNH) {
        // BatchNorm-backward head (EpiX: acc = bn_h, bn_stats = [mean | rstd | scale | shift] x N,
        // bn_part = partials, post_act = act code, bn_p = dropout p).  Thread (c = tid & 31, r0 = tid >> 5)
        // owns column chunk c of rows r0 + 16 it, loads h for EPG rows before use, stores dz and keeps
        // its 8 columns' running sums; the tile's 16 per-column partials are then combined in fixed order.
        // The epilogue runs while the CU's MFMAs idle (one workgroup per CU), so its VALU count is the
        // cost: the activation is a compile-time branch of the row loop (a per-element runtime branch
        // split every row into 8 basic blocks), tanh' = 4 r (1 - r) with r = 1 / (exp(2z) + 1) and the
        // exp2 scale folded into the BatchNorm affine; the second partial is sum dz * (h - mean) (the
        // finalize applies rstd once per column).
        constexpr int EPI = BG * 32 / NT3;
        const int c = tid & 31, r0 = tid >> 5;
        const int n = n0 + c * 8;
        const bool col_ok = n < g.N;
        float bmu[8], bsc[8], bsh[8], bs1[8], bs2[8];
        const int act_c = ex.post_act;
        const float zs = act_c == 1 ? 2.8853900817779268f : 1.f;  // 2 log2(e): exp(2z) = exp2(zs z)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int nq = col_ok ? n + q : 0;
          bmu[q] = ex.bn_stats[nq];
          bsc[q] = ex.bn_stats[2 * g.N + nq] * zs;
          bsh[q] = ex.bn_stats[3 * g.N + nq] * zs;
          bs1[q] = 0.f;
          bs2[q] = 0.f;
        }
        // vmcnt counts stores as well as loads: a load the waitcnt pass still thinks outstanding (the h
        // prefetch, retired by the main loop's inline-asm waits it cannot see; the column constants) makes
        // it wait with vmcnt(0) -- i.e. for every dz store issued so far -- before the first use in each
        // row.  One counted wait here retires them all for the pass; the rows are straight-line code (no
        // per-row skip: out-of-range rows have dz = 0 and h = 0 and only their store is predicated).
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt unconstrained
        auto rows = [&](auto actc) {
          constexpr int A = decltype(actc)::value;
#pragma unroll
          for (int it = 0; it < EPI; ++it) {
            const int r = r0 + 16 * it;
            const int m = m0 + r;
            const short8 v = ct_read(Ct, r, c);
            const long off = (long)m * ldy + n;
            float ks[8];
            drop_scales<8>(ex.bn_seed, (uint64_t)off, ex.bn_p, ks);
            short8 o;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const float hv = bf2f((bf16_t)hpre[it][q]);
              float d = bf2f((bf16_t)v[q]) * ks[q];
              if constexpr (A == 1) {
                const float rr = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(hv * bsc[q] + bsh[q]) + 1.f);
                d *= 4.f * (rr - rr * rr);
              } else if constexpr (A == 2) {
                d = hv * bsc[q] + bsh[q] > 0.f ? d : 0.f;
              }
              bs1[q] += d;
              bs2[q] += d * (hv - bmu[q]);
              o[q] = (short)f2bf(d);
            }
            if (m < g.M && col_ok) *reinterpret_cast<short8*>(Y + off) = o;
          }
        };
        if (act_c == 1) rows(std::integral_constant<int, 1>{});  // tanh (PostNet); ReLU is rejected on the host
        else rows(std::integral_constant<int, 0>{});
        // every Ct read is done: reuse the staging LDS for the partials.  LDS-only barriers: __syncthreads
        // would also drain this thread's 16 dz stores (vmcnt counts stores), ~7 us per tile-round chip-wide
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        float* red = reinterpret_cast<float*>(smem);  // [2][16][256]
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          red[r0 * 256 + c * 8 + q] = bs1[q];
          red[4096 + r0 * 256 + c * 8 + q] = bs2[q];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const int which = tid >> 8, col = tid & 255;  // threads 0..255: sum dz, 256..511: sum dz*xhat
        if (n0 + col < g.N) {
          float a = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) a += red[which * 4096 + r * 256 + col];
          ex.bn_part[((long)which * nM + tm) * g.N + n0 + col] = a;
        }
        return;
      } else {  // !EPI_BNH: the BNH instantiation compiles none of the code below
      const bool xon = ex.acc || ex.y2 || ex.post_act || ex.scale != 1.f || ex.mask_in;
      // Thread (c = tid & 31, r0 = tid >> 5) owns the 16-B column chunk c of rows r0 + 16 it.  The
      // global operands of EPG rows (aux / residual / accumulator segments, mask bytes, sequence
      // lengths) are all loaded before any is used: one loop iteration per row would expose a full
      // memory round trip per row (16 in a row per tile -- the K = 256 ReLU-mask data gradient
      // spent most of its time there).  All 16 rows are loaded before the first store (the accumulators
      // are dead here, 3 x 16 x 16 B fit): a second load batch after stores would wait for those stores
      // too (vmcnt counts both).  Same arithmetic, same order as the one-row form.
      constexpr int EPI = BG * 32 / NT3;  // 16 rows per thread
      constexpr int EPG = 16;             // rows per load batch: all 16 before the first store (see below)
      const int c = tid & 31, r0 = tid >> 5;
      const int n = n0 + c * 8;
      const bool col_ok = n < g.N;
      const bool loads = aux || resid || ex.acc || ex.mask_in || lens;
      if (!loads && !xon) {  // store-only epilogue (+ the ReLU bitmask): the plain row loop
        for (int e = tid; e < BG * 32; e += NT3) {
          const int r = e >> 5, cc = e & 31;
          const int m = m0 + r, nn = n0 + cc * 8;
          if (m >= g.M || nn >= g.N) continue;
          const short8 v = ct_read(Ct, r, cc);
          if (ex.mask_out) {
            unsigned bits = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) bits |= (unsigned)((short)v[q] > 0) << q;
            ex.mask_out[(long)m * (g.N >> 3) + (nn >> 3)] = (unsigned char)bits;
          }
          *reinterpret_cast<short8*>(Y + (long)m * ldy + nn) = v;
        }
        return;
      }
#pragma unroll
      for (int g0 = 0; g0 < EPI; g0 += EPG) {
        short8 va[EPG], vr[EPG], vc[EPG];
        unsigned mb[EPG];
        bool vv[EPG];
        if (loads) {
#pragma unroll
          for (int u = 0; u < EPG; ++u) {
            const int m = m0 + r0 + 16 * (g0 + u);
            const bool in = col_ok && m < g.M;
            const long off = (long)m * ldy + n;
            if (in && aux) va[u] = *reinterpret_cast<const short8*>(aux + off);
            if (in && resid) vr[u] = *reinterpret_cast<const short8*>(resid + off);
            if (in && ex.acc) vc[u] = *reinterpret_cast<const short8*>(ex.acc + off);
            if constexpr (EPIM == EPI_MASK) mb[u] = mpre[g0 + u];
            else mb[u] = (in && ex.mask_in) ? (unsigned)ex.mask_in[(long)m * (g.N >> 3) + (n >> 3)] : 0xffu;
            vv[u] = true;
            if (in && lens) {
              const int bb = m / g.L, tt = m - bb * g.L;
              vv[u] = tt < (int)lens[bb];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < EPG; ++u) {
          const int r = r0 + 16 * (g0 + u);
          const int m = m0 + r;
          if (m >= g.M || !col_ok) continue;
          short8 v = ct_read(Ct, r, c);
          const bool valid = loads ? vv[u] : true;
          const long off = (long)m * ldy + n;
          if (ex.mask_out) {  // ReLU output > 0  <=>  its bf16 bits are a positive non-zero value
            unsigned bits = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) bits |= (unsigned)((short)v[q] > 0) << q;
            ex.mask_out[(long)m * (g.N >> 3) + (n >> 3)] = (unsigned char)bits;
          }
          if (aux || resid || !valid || xon) {
            float f[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] = bf2f((bf16_t)v[q]);
            if (aux) {
#pragma unroll
              for (int q = 0; q < 8; ++q) f[q] = bf2f((bf16_t)va[u][q]) > 0.f ? f[q] : 0.f;
            }
            if (ex.mask_in) {
#pragma unroll
              for (int q = 0; q < 8; ++q) f[q] = (mb[u] >> q) & 1u ? f[q] : 0.f;
            }
            if (resid) {
#pragma unroll
              for (int q = 0; q < 8; ++q) f[q] += bf2f((bf16_t)vr[u][q]);
            }
            if (ex.acc) {
#pragma unroll
              for (int q = 0; q < 8; ++q) f[q] += bf2f((bf16_t)vc[u][q]);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] = valid ? f[q] * ex.scale : 0.f;
            if (ex.y2) {
              short8 o2;
#pragma unroll
              for (int q = 0; q < 8; ++q) o2[q] = (short)f2bf(f[q] > 0.f ? f[q] : 0.1f * f[q]);
              *reinterpret_cast<short8*>(ex.y2 + off) = o2;
            }
            if (ex.post_act == ACT_LRELU) {
#pragma unroll
              for (int q = 0; q < 8; ++q) f[q] = f[q] > 0.f ? f[q] : 0.1f * f[q];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = (short)f2bf(f[q]);
          }
          *reinterpret_cast<short8*>(Y + off) = v;
        }
      }
      return;
      }  // !EPI_BNH
    }
  }
  if constexpr (EPIM == EPI_BNH) return;  // unreachable: conv_gemm_impl validates the staged-path shape
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + (lane & 15);
    if (m >= g.M) continue;
    bool valid = true;
    if (lens) {
      const int bb = m / g.L, tt = m - bb * g.L;
      valid = tt < (int)lens[bb];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= g.N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      epi_store4<OUT_F32>(v, m, n, bias, aux, resid, valid, act, ldy, Yv);
    }
  }
}

template <bool OUT_F32, bool FASTK, bool PACKED, bool BUF = false, int EPIM = EPI_GEN, bool STG = false>
__global__ void __launch_bounds__(NT3, 1) conv_gemm_big64_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                               const float* __restrict__ bias,
                                                               const bf16_t* __restrict__ aux,
                                                               const bf16_t* __restrict__ resid,
                                                               const int64_t* __restrict__ lens, void* __restrict__ Yv,
                                                               ConvGeom g, int act, int ldy, EpiX ex) {
  big64_tile<OUT_F32, FASTK, PACKED, BUF, EPIM, STG>(X, W, bias, aux, resid, lens, Yv, g, act, ldy, ex, blockIdx.x);
}


// ----------------------------------------------------------------------------
// Weight gradient.  Tile: 128 (n = cout) x 128 (k = tap*Cin + cin), reduction over
// rows m in steps of RB = 64.  LDS image per operand: [64 rows][128 cols] bf16,
// 256-B rows, 8-B column chunks XOR-swizzled by f(row) = ((row&3) | ((row>>3)&1)<<2) << 2
// so the 32 lanes of a half-wave hit 32 distinct 8-B slots in ds_read_b64_tr_b16.
// ----------------------------------------------------------------------------
constexpr int RB = 64;

__device__ __forceinline__ int swz_tr(int row, int cc /*8-B chunk 0..31*/) {
  const int f = ((row & 3) | (((row >> 3) & 1) << 2)) << 2;
  return row * 256 + ((cc ^ f) << 3);
}

__device__ __forceinline__ short4v ds_read_tr(const char* p) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

template <bool PACKED>
__global__ void __launch_bounds__(NT, 2) conv_wgrad_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                                                           float* __restrict__ slabs, float* __restrict__ bias_slabs,
                                                           ConvGeom g, int rows_per_split) {
  const void* const g_zero_chunk = zero_chunk_ptr();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nN = (g.N + 127) / 128;  // cout tiles
  const int nK = (g.K + 127) / 128;  // k tiles
  const int tile = blockIdx.x % (nN * nK);
  const int split = blockIdx.x / (nN * nK);
  const int tn = tile / nK, tk = tile % nK;
  const int n0 = tn * 128, k0 = tk * 128;
  const int r_begin = split * rows_per_split;
  const int r_end = min(g.M, r_begin + rows_per_split);
  // wave index as a scalar: LDS-DMA destinations (M0) and per-wave offsets stay in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 1, wk = wave & 1;
  const float invCin = 1.f / (float)g.Cin;

  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};

  // LDS-DMA staging: a wave instruction fills 4 rows x 256 B; lane -> (row rr, physical 16-B chunk p16);
  // the tr-read swizzle f(row) permutes 16-B chunks by f>>1, applied on the source side.
  int rr[4], c_n[4], c_tap[4], c_cin[4];
  bool c_kok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 4 + wave) * 4 + (lane >> 4);
    rr[i] = row;
    const int f = ((row & 3) | (((row >> 3) & 1) << 2)) << 2;
    const int c16 = (lane & 15) ^ (f >> 1);
    c_n[i] = n0 + c16 * 8;
    const int k = k0 + c16 * 8;
    c_kok[i] = k < g.K;
    c_tap[i] = c_kok[i] ? (int)(((float)k + 0.5f) * invCin) : 0;
    c_cin[i] = k - c_tap[i] * g.Cin;
  }
  // per-row time index t = m mod L, advanced incrementally (stage() is called for r0 = r_begin, +RB, ...)
  int tcur[4], shift[4];
  // PACKED: (position, length) of the next stage's rows, loaded one stage ahead with a clamped
  // (branch-free) index so the read never sits in front of the operand DMA
  int2 rnext[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    shift[i] = c_tap[i] * g.dil - g.pad;
    if constexpr (PACKED) rnext[i] = g.rinfo[min(r_begin + rr[i], g.M - 1)];
    else tcur[i] = (r_begin + rr[i]) % g.L;
  }
  auto stage = [&](int r0, int buf) {
    char* Ys = smem + buf * (2 * RB * 256);
    char* Xs = Ys + RB * 256;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + rr[i];
      const bool mok = m < r_end;
      int ts, lim;
      if constexpr (PACKED) {
        ts = rnext[i].x + shift[i];
        lim = rnext[i].y;
        rnext[i] = g.rinfo[min(m + RB, g.M - 1)];
      } else {
        ts = tcur[i] + shift[i];
        lim = g.L;
      }
      const bool xok = mok && c_kok[i] && ts >= 0 && ts < lim;
      const void* sy = (mok && c_n[i] < g.N) ? (const void*)(dY + (long)m * g.N + c_n[i]) : (const void*)g_zero_chunk;
      const void* sx = xok ? (const void*)(X + (long)(m + shift[i]) * g.Cin + c_cin[i]) : (const void*)g_zero_chunk;
      glds16(sy, Ys + (i * 4 + wave) * 4 * 256);
      glds16(sx, Xs + (i * 4 + wave) * 4 * 256);
      if constexpr (!PACKED) {
        int t = tcur[i] + RB;
        while (t >= g.L) t -= g.L;
        tcur[i] = t;
      }
    }
  };
  // bias gradient (column sums of dY) for the k-tile-0 blocks, read back from the LDS image
  const bool do_bias = bias_slabs != nullptr && tk == 0;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int bc16 = tid & 15;

  const int nsteps = (r_end - r_begin + RB - 1) / RB;
  if (nsteps > 0) stage(r_begin, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) stage(r_begin + (s + 1) * RB, buf ^ 1);
    const char* Ys = smem + buf * (2 * RB * 256);
    const char* Xs = Ys + RB * 256;
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (tid >> 4) + 16 * j;
        const short8 v = *reinterpret_cast<const short8*>(Ys + swz_tr(row, bc16 * 2));
#pragma unroll
        for (int t = 0; t < 8; ++t) bsum[t] += bf2f((bf16_t)v[t]);
      }
    }
#pragma unroll
    for (int kk = 0; kk < RB / 32; ++kk) {
      short8 fa[4], fb[4];
      const int rbase = kk * 32 + grp * 8 + q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ca = (wn * 64 + i * 16) / 4 + p;
        const int cb = (wk * 64 + i * 16) / 4 + p;
        short4v a0 = ds_read_tr(Ys + swz_tr(rbase, ca));
        short4v a1 = ds_read_tr(Ys + swz_tr(rbase + 4, ca));
        short4v b0 = ds_read_tr(Xs + swz_tr(rbase, cb));
        short4v b1 = ds_read_tr(Xs + swz_tr(rbase + 4, cb));
        fa[i] = (short8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        fb[i] = (short8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (do_bias) {  // reduce the 16 row-groups that share a column chunk, one partial per split
    float* red = reinterpret_cast<float*>(smem);  // [16][128]
#pragma unroll
    for (int t = 0; t < 8; ++t) red[(tid >> 4) * 128 + bc16 * 8 + t] = bsum[t];
    __syncthreads();
    if (tid < 128 && n0 + tid < g.N) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) t += red[j * 128 + tid];
      bias_slabs[(long)split * g.N + n0 + tid] = t;
    }
  }
  // partial slab [split][N][K] fp32
  float* S = slabs + (long)split * g.N * g.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wk * 64 + j * 16 + (lane & 15);
        if (n < g.N && k < g.K) S[(long)n * g.K + k] = acc[i][j][r];
      }
}


// LDS helpers of the 256x256 weight-gradient kernel (64-row dY / X images, 512-B rows)

// ds_read_b64_tr_b16 as inline asm: the builtin carries no LDS alias information, so the
// compiler's waitcnt pass drains EVERY in-flight LDS-DMA (vmcnt(0)) before it -- which
// serialises the ring.  The asm form is invisible to that pass; the caller waits with
// lgkm_wait_tie() before consuming the fragments.
__device__ __forceinline__ short4v ds_read_tr_asm(const char* p) {
  short4v r;
  const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
// ... with a DS immediate offset: fragments that differ by a constant (the +4-row half, the k-half, the stage
// buffer) share one address register -- no per-read v_add in the read segment
template <int OFF>
__device__ __forceinline__ short4v ds_read_tr_off(unsigned addr) {
  short4v r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
// s_waitcnt lgkmcnt(0) that the fragments data-depend on (MFMAs cannot be hoisted above it)
__device__ __forceinline__ void lgkm_wait_tie(short8 (&fa)[4], short8 (&fb)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(fa[0]), "+v"(fa[1]), "+v"(fa[2]), "+v"(fa[3]), "+v"(fb[0]), "+v"(fb[1]), "+v"(fb[2]),
                 "+v"(fb[3]));
}

__device__ __forceinline__ int swz_tr512(int row, int cc /*8-B chunk 0..63*/) {
  const int f = ((row & 3) | (((row >> 3) & 1) << 2)) << 2;
  return row * 512 + ((cc ^ f) << 3);
}

constexpr int WB64_STAGE = 2 * 64 * 512;  // 64 KiB: dY [64][256] + X [64][256]

// lgkmcnt(0) that the fragments depend on (the inline-asm LDS reads are invisible to the compiler's
// waitcnt pass, so the MFMAs consuming them must not be scheduled above the wait)
__device__ __forceinline__ void lgkm_tie(short8 (&a)[2][4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0][0]), "+v"(a[0][1]), "+v"(a[0][2]), "+v"(a[0][3]), "+v"(a[1][0]), "+v"(a[1][1]),
                 "+v"(a[1][2]), "+v"(a[1][3]));
}
__device__ __forceinline__ void lgkm_tie(short8 (&b)[2][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[1][0]), "+v"(b[1][1]));
}

template <bool PACKED, bool IMM, bool BUF, bool PP = false>
__global__ void __launch_bounds__(NT3, 1) conv_wgrad_big64_kernel(const bf16_t* __restrict__ X,
                                                                const bf16_t* __restrict__ dY,
                                                                float* __restrict__ slabs,
                                                                float* __restrict__ bias_slabs, ConvGeom g,
                                                                int rows_per_split) {
  const void* const g_zero_chunk = zero_chunk_ptr();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nN = (g.N + 255) / 256;
  const int nK = (g.K + 255) / 256;
  const int tiles = nN * nK;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wg % tiles, split = wg / tiles;
  const int tn = tile / nK, tk = tile % nK;
  const int n0 = tn * 256, k0 = tk * 256;
  const int r_begin = split * rows_per_split;
  const int r_end = min(g.M, r_begin + rows_per_split);
  // wave index as a scalar: LDS-DMA destinations (M0) and per-wave offsets stay in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 2, wk = wave & 3;
  const float invCin = 1.f / (float)g.Cin;
  if (!PP && g.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);

  float4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};

  // DMA: a wave instruction = 2 rows of 512 B; each image 32 rows = 16 instructions = 2 per wave
  int drow[4];
  const bf16_t* ysrc[4];
  bool yok[4];
  int xshift[4], xcin[4];
  bool xkok[4];
  int t_cur[4];
  // packed rows: (position, length) of each staged row from the rinfo table, prefetched one stage
  // ahead of its use so the DMA issue never waits on it (no per-step sequence walk)
  int2 ri_nxt[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 2 * (i * 8 + wave) + (lane >> 5);
    drow[i] = row;
    const int f = ((row & 3) | (((row >> 3) & 1) << 2)) << 2;
    const int c16 = (lane & 31) ^ (f >> 1);
    const int n = n0 + c16 * 8;
    yok[i] = n < g.N;
    ysrc[i] = dY + (yok[i] ? n : 0);
    const int k = k0 + c16 * 8;
    xkok[i] = k < g.K;
    const int tap = xkok[i] ? (int)(((float)k + 0.5f) * invCin) : 0;
    xcin[i] = k - tap * g.Cin;
    xshift[i] = tap * g.dil - g.pad;
    const int m = r_begin + row;
    if constexpr (!PACKED) t_cur[i] = m % g.L;
  }
  // BUF: the rinfo rows through a descriptor bounded at r_end (past it: (0, 0) = every tap invalid),
  // no exec-masked load blocks
  const __amdgpu_buffer_rsrc_t rR = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.rinfo, 0, (BUF && PACKED) ? r_end * 8 : 0, 0x00020000);
  auto load_ri = [&](int r0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + drow[i];
      if constexpr (BUF) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rR, m * 8, 0, 0);
        ri_nxt[i] = make_int2((int)v[0], (int)v[1]);
      } else {
        ri_nxt[i] = m < r_end ? g.rinfo[m] : make_int2(0, 0);
      }
    }
  };
  if constexpr (PACKED) load_ri(r_begin);
  // BUF: LDS-DMA through buffer descriptors -- dY over the rows of this split (a row past r_end or a
  // column past N is out of range and lands as zeros), X over rows [-pad, M) -- with loop-invariant
  // 32-bit per-lane offsets plus one 32-bit add per row and step: no 64-bit address math, no
  // exec-masked address blocks and no zero-chunk selects in the stage issue (out-of-range = zeros)
  const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dY + (long)r_begin * g.N), 0, BUF ? (r_end - r_begin) * g.N * 2 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(X - (long)g.pad * g.Cin), 0, BUF ? (g.M + g.pad) * g.Cin * 2 : 0, 0x00020000);
  int yvo[4], xvo[4];
  constexpr int kOOB = (int)0x80000000;
  const bool x_always = g.ks == 1 && g.pad == 0;  // Linear / k = 1: every X row of a valid dY row is valid
  if constexpr (BUF) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      yvo[i] = yok[i] ? (drow[i] * g.N + (int)(ysrc[i] - dY)) * 2 : kOOB;
      xvo[i] = xkok[i] ? ((drow[i] + xshift[i] + g.pad) * g.Cin + xcin[i]) * 2 : kOOB;
    }
  }
  // LDS: dY images of the two stages at 0 / 32 KiB, X images at 64 / 96 KiB, so that every
  // fragment read is a loop-invariant per-lane base + an immediate (stage, k-half, +4 rows)
  // BUF: the dY and X halves of a stage, issued separately by the ping-pong loop
  auto stage_y = [&](int r0, int buf) {
    char* Ys = smem + buf * 32768;
    const int dy_off = (r0 - r_begin) * g.N * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) buf_lds16(rY, yvo[i] + dy_off, 0, Ys + (i * 8 + wave) * 1024);
  };
  auto stage_x = [&](int r0, int buf) {
    char* Xs = smem + 65536 + buf * 32768;
    const int x_off = r0 * g.Cin * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool ok = true;
      if (!x_always) {
        int ts, lim;
        if constexpr (PACKED) {
          ts = ri_nxt[i].x + xshift[i];
          lim = ri_nxt[i].y;
        } else {
          ts = t_cur[i] + xshift[i];
          lim = g.L;
          int t = t_cur[i] + 64;
          while (t >= g.L) t -= g.L;
          t_cur[i] = t;
        }
        ok = (unsigned)ts < (unsigned)lim;
      }
      buf_lds16(rX, ok ? xvo[i] + x_off : kOOB, 0, Xs + (i * 8 + wave) * 1024);
    }
  };
  auto stage = [&](int r0, int buf) {
    char* Ys = smem + buf * 32768;
    char* Xs = smem + 65536 + buf * 32768;
    if constexpr (BUF) {
      const int dy_off = (r0 - r_begin) * g.N * 2, x_off = r0 * g.Cin * 2;
#pragma unroll
      for (int i = 0; i < 4; ++i) buf_lds16(rY, yvo[i] + dy_off, 0, Ys + (i * 8 + wave) * 1024);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bool ok = true;
        if (!x_always) {
          int ts, lim;
          if constexpr (PACKED) {
            ts = ri_nxt[i].x + xshift[i];
            lim = ri_nxt[i].y;
          } else {
            ts = t_cur[i] + xshift[i];
            lim = g.L;
            int t = t_cur[i] + 64;
            while (t >= g.L) t -= g.L;
            t_cur[i] = t;
          }
          ok = (unsigned)ts < (unsigned)lim;
        }
        buf_lds16(rX, ok ? xvo[i] + x_off : kOOB, 0, Xs + (i * 8 + wave) * 1024);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + drow[i];
      glds16((yok[i] && m < r_end) ? (const void*)(ysrc[i] + (long)m * g.N) : (const void*)g_zero_chunk,
             Ys + (i * 8 + wave) * 1024);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + drow[i];
      int ts, lim;
      if constexpr (PACKED) {
        ts = ri_nxt[i].x + xshift[i];
        lim = ri_nxt[i].y;
      } else {
        ts = t_cur[i] + xshift[i];
        lim = g.L;
        int t = t_cur[i] + 64;
        while (t >= g.L) t -= g.L;
        t_cur[i] = t;
      }
      const bool ok = xkok[i] && m < r_end && ts >= 0 && ts < lim;
      glds16(ok ? (const void*)(X + (long)(m + xshift[i]) * g.Cin + xcin[i]) : (const void*)g_zero_chunk,
             Xs + (i * 8 + wave) * 1024);
    }
  };
  const bool do_bias = bias_slabs != nullptr && tk == 0;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int bc16 = tid & 31;

  const int nsteps = (r_end - r_begin + 64 - 1) / 64;
  if (nsteps > 0) stage(r_begin, 0);
  if constexpr (PACKED) load_ri(r_begin + 64);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (PP) {
    // Ping-pong schedule (see conv_gemm_big64_kernel): the two wave groups are the two 128-row halves
    // of the dW tile (one wave of each per SIMD), 4 phases per 64-row step, one 64 (n) x 32 (k)
    // quadrant of the wave's 128 x 64 each; group 1 runs one barrier behind group 0.  Step st+1 is
    // DMA'd in phases 0 (dY) / 1 (X, then the rinfo rows of step st+2) of step st and retired before
    // the barrier that ends phase 3; the bias column sums read the dY image in the (otherwise
    // empty) phase-3 read slot.
    if constexpr (PACKED) {  // retired by the vmcnt(0) above (see the end of the step loop)
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(ri_nxt[i].x), "+v"(ri_nxt[i].y));
    }
    pp_barrier();
    if (wn == 1) pp_barrier();
    const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    short8 fa[2][4], fb0[2][2], fb1[2][2];
    auto mma = [&](short8 (&a)[2][4], short8 (&b)[2][2], int i0, int j0) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][i], b[kk][j], acc[i0 + i][j0 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    // per-lane fragment bases (stage 0, k-half 0): dY columns of the wave's 8 16-col blocks, X columns of
    // its 4; the +4-row half (2 KiB), the k-half (16 KiB) and the stage (32 KiB) are DS immediates
    unsigned fab[8], fbb[4];
    {
      const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)smem;
#pragma unroll
      for (int i = 0; i < 8; ++i) fab[i] = lds0 + swz_tr512(grp * 8 + q, (wn * 128 + i * 16) / 4 + p);
#pragma unroll
      for (int j = 0; j < 4; ++j) fbb[j] = lds0 + 65536 + swz_tr512(grp * 8 + q, (wk * 64 + j * 16) / 4 + p);
    }
    auto rd = [&](unsigned base, auto offc) {
      constexpr int O = decltype(offc)::value;
      const short4v v0 = ds_read_tr_off<O>(base);
      const short4v v1 = ds_read_tr_off<O + 2048>(base);
      return (short8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 16384>;
    using I2 = std::integral_constant<int, 32768>;
    using I3 = std::integral_constant<int, 32768 + 16384>;
    auto step = [&](int st, auto bufc) {
      constexpr int buf = decltype(bufc)::value;
      using K0 = std::conditional_t<buf == 0, I0, I2>;  // k-half 0 / 1 of this stage
      using K1 = std::conditional_t<buf == 0, I1, I3>;
      const char* Ys = smem + buf * 32768;
      const bool more = st + 1 < nsteps;
      // phase 0: n rows 0-63 of the wave's half, k columns 0-31
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        fb0[0][j] = rd(fbb[j], K0{});
        fb0[1][j] = rd(fbb[j], K1{});
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[0][i] = rd(fab[i], K0{});
        fa[1][i] = rd(fab[i], K1{});
      }
      if (more) stage_y(r_begin + (st + 1) * 64, buf ^ 1);
      pp_barrier();
      lgkm_tie(fa);
      lgkm_tie(fb0);
      mma(fa, fb0, 0, 0);
      pp_barrier();
      // phase 1: n rows 0-63, k columns 32-63
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        fb1[0][j] = rd(fbb[2 + j], K0{});
        fb1[1][j] = rd(fbb[2 + j], K1{});
      }
      if (more) {
        stage_x(r_begin + (st + 1) * 64, buf ^ 1);
        if constexpr (PACKED) load_ri(r_begin + (st + 2) * 64);
      }
      pp_barrier();
      lgkm_tie(fb1);
      mma(fa, fb1, 0, 2);
      pp_barrier();
      // phase 2: n rows 64-127, k columns 32-63
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[0][i] = rd(fab[4 + i], K0{});
        fa[1][i] = rd(fab[4 + i], K1{});
      }
      pp_barrier();
      lgkm_tie(fa);
      mma(fa, fb1, 4, 2);
      pp_barrier();
      // phase 3: n rows 64-127, k columns 0-31 (fragments in registers); bias sums in the read slot
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = (tid >> 5) + 16 * j;
          const int f = ((row & 3) | (((row >> 3) & 1) << 2)) << 2;
          const short8 v = *reinterpret_cast<const short8*>(Ys + row * 512 + ((bc16 ^ (f >> 1)) << 4));
#pragma unroll
          for (int t = 0; t < 8; ++t) bsum[t] += bf2f((bf16_t)v[t]);
        }
      }
      if (wn == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      pp_barrier();
      mma(fa, fb0, 4, 0);
      if (wn == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      pp_barrier();
      if constexpr (PACKED) {
        // the rinfo rows of step st+2 are retired by the vmcnt(0) above; re-define them through an
        // empty asm so the compiler's waitcnt pass (which cannot see that wait) does not make the
        // next step's X stage wait for the dY DMA issued just before it
        int2* rn = ri_nxt;  // (named here: an asm operand alone does not capture it in the generic lambda)
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(rn[i].x), "+v"(rn[i].y));
      }
    };
    // two steps per iteration: the stage buffer is a compile-time immediate in each body
    for (int st = 0; st < nsteps; st += 2) {
      step(st, std::integral_constant<int, 0>{});
      if (st + 1 < nsteps) step(st + 1, std::integral_constant<int, 1>{});
    }
    if (wn == 0) pp_barrier();
  } else {
  __builtin_amdgcn_s_barrier();
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  typedef short v4s __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  const __attribute__((address_space(3))) char* lds0 = (const __attribute__((address_space(3))) char*)smem;
  int fa_off[8], fb_off[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) fa_off[i] = swz_tr512(grp * 8 + q, (wn * 128 + i * 16) / 4 + p);
#pragma unroll
  for (int j = 0; j < 4; ++j) fb_off[j] = 65536 + swz_tr512(grp * 8 + q, (wk * 64 + j * 16) / 4 + p);
  auto tr = [&](int off) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(lds0 + off)); };
  auto step = [&](int st, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    if (st + 1 < nsteps) {
      stage(r_begin + (st + 1) * 64, buf ^ 1);
      if constexpr (PACKED) load_ri(r_begin + (st + 2) * 64);
    }
    if (do_bias) {
      const char* Ys = smem + buf * 32768;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (tid >> 5) + 16 * j;
        const int f = ((row & 3) | (((row >> 3) & 1) << 2)) << 2;
        const short8 v = *reinterpret_cast<const short8*>(Ys + row * 512 + ((bc16 ^ (f >> 1)) << 4));
#pragma unroll
        for (int t = 0; t < 8; ++t) bsum[t] += bf2f((bf16_t)v[t]);
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int imm = buf * 32768 + kk * 16384;  // compile-time after unrolling
      short8 fa[8], fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const short4v b0 = tr(fb_off[j] + imm), b1 = tr(fb_off[j] + imm + 2048);
        fb[j] = (short8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const short4v a0 = tr(fa_off[i] + imm), a1 = tr(fa_off[i] + imm + 2048);
        fa[i] = (short8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  if constexpr (IMM) {
    // two steps per iteration: the stage index is a compile-time constant in each body
    for (int st = 0; st < nsteps; st += 2) {
      step(st, std::integral_constant<int, 0>{});
      if (st + 1 < nsteps) step(st + 1, std::integral_constant<int, 1>{});
    }
  } else {  // all 24 fragment reads of a k-half issued, one wait, 32 MFMAs
    // fragment reads from per-block base registers + DS immediates (+4 rows, k-half, stage buffer), the
    // loop unrolled over the two stage buffers (as in the ping-pong loop: no v_add per read)
    unsigned fab[8], fbb[4];
    {
      const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)smem;
#pragma unroll
      for (int i = 0; i < 8; ++i) fab[i] = lds0 + swz_tr512(grp * 8 + q, (wn * 128 + i * 16) / 4 + p);
#pragma unroll
      for (int j = 0; j < 4; ++j) fbb[j] = lds0 + 65536 + swz_tr512(grp * 8 + q, (wk * 64 + j * 16) / 4 + p);
    }
    auto rd = [&](unsigned base, auto offc) {
      constexpr int O = decltype(offc)::value;
      const short4v v0 = ds_read_tr_off<O>(base);
      const short4v v1 = ds_read_tr_off<O + 2048>(base);
      return (short8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    };
    auto step = [&](int st, auto bufc) {
      constexpr int buf = decltype(bufc)::value;
      if (st + 1 < nsteps) {
        stage(r_begin + (st + 1) * 64, buf ^ 1);
        if constexpr (PACKED) load_ri(r_begin + (st + 2) * 64);
      }
      const char* Ys = smem + buf * 32768;
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = (tid >> 5) + 16 * j;
          const int f = ((row & 3) | (((row >> 3) & 1) << 2)) << 2;
          const short8 v = *reinterpret_cast<const short8*>(Ys + row * 512 + ((bc16 ^ (f >> 1)) << 4));
#pragma unroll
          for (int t = 0; t < 8; ++t) bsum[t] += bf2f((bf16_t)v[t]);
        }
      }
      auto khalf = [&](auto offc) {
        short8 fa[8], fb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = rd(fbb[j], offc);
#pragma unroll
        for (int i = 0; i < 8; ++i) fa[i] = rd(fab[i], offc);
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(fa[0]), "+v"(fa[1]), "+v"(fa[2]), "+v"(fa[3]), "+v"(fa[4]), "+v"(fa[5]), "+v"(fa[6]),
                       "+v"(fa[7]), "+v"(fb[0]), "+v"(fb[1]), "+v"(fb[2]), "+v"(fb[3]));
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      };
      khalf(std::integral_constant<int, buf * 32768>{});
      khalf(std::integral_constant<int, buf * 32768 + 16384>{});
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    };
    for (int st = 0; st < nsteps; st += 2) {
      step(st, std::integral_constant<int, 0>{});
      if (st + 1 < nsteps) step(st + 1, std::integral_constant<int, 1>{});
    }
  }
  }
  if (do_bias) {
    float* red = reinterpret_cast<float*>(smem);  // [16][256]
#pragma unroll
    for (int t = 0; t < 8; ++t) red[(tid >> 5) * 256 + bc16 * 8 + t] = bsum[t];
    __syncthreads();
    if (tid < 256 && n0 + tid < g.N) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) t += red[j * 256 + tid];
      bias_slabs[(long)split * g.N + n0 + tid] = t;
    }
  }
  float* S = slabs + (long)split * g.N * g.K;
  if ((g.K & 3) == 0) {
    // slab tile through LDS in two 128-row halves (rows padded to 1088 B: the 2 rows x 16 k of a
    // ds_write_b32 half-wave land on distinct banks): float4 stores of whole 1-KiB rows instead of
    // 64-B pieces.  The stage buffers and the cu table are dead after the main loop.
    constexpr int RSF = 1088;
    char* Ct = smem;
    // barriers between the halves order LDS only: __syncthreads would also drain the first half's
    // 128 KiB of slab stores (vmcnt counts stores) before the second half could be staged
    auto lds_barrier = [] {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (half == 0) __syncthreads();
      else lds_barrier();
      if (wn == half) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int nl = i * 16 + (lane >> 4) * 4 + r;
              const int kl = wk * 64 + j * 16 + (lane & 15);
              *reinterpret_cast<float*>(Ct + nl * RSF + kl * 4) = acc[i][j][r];
            }
      }
      lds_barrier();
      for (int e = tid; e < 128 * 64; e += NT3) {
        const int nl = e >> 6, c4 = e & 63;
        const int n = n0 + half * 128 + nl, k = k0 + c4 * 4;
        if (n < g.N && k < g.K)
          *reinterpret_cast<float4*>(S + (long)n * g.K + k) = *reinterpret_cast<const float4*>(Ct + nl * RSF + c4 * 16);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 128 + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wk * 64 + j * 16 + (lane & 15);
        if (n < g.N && k < g.K) S[(long)n * g.K + k] = acc[i][j][r];
      }
}

// Register-staged variant (faster at large K = ks*Cin; the LDS-DMA one wins at K <= 1024).
template <bool PACKED>
__global__ void __launch_bounds__(NT, 2) conv_wgrad_reg_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                                                           float* __restrict__ slabs, float* __restrict__ bias_slabs,
                                                           ConvGeom g, int rows_per_split) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nN = (g.N + 127) / 128;  // cout tiles
  const int nK = (g.K + 127) / 128;  // k tiles
  const int tile = blockIdx.x % (nN * nK);
  const int split = blockIdx.x / (nN * nK);
  const int tn = tile / nK, tk = tile % nK;
  const int n0 = tn * 128, k0 = tk * 128;
  const int r_begin = split * rows_per_split;
  const int r_end = min(g.M, r_begin + rows_per_split);
  // wave index as a scalar: LDS-DMA destinations (M0) and per-wave offsets stay in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 1, wk = wave & 1;
  const float invCin = 1.f / (float)g.Cin;

  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};

  // staging: each operand tile = 64 rows x 128 cols bf16 = 1024 x 16-B chunks; 4 per thread
  // chunk e = tid + 256*i: row = e / 16, c16 = e % 16 (16-B chunk = two 8-B chunks)
  const int c16 = tid & 15;
  const int k_ld = k0 + c16 * 8;
  int tap = 0, cin = 0;
  const bool k_ok = k_ld < g.K;
  if (k_ok) {
    tap = (int)(((float)k_ld + 0.5f) * invCin);
    cin = k_ld - tap * g.Cin;
  }
  const int n_ld = n0 + c16 * 8;
  short8 rx[4], ry[4];
  int tcur[4];
  const int xshift = tap * g.dil - g.pad;
  // packed rows: (position, length) of the rows of the NEXT gload, prefetched one step ahead so
  // the table read never sits in front of the operand loads
  int2 rnext[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = r_begin + (tid >> 4) + 16 * i;
    if constexpr (PACKED) rnext[i] = g.rinfo[min(m, g.M - 1)];
    else tcur[i] = m % g.L;
  }
  auto gload = [&](int r0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + (tid >> 4) + 16 * i;
      short8 vx = {0, 0, 0, 0, 0, 0, 0, 0}, vy = {0, 0, 0, 0, 0, 0, 0, 0};
      int ts, lim;
      if constexpr (PACKED) {  // clamped, branch-free prefetch of the next step's row table
        ts = rnext[i].x + xshift;
        lim = rnext[i].y;
        rnext[i] = g.rinfo[min(m + RB, g.M - 1)];
      } else {
        ts = tcur[i] + xshift;
        lim = g.L;
      }
      if (m < r_end) {
        if (n_ld < g.N) vy = *reinterpret_cast<const short8*>(dY + (long)m * g.N + n_ld);
        if (k_ok && ts >= 0 && ts < lim) vx = *reinterpret_cast<const short8*>(X + (long)(m + xshift) * g.Cin + cin);
      }
      rx[i] = vx;
      ry[i] = vy;
      if constexpr (!PACKED) {
        int t = tcur[i] + RB;
        while (t >= g.L) t -= g.L;
        tcur[i] = t;
      }
    }
  };
  // bias gradient (column sums of dY) rides on the staging registers of the k-tile-0 blocks
  const bool do_bias = bias_slabs != nullptr && tk == 0;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto bias_acc = [&]() {
    if (!do_bias) return;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) bsum[q] += bf2f((bf16_t)ry[i][q]);
  };
  auto lstore = [&](int buf) {
    char* Ys = smem + buf * (2 * RB * 256);
    char* Xs = Ys + RB * 256;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 4) + 16 * i;
      *reinterpret_cast<short8*>(Ys + swz_tr(row, c16 * 2)) = ry[i];
      *reinterpret_cast<short8*>(Xs + swz_tr(row, c16 * 2)) = rx[i];
    }
  };

  const int nsteps = (r_end - r_begin + RB - 1) / RB;
  if (nsteps > 0) {
    gload(r_begin);
    bias_acc();
    lstore(0);
  }
  __syncthreads();
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) {
      gload(r_begin + (s + 1) * RB);
      bias_acc();
    }
    const char* Ys = smem + buf * (2 * RB * 256);
    const char* Xs = Ys + RB * 256;
#pragma unroll
    for (int kk = 0; kk < RB / 32; ++kk) {
      short8 fa[4], fb[4];
      const int rbase = kk * 32 + grp * 8 + q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ca = (wn * 64 + i * 16) / 4 + p;  // 8-B chunk of the A (dY) column block
        const int cb = (wk * 64 + i * 16) / 4 + p;
        short4v a0 = ds_read_tr(Ys + swz_tr(rbase, ca));
        short4v a1 = ds_read_tr(Ys + swz_tr(rbase + 4, ca));
        short4v b0 = ds_read_tr(Xs + swz_tr(rbase, cb));
        short4v b1 = ds_read_tr(Xs + swz_tr(rbase + 4, cb));
        fa[i] = (short8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        fb[i] = (short8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nsteps) lstore(buf ^ 1);
    __syncthreads();
  }
  if (do_bias) {  // reduce the 16 row-groups that share a column chunk, one partial per split
    float* red = reinterpret_cast<float*>(smem);  // [16][128]
#pragma unroll
    for (int q = 0; q < 8; ++q) red[(tid >> 4) * 128 + c16 * 8 + q] = bsum[q];
    __syncthreads();
    if (tid < 128 && n0 + tid < g.N) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) t += red[j * 128 + tid];
      bias_slabs[(long)split * g.N + n0 + tid] = t;
    }
  }
  // partial slab [split][N][K] fp32
  float* S = slabs + (long)split * g.N * g.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wk * 64 + j * 16 + (lane & 15);
        if (n < g.N && k < g.K) S[(long)n * g.K + k] = acc[i][j][r];
      }
}

// Skinny-M implicit-GEMM conv (M <= g_skinny_maxm = 1024 rows: a batch-1 utterance's phonemes and frames, the first
// vocoder stages, per-utterance style vectors): the tile machinery above pays a 256-row prologue / epilogue for a
// handful of rows and leaves most CUs idle.  Here a block of NWV waves owns a 16-row x 16-column output tile and
// splits the k-steps (32 deep) over its waves, operands straight from global memory in the MFMA fragment layout
// (no LDS staging: the A rows are a few KiB, every weight fragment is read once per row block), the partial tiles
// summed in LDS in a fixed order, then the conv_gemm epilogue (bias, activation, ReLU-aux mask, residual, row
// validity, fp32 out, EpiX tail).  Grid = N/16 x M/16 blocks.  (A 32 x 64 tile per block -- fewer fragment loads
// per MFMA -- measured slower: fewer blocks; profiles/r6_b1_latency.txt.)
// Cin % 32 == 0: a k-step never straddles a tap; otherwise (Cin % 8 == 0) each lane finds the tap of its 8-channel
// chunk and K is padded to the k-step with zeros.  N % 16 == 0.  A ConvTranspose 3-tap form (ksplit) is
// computed in full: its zero tap adds exact zeros, so the result is bitwise the same with or without the skip.
template <int NWV, bool AL = true>  // AL: Cin % 32 == 0 (k-steps never straddle a tap); else per-lane taps, K padded
__global__ void __launch_bounds__(64 * NWV) skinny_gemm_kernel(const bf16_t* __restrict__ X,
                                                               const bf16_t* __restrict__ W,
                                                               const float* __restrict__ bias,
                                                               const bf16_t* __restrict__ aux,
                                                               const bf16_t* __restrict__ resid,
                                                               const int64_t* __restrict__ lens, void* Y, int out_f32,
                                                               ConvGeom g, int act, int ldy, EpiX ex) {
  __shared__ float red[NWV][64][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * 16;
  const int r = m0 + (lane & 15), ks8 = 8 * (lane >> 4);
  const int K = g.K, nk = AL ? K / 32 : (K + 31) / 32;
  int2 rp = make_int2(0, 0);
  if (r < g.M) rp = row_pos(g, r);
  const bf16_t* wrow = W + (long)(n0 + (lane & 15)) * K + ks8;
  float4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int st = wave; st < nk; st += NWV) {
    const int k0 = st * 32;
    short8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (AL) {
      const int tap = k0 / g.Cin, c0 = k0 - tap * g.Cin;
      const int sp = rp.x + tap * g.dil - g.pad;  // source position in the row's sequence
      if (r < g.M && sp >= 0 && sp < rp.y)
        a = *reinterpret_cast<const short8*>(X + (long)(r + sp - rp.x) * g.Cin + c0 + ks8);
      b = *reinterpret_cast<const short8*>(wrow + k0);
    } else {  // Cin % 8 == 0: the lane's 8-channel chunk lies within one tap; chunks past K are zero
      const int k = k0 + ks8;
      if (k < K) {
        const int tap = k / g.Cin, c = k - tap * g.Cin;
        const int sp = rp.x + tap * g.dil - g.pad;
        if (r < g.M && sp >= 0 && sp < rp.y)
          a = *reinterpret_cast<const short8*>(X + (long)(r + sp - rp.x) * g.Cin + c);
        b = *reinterpret_cast<const short8*>(wrow + k0);
      }
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][lane][i] = acc[i];
  __syncthreads();
  if (tid >= 256) return;
  // thread t: output (row 4 * (t >> 6) + (t & 3), col (t >> 2) & 15) -- i.e. lane L = (t >> 2) & 15 | (t >> 6) << 4
  const int L = ((tid >> 2) & 15) | ((tid >> 6) << 4), i = tid & 3;
  const int m = m0 + 4 * (L >> 4) + i, n = n0 + (L & 15);
  if (m >= g.M) return;
  float v = 0.f;
#pragma unroll
  for (int w = 0; w < NWV; ++w) v += red[w][L][i];
  if (bias) v += bias[n];
  if (act == ACT_RELU) v = fmaxf(v, 0.f);
  else if (act == ACT_LRELU) v = v > 0.f ? v : 0.1f * v;
  else if (act == ACT_TANH) v = tanhf(v);
  const long off = (long)m * ldy + n;
  if (aux) v = bf2f(aux[off]) > 0.f ? v : 0.f;
  if (resid) v += bf2f(resid[off]);
  bool valid = true;
  if (lens) {
    const int bb = m / g.L;
    valid = m - bb * g.L < (int)lens[bb];
  }
  if (!valid) v = 0.f;
  if (out_f32) {
    reinterpret_cast<float*>(Y)[off] = v;
    return;
  }
  if (ex.acc) v += bf2f(ex.acc[off]);
  v = valid ? v * ex.scale : 0.f;
  if (ex.y2) ex.y2[off] = f2bf(v > 0.f ? v : 0.1f * v);
  if (ex.post_act == ACT_LRELU) v = v > 0.f ? v : 0.1f * v;
  reinterpret_cast<bf16_t*>(Y)[off] = f2bf(v);
}

// Split-K finish: out[m][n] = epilogue( sum_s P[s][m][n] ) in a fixed slice order, with the
// epi_store4 semantics (bias, activation, ReLU-aux mask, residual, row validity) and, for bf16 output, the
// big64 EpiX tail (accumulate, scale, leaky-ReLU copy y2, post activation).  8 columns per thread (two
// float4 per slice).
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ P, int S, long M, int N,
                                                            const float* __restrict__ bias,
                                                            const bf16_t* __restrict__ aux,
                                                            const bf16_t* __restrict__ resid,
                                                            const int64_t* __restrict__ lens, int L, int act,
                                                            int out_f32, void* Y,
                                                            const bf16_t* xacc, bf16_t* y2,
                                                            float scale, int post_act) {
  const int n8 = N >> 3;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= M * n8) return;
  const long m = e / n8;
  const int n = (int)(e - m * n8) * 8;
  const long off = m * N + n;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int sl = 0; sl < S; ++sl) {
    const float4* p = reinterpret_cast<const float4*>(P + (long)sl * M * N + off);
    const float4 a = p[0], b = p[1];
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (bias) v[q] += bias[n + q];
    if (act == ACT_RELU) v[q] = fmaxf(v[q], 0.f);
    else if (act == ACT_LRELU) v[q] = v[q] > 0.f ? v[q] : 0.1f * v[q];
    else if (act == ACT_TANH) v[q] = tanhf(v[q]);
  }
  if (aux) {
    const short8 x = *reinterpret_cast<const short8*>(aux + off);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = bf2f((bf16_t)x[q]) > 0.f ? v[q] : 0.f;
  }
  if (resid) {
    const short8 x = *reinterpret_cast<const short8*>(resid + off);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += bf2f((bf16_t)x[q]);
  }
  bool valid = true;
  if (lens) {
    const long b = m / L;
    valid = m - b * L < lens[b];
    if (!valid) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = 0.f;
    }
  }
  if (out_f32) {
    float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(Y) + off);
    o[0] = make_float4(v[0], v[1], v[2], v[3]);
    o[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    if (xacc) {
      const short8 x = *reinterpret_cast<const short8*>(xacc + off);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += bf2f((bf16_t)x[q]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = valid ? v[q] * scale : 0.f;
    if (y2) {
      short8 o2;
#pragma unroll
      for (int q = 0; q < 8; ++q) o2[q] = (short)f2bf(v[q] > 0.f ? v[q] : 0.1f * v[q]);
      *reinterpret_cast<short8*>(y2 + off) = o2;
    }
    if (post_act == ACT_LRELU) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = v[q] > 0.f ? v[q] : 0.1f * v[q];
    }
    short8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (short)f2bf(v[q]);
    *reinterpret_cast<short8*>(reinterpret_cast<bf16_t*>(Y) + off) = o;
  }
}

// Split-parallel slab reduction: block = 64 float4 columns x 4 split lanes; lane l sums the slabs
// l, l+4, ... (4 independent float4 loads in flight per thread, every block of the grid busy even
// for a single 256x256 weight), the 4 lane sums are combined in LDS in a fixed order -> the same
// bits on every run.  Blocks past the dW part reduce the bias slabs the same way.
__global__ void __launch_bounds__(256) wgrad_reduce4_kernel(const float* __restrict__ slabs, float* __restrict__ dW,
                                                            const float* __restrict__ bslabs, float* __restrict__ db,
                                                            int splits, int N, int Cin, int ks, int nb_main) {
  __shared__ float4 red[4][64];
  const long K = (long)Cin * ks;
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const bool bias_blk = (int)blockIdx.x >= nb_main;
  const long stride = bias_blk ? (long)N : (long)N * K;   // floats between consecutive slabs
  const long ncol4 = bias_blk ? (N + 3) / 4 : (long)N * K / 4;
  const long c4 = (long)(bias_blk ? blockIdx.x - nb_main : blockIdx.x) * 64 + cl;
  const float* base = bias_blk ? bslabs : slabs;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 < ncol4) {
    if (bias_blk && (N & 3)) {  // scalar tail-safe bias path (N % 4 != 0)
      for (int q = 0; q < 4; ++q) {
        const long n = c4 * 4 + q;
        if (n >= N) break;
        float t = 0.f;
        for (int sp = sl; sp < splits; sp += 4) t += base[(long)sp * stride + n];
        (&acc.x)[q] = t;
      }
    } else {
#pragma unroll 4
      for (int sp = sl; sp < splits; sp += 4) {
        const float4 v = reinterpret_cast<const float4*>(base + (long)sp * stride)[c4];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
  }
  red[sl][cl] = acc;
  __syncthreads();
  if (sl != 0 || c4 >= ncol4) return;
  const float4 a = red[0][cl], b = red[1][cl], c = red[2][cl], d = red[3][cl];
  const float4 t = make_float4((a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y), (a.z + b.z) + (c.z + d.z),
                               (a.w + b.w) + (c.w + d.w));
  if (bias_blk) {
    for (int q = 0; q < 4; ++q)
      if (c4 * 4 + q < N) db[c4 * 4 + q] = (&t.x)[q];
    return;
  }
  const long e = c4 * 4;
  const long n = e / K;
  const int k = (int)(e - n * K);
  const int tap = k / Cin, cin = k - tap * Cin;  // the 4 k share a tap (Cin % 4 == 0)
  if (ks == 1) {  // scalar stores: dW may be an arena slot without 16-B alignment
    float* dst = dW + n * Cin + cin;
    dst[0] = t.x;
    dst[1] = t.y;
    dst[2] = t.z;
    dst[3] = t.w;
  } else {
    float* dst = dW + (n * Cin + cin) * ks + tap;
    dst[0] = t.x;
    dst[ks] = t.y;
    dst[2 * ks] = t.z;
    dst[3 * ks] = t.w;
  }
}

// ks > 1: one block per output row n; slab row read coalesced (float4 over k = tap*Cin + cin),
// summed over splits, transposed through LDS to the [cin][tap] order of dW, written contiguously.
__global__ void __launch_bounds__(256) wgrad_reduce_rows_kernel(const float* __restrict__ slabs,
                                                                float* __restrict__ dW,
                                                                const float* __restrict__ bslabs,
                                                                float* __restrict__ db, int splits, int N, int Cin,
                                                                int ks) {
  extern __shared__ float row[];
  const int n = blockIdx.x;
  const int K = Cin * ks;
  const long total = (long)N * K;
  const float* src = slabs + (long)n * K;
  for (int k4 = threadIdx.x; k4 < K / 4; k4 += 256) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int sp = 0; sp < splits; ++sp) {
      const float4 v = reinterpret_cast<const float4*>(src + (long)sp * total)[k4];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    const int k = k4 * 4;
    const int tap = k / Cin, cin = k - tap * Cin;  // the 4 k share a tap (Cin % 4 == 0)
    row[(cin + 0) * ks + tap] = acc.x;
    row[(cin + 1) * ks + tap] = acc.y;
    row[(cin + 2) * ks + tap] = acc.z;
    row[(cin + 3) * ks + tap] = acc.w;
  }
  if (bslabs && threadIdx.x == 0) {
    float sb = 0.f;
    for (int sp = 0; sp < splits; ++sp) sb += bslabs[(long)sp * N + n];
    db[n] = sb;
  }
  __syncthreads();
  float* dst = dW + (long)n * K;
  for (int k = threadIdx.x; k < K; k += 256) dst[k] = row[k];
}

// db[n] = sum_m dY[m, n]: per row-chunk partials part[chunk][n], finished by a fixed-order column
// sum (k_reduce.hip) -- deterministic
__global__ void __launch_bounds__(256) colsum_kernel(const bf16_t* __restrict__ dY, float* __restrict__ part, long M,
                                                     int N, int rows_per_block) {
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min(M, r0 + rows_per_block);
  for (int n = blockIdx.x * 256 + threadIdx.x; n < N; n += gridDim.x * 256) {
    float s = 0.f;
    for (long r = r0; r < r1; ++r) s += bf2f(dY[r * N + n]);
    part[(long)blockIdx.y * N + n] = s;
  }
}

}  // namespace

static bool g_force_lds_epilogue = false;
static int g_gemm_variant = -1;  // -1 auto, 0: register staging, 1: LDS-DMA 128x128, 2: LDS-DMA 3-stage ring 256x128
// s_setprio 1 for waves 4-7 of the 8-wave big64 blocks (MI355X_MICROARCH "static priority for the
// younger half"), measured per kernel (tools/exp_prio.py): weight gradients on packed rows -2..-4 %,
// others neutral -> on for wgrad; forward mixed (k9 N = 1024 fwd -4 %, k9 N = 256 dgrad +8 %) -> on for
// N >= 1024 convs only
static int g_gemm_prio = -1, g_wgrad_prio = 1;  // forward -1: auto (on for wide k > 1 convs only)
SSAMD_API void ssamd_gemm_set_prio(int v) { g_gemm_prio = v; }
static int g_gemm_ngrp = 1;  // 256x256 tile order: N-tile groups (tile_of); experiment knob
SSAMD_API void ssamd_gemm_set_ngrp(int v) { g_gemm_ngrp = v; }
SSAMD_API void ssamd_wgrad_set_prio(int v) { g_wgrad_prio = v; }
static int g_splitk = -1;        // -1 auto, 0 off, S > 1 forced slices (big64 split-K + reduce)
static int g_ring_maxk = 0, g_ring_maxn = 256;  // 0: the 256x128 ring only for <= 64 big tiles (A/B knob)
static int g_splitk_tiny = 3;    // min k-steps per slice for <= 8 tiles (0: the general rule only)
static int g_skinny = 1;         // skinny_gemm_kernel for M <= g_skinny_maxm rows (0: off, A/B)
// 8-wave skinny blocks from this many k-steps (0: always 4 waves).  Batch 1: 4 waves 1.674 / 1.676 ms, 8 from 16
// steps 1.625 / 1.624 / 1.605, from 8 steps 1.613 / 1.618; 16 waves from 32 or 64 steps no better (r6_b1_latency.txt)
static int g_skinny_w8 = 16;
static int g_skinny_maxm = 1024;
static int g_skinny_any_cin = 1;  // the skinny kernel also for Cin % 32 != 0 (per-lane taps; 0: tile kernels, A/B)  // measured at batch 1: 64 -> 2.19 ms, 128 -> 1.80, 1024 -> 1.76 (r6_b1_latency.txt)
static int g_num_cus_gemm = 256;
// Split-K fp32 partials: one workspace per (device, stream).  A process-global buffer would hand a
// foreign-device pointer to a second GPU and let GEMMs on two streams race on the same partials.
struct SplitKWs { int dev; hipStream_t s; void* p; size_t bytes; };
static SplitKWs g_splitk_ws[32];
static int g_splitk_nws = 0;
static std::mutex g_splitk_mu;
// Workspace of >= need bytes for (current device, s), or nullptr.  Sized once to 64 MiB (S * tiles <=
// 256 CUs bounds every split-K workspace by 256 tiles x 256 KiB): a regrow would hipFree, a device-wide
// synchronisation in the middle of a training step.
static bool g_ws_retain = false;
static hipStreamCaptureStatus g_cap_status;
SSAMD_API void ssamd_gemm_retain_workspaces(int v) { g_ws_retain = v != 0; }

static void* splitk_workspace(hipStream_t s, size_t need) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_splitk_mu);
  SplitKWs* e = nullptr;
  for (int i = 0; i < g_splitk_nws; ++i)
    if (g_splitk_ws[i].dev == dev && g_splitk_ws[i].s == s) e = &g_splitk_ws[i];
  if (!e) {
    if (g_splitk_nws == 32) return nullptr;
    e = &g_splitk_ws[g_splitk_nws++];
    *e = SplitKWs{dev, s, nullptr, 0};
  }
  if (need > e->bytes) {
    const size_t want = need > ((size_t)64 << 20) ? need : ((size_t)64 << 20);
    // a captured HIP graph holds the old address: once graphs exist (ssamd_gemm_retain_workspaces) the old buffer
    // is kept (leaked) instead of freed; during a capture no allocation is legal at all (-4: warm the shape first)
    if (g_ws_retain) {
      if (hipStreamIsCapturing(s, &g_cap_status) == hipSuccess && g_cap_status != hipStreamCaptureStatusNone)
        return nullptr;
    } else if (e->p) {
      (void)hipFree(e->p);
    }
    e->p = nullptr;
    e->bytes = 0;
    if (hipMalloc(&e->p, want) != hipSuccess) return nullptr;
    e->bytes = want;
  }
  return e->p;
}
SSAMD_API void ssamd_gemm_set_splitk(int v) { g_splitk = v; }
SSAMD_API void ssamd_gemm_set_splitk_tiny(int v) { g_splitk_tiny = v; }
SSAMD_API void ssamd_gemm_set_ring_maxk(int v) { g_ring_maxk = v; }
SSAMD_API void ssamd_gemm_set_skinny(int v) { g_skinny = v; }
SSAMD_API void ssamd_gemm_set_skinny_maxm(int v) { g_skinny_maxm = v; }
SSAMD_API void ssamd_gemm_set_skinny_w8(int v) { g_skinny_w8 = v; }
SSAMD_API void ssamd_gemm_set_skinny_any_cin(int v) { g_skinny_any_cin = v; }
SSAMD_API void ssamd_gemm_set_ring_maxn(int v) { g_ring_maxn = v; }

SSAMD_API void ssamd_gemm_set_epilogue(int lds_staged) { g_force_lds_epilogue = lds_staged != 0; }
SSAMD_API void ssamd_gemm_set_variant(int v) { g_gemm_variant = v; }

static int g_gemm_buf = 1;  // big64 (FASTK) LDS-DMA through buffer descriptors (0: flat global_load_lds)
SSAMD_API void ssamd_gemm_set_buf(int v) { g_gemm_buf = v; }
// big64 buffer-descriptor path: 1 = the staggered 8-phase main loop for K >= 512 (tools/exp_stg.py: +5 % on
// the k9 convs and K = 1024, +2 % PostNet k5, -1..4 % at K = 256 where the prologue / epilogue dominate)
static int g_gemm_stg = 1;
static int g_gemm_mask_pre = 1;  // EPI_MASK for the ReLU-mask data gradient (0: the generic epilogue, A/B)
static int g_gemm_bnh_stg = 1;   // the BatchNorm-backward-head data gradient on the staggered main loop (0: A/B)
SSAMD_API void ssamd_gemm_set_bnh_stg(int v) { g_gemm_bnh_stg = v; }
SSAMD_API void ssamd_gemm_set_mask_pre(int v) { g_gemm_mask_pre = v; }
SSAMD_API void ssamd_gemm_set_stg(int v) { g_gemm_stg = v; }

// every byte offset of the descriptors must stay below the out-of-range marker 0x80000000
static bool big64_buf_ok(const ConvGeom& g) {
  return g_gemm_buf != 0 && (long)(g.M + g.pad) * g.Cin * 2 < (1L << 31) && (long)g.N * g.K * 2 + 512 < (1L << 31);
}

static ConvGeom make_geom(int B, int L, int Cin, int ks, int dil, int pad, int N) {
  ConvGeom g;
  g.B = B; g.L = L; g.Cin = Cin; g.ks = ks; g.dil = dil; g.pad = pad;
  g.M = B * L; g.N = N; g.K = ks * Cin;
  g.rinfo = nullptr;
  g.cu = nullptr;
  g.nseq = 0;
  g.ksplit = 0;
  g.prio = g_gemm_prio < 0 ? (N >= 1024 && ks > 1) : g_gemm_prio;
  const int nN = (N + 255) / 256;
  g.ngrp = (g_gemm_ngrp > 1 && nN % g_gemm_ngrp == 0) ? g_gemm_ngrp : 1;
  return g;
}

static int conv_gemm_impl(const bf16_t* X, const bf16_t* W, const float* bias, const bf16_t* aux,
                          const bf16_t* resid, const int64_t* lens, void* Y, int out_f32, int B, int L, int Cin,
                          int ks, int dil, int pad, int N, int act, int ldy, const int* rinfo, EpiX ex, hipStream_t s,
                          bool bnh = false, int ksplit = 0) {
  if (Cin % 8 != 0) return -2;
  if ((long)B * L == 0 || N == 0) return 0;
  ConvGeom g = make_geom(B, L, Cin, ks, dil, pad, N);
  g.rinfo = reinterpret_cast<const int2*>(rinfo);
  if (ksplit > 0 && ks == 3 && Cin % 64 == 0 && ksplit % 256 == 0 && ksplit < N) g.ksplit = ksplit;
  const int nwg = ((g.M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const size_t lds = (size_t)BM * CSTRIDE * 4;  // >= 2 stages x (A+B) = 64 KiB
  static bool lds_set = false;
  if (!lds_set) {
    allow_lds(conv_gemm_kernel<true, false>, lds);
    allow_lds(conv_gemm_kernel<false, false>, lds);
    lds_set = true;
  }
  // register epilogue needs N % 4 == 0 and an 8-B aligned ldy; LDS-staged epilogue otherwise
  const bool reg = (N % 4 == 0) && (ldy % 4 == 0) && !g_force_lds_epilogue;
  const size_t lds_reg = (size_t)2 * 2 * BM * BK * 2;
  int variant = g_gemm_variant;
  // measured on MI355X (tools/bench_kernels.py): the 256x256 tile with a BK=64 double buffer wins for
  // every N >= 256 shape (+3..15 % over the 256x128 ring, +4..8 % over 256x256 with a BK=32 4-stage ring);
  // the 256x128 ring for narrower N when K-slabs are tap-aligned, LDS-DMA 128x128 otherwise
  if (variant < 0) variant = N >= 256 ? 4 : (Cin % BK == 0) ? 2 : 1;
  // Few 256x256 tiles (encoder / variance-predictor GEMMs at M = B*T ~ 5k-30k rows with N = 256): the
  // big tile leaves most of the 256 CUs idle; the 256x128 ring (or the 128x128 LDS-DMA kernel) doubles
  // (quadruples) the tile count.  Measured at M = 14k (tools/exp_small_m.py): -20..36 % time for every
  // N = 256 shape (k9 dgrad 219 -> 141 us), while N >= 768 keeps the 256x256 tile.
  if (g_gemm_variant < 0 && N >= 256 && N <= 256 && ((g.M + BG - 1) / BG) * ((N + BG - 1) / BG) <= 64)
    variant = (Cin % BK == 0) ? 2 : 1;
  // (A/B) the 256x128 ring also for short-K GEMMs with more tiles (K <= g_ring_maxk, N <= g_ring_maxn)
  if (g_gemm_variant < 0 && g_ring_maxk > 0 && N >= 256 && N <= g_ring_maxn && g.K <= g_ring_maxk &&
      Cin % BK == 0)
    variant = 2;
  // Skinny M (<= g_skinny_maxm rows): 16 x 16 output tiles, k split over the block's waves (skinny_gemm_kernel)
  if (g_skinny && g.M <= g_skinny_maxm && (Cin % 32 == 0 || g_skinny_any_cin) && N % 16 == 0 && !bnh && !ex.mask_out && !ex.mask_in &&
      act >= 0 && (ex.post_act == 0 || ex.post_act == ACT_LRELU) && (!out_f32 || !(ex.acc || ex.y2 || ex.post_act ||
      ex.scale != 1.f))) {
    const dim3 grid(N / 16, (g.M + 15) / 16);
    const bool w8 = g_skinny_w8 > 0 && g.K / 32 >= g_skinny_w8;  // long K: 8 waves split it (shorter chains)
    if (Cin % 32 == 0) {
      if (w8)
        hipLaunchKernelGGL((skinny_gemm_kernel<8, true>), grid, dim3(512), 0, s, X, W, bias, aux, resid, lens, Y,
                           out_f32, g, act, ldy, ex);
      else
        hipLaunchKernelGGL((skinny_gemm_kernel<4, true>), grid, dim3(256), 0, s, X, W, bias, aux, resid, lens, Y,
                           out_f32, g, act, ldy, ex);
    } else {  // Cin % 8 == 0 (conv_pre / PostNet conv 0 over 80 mel channels, the GST's first im2col layer)
      if (w8)
        hipLaunchKernelGGL((skinny_gemm_kernel<8, false>), grid, dim3(512), 0, s, X, W, bias, aux, resid, lens, Y,
                           out_f32, g, act, ldy, ex);
      else
        hipLaunchKernelGGL((skinny_gemm_kernel<4, false>), grid, dim3(256), 0, s, X, W, bias, aux, resid, lens, Y,
                           out_f32, g, act, ldy, ex);
    }
    return (int)hipGetLastError();
  }
  // Split-K for few 256x256 tiles with a long K (encoder-sized M, k = 9 data gradients, K = 9216):
  // S slices of the k range as extra blocks writing fp32 partials, one fixed-order reduce kernel
  // applies the epilogue.  Measured (tools/exp_splitk.py) on the tile-poor shapes only.
  {
    const int tiles = ((g.M + BG - 1) / BG) * ((N + BG - 1) / BG);
    const int nk64 = (g.K + 63) / 64;
    // the reduce applies EpiX's accumulate / scale / y2 / post activation (bf16 output, as the big64 epilogue)
    const bool xon = ex.acc || ex.y2 || ex.post_act || ex.scale != 1.f;
    const bool plain = !(ex.mask_out || ex.mask_in || bnh) && (!xon || (!out_f32 && (ex.post_act == 0 ||
                                                                                     ex.post_act == ACT_LRELU)));
    int S = 0;
    if (g_splitk > 0) S = g_splitk;
    else if (g_splitk < 0 && g_gemm_variant < 0 && tiles <= 128 && nk64 >= 16)
      // as many slices as keep the split grid within ONE wave of blocks (a second partial wave
      // costs more than it saves: M = 10800 / 43 tiles: S = 4 81 us, S = 6 111 us, unsplit 149 us)
      S = min(min(8, g_num_cus_gemm / tiles), nk64 / 6);
    // a handful of tiles at <= 1024 rows (batch-1 inference: one utterance's phonemes / frames / first vocoder
    // stages) is a serial chain of k-steps on a few CUs: shorter slices (>= g_splitk_tiny k-steps each), also
    // for the shorter K of the k = 3 convs
    if (g_splitk < 0 && g_gemm_variant < 0 && g_splitk_tiny > 0 && tiles <= 8 && g.M <= 1024 &&
        nk64 >= 2 * g_splitk_tiny)
      S = max(S, min(8, nk64 / g_splitk_tiny));
    if (S > 1 && plain && reg && N >= 256 && (N % 8) == 0 && ldy == N && act >= 0 && (ldy % 8) == 0) {
      void* ws = splitk_workspace(s, (size_t)S * g.M * N * sizeof(float));
      if (!ws) return -4;
      static bool sk_set = false;
      if (!sk_set) {
        allow_lds(conv_gemm_big64_kernel<true, true, false>, B64_LDS);
        allow_lds(conv_gemm_big64_kernel<true, false, false>, B64_LDS);
        allow_lds(conv_gemm_big64_kernel<true, true, true>, B64_LDS);
        allow_lds(conv_gemm_big64_kernel<true, false, true>, B64_LDS);
        allow_lds(conv_gemm_big64_kernel<true, true, false, true>, B64_LDS);
        allow_lds(conv_gemm_big64_kernel<true, true, true, true>, B64_LDS);
        sk_set = true;
      }
      const bool fastk = (Cin % 64) == 0;
      const bool bf = fastk && big64_buf_ok(g);
      auto kfn = g.rinfo ? (bf ? conv_gemm_big64_kernel<true, true, true, true>
                               : fastk ? conv_gemm_big64_kernel<true, true, true> : conv_gemm_big64_kernel<true, false, true>)
                         : (bf ? conv_gemm_big64_kernel<true, true, false, true>
                               : fastk ? conv_gemm_big64_kernel<true, true, false> : conv_gemm_big64_kernel<true, false, false>);
      hipLaunchKernelGGL(kfn, dim3(tiles, S), dim3(NT3), B64_LDS, s, X, W, nullptr, nullptr, nullptr, nullptr,
                         ws, g, 0, N, EpiX{});
      const long nthr = (long)g.M * (N / 8);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(cdiv(nthr, 256)), dim3(256), 0, s,
                         reinterpret_cast<const float*>(ws), S, (long)g.M, N, bias, aux, resid, lens, g.L,
                         act, out_f32, Y, ex.acc, ex.y2, ex.scale, ex.post_act);
      return (int)hipGetLastError();
    }
  }
  if (bnh) {  // BatchNorm-backward head (EpiX aliases: acc = bn_h, ln_w = stats, mean = partials): big64 only
    if (N < 256 || (N % 8) || ldy != N || out_f32 || !reg || act != 0 || ex.post_act == 2 || aux || resid || lens || !ex.acc ||
        !ex.bn_stats || !ex.bn_part || rinfo || ex.y2 || ex.mask_out || ex.mask_in)
      return -3;
    variant = 4;
  } else {
  if (ex.mask_out || ex.mask_in) {  // the bitmask lives in the big64 LDS-staged epilogue only
    if (N < 256 || (N % 8) || ldy != N || out_f32 || !reg || act < 0) return -3;
    if (ex.mask_out && act != ACT_RELU) return -3;
    variant = 4;
  }
  const bool xon = ex.acc || ex.y2 || ex.post_act || ex.scale != 1.f;
  if (xon) {  // only the big64 (LDS-staged bf16 epilogue) and ring kernels implement EpiX
    if (out_f32 || !reg || (N % 8) || (ldy % 8) || act < 0) return -3;
    if (N >= 256) variant = 4;
    else if (variant != 2) return -3;
  }
  }  // !bnh
  if (reg && variant == 4 && N >= 256) {
    static bool b64_set = false;
    if (!b64_set) {
      allow_lds(conv_gemm_big64_kernel<true, true, false>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, false>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<true, false, false>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, false, false>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<true, true, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<true, false, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, false, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<true, true, false, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, false, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<true, true, true, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, true, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, false, true, EPI_BNH>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, false, true, EPI_BNH, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, false, false, EPI_BNH>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, false, false, false, EPI_BNH>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, false, true, EPI_GEN, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, true, true, EPI_GEN, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<true, true, false, true, EPI_GEN, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<true, true, true, true, EPI_GEN, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, false, true, EPI_MASK>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, true, true, EPI_MASK>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, false, true, EPI_MASK, true>, B64_LDS);
      allow_lds(conv_gemm_big64_kernel<false, true, true, true, EPI_MASK, true>, B64_LDS);
      b64_set = true;
    }
    const int nwgb = ((g.M + BG - 1) / BG) * ((N + BG - 1) / BG);
    const bool fastk = (Cin % 64) == 0;
    const size_t LB = B64_LDS;
    // the ReLU-mask data gradient with nothing else in its epilogue: mask bytes prefetched (EPI_MASK)
    const bool mask_pre = ex.mask_in && !ex.mask_out && !bnh && !aux && !resid && !lens && !ex.acc && !ex.y2 &&
                          !ex.post_act && ex.scale == 1.f && !out_f32 && act >= 0 && ldy == N;
#define B64_LAUNCH(F32, FK)                                                                              \
    do {                                                                                                 \
      auto kfn = g.rinfo ? conv_gemm_big64_kernel<F32, FK, true, BF> : conv_gemm_big64_kernel<F32, FK, false, BF>; \
      const bool stg_ = g_gemm_stg && g.K >= 512;                                                        \
      int grid_x = nwgb;                                                                                 \
      if constexpr (!F32) {                                                                              \
        if (bnh) kfn = conv_gemm_big64_kernel<false, FK, false, BF, EPI_BNH>;                           \
      }                                                                                                  \
      if constexpr (BF) {                                                                                \
        if (stg_ && !bnh)                                                                                \
          kfn = g.rinfo ? conv_gemm_big64_kernel<F32, true, true, true, EPI_GEN, true>                   \
                        : conv_gemm_big64_kernel<F32, true, false, true, EPI_GEN, true>;                 \
        if constexpr (!F32) {                                                                            \
          if (stg_ && bnh && g_gemm_bnh_stg) kfn = conv_gemm_big64_kernel<false, true, false, true, EPI_BNH, true>; \
        }                                                                                                \
        if constexpr (!F32) {                                                                            \
          if (g_gemm_mask_pre && mask_pre)                                                               \
            kfn = stg_ ? (g.rinfo ? conv_gemm_big64_kernel<false, true, true, true, EPI_MASK, true>       \
                                  : conv_gemm_big64_kernel<false, true, false, true, EPI_MASK, true>)    \
                       : (g.rinfo ? conv_gemm_big64_kernel<false, true, true, true, EPI_MASK>             \
                                  : conv_gemm_big64_kernel<false, true, false, true, EPI_MASK>);         \
        }                                                                                                \
      }                                                                                                  \
      hipLaunchKernelGGL(kfn, dim3(grid_x), dim3(NT3), LB, s, X, W, bias, aux, resid, lens, Y, g, act, ldy, ex); \
    } while (0)
    const bool bf = fastk && big64_buf_ok(g);
    if (out_f32) {
      if (bf) { constexpr bool BF = true; B64_LAUNCH(true, true); }
      else if (fastk) { constexpr bool BF = false; B64_LAUNCH(true, true); }
      else { constexpr bool BF = false; B64_LAUNCH(true, false); }
    } else {
      if (bf) { constexpr bool BF = true; B64_LAUNCH(false, true); }
      else if (fastk) { constexpr bool BF = false; B64_LAUNCH(false, true); }
      else { constexpr bool BF = false; B64_LAUNCH(false, false); }
    }
#undef B64_LAUNCH
  } else if (reg && variant >= 2) {
    static bool ring_set = false;
    if (!ring_set) {
      allow_lds(conv_gemm_ring_kernel<true, true, false>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<false, true, false>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<true, false, false>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<false, false, false>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<true, true, true>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<false, true, true>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<true, false, true>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<false, false, true>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<true, true, false, true>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<false, true, false, true>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<true, true, true, true>, NSTAGE * STAGE_BYTES);
      allow_lds(conv_gemm_ring_kernel<false, true, true, true>, NSTAGE * STAGE_BYTES);
      ring_set = true;
    }
    const int nwg3 = ((g.M + BM3 - 1) / BM3) * ((N + BN - 1) / BN);
    const bool fastk = (Cin % BK) == 0;
    const size_t L3 = NSTAGE * STAGE_BYTES;
#define RING_LAUNCH(F32, FK)                                                                        \
    do {                                                                                            \
      auto kfn = g.rinfo ? conv_gemm_ring_kernel<F32, FK, true, BF> : conv_gemm_ring_kernel<F32, FK, false, BF>; \
      hipLaunchKernelGGL(kfn, dim3(nwg3), dim3(NT3), L3, s, X, W, bias, aux, resid, lens, Y, g, act, ldy, ex); \
    } while (0)
    const bool bf = fastk && big64_buf_ok(g);
    if (out_f32) {
      if (bf) { constexpr bool BF = true; RING_LAUNCH(true, true); }
      else if (fastk) { constexpr bool BF = false; RING_LAUNCH(true, true); }
      else { constexpr bool BF = false; RING_LAUNCH(true, false); }
    } else {
      if (bf) { constexpr bool BF = true; RING_LAUNCH(false, true); }
      else if (fastk) { constexpr bool BF = false; RING_LAUNCH(false, true); }
      else { constexpr bool BF = false; RING_LAUNCH(false, false); }
    }
#undef RING_LAUNCH
  } else if (reg && variant == 1) {
    if (out_f32)
      hipLaunchKernelGGL((conv_gemm_glds_kernel<true>), dim3(nwg), dim3(NT), lds_reg, s, X, W, bias, aux, resid, lens,
                         Y, g, act, ldy);
    else
      hipLaunchKernelGGL((conv_gemm_glds_kernel<false>), dim3(nwg), dim3(NT), lds_reg, s, X, W, bias, aux, resid, lens,
                         Y, g, act, ldy);
  } else if (reg) {
    if (out_f32)
      hipLaunchKernelGGL((conv_gemm_kernel<true, true>), dim3(nwg), dim3(NT), lds_reg, s, X, W, bias, aux, resid, lens,
                         Y, g, act, ldy);
    else
      hipLaunchKernelGGL((conv_gemm_kernel<false, true>), dim3(nwg), dim3(NT), lds_reg, s, X, W, bias, aux, resid, lens,
                         Y, g, act, ldy);
  } else if (out_f32) {
    hipLaunchKernelGGL((conv_gemm_kernel<true, false>), dim3(nwg), dim3(NT), lds, s, X, W, bias, aux, resid, lens, Y, g,
                       act, ldy);
  } else {
    hipLaunchKernelGGL((conv_gemm_kernel<false, false>), dim3(nwg), dim3(NT), lds, s, X, W, bias, aux, resid, lens, Y,
                       g, act, ldy);
  }
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_conv_gemm(const bf16_t* X, const bf16_t* W, const float* bias, const bf16_t* aux,
                              const bf16_t* resid, const int64_t* lens, void* Y, int out_f32, int B, int L, int Cin,
                              int ks, int dil, int pad, int N, int act, int ldy, const int* rinfo, hipStream_t s) {
  EpiX ex{};
  ex.scale = 1.f;
  return conv_gemm_impl(X, W, bias, aux, resid, lens, Y, out_f32, B, L, Cin, ks, dil, pad, N, act, ldy, rinfo, ex, s);
}

// conv_gemm with the extended epilogue (see EpiX): acc (may alias Y), y2 = lrelu(v), scale, post_act.
SSAMD_API int ssamd_conv_gemm_ex(const bf16_t* X, const bf16_t* W, const float* bias, const bf16_t* resid, void* Y,
                                 int B, int L, int Cin, int ks, int dil, int pad, int N, int act, const bf16_t* acc,
                                 bf16_t* y2, float scale, int post_act, hipStream_t s) {
  EpiX ex{};
  ex.acc = acc;
  ex.y2 = y2;
  ex.scale = scale;
  ex.post_act = post_act;
  return conv_gemm_impl(X, W, bias, nullptr, resid, nullptr, Y, 0, B, L, Cin, ks, dil, pad, N, act, N, nullptr, ex, s);
}

// ssamd_conv_gemm_ex for the 3-tap ConvTranspose form (hifigan convT_as_conv3): ksplit = (stride / 2) * Cout,
// the first output column of the phases that read taps {1, 2} (see ConvGeom::ksplit); ignored unless ks == 3,
// Cin % 64 == 0 and ksplit % 256 == 0 (the weights' zero tap is then skipped per 256-column tile).
SSAMD_API int ssamd_conv_gemm_ex2(const bf16_t* X, const bf16_t* W, const float* bias, const bf16_t* resid, void* Y,
                                  int B, int L, int Cin, int ks, int dil, int pad, int N, int act, const bf16_t* acc,
                                  bf16_t* y2, float scale, int post_act, int ksplit, hipStream_t s) {
  EpiX ex{};
  ex.acc = acc;
  ex.y2 = y2;
  ex.scale = scale;
  ex.post_act = post_act;
  return conv_gemm_impl(X, W, bias, nullptr, resid, nullptr, Y, 0, B, L, Cin, ks, dil, pad, N, act, N, nullptr, ex, s,
                        false, ksplit);
}

// ssamd_conv_gemm_ex2 on packed rows (B = 1, L = R): rinfo [R] int2 {position, length} zero-pads every conv at its
// own sequence's ends (the length-exact vocoder's GEMM stages, k_vocoder.hip ssamd_voc_rinfo).
SSAMD_API int ssamd_conv_gemm_ex3(const bf16_t* X, const bf16_t* W, const float* bias, const bf16_t* resid, void* Y,
                                  int R, int Cin, int ks, int dil, int pad, int N, int act, const bf16_t* acc,
                                  bf16_t* y2, float scale, int post_act, int ksplit, const int* rinfo, hipStream_t s) {
  if (!rinfo) return -2;
  EpiX ex{};
  ex.acc = acc;
  ex.y2 = y2;
  ex.scale = scale;
  ex.post_act = post_act;
  return conv_gemm_impl(X, W, bias, nullptr, resid, nullptr, Y, 0, 1, R, Cin, ks, dil, pad, N, act, N, rinfo, ex, s,
                        false, ksplit);
}

// Data gradient of a conv whose input came out of BatchNorm (+act, dropout): Y = dz (see EpiX.bn_*) and the
// per-M-tile column partials bn_part [2][ceil(M/256)][N] of dz and dz * (h - mean) (ssamd_bn_bwd_dz applies rstd).
SSAMD_API int ssamd_conv_gemm_bnbwd(const bf16_t* X, const bf16_t* W, void* Y, int B, int L, int Cin, int ks, int dil,
                                    int pad, int N, const bf16_t* bn_h, const float* bn_stats, float* bn_part,
                                    int bn_act, float p, unsigned long long seed, hipStream_t s) {
  if (!bn_h || !bn_stats || !bn_part) return -2;
  EpiX ex{};
  ex.scale = 1.f;
  ex.acc = bn_h;
  ex.bn_stats = bn_stats;
  ex.bn_part = bn_part;
  ex.post_act = bn_act;
  ex.bn_p = p;
  ex.bn_seed = seed;
  return conv_gemm_impl(X, W, nullptr, nullptr, nullptr, nullptr, Y, 0, B, L, Cin, ks, dil, pad, N, 0, N, nullptr, ex, s,
                        true);
}

// conv_gemm with a ReLU bitmask: mask_out (act must be ReLU) stores bit (y > 0) per output element,
// mask_in zeroes the outputs whose bit is clear (the dgrad of a ReLU layer).  [M][N/8] bytes.
SSAMD_API int ssamd_conv_gemm_mask(const bf16_t* X, const bf16_t* W, const float* bias, void* Y, int B, int L,
                                   int Cin, int ks, int dil, int pad, int N, int act, const int* rinfo,
                                   unsigned char* mask_out, const unsigned char* mask_in, hipStream_t s) {
  EpiX ex{};
  ex.scale = 1.f;
  ex.mask_out = mask_out;
  ex.mask_in = mask_in;
  return conv_gemm_impl(X, W, bias, nullptr, nullptr, nullptr, Y, 0, B, L, Cin, ks, dil, pad, N, act, N, rinfo, ex, s);
}

static int g_wgrad_imm = -1;  // -1 auto, 0 / 1: force the big64 wgrad read schedule
SSAMD_API void ssamd_wgrad_set_imm(int v) { g_wgrad_imm = v; }
static int g_wgrad_buf = 1;  // big64 wgrad LDS-DMA through buffer descriptors (0: flat global_load_lds)
SSAMD_API void ssamd_wgrad_set_buf(int v) { g_wgrad_buf = v; }
// big64 wgrad (buffer-descriptor path) ping-pong main loop: -1 auto = on packed rows (decoder k9 wgrad
// 646 -> 519 us vs 718 before, tools/exp_wgrad_pp.py), off on plain rows (PostNet k5 -14 %)
static int g_wgrad_pp = -1;
SSAMD_API void ssamd_wgrad_set_pp(int v) { g_wgrad_pp = v; }

// Workspace: splits * N * ks*Cin floats.  Returns the number of splits used via *splits_used.
// ws: splits*N*ks*Cin (+ splits*N when db != null) floats.  db (optional): fused bias gradient.
static void launch_reduce(const float* ws, float* dW, const float* bws, float* db, int splits, int N, int Cin, int ks,
                          int blocks, hipStream_t s) {
  const int K = Cin * ks;
  (void)blocks;
  // many output rows of a k > 1 conv: one block per row keeps the dW stores contiguous; otherwise
  // (Linear / k = 1 weights, few rows) the split-parallel kernel keeps every CU busy
  if (ks > 1 && N >= 256 && (size_t)K * 4 <= 65536) {
    hipLaunchKernelGGL(wgrad_reduce_rows_kernel, dim3(N), dim3(256), (size_t)K * 4, s, ws, dW, bws, db, splits, N, Cin,
                       ks);
    return;
  }
  const int nb_main = (int)cdiv((long)N * K / 4, 64L);
  const int nb_bias = bws ? (int)cdiv((long)(N + 3) / 4, 64L) : 0;
  hipLaunchKernelGGL(wgrad_reduce4_kernel, dim3(nb_main + nb_bias), dim3(256), 0, s, ws, dW, bws, db, splits, N, Cin,
                     ks, nb_main);
}

// Split-M count of the 256x256 weight-gradient kernel (one block per CU): the blocks run in
// ceil(tiles * S / CUs) rounds of ceil(M / S / 64) row steps each, and every split adds a 256x256
// fp32 slab to write and reduce (~8 % of a 64-row step per slab tile).  The old fixed target of 512
// blocks left partial rounds (packed k9 wgrad: 36 tiles x 15 = 540 blocks = 2.1 rounds -> 3) and,
// capped by the 128x128 kernels' split limit, single-tile weights ran on 64 CUs.
static int g_cus_dev[64];
static int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!g_cus_dev[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    g_cus_dev[dev] = n;
  }
  return g_cus_dev[dev];
}
static int g_wgrad_blocks = 0;   // > 0: fixed split-M target (blocks per launch) instead of the cost model
// > 0: plan the split-M rounds for this many CUs instead of the device's (a weight gradient on the side
// stream then leaves the other CUs to the data-gradient chain instead of holding every CU's LDS)
// The budget applies to launches on ONE stream (the weight-gradient side stream): a main-stream weight
// gradient (first step, --no-side-wgrad) keeps the whole-device plan, so the split-M count -- and with it
// the fp32 reduction order -- of a main-stream launch does not depend on the side-stream setting.
static int g_wgrad_cus = 0;
static hipStream_t g_wgrad_cus_stream = nullptr;
static int choose_wgrad_splits(int tiles, int M, int max_splits, long ws_splits, int cus) {
  const int steps_all = (M + 63) / 64;
  int smax = max_splits;
  if (smax > steps_all / 4) smax = steps_all / 4 > 0 ? steps_all / 4 : 1;  // >= 4 row steps per split
  if ((long)smax > ws_splits) smax = (int)ws_splits;
  if (smax < 1) return (int)(ws_splits >= 1 ? 1 : 0);
  if (g_wgrad_blocks > 0) {
    const int sp = (g_wgrad_blocks + tiles - 1) / tiles;
    return sp < smax ? sp : smax;
  }
  int best = 1;
  double best_c = 1e30;
  for (int sp = 1; sp <= smax; ++sp) {
    const long rounds = ((long)tiles * sp + cus - 1) / cus;
    const long steps = (steps_all + sp - 1) / sp;
    const double c = (double)rounds * (double)steps + 0.08 * (double)sp * tiles;
    if (c < best_c - 1e-9) { best_c = c; best = sp; }
  }
  return best;
}

static int g_wgrad_variant = -1;  // -1 auto (256x256 BK=64 when it applies), 0: force the 128x128 kernels
SSAMD_API void ssamd_wgrad_set_blocks(int b) { g_wgrad_blocks = b > 0 ? b : 0; }
SSAMD_API void ssamd_wgrad_set_cus(hipStream_t s, int n) {
  g_wgrad_cus = n > 0 ? n : 0;
  g_wgrad_cus_stream = s;
}
SSAMD_API void ssamd_wgrad_set_variant(int v) { g_wgrad_variant = v; }

SSAMD_API int ssamd_conv_wgrad(const bf16_t* X, const bf16_t* dY, float* ws, long ws_floats, float* dW, float* db,
                               int B, int L, int Cin, int ks, int dil, int pad, int N, int max_splits, const int* rinfo,
                               const int64_t* cu, int nseq, hipStream_t s) {
  if (Cin % 8 != 0 || N % 8 != 0) return -2;
  ConvGeom g = make_geom(B, L, Cin, ks, dil, pad, N);
  g.rinfo = reinterpret_cast<const int2*>(rinfo);
  g.cu = cu;
  g.nseq = nseq;
  g.prio = g_wgrad_prio;
  const long slab = (long)N * g.K;
  if (g.M == 0) {
    hipMemsetAsync(dW, 0, slab * sizeof(float), s);
    if (db) hipMemsetAsync(db, 0, N * sizeof(float), s);
    return (int)hipGetLastError();
  }
  const bool packed = rinfo != nullptr;
  // 256x256 kernel (split-M slabs + fixed-order reduce) when there are >= 2 output tiles; variant 0
  // forces the 128x128 kernels (the choice for single-tile and narrow problems)
  const bool big = g_wgrad_variant != 0 && N >= 256 && g.K >= 256 && (long)N * g.K >= 2L * 256 * 256 &&
                   (!packed || (cu != nullptr && nseq > 0 && nseq < 8192));
  if (big) {
    static bool b64_set = false;
    if (!b64_set) {
      allow_lds(conv_wgrad_big64_kernel<false, false, false>, 160 * 1024);
      allow_lds(conv_wgrad_big64_kernel<true, false, false>, 160 * 1024);
      allow_lds(conv_wgrad_big64_kernel<false, true, false>, 160 * 1024);
      allow_lds(conv_wgrad_big64_kernel<true, true, false>, 160 * 1024);
      allow_lds(conv_wgrad_big64_kernel<false, false, true>, 160 * 1024);
      allow_lds(conv_wgrad_big64_kernel<true, false, true>, 160 * 1024);
      allow_lds(conv_wgrad_big64_kernel<false, true, true>, 160 * 1024);
      allow_lds(conv_wgrad_big64_kernel<true, true, true>, 160 * 1024);
      allow_lds(conv_wgrad_big64_kernel<false, false, true, true>, 160 * 1024);
      allow_lds(conv_wgrad_big64_kernel<true, false, true, true>, 160 * 1024);
      b64_set = true;
    }
    const int tiles = ((N + 255) / 256) * ((g.K + 255) / 256);
    const bool on = g_wgrad_cus_stream == reinterpret_cast<hipStream_t>(-1) || s == g_wgrad_cus_stream;
    const int cus = (g_wgrad_cus > 0 && on) ? g_wgrad_cus : device_cus();
    int splits = choose_wgrad_splits(tiles, g.M, max_splits, ws_floats / (slab + N), cus);
    if (splits < 1) return -3;
    int rows_per_split = (g.M + splits - 1) / splits;
    rows_per_split = (rows_per_split + 63) / 64 * 64;
    splits = (g.M + rows_per_split - 1) / rows_per_split;
    float* bws = db ? ws + (long)splits * slab : nullptr;
    size_t lds = 2 * WB64_STAGE;
    if (lds < 128 * 1088) lds = 128 * 1088;  // the LDS-staged slab epilogue tile
    // immediate-offset fragment reads: measured faster on packed rows (the decoder FFN), the
    // single-wait schedule on plain rows (tools/exp_packed_wgrad.py); g_wgrad_imm overrides
    const bool imm = g_wgrad_imm < 0 ? packed : g_wgrad_imm != 0;
    // buffer-descriptor DMA needs every byte offset in 31 bits (out-of-range marker 0x80000000)
    const bool bufok = g_wgrad_buf != 0 && (long)(g.M + pad) * Cin * 2 < (1L << 31) &&
                       (long)rows_per_split * N * 2 < (1L << 31);
    auto wb = bufok ? (packed ? (imm ? conv_wgrad_big64_kernel<true, true, true> : conv_wgrad_big64_kernel<true, false, true>)
                              : (imm ? conv_wgrad_big64_kernel<false, true, true> : conv_wgrad_big64_kernel<false, false, true>))
                    : (packed ? (imm ? conv_wgrad_big64_kernel<true, true, false> : conv_wgrad_big64_kernel<true, false, false>)
                              : (imm ? conv_wgrad_big64_kernel<false, true, false> : conv_wgrad_big64_kernel<false, false, false>));
    if (bufok && (g_wgrad_pp < 0 ? packed : g_wgrad_pp != 0))
      wb = packed ? conv_wgrad_big64_kernel<true, false, true, true> : conv_wgrad_big64_kernel<false, false, true, true>;
    hipLaunchKernelGGL(wb, dim3(tiles * splits), dim3(NT3), lds, s, X, dY, ws, bws, g, rows_per_split);
    const int blocks = (int)min((slab + 255) / 256, 8192L);
    launch_reduce(ws, dW, bws, db, splits, N, Cin, ks, blocks, s);
    return (int)hipGetLastError();
  }
  const int tiles = ((N + 127) / 128) * ((g.K + 127) / 128);
  int splits = (1536 + tiles - 1) / tiles;
  const int max_by_rows = (g.M + 511) / 512;
  if (splits > max_by_rows) splits = max_by_rows;
  if (splits > max_splits) splits = max_splits;
  if ((long)splits * (slab + N) > ws_floats) splits = (int)(ws_floats / (slab + N));
  if (splits < 1) return -3;
  int rows_per_split = (g.M + splits - 1) / splits;
  rows_per_split = (rows_per_split + RB - 1) / RB * RB;
  splits = (g.M + rows_per_split - 1) / rows_per_split;
  float* bws = db ? ws + (long)splits * slab : nullptr;
  auto wreg = g.rinfo ? conv_wgrad_reg_kernel<true> : conv_wgrad_reg_kernel<false>;
  auto wdma = g.rinfo ? conv_wgrad_kernel<true> : conv_wgrad_kernel<false>;
  if (g.K > 1024)
    hipLaunchKernelGGL(wreg, dim3(tiles * splits), dim3(NT), 2 * 2 * RB * 256, s, X, dY, ws, bws, g,
                       rows_per_split);
  else
    hipLaunchKernelGGL(wdma, dim3(tiles * splits), dim3(NT), 2 * 2 * RB * 256, s, X, dY, ws, bws, g,
                       rows_per_split);
  const long total = slab;
  int blocks = (int)min((total + 255) / 256, 8192L);
  launch_reduce(ws, dW, bws, db, splits, N, Cin, ks, blocks, s);
  return (int)hipGetLastError();
}

SSAMD_API long ssamd_colsum_ws(long M, int N) { return (long)cdiv(M, 256) * N + seg_colsum_ws(1, N); }

SSAMD_API int ssamd_colsum(const bf16_t* dY, float* db, long M, int N, float* ws, long ws_floats, hipStream_t s) {
  if (M == 0) return (int)hipMemsetAsync(db, 0, (size_t)N * sizeof(float), s);
  const int rpb = 256;
  const int chunks = cdiv(M, rpb);
  if (ws_floats < ssamd_colsum_ws(M, N)) return -3;
  dim3 grid((N + 255) / 256, chunks);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, s, dY, ws, M, N, rpb);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  return ssamd_seg_colsum(ws, N, 1, chunks, N, db, 0, 0, N, nullptr, ws + (long)chunks * N, seg_colsum_ws(1, N), s);
}

SSAMD_DROP_SALT_LOADER(gemm)
