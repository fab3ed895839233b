// Fused multi-head self-attention with key-padding mask (flash-style, O(L) memory).
//
// Reference math: transformer/Modules.py:14-23 + SubLayers.py:39-57 -- softmax over
// keys of QK^T / sqrt(d_k), keys >= len[b] masked to -inf, times V.  Heads are read
// straight out of the fused QKV projection output qkv[B, L, 3*H*D] (channel h*D+d of
// each third), the output is written head-interleaved o[B, L, H*D]; no permute copies.
//
// Forward (per block: 64 queries of one (b, h), 4 waves x 16 queries):
//   S^T = K Q^T is computed "swapped" (A = K tile from LDS, B = Q fragments kept in
//   registers) so that the 16x16 accumulator puts ONE query per lane column; the
//   online softmax is then lane-local plus two cross-group shuffles, and the bf16
//   P^T accumulator is *directly* the B operand of O^T += V^T P^T (key order
//   permuted consistently on both operands).  V^T fragments come from LDS through
//   ds_read_b64_tr_b16.  Scores live in the log2 domain (exp2); lse is stored as
//   log2-domain m + log2(l) per (b, h, q).
// Backward (FA2 split, no atomics, deterministic):
//   delta = rowsum(dO * O);  kernel dKdV: per 64-key block, key on the MFMA lane,
//   stream query tiles: S, dP -> P, dS are already the B operands of dV^T += dO^T P and
//   dK^T += Q^T dS;  kernel dQ: per 64-query block, swapped again (query on the lane),
//   dQ^T += K^T dS^T.  Every LDS image is XOR-swizzled for its read instruction
//   (ds_read_b128 row reads / ds_read_b64_tr_b16 transposed reads).
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int TQ = 64;   // queries per block
constexpr int TK = 64;   // keys per tile

__device__ __forceinline__ short4v tr_read(const char* p) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

// D = 128 (256-B rows): ONE swizzle serves both read kinds, so a tensor needs a single LDS
// image.  16-B chunk c of row r sits at c ^ h(r), h = {0,2,..,14, 9,11,13,15, 1,3,5,7}[r % 16]:
// the ds_read_b128 lane groups (rows {0-3,12-15} at chunk c, rows 4-11 at c+1, and the
// mirrored groups) hit 16 distinct slots because h(rows 0-3,12-15) and h(rows 4-11)^1 are
// disjoint, and the ds_read_b64_tr_b16 half-waves (8 consecutive rows x 4 chunks) because
// h(r) >> 1 is a permutation of 0..7 on rows 0-7 and on rows 8-15.
template <int D>
constexpr bool kUnified = (D == 128);
__device__ __forceinline__ int uni_h(int row) {
  const int r = row & 15;
  return r < 8 ? 2 * r : (2 * r + 9) & 15;
}
// [rows][D] bf16 image read by 16-B rows (MFMA A/B "row" fragments)
template <int D>
__device__ __forceinline__ int row_off(int row, int c16) {
  if constexpr (kUnified<D>) return row * 256 + ((c16 ^ uni_h(row)) << 4);
  constexpr int RPB = 256 / (2 * D);  // rows per 256-B bank row
  constexpr int CPR = D / 8;          // 16-B chunks per row
  return row * (2 * D) + ((c16 ^ ((row / RPB) % CPR)) << 4);
}
// [rows][D] bf16 image read by ds_read_b64_tr_b16 (8-B chunks)
template <int D>
__device__ __forceinline__ int tr_off(int row, int c8) {
  if constexpr (kUnified<D>) return row * 256 + ((c8 ^ (2 * uni_h(row))) << 3);
  constexpr int RPB = 256 / (2 * D);
  constexpr int CPR4 = D / 16;  // (8-B chunks per row) / 4
  return row * (2 * D) + ((c8 ^ (((row / RPB) % CPR4) << 2)) << 3);
}

// stage a [64][D] tile (rows r0.., channel offset coff) of the [B*L, RS] matrix into registers
template <int D>
__device__ __forceinline__ void load_tile(const bf16_t* base, long row0, int nvalid, int RS, short8* regs) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
    const int e = threadIdx.x + NT * i;
    const int r = e / CPR, c = e % CPR;
    short8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < nvalid) v = *reinterpret_cast<const short8*>(base + (row0 + r) * (long)RS + c * 8);
    regs[i] = v;
  }
}
template <int D>
__device__ __forceinline__ void store_row_img(char* img, const short8* regs) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
    const int e = threadIdx.x + NT * i;
    *reinterpret_cast<short8*>(img + row_off<D>(e / CPR, e % CPR)) = regs[i];
  }
}
template <int D>
__device__ __forceinline__ void store_tr_img(char* img, const short8* regs) {
  if constexpr (kUnified<D>) {
    store_row_img<D>(img, regs);
    return;
  }
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
    const int e = threadIdx.x + NT * i;
    *reinterpret_cast<short8*>(img + tr_off<D>(e / CPR, 2 * (e % CPR))) = regs[i];
  }
}

__device__ __forceinline__ short8 pack8(const float4v& a, const float4v& b) {
  short8 r;
  r[0] = (short)f2bf(a[0]); r[1] = (short)f2bf(a[1]); r[2] = (short)f2bf(a[2]); r[3] = (short)f2bf(a[3]);
  r[4] = (short)f2bf(b[0]); r[5] = (short)f2bf(b[1]); r[6] = (short)f2bf(b[2]); r[7] = (short)f2bf(b[3]);
  return r;
}

// Online-softmax update of one 64-key tile (scores st = raw Q.K, query on the lane column, keys
// 4g + r of each 16-key fragment on the lane's 4 accumulator slots).  VALU-lean form -- the
// loop is VALU-issue bound (MI355X_MICROARCH: 4 cycles per VALU, 8 per v_exp beside 16-cycle
// MFMAs): raw v_exp_f32 (no denormal-range fix-up: softmax terms below 2^-126 are 0 anyway),
// the key mask only on the one tile that straddles len, scale and max folded into one FMA,
// the running max deferred (moved only by jumps > kMaxSlack, so the O rescale is rare), and l kept as a
// per-lane partial
// (the 4 lane groups of a query share m, so the cross-group sum is deferred to the end).
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
constexpr float kMaxSlack = 8.f;

template <int NF, int D>
__device__ __forceinline__ void online_softmax(float4v (&st)[NF][4], float (&m)[NF], float (&l)[NF],
                                               float4v (&oacc)[NF][D / 16], int key0, int len, float scale_log2,
                                               int g) {
  if (key0 + TK > len) {
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (key0 + kf * 16 + 4 * g + r >= len)
#pragma unroll
          for (int f = 0; f < NF; ++f) st[f][kf][r] = -INFINITY;
  }
  bool rescale = false;
  float alpha[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    float mx = fmaxf(fmaxf(st[f][0][0], st[f][0][1]), fmaxf(st[f][0][2], st[f][0][3]));
#pragma unroll
    for (int kf = 1; kf < 4; ++kf)
      mx = fmaxf(mx, fmaxf(fmaxf(st[f][kf][0], st[f][kf][1]), fmaxf(st[f][kf][2], st[f][kf][3])));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    // deferred max: the running max moves only when a tile's max exceeds it by more than kMaxSlack (log2
    // units), so the O rescale runs on the first tile and on rare jumps instead of whenever any query's max
    // creeps up; unnormalised p stay <= 2^kMaxSlack (exact in fp32 / bf16 range), l and O share the factor
    const float cand = mx * scale_log2;               // the tile always holds a valid key: cand finite
    const bool up = cand > m[f] + kMaxSlack;          // m = -inf on the first tile -> up
    const float mn = up ? cand : m[f];
    alpha[f] = fast_exp2(m[f] - mn);                  // 1 when the max stays, 0 on the first tile
    rescale |= up;
    const float nb = -mn;
    float ls = 0.f;
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = fast_exp2(fmaf(st[f][kf][r], scale_log2, nb));
        st[f][kf][r] = pv;
        ls += pv;
      }
    l[f] = fmaf(l[f], alpha[f], ls);
    m[f] = mn;
  }
  if (__any(rescale)) {
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int i = 0; i < D / 16; ++i) oacc[f][i] *= alpha[f];
  }
}

// per-lane partial -> the query's full softmax denominator (sum over the 4 lane groups)
__device__ __forceinline__ float lsum_groups(float l) {
  l += __shfl_xor(l, 16, 64);
  return l + __shfl_xor(l, 32, 64);
}

// A fragment (16 rows x 32) of a transposed image: rows = reduction keys/queries in the
// permuted order {base + 4g + q} u {base + 16 + 4g + q}, columns col0 .. col0+15.
template <int D>
__device__ __forceinline__ short8 tr_frag(const char* img, int base, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int c8 = col0 / 4 + p;
  short4v a = tr_read(img + tr_off<D>(base + 4 * g + q, c8));
  short4v b = tr_read(img + tr_off<D>(base + 16 + 4 * g + q, c8));
  return (short8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// ------------------------------------------------------------------------------ forward
// NF = query fragments (of 16) per wave: each LDS fragment read feeds NF MFMAs.
template <int D, int NF>
__global__ void __launch_bounds__(NT) attn_fwd_kernel(const bf16_t* __restrict__ qkv, const int64_t* __restrict__ lens,
                                                      const int64_t* __restrict__ cu,
                                                      bf16_t* __restrict__ out, float* __restrict__ lse, int L, int H,
                                                      float scale_log2) {
  __shared__ __attribute__((aligned(16))) char smem[2 * TK * D * 2];
  char* Ks = smem;
  char* Vs = smem + TK * D * 2;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int RS = 3 * H * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int len = (int)lens[b];
  // packed variable-length rows (cu = row offsets): only rows < len exist for sequence b
  const long rowb = cu ? (long)cu[b] : (long)b * L;
  const int Lq = cu ? len : L;
  const bf16_t* Qp = qkv + h * D;
  const bf16_t* Kp = qkv + H * D + h * D;
  const bf16_t* Vp = qkv + 2 * H * D + h * D;
  int qv[NF];
  short8 qf[NF][D / 32];
  if (blockIdx.x * (64 * NF) >= len) {
    // query rows past the sequence length are defined as zero output (they are masked
    // downstream): a fully padded query block only writes zeros
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int q = blockIdx.x * (64 * NF) + wave * (16 * NF) + f * 16 + (lane & 15);
      if (q >= Lq) continue;
      bf16_t* op = out + (rowb + q) * (long)(H * D) + h * D;
#pragma unroll
      for (int df = 0; df < D / 16; ++df) *reinterpret_cast<short4v*>(op + df * 16 + 4 * g) = (short4v){0, 0, 0, 0};
      if (g == 0) lse[(long)bh * L + q] = INFINITY;
    }
    return;
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    qv[f] = blockIdx.x * (64 * NF) + wave * (16 * NF) + f * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      short8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qv[f] < len) v = *reinterpret_cast<const short8*>(Qp + (rowb + qv[f]) * RS + s * 32 + 8 * g);
      qf[f][s] = v;
    }
  }
  float4v oacc[NF][D / 16];
  float m[NF], l[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    m[f] = -INFINITY;
    l[f] = 0.f;
#pragma unroll
    for (int i = 0; i < D / 16; ++i) oacc[f][i] = (float4v){0.f, 0.f, 0.f, 0.f};
  }

  const int nkt = (len + TK - 1) / TK;
  short8 rk[D / 32], rv[D / 32];
  if (nkt > 0) {
    load_tile<D>(Kp, rowb, min(TK, len), RS, rk);
    load_tile<D>(Vp, rowb, min(TK, len), RS, rv);
  }
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    store_row_img<D>(Ks, rk);
    store_tr_img<D>(Vs, rv);
    __syncthreads();
    if (kt + 1 < nkt) {
      const int k1 = (kt + 1) * TK;
      load_tile<D>(Kp, rowb + k1, min(TK, len - k1), RS, rk);
      load_tile<D>(Vp, rowb + k1, min(TK, len - k1), RS, rv);
    }
    float4v st[NF][4];
#pragma unroll
    for (int kf = 0; kf < 4; ++kf) {
#pragma unroll
      for (int f = 0; f < NF; ++f) st[f][kf] = (float4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
        const short8 a = *reinterpret_cast<const short8*>(Ks + row_off<D>(kf * 16 + (lane & 15), s * 4 + g));
#pragma unroll
        for (int f = 0; f < NF; ++f) st[f][kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[f][s], st[f][kf], 0, 0, 0);
      }
    }
    online_softmax<NF, D>(st, m, l, oacc, kt * TK, len, scale_log2, g);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      short8 pb[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) pb[f] = pack8(st[f][2 * hh], st[f][2 * hh + 1]);
#pragma unroll
      for (int df = 0; df < D / 16; ++df) {
        const short8 a = tr_frag<D>(Vs, hh * 32, df * 16, lane);
#pragma unroll
        for (int f = 0; f < NF; ++f) oacc[f][df] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[f], oacc[f][df], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) l[f] = lsum_groups(l[f]);
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    if (qv[f] >= Lq) continue;
    const float inv = (l[f] > 0.f && qv[f] < len) ? 1.f / l[f] : 0.f;
    bf16_t* op = out + (rowb + qv[f]) * (long)(H * D) + h * D;
#pragma unroll
    for (int df = 0; df < D / 16; ++df) {
      short4v v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (short)f2bf(oacc[f][df][r] * inv);
      *reinterpret_cast<short4v*>(op + df * 16 + 4 * g) = v;
    }
    if (g == 0) lse[(long)bh * L + qv[f]] = (l[f] > 0.f && qv[f] < len) ? m[f] + log2f(l[f]) : INFINITY;
  }
}

// LDS-DMA (global_load_lds, 16 B per lane, lane-linear destination) for the attention tiles
__device__ __attribute__((aligned(16))) bf16_t a_zero_chunk[8];
__device__ __forceinline__ void a_glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Buffer-resource LDS-DMA: a descriptor over the rows of ONE sequence (bytes = len rows), so a
// tile row past len is out of range and lands as zeros (no per-row select, no 64-bit address
// math per tile); the per-lane part is a loop-invariant 32-bit voffset, the tile offset a
// scalar soffset.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t seq_rsrc(const bf16_t* base, int nrows, int row_stride) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nrows * row_stride * 2, 0x00020000);
}
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, soff,
                                           0, 0);
}

template <int NF>
__global__ void __launch_bounds__(NT, 2) attn_fwd_dma_kernel(const bf16_t* __restrict__ qkv, const int64_t* __restrict__ lens,
                                                      const int64_t* __restrict__ cu,
                                                      bf16_t* __restrict__ out, float* __restrict__ lse, int L, int H,
                                                      float scale_log2) {
  constexpr int D = 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (K, V) tiles, unified swizzle
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int RS = 3 * H * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4;
  const int len = (int)lens[b];
  // packed variable-length rows (cu = row offsets): only rows < len exist for sequence b
  const long rowb = cu ? (long)cu[b] : (long)b * L;
  const int Lq = cu ? len : L;
  const bf16_t* Qp = qkv + h * D;
  const bf16_t* Kp = qkv + H * D + h * D;
  const bf16_t* Vp = qkv + 2 * H * D + h * D;
  int qv[NF];
  short8 qf[NF][D / 32];
  if (blockIdx.x * (64 * NF) >= len) {
    // query rows past the sequence length are defined as zero output (they are masked
    // downstream): a fully padded query block only writes zeros
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int q = blockIdx.x * (64 * NF) + wave * (16 * NF) + f * 16 + (lane & 15);
      if (q >= Lq) continue;
      bf16_t* op = out + (rowb + q) * (long)(H * D) + h * D;
#pragma unroll
      for (int df = 0; df < D / 16; ++df) *reinterpret_cast<short4v*>(op + df * 16 + 4 * g) = (short4v){0, 0, 0, 0};
      if (g == 0) lse[(long)bh * L + q] = INFINITY;
    }
    return;
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    qv[f] = blockIdx.x * (64 * NF) + wave * (16 * NF) + f * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      short8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qv[f] < len) v = *reinterpret_cast<const short8*>(Qp + (rowb + qv[f]) * RS + s * 32 + 8 * g);
      qf[f][s] = v;
    }
  }
  float4v oacc[NF][D / 16];
  float m[NF], l[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    m[f] = -INFINITY;
    l[f] = 0.f;
#pragma unroll
    for (int i = 0; i < D / 16; ++i) oacc[f][i] = (float4v){0.f, 0.f, 0.f, 0.f};
  }

  const int nkt = (len + TK - 1) / TK;
  // K / V tiles go global -> LDS by DMA (no staging registers, no ds_write), row-major with the
  // unified swizzle applied on the source side; V^T fragments are read with ds_read_b64_tr_b16.
  const __amdgpu_buffer_rsrc_t rK = seq_rsrc(Kp + rowb * RS, len, RS), rV = seq_rsrc(Vp + rowb * RS, len, RS);
  int voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 4 + wave) * 4 + (lane >> 4);
    voff[i] = (row * RS + ((lane & 15) ^ uni_h(row)) * 8) * 2;
  }
  auto issue = [&](int key0, int buf) {
    char* Kd = smem + buf * (2 * TK * D * 2);
    char* Vd = Kd + TK * D * 2;
    const int soff = key0 * RS * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      buf_lds16(rK, voff[i], soff, Kd + (i * 4 + wave) * 1024);
      buf_lds16(rV, voff[i], soff, Vd + (i * 4 + wave) * 1024);
    }
  };
  if (nkt > 0) issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) issue((kt + 1) * TK, buf ^ 1);
    const char* Ks = smem + buf * (2 * TK * D * 2);
    const char* Vs = Ks + TK * D * 2;
    float4v st[NF][4];
#pragma unroll
    for (int kf = 0; kf < 4; ++kf) {
#pragma unroll
      for (int f = 0; f < NF; ++f) st[f][kf] = (float4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
        const short8 a = *reinterpret_cast<const short8*>(Ks + row_off<D>(kf * 16 + (lane & 15), s * 4 + g));
#pragma unroll
        for (int f = 0; f < NF; ++f) st[f][kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[f][s], st[f][kf], 0, 0, 0);
      }
    }
    online_softmax<NF, D>(st, m, l, oacc, kt * TK, len, scale_log2, g);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      short8 pb[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) pb[f] = pack8(st[f][2 * hh], st[f][2 * hh + 1]);
#pragma unroll
      for (int df = 0; df < D / 16; ++df) {
        const short8 a = tr_frag<D>(Vs, hh * 32, df * 16, lane);
#pragma unroll
        for (int f = 0; f < NF; ++f) oacc[f][df] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[f], oacc[f][df], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // next tile landed, this one consumed
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) l[f] = lsum_groups(l[f]);
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    if (qv[f] >= Lq) continue;
    const float inv = (l[f] > 0.f && qv[f] < len) ? 1.f / l[f] : 0.f;
    bf16_t* op = out + (rowb + qv[f]) * (long)(H * D) + h * D;
#pragma unroll
    for (int df = 0; df < D / 16; ++df) {
      short4v v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (short)f2bf(oacc[f][df][r] * inv);
      *reinterpret_cast<short4v*>(op + df * 16 + 4 * g) = v;
    }
    if (g == 0) lse[(long)bh * L + qv[f]] = (l[f] > 0.f && qv[f] < len) ? m[f] + log2f(l[f]) : INFINITY;
  }
}

// ------------------------------------------------------------------------------ backward
// delta[row * H + h] = sum_d dO * O: 8 channels (16 B) per lane, D/8 lanes per (row, head)
__global__ void __launch_bounds__(NT) attn_delta_kernel(const bf16_t* __restrict__ o, const bf16_t* __restrict__ dO,
                                                        float* __restrict__ delta, long rows, int H, int D) {
  const int lpr = D / 8;  // lanes per (row, head): 4 (D=32) .. 16 (D=128), a power of two
  const long e = blockIdx.x * (long)NT + threadIdx.x;
  const long wid = e / lpr;
  const int c = (int)(e - wid * lpr);
  float s = 0.f;
  if (wid < rows * H) {
    const long off = wid * D + c * 8;  // [rows, H*D] row-major == (row*H + h)*D
    const short8 a = *reinterpret_cast<const short8*>(o + off);
    const short8 b = *reinterpret_cast<const short8*>(dO + off);
#pragma unroll
    for (int q = 0; q < 8; ++q) s += bf2f((bf16_t)a[q]) * bf2f((bf16_t)b[q]);
  }
  for (int w = lpr >> 1; w > 0; w >>= 1) s += __shfl_xor(s, w, 64);
  if (c == 0 && wid < rows * H) delta[wid] = s;
}

// NF = key fragments (of 16) per wave; block = 4 waves x 16*NF keys
template <int D, int NF>
__global__ void __launch_bounds__(NT) attn_bwd_dkdv_kernel(const bf16_t* __restrict__ qkv,
                                                           const int64_t* __restrict__ lens,
                                                           const int64_t* __restrict__ cu,
                                                           const bf16_t* __restrict__ dO, const float* __restrict__ lse,
                                                           const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
                                                           int L, int H, float scale_log2, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NIMG = kUnified<D> ? 2 : 4;  // unified swizzle: row and transposed reads share an image
  char* Qr = smem;
  char* Qt = kUnified<D> ? Qr : Qr + TQ * D * 2;
  char* Dr = kUnified<D> ? Qr + TQ * D * 2 : Qt + TQ * D * 2;
  char* Dt = kUnified<D> ? Dr : Dr + TQ * D * 2;
  // per-query lse / delta of the current tile, staged with the Q / dO images (the global
  // loads ride with the tile prefetch instead of stalling the softmax every iteration)
  float* Ls = reinterpret_cast<float*>(smem + NIMG * TQ * D * 2);
  float* Ds = Ls + TQ;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int RS = 3 * H * D, OS = H * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int len = (int)lens[b];
  // packed variable-length rows (cu = row offsets): only rows < len exist for sequence b
  const long rowb = cu ? (long)cu[b] : (long)b * L;
  const int Lq = cu ? len : L;
  const int kblk0 = blockIdx.x * (64 * NF);
  auto load_ld = [&](int q0) -> float {  // thread t < 64: lse of query q0+t; 64 <= t < 128: delta
    const int qq = q0 + (tid & 63);
    if (tid >= 128) return 0.f;
    if (qq >= len) return tid < 64 ? INFINITY : 0.f;  // P = exp2(-inf) = 0, dS = 0: no query mask
    return tid < 64 ? lse[(long)bh * L + qq] : delta[(rowb + qq) * H + h];
  };
  const bf16_t* Qp = qkv + h * D;
  const bf16_t* Kp = qkv + H * D + h * D;
  const bf16_t* Vp = qkv + 2 * H * D + h * D;
  const bf16_t* dOp = dO + h * D;

  int keyv[NF];
  bool kval[NF];
  short8 kb[NF][D / 32], vb[NF][D / 32];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    keyv[f] = kblk0 + wave * (16 * NF) + f * 16 + (lane & 15);
    kval[f] = keyv[f] < len;
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      short8 kv = {0, 0, 0, 0, 0, 0, 0, 0}, vv = {0, 0, 0, 0, 0, 0, 0, 0};
      if (keyv[f] < Lq) {
        kv = *reinterpret_cast<const short8*>(Kp + (rowb + keyv[f]) * RS + s * 32 + 8 * g);
        vv = *reinterpret_cast<const short8*>(Vp + (rowb + keyv[f]) * RS + s * 32 + 8 * g);
      }
      kb[f][s] = kv;
      vb[f][s] = vv;
    }
  }
  float4v dk[NF][D / 16], dv[NF][D / 16];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int i = 0; i < D / 16; ++i) dk[f][i] = dv[f][i] = (float4v){0.f, 0.f, 0.f, 0.f};

  // fully masked key block -> zero grads; query rows >= len have zero output -> no contribution
  const int nqt = (kblk0 < len) ? (len + TQ - 1) / TQ : 0;
  short8 rq[D / 32], rd[D / 32];
  float rld = 0.f;
  if (nqt > 0) {
    load_tile<D>(Qp, rowb, min(TQ, len), RS, rq);
    load_tile<D>(dOp, rowb, min(TQ, len), OS, rd);
    rld = load_ld(0);
  }
  for (int qt = 0; qt < nqt; ++qt) {
    __syncthreads();
    store_row_img<D>(Qr, rq);
    if constexpr (!kUnified<D>) store_tr_img<D>(Qt, rq);
    store_row_img<D>(Dr, rd);
    if constexpr (!kUnified<D>) store_tr_img<D>(Dt, rd);
    if (tid < 128) Ls[tid] = rld;  // Ls[0..63] = lse, Ds = Ls + 64 = delta
    __syncthreads();
    if (qt + 1 < nqt) {
      const int q1 = (qt + 1) * TQ;
      load_tile<D>(Qp, rowb + q1, min(TQ, len - q1), RS, rq);
      load_tile<D>(dOp, rowb + q1, min(TQ, len - q1), OS, rd);
      rld = load_ld(q1);
    }
    float4v sp[NF][4], dp[NF][4];
#pragma unroll
    for (int qf = 0; qf < 4; ++qf) {
#pragma unroll
      for (int f = 0; f < NF; ++f) sp[f][qf] = dp[f][qf] = (float4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
        const short8 aq = *reinterpret_cast<const short8*>(Qr + row_off<D>(qf * 16 + (lane & 15), s * 4 + g));
        const short8 ad = *reinterpret_cast<const short8*>(Dr + row_off<D>(qf * 16 + (lane & 15), s * 4 + g));
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          sp[f][qf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, kb[f][s], sp[f][qf], 0, 0, 0);
          dp[f][qf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad, vb[f][s], dp[f][qf], 0, 0, 0);
        }
      }
    }
    // P = exp2(S*c - lse2[q]); dS = P * (dP - delta[q]); rows = queries qt*64 + qf*16 + 4g + r
#pragma unroll
    for (int qf = 0; qf < 4; ++qf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // key columns past len only feed their own (discarded) dK / dV column: no key mask
        const int ql = qf * 16 + 4 * g + r;
        const float nlq = -Ls[ql];
        const float dq = Ds[ql];
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const float pv = fast_exp2(fmaf(sp[f][qf][r], scale_log2, nlq));
          sp[f][qf][r] = pv;
          dp[f][qf][r] = pv * (dp[f][qf][r] - dq);
        }
      }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      short8 pb[NF], sb[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        pb[f] = pack8(sp[f][2 * hh], sp[f][2 * hh + 1]);
        sb[f] = pack8(dp[f][2 * hh], dp[f][2 * hh + 1]);
      }
#pragma unroll
      for (int df = 0; df < D / 16; ++df) {
        const short8 ado = tr_frag<D>(Dt, hh * 32, df * 16, lane);
        const short8 aq = tr_frag<D>(Qt, hh * 32, df * 16, lane);
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          dv[f][df] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ado, pb[f], dv[f][df], 0, 0, 0);
          dk[f][df] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, sb[f], dk[f][df], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    if (keyv[f] >= Lq) continue;
    bf16_t* dkp = dqkv + (rowb + keyv[f]) * RS + H * D + h * D;
    bf16_t* dvp = dqkv + (rowb + keyv[f]) * RS + 2 * H * D + h * D;
#pragma unroll
    for (int df = 0; df < D / 16; ++df) {
      short4v a, c;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = (short)f2bf(kval[f] ? dk[f][df][r] * scale : 0.f);
        c[r] = (short)f2bf(kval[f] ? dv[f][df][r] : 0.f);
      }
      *reinterpret_cast<short4v*>(dkp + df * 16 + 4 * g) = a;
      *reinterpret_cast<short4v*>(dvp + df * 16 + 4 * g) = c;
    }
  }
}

template <int NF, int MINB>
__global__ void __launch_bounds__(NT, MINB) attn_bwd_dkdv_dma_kernel(const bf16_t* __restrict__ qkv,
                                                           const int64_t* __restrict__ lens,
                                                           const int64_t* __restrict__ cu,
                                                           const bf16_t* __restrict__ dO, const float* __restrict__ lse,
                                                           const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
                                                           int L, int H, float scale_log2, float scale) {
  constexpr int D = 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // per buffer: Q image, dO image (unified swizzle, DMA'd), lse[64], delta[64]
  constexpr int BUFB = 2 * TQ * D * 2 + 2 * TQ * 4;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int RS = 3 * H * D, OS = H * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4;
  const int len = (int)lens[b];
  // packed variable-length rows (cu = row offsets): only rows < len exist for sequence b
  const long rowb = cu ? (long)cu[b] : (long)b * L;
  const int Lq = cu ? len : L;
  const int kblk0 = blockIdx.x * (64 * NF);
  auto load_ld = [&](int q0) -> float {  // thread t < 64: lse of query q0+t; 64 <= t < 128: delta
    const int qq = q0 + (tid & 63);
    if (tid >= 128) return 0.f;
    if (qq >= len) return tid < 64 ? INFINITY : 0.f;  // P = exp2(-inf) = 0, dS = 0: no query mask
    return tid < 64 ? lse[(long)bh * L + qq] : delta[(rowb + qq) * H + h];
  };
  const bf16_t* Qp = qkv + h * D;
  const bf16_t* Kp = qkv + H * D + h * D;
  const bf16_t* Vp = qkv + 2 * H * D + h * D;
  const bf16_t* dOp = dO + h * D;

  int keyv[NF];
  bool kval[NF];
  short8 kb[NF][D / 32], vb[NF][D / 32];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    keyv[f] = kblk0 + wave * (16 * NF) + f * 16 + (lane & 15);
    kval[f] = keyv[f] < len;
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      short8 kv = {0, 0, 0, 0, 0, 0, 0, 0}, vv = {0, 0, 0, 0, 0, 0, 0, 0};
      if (keyv[f] < Lq) {
        kv = *reinterpret_cast<const short8*>(Kp + (rowb + keyv[f]) * RS + s * 32 + 8 * g);
        vv = *reinterpret_cast<const short8*>(Vp + (rowb + keyv[f]) * RS + s * 32 + 8 * g);
      }
      kb[f][s] = kv;
      vb[f][s] = vv;
    }
  }
  float4v dk[NF][D / 16], dv[NF][D / 16];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int i = 0; i < D / 16; ++i) dk[f][i] = dv[f][i] = (float4v){0.f, 0.f, 0.f, 0.f};

  // fully masked key block -> zero grads; query rows >= len have zero output -> no contribution
  const int nqt = (kblk0 < len) ? (len + TQ - 1) / TQ : 0;
  const __amdgpu_buffer_rsrc_t rQ = seq_rsrc(Qp + rowb * RS, len, RS), rD = seq_rsrc(dOp + rowb * OS, len, OS);
  int voq[4], vod[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 4 + wave) * 4 + (lane >> 4);
    const int c = (lane & 15) ^ uni_h(row);
    voq[i] = (row * RS + c * 8) * 2;
    vod[i] = (row * OS + c * 8) * 2;
  }
  auto issue = [&](int q0, int buf) {
    char* Qd = smem + buf * BUFB;
    char* Dd = Qd + TQ * D * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      buf_lds16(rQ, voq[i], q0 * RS * 2, Qd + (i * 4 + wave) * 1024);
      buf_lds16(rD, vod[i], q0 * OS * 2, Dd + (i * 4 + wave) * 1024);
    }
  };
  auto stash_ld = [&](int buf, float v) {
    if (tid < 128) reinterpret_cast<float*>(smem + buf * BUFB + 2 * TQ * D * 2)[tid] = v;
  };
  if (nqt > 0) {
    issue(0, 0);
    stash_ld(0, load_ld(0));
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int qt = 0; qt < nqt; ++qt) {
    const int buf = qt & 1;
    float rld = 0.f;
    if (qt + 1 < nqt) {
      issue((qt + 1) * TQ, buf ^ 1);
      rld = load_ld((qt + 1) * TQ);
    }
    const char* Qr = smem + buf * BUFB;
    const char* Dr = Qr + TQ * D * 2;
    const char* Qt = Qr;  // unified swizzle: transposed reads from the same images
    const char* Dt = Dr;
    const float* Ls = reinterpret_cast<const float*>(Qr + 2 * TQ * D * 2);
    const float* Ds = Ls + TQ;
    float4v sp[NF][4], dp[NF][4];
#pragma unroll
    for (int qf = 0; qf < 4; ++qf) {
#pragma unroll
      for (int f = 0; f < NF; ++f) sp[f][qf] = dp[f][qf] = (float4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
        const short8 aq = *reinterpret_cast<const short8*>(Qr + row_off<D>(qf * 16 + (lane & 15), s * 4 + g));
        const short8 ad = *reinterpret_cast<const short8*>(Dr + row_off<D>(qf * 16 + (lane & 15), s * 4 + g));
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          sp[f][qf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, kb[f][s], sp[f][qf], 0, 0, 0);
          dp[f][qf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad, vb[f][s], dp[f][qf], 0, 0, 0);
        }
      }
    }
    // P = exp2(S*c - lse2[q]); dS = P * (dP - delta[q]); rows = queries qt*64 + qf*16 + 4g + r
#pragma unroll
    for (int qf = 0; qf < 4; ++qf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // key columns past len only feed their own (discarded) dK / dV column: no key mask
        const int ql = qf * 16 + 4 * g + r;
        const float nlq = -Ls[ql];
        const float dq = Ds[ql];
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const float pv = fast_exp2(fmaf(sp[f][qf][r], scale_log2, nlq));
          sp[f][qf][r] = pv;
          dp[f][qf][r] = pv * (dp[f][qf][r] - dq);
        }
      }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      short8 pb[NF], sb[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        pb[f] = pack8(sp[f][2 * hh], sp[f][2 * hh + 1]);
        sb[f] = pack8(dp[f][2 * hh], dp[f][2 * hh + 1]);
      }
#pragma unroll
      for (int df = 0; df < D / 16; ++df) {
        const short8 ado = tr_frag<D>(Dt, hh * 32, df * 16, lane);
        const short8 aq = tr_frag<D>(Qt, hh * 32, df * 16, lane);
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          dv[f][df] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ado, pb[f], dv[f][df], 0, 0, 0);
          dk[f][df] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, sb[f], dk[f][df], 0, 0, 0);
        }
      }
    }
    if (qt + 1 < nqt) stash_ld(buf ^ 1, rld);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    if (keyv[f] >= Lq) continue;
    bf16_t* dkp = dqkv + (rowb + keyv[f]) * RS + H * D + h * D;
    bf16_t* dvp = dqkv + (rowb + keyv[f]) * RS + 2 * H * D + h * D;
#pragma unroll
    for (int df = 0; df < D / 16; ++df) {
      short4v a, c;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = (short)f2bf(kval[f] ? dk[f][df][r] * scale : 0.f);
        c[r] = (short)f2bf(kval[f] ? dv[f][df][r] : 0.f);
      }
      *reinterpret_cast<short4v*>(dkp + df * 16 + 4 * g) = a;
      *reinterpret_cast<short4v*>(dvp + df * 16 + 4 * g) = c;
    }
  }
}

// NF = query fragments per wave; block = 4 waves x 16*NF queries
template <int D, int NF>
__global__ void __launch_bounds__(NT) attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv, const int64_t* __restrict__ lens,
                                                         const int64_t* __restrict__ cu,
                                                         const bf16_t* __restrict__ dO, const float* __restrict__ lse,
                                                         const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
                                                         int L, int H, float scale_log2, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kr = smem;
  char* Kt = kUnified<D> ? Kr : Kr + TK * D * 2;
  char* Vr = Kt + TK * D * 2;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int RS = 3 * H * D, OS = H * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int len = (int)lens[b];
  // packed variable-length rows (cu = row offsets): only rows < len exist for sequence b
  const long rowb = cu ? (long)cu[b] : (long)b * L;
  const int Lq = cu ? len : L;
  const bf16_t* Qp = qkv + h * D;
  const bf16_t* Kp = qkv + H * D + h * D;
  const bf16_t* Vp = qkv + 2 * H * D + h * D;

  int qv[NF];
  float lq[NF], dd[NF];
  short8 qf[NF][D / 32], df_[NF][D / 32];
  if (blockIdx.x * (64 * NF) >= len) {  // padded query block: dQ = 0
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int q = blockIdx.x * (64 * NF) + wave * (16 * NF) + f * 16 + (lane & 15);
      if (q >= Lq) continue;
      bf16_t* dqp = dqkv + (rowb + q) * RS + h * D;
#pragma unroll
      for (int df = 0; df < D / 16; ++df) *reinterpret_cast<short4v*>(dqp + df * 16 + 4 * g) = (short4v){0, 0, 0, 0};
    }
    return;
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    qv[f] = blockIdx.x * (64 * NF) + wave * (16 * NF) + f * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      short8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qv[f] < len) {
        a = *reinterpret_cast<const short8*>(Qp + (rowb + qv[f]) * RS + s * 32 + 8 * g);
        c = *reinterpret_cast<const short8*>(dO + (rowb + qv[f]) * OS + h * D + s * 32 + 8 * g);
      }
      qf[f][s] = a;
      df_[f][s] = c;
    }
    lq[f] = qv[f] < len ? lse[(long)bh * L + qv[f]] : 0.f;
    dd[f] = qv[f] < len ? delta[(rowb + qv[f]) * H + h] : 0.f;
  }
  float4v dq[NF][D / 16];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int i = 0; i < D / 16; ++i) dq[f][i] = (float4v){0.f, 0.f, 0.f, 0.f};

  const int nkt = (len + TK - 1) / TK;
  short8 rk[D / 32], rv[D / 32];
  if (nkt > 0) {
    load_tile<D>(Kp, rowb, min(TK, len), RS, rk);
    load_tile<D>(Vp, rowb, min(TK, len), RS, rv);
  }
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    store_row_img<D>(Kr, rk);
    if constexpr (!kUnified<D>) store_tr_img<D>(Kt, rk);
    store_row_img<D>(Vr, rv);
    __syncthreads();
    if (kt + 1 < nkt) {
      const int k1 = (kt + 1) * TK;
      load_tile<D>(Kp, rowb + k1, min(TK, len - k1), RS, rk);
      load_tile<D>(Vp, rowb + k1, min(TK, len - k1), RS, rv);
    }
    float4v st[NF][4], dpt[NF][4];
#pragma unroll
    for (int kf = 0; kf < 4; ++kf) {
#pragma unroll
      for (int f = 0; f < NF; ++f) st[f][kf] = dpt[f][kf] = (float4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
        const short8 ak = *reinterpret_cast<const short8*>(Kr + row_off<D>(kf * 16 + (lane & 15), s * 4 + g));
        const short8 av = *reinterpret_cast<const short8*>(Vr + row_off<D>(kf * 16 + (lane & 15), s * 4 + g));
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          st[f][kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, qf[f][s], st[f][kf], 0, 0, 0);
          dpt[f][kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, df_[f][s], dpt[f][kf], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // queries past len have zero Q / dO, lse = delta = 0 -> dS = 0: no query mask.  Keys past
        // len (zero K / V rows) are masked on the one tile that straddles len only: their dS
        // meets a zero K row, but exp2(-lse) could overflow for a row of very negative scores.
        if (kt * TK + TK > len && kt * TK + kf * 16 + 4 * g + r >= len) {
#pragma unroll
          for (int f = 0; f < NF; ++f) st[f][kf][r] = -INFINITY;
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const float pv = fast_exp2(fmaf(st[f][kf][r], scale_log2, -lq[f]));
          st[f][kf][r] = pv * (dpt[f][kf][r] - dd[f]);
        }
      }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      short8 sb[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) sb[f] = pack8(st[f][2 * hh], st[f][2 * hh + 1]);
#pragma unroll
      for (int df = 0; df < D / 16; ++df) {
        const short8 ak = tr_frag<D>(Kt, hh * 32, df * 16, lane);
#pragma unroll
        for (int f = 0; f < NF; ++f) dq[f][df] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, sb[f], dq[f][df], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    if (qv[f] >= Lq) continue;
    bf16_t* dqp = dqkv + (rowb + qv[f]) * RS + h * D;
#pragma unroll
    for (int df = 0; df < D / 16; ++df) {
      short4v a;
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = (short)f2bf(dq[f][df][r] * scale);
      *reinterpret_cast<short4v*>(dqp + df * 16 + 4 * g) = a;
    }
  }
}

template <int NF, int MINB>
__global__ void __launch_bounds__(NT, MINB) attn_bwd_dq_dma_kernel(const bf16_t* __restrict__ qkv, const int64_t* __restrict__ lens,
                                                         const int64_t* __restrict__ cu,
                                                         const bf16_t* __restrict__ dO, const float* __restrict__ lse,
                                                         const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
                                                         int L, int H, float scale_log2, float scale) {
  constexpr int D = 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (K, V) unified images, DMA'd
  constexpr int BUFB = 2 * TK * D * 2;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int RS = 3 * H * D, OS = H * D;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4;
  const int len = (int)lens[b];
  // packed variable-length rows (cu = row offsets): only rows < len exist for sequence b
  const long rowb = cu ? (long)cu[b] : (long)b * L;
  const int Lq = cu ? len : L;
  const bf16_t* Qp = qkv + h * D;
  const bf16_t* Kp = qkv + H * D + h * D;
  const bf16_t* Vp = qkv + 2 * H * D + h * D;

  int qv[NF];
  float lq[NF], dd[NF];
  short8 qf[NF][D / 32], df_[NF][D / 32];
  if (blockIdx.x * (64 * NF) >= len) {  // padded query block: dQ = 0
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int q = blockIdx.x * (64 * NF) + wave * (16 * NF) + f * 16 + (lane & 15);
      if (q >= Lq) continue;
      bf16_t* dqp = dqkv + (rowb + q) * RS + h * D;
#pragma unroll
      for (int df = 0; df < D / 16; ++df) *reinterpret_cast<short4v*>(dqp + df * 16 + 4 * g) = (short4v){0, 0, 0, 0};
    }
    return;
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    qv[f] = blockIdx.x * (64 * NF) + wave * (16 * NF) + f * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      short8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qv[f] < len) {
        a = *reinterpret_cast<const short8*>(Qp + (rowb + qv[f]) * RS + s * 32 + 8 * g);
        c = *reinterpret_cast<const short8*>(dO + (rowb + qv[f]) * OS + h * D + s * 32 + 8 * g);
      }
      qf[f][s] = a;
      df_[f][s] = c;
    }
    lq[f] = qv[f] < len ? lse[(long)bh * L + qv[f]] : 0.f;
    dd[f] = qv[f] < len ? delta[(rowb + qv[f]) * H + h] : 0.f;
  }
  float4v dq[NF][D / 16];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int i = 0; i < D / 16; ++i) dq[f][i] = (float4v){0.f, 0.f, 0.f, 0.f};

  const int nkt = (len + TK - 1) / TK;
  const __amdgpu_buffer_rsrc_t rK = seq_rsrc(Kp + rowb * RS, len, RS), rV = seq_rsrc(Vp + rowb * RS, len, RS);
  int voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 4 + wave) * 4 + (lane >> 4);
    voff[i] = (row * RS + ((lane & 15) ^ uni_h(row)) * 8) * 2;
  }
  auto issue = [&](int key0, int buf) {
    char* Kd = smem + buf * BUFB;
    char* Vd = Kd + TK * D * 2;
    const int soff = key0 * RS * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      buf_lds16(rK, voff[i], soff, Kd + (i * 4 + wave) * 1024);
      buf_lds16(rV, voff[i], soff, Vd + (i * 4 + wave) * 1024);
    }
  };
  if (nkt > 0) issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) issue((kt + 1) * TK, buf ^ 1);
    const char* Kr = smem + buf * BUFB;
    const char* Kt = Kr;
    const char* Vr = Kr + TK * D * 2;
    float4v st[NF][4], dpt[NF][4];
#pragma unroll
    for (int kf = 0; kf < 4; ++kf) {
#pragma unroll
      for (int f = 0; f < NF; ++f) st[f][kf] = dpt[f][kf] = (float4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
        const short8 ak = *reinterpret_cast<const short8*>(Kr + row_off<D>(kf * 16 + (lane & 15), s * 4 + g));
        const short8 av = *reinterpret_cast<const short8*>(Vr + row_off<D>(kf * 16 + (lane & 15), s * 4 + g));
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          st[f][kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, qf[f][s], st[f][kf], 0, 0, 0);
          dpt[f][kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, df_[f][s], dpt[f][kf], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // queries past len have zero Q / dO, lse = delta = 0 -> dS = 0: no query mask.  Keys past
        // len (zero K / V rows) are masked on the one tile that straddles len only: their dS
        // meets a zero K row, but exp2(-lse) could overflow for a row of very negative scores.
        if (kt * TK + TK > len && kt * TK + kf * 16 + 4 * g + r >= len) {
#pragma unroll
          for (int f = 0; f < NF; ++f) st[f][kf][r] = -INFINITY;
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const float pv = fast_exp2(fmaf(st[f][kf][r], scale_log2, -lq[f]));
          st[f][kf][r] = pv * (dpt[f][kf][r] - dd[f]);
        }
      }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      short8 sb[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) sb[f] = pack8(st[f][2 * hh], st[f][2 * hh + 1]);
#pragma unroll
      for (int df = 0; df < D / 16; ++df) {
        const short8 ak = tr_frag<D>(Kt, hh * 32, df * 16, lane);
#pragma unroll
        for (int f = 0; f < NF; ++f) dq[f][df] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, sb[f], dq[f][df], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    if (qv[f] >= Lq) continue;
    bf16_t* dqp = dqkv + (rowb + qv[f]) * RS + h * D;
#pragma unroll
    for (int df = 0; df < D / 16; ++df) {
      short4v a;
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = (short)f2bf(dq[f][df][r] * scale);
      *reinterpret_cast<short4v*>(dqp + df * 16 + 4 * g) = a;
    }
  }
}

}  // namespace

// NF (fragments per wave) chosen from measurement on MI355X: the forward keeps 2 waves/SIMD
// with NF = 1; the D >= 64 backward is LDS-read bound and gains from NF = 2.
static int g_nf32_fwd = 2, g_nf32_bwd = 2;  // D = 32 (reference encoder, 8 heads): measured NF=2 -6 % fwd, -2 % bwd vs 1; 4 spills
SSAMD_API void ssamd_attn_set_nf32(int fwd, int bwd) {
  g_nf32_fwd = fwd;
  g_nf32_bwd = bwd;
}
#define ATTN_DISPATCH(D, FWD, ...)                                                                 \
  switch (D) {                                                                                     \
    case 32: {                                                                                     \
      constexpr int DD = 32;                                                                       \
      const int nf32 = FWD ? g_nf32_fwd : g_nf32_bwd;                                              \
      if (nf32 == 4) { constexpr int NF = 4; __VA_ARGS__; }                                         \
      else if (nf32 == 2) { constexpr int NF = 2; __VA_ARGS__; }                                    \
      else { constexpr int NF = 1; __VA_ARGS__; }                                                   \
      break;                                                                                       \
    }                                                                                              \
    case 64: { constexpr int DD = 64; constexpr int NF = FWD ? 1 : 2; __VA_ARGS__; break; }       \
    case 128: { constexpr int DD = 128; constexpr int NF = FWD ? 1 : 2; __VA_ARGS__; break; }     \
    default: return -1;                                                                            \
  }

static const float kLog2e = 1.4426950408889634f;
static int g_fwd_dma = 1, g_fwd_nf = 2;  // measured (L=800, D=128): DMA NF=2 at 2 waves/SIMD 0.169 ms, DMA NF=1 0.227, registers 0.222
SSAMD_API void ssamd_attn_set_fwd(int dma, int nf) {
  g_fwd_dma = dma;
  g_fwd_nf = nf;
}
static int g_nf_kv = 1, g_nf_q = 2;  // measured (D=128, L=800): LDS-DMA dK/dV NF=1 (2 waves/SIMD), LDS-DMA dQ NF=2: bwd 0.599 ms (from 0.793)
static int g_kv_dma = 1, g_q_dma = 1;
SSAMD_API void ssamd_attn_set_kv_dma(int v) { g_kv_dma = v; }
SSAMD_API void ssamd_attn_set_q_dma(int v, int nf) {
  g_q_dma = v;
  g_nf_q = nf;
}  // measured on MI355X (D=128): dK/dV NF=2, dQ NF=1 -> -14 %
SSAMD_API void ssamd_attn_set_nf(int nf_kv, int nf_q) {
  g_nf_kv = nf_kv;
  g_nf_q = nf_q;
}

template <int DD, int NF>
static void launch_dkdv(const bf16_t* qkv, const int64_t* lens, const int64_t* cu, const bf16_t* dO, const float* lse,
                        const float* delta, bf16_t* dqkv, int B, int L, int H, float scale, hipStream_t s) {
  dim3 grid(cdiv(L, 64 * NF), B * H);
  constexpr size_t lds_kv = (kUnified<DD> ? 2 : 4) * TQ * DD * 2 + 2 * TQ * 4;
  static const bool lds_once = (allow_lds(attn_bwd_dkdv_kernel<DD, NF>, lds_kv), true);
  (void)lds_once;
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<DD, NF>), grid, dim3(NT), lds_kv, s, qkv, lens, cu, dO, lse, delta, dqkv, L,
                     H, scale * kLog2e, scale);
}

template <int DD, int NF>
static void launch_dq(const bf16_t* qkv, const int64_t* lens, const int64_t* cu, const bf16_t* dO, const float* lse,
                      const float* delta, bf16_t* dqkv, int B, int L, int H, float scale, hipStream_t s) {
  dim3 grid(cdiv(L, 64 * NF), B * H);
  hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, NF>), grid, dim3(NT), (kUnified<DD> ? 2 : 3) * TK * DD * 2, s, qkv, lens,
                     cu, dO, lse, delta, dqkv, L, H, scale * kLog2e, scale);
}

// cu (optional): packed rows, sequence b = rows cu[b] .. cu[b]+lens[b]-1; L = longest sequence.
SSAMD_API int ssamd_attn_fwd(const bf16_t* qkv, const int64_t* lens, const int64_t* cu, bf16_t* out, float* lse, int B,
                             int L, int H, int D, float scale, hipStream_t s) {
  if ((long)B * L == 0) return 0;
  if (D == 128 && g_fwd_dma) {  // LDS-DMA K/V tiles, NF query fragments per wave
    if (g_fwd_nf == 2) {
      dim3 grid(cdiv(L, 128), B * H);
      hipLaunchKernelGGL((attn_fwd_dma_kernel<2>), grid, dim3(NT), 4 * TK * 128 * 2, s, qkv, lens, cu, out, lse, L,
                         H, scale * kLog2e);
    } else {
      dim3 grid(cdiv(L, 64), B * H);
      hipLaunchKernelGGL((attn_fwd_dma_kernel<1>), grid, dim3(NT), 4 * TK * 128 * 2, s, qkv, lens, cu, out, lse, L,
                         H, scale * kLog2e);
    }
    return (int)hipGetLastError();
  }
  ATTN_DISPATCH(D, true, {
    dim3 grid(cdiv(L, 64 * NF), B * H);
    hipLaunchKernelGGL((attn_fwd_kernel<DD, NF>), grid, dim3(NT), 0, s, qkv, lens, cu, out, lse, L, H,
                       scale * kLog2e);
  });
  return (int)hipGetLastError();
}

// lse: [B, H, L] log2-domain; delta workspace: [rows*H] fp32 (rows = B*L, or the packed row count)
SSAMD_API int ssamd_attn_bwd(const bf16_t* qkv, const int64_t* lens, const int64_t* cu, const bf16_t* o,
                             const float* lse, const bf16_t* dO, bf16_t* dqkv, float* delta, long rows, int B, int L,
                             int H, int D, float scale, hipStream_t s) {
  if ((long)B * L == 0 || rows == 0) return 0;
  hipLaunchKernelGGL(attn_delta_kernel, dim3(cdiv(rows * H * (D / 8), NT)), dim3(NT), 0, s, o, dO, delta, rows, H, D);
  if (D == 128) {  // fragments per wave of the two kernels: runtime-tunable (measured defaults)
    if (g_kv_dma) {
      constexpr size_t lds = 2 * (2 * TQ * 128 * 2 + 2 * TQ * 4);
      if (g_nf_kv == 1) {
        static const bool once1 = (allow_lds(attn_bwd_dkdv_dma_kernel<1, 2>, lds), true);
        (void)once1;
        hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<1, 2>), dim3(cdiv(L, 64), B * H), dim3(NT), lds, s, qkv, lens,
                           cu, dO, lse, delta, dqkv, L, H, scale * kLog2e, scale);
      } else {
        static const bool once2 = (allow_lds(attn_bwd_dkdv_dma_kernel<2, 1>, lds), true);
        (void)once2;
        hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<2, 1>), dim3(cdiv(L, 128), B * H), dim3(NT), lds, s, qkv, lens,
                           cu, dO, lse, delta, dqkv, L, H, scale * kLog2e, scale);
      }
    } else if (g_nf_kv == 1) launch_dkdv<128, 1>(qkv, lens, cu, dO, lse, delta, dqkv, B, L, H, scale, s);
    else launch_dkdv<128, 2>(qkv, lens, cu, dO, lse, delta, dqkv, B, L, H, scale, s);
    if (g_q_dma) {
      constexpr size_t lds = 2 * 2 * TK * 128 * 2;  // 64 KiB
      if (g_nf_q == 1)
        hipLaunchKernelGGL((attn_bwd_dq_dma_kernel<1, 2>), dim3(cdiv(L, 64), B * H), dim3(NT), lds, s, qkv, lens, cu,
                           dO, lse, delta, dqkv, L, H, scale * kLog2e, scale);
      else
        hipLaunchKernelGGL((attn_bwd_dq_dma_kernel<2, 2>), dim3(cdiv(L, 128), B * H), dim3(NT), lds, s, qkv, lens,
                           cu, dO, lse, delta, dqkv, L, H, scale * kLog2e, scale);
    } else if (g_nf_q == 1) launch_dq<128, 1>(qkv, lens, cu, dO, lse, delta, dqkv, B, L, H, scale, s);
    else launch_dq<128, 2>(qkv, lens, cu, dO, lse, delta, dqkv, B, L, H, scale, s);
  } else {
    ATTN_DISPATCH(D, false, {
      launch_dkdv<DD, NF>(qkv, lens, cu, dO, lse, delta, dqkv, B, L, H, scale, s);
      launch_dq<DD, NF>(qkv, lens, cu, dO, lse, delta, dqkv, B, L, H, scale, s);
    });
  }
  return (int)hipGetLastError();
}
