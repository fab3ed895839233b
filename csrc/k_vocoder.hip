// HiFi-GAN MRF residual layer, fused (reference hifigan/models.py:20-103 ResBlock1):
//
//     y = x + conv2( lrelu( conv1_d( lrelu(x) ) + b1 ) ) + b2          [channel-last, C channels]
//     out = (acc_in + y) * out_scale   (optional: the MRF branch sum / mean, in place)
//     [-> lrelu(out): the next upsampling conv's input activation, when post_lrelu]
//
// for the high-rate stages (C = 32 / 64 / 128 at 256 / 128 / 64x the mel rate), where a generic
// GEMM tile wastes N width and every separate lrelu / add pass re-streams GBs of activations.
// One workgroup (4 waves; 8 for C = 128) owns BM (~118-250, see RB) output rows of one utterance:
//   1. stage lrelu(x) for the rows both convs need (halo d*(K-1)/2 + (K-1)/2 each side, zero
//      outside [0, T)) into LDS;
//   2. conv1 (dilation d) for BM + K-1 rows on v_mfma_f32_16x16x32_bf16: A fragments from the
//      LDS tile at row offset tap*d, B fragments (weights [C][K][C], L2-resident, shared by all
//      blocks) DMA-staged per (tap, 32-deep chunk) into an LDS ring; + b1, lrelu, zero outside
//      [0, T) -> t1 tile in LDS (bf16);
//   3. conv2 (dilation 1) over the t1 tile, + b2 -> fp32 tile in LDS (aliases the x tile);
//   4. coalesced 16-B epilogue: + x (residual), + acc_in, * out_scale -> out.
// Each activation byte is read once (plus the halo) and written once per layer: the unfused
// path (lrelu, conv, lrelu-epilogue conv, add) moves ~4x more.
#include "common.h"

namespace {

constexpr int MAXD = 5;

// Work split: NW waves = WR (row groups) x WC (column groups); each wave owns RPW 16-row blocks
// x NSW 16-column sub-tiles, so a 32-deep step costs RPW + NSW ds_read_b128 for RPW * NSW MFMAs
// (C = 128: 2 + 4 reads / 8 MFMAs, under the LDS array's 1 read per 16-cycle MFMA at 2 waves per
// SIMD).  The output tile BM = 16 * RPW * WR - (K - 1) is chosen so that conv1's BM + K - 1 rows
// fill the row blocks exactly (no straggler block on one wave).
// (Measured and lost: C = 128 at one wave per SIMD with a 64 x 64 wave tile -- 8 fragment reads per 16
// MFMAs instead of 6 per 8 -- K = 7 5.25 -> 5.85 ms, K = 3 3.47 -> 4.00 ms: the second wave per SIMD
// hides more than the saved LDS reads.)
// BIG_ (the "tall" per-layer tile, resblock_layer_tall_kernel): 8 waves of 64 x 64 (RPW_ = 4 row blocks x 4
// sub-tiles), 8 fragment reads per 16 MFMAs instead of 6 per 8 -- the LDS-read-bound conv loop moves 1/3 fewer bytes
// per MFMA and the weight slices are staged once per 256 (C = 128) / 512 (C = 64) rows instead of per 128 / 64.  The
// x tile, the t1 tile and the fp32 output tile share one LDS region (each is dead before the next is written:
// extra barriers after each conv), the weight ring sits behind the x tile.
// NW_ (> 0): waves per block of a tall tile -- 4 gives the "half" tall block (the same 64 x 64 wave tile on half the
// rows and LDS), two of which share a CU so one block's staging / epilogue phases run under the other's MFMAs
template <int C_, int K_, int RPW_ = 2, bool BIG_ = false, int NW_ = 0>
struct RB {
  static constexpr int C = C_;
  static constexpr int K = K_;
  static constexpr bool BIG = BIG_;
  static constexpr int NW = NW_ > 0 ? NW_ : (BIG ? 8 : (C >= 128 ? 8 : 4));  // waves per block
  static constexpr int NT = 64 * NW;
  // column groups: 64 columns per wave in the tall tile (C = 256: 4 x 2 waves), else 2 groups from C = 128 up
  static constexpr int WC = BIG ? (C >= 64 ? C / 64 : 1) : (C >= 128 ? 2 : 1);
  static constexpr int WR = NW / WC;                // row groups
  static constexpr int RPW = RPW_;                  // row blocks per wave
  static constexpr int H2 = (K - 1) / 2;
  static constexpr int NRB1 = RPW * WR;             // conv1 row blocks
  static constexpr int R1P = NRB1 * 16;             // t1 rows (= R1: no padding)
  static constexpr int R1 = R1P;
  static constexpr int BM = R1 - 2 * H2;            // output rows per block
  static constexpr int NRB2 = (BM + 15) / 16;
  // LDS pitch (bf16) of the activation tiles: the A-fragment ds_read_b128 of lane l reads row l & 15 at
  // 16-B column chunk l >> 4, so its bank quad is (p * row + chunk) mod 16 for a pitch of 4p dwords.
  // The b128 lane groups ({0-3,12-15,20-27}, ...) hit 16 distinct quads iff p = 2 (mod 4), i.e. a pitch
  // of C + 16 bf16 for C = 32 / 64 / 128 (p = 6 / 10 / 18).  C + 8 (p odd) left a 2-way conflict in
  // every group: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 0.40-0.48 (profiles/r2_v2_pmc_step_summary.txt).
  static constexpr int LDC = C + 16;
  static constexpr int RX = R1P + (K - 1) * MAXD;  // staged x rows at the largest dilation
  static constexpr int NS = C / 16;                // 16-wide output sub-tiles
  static constexpr int NSW = NS / WC;              // sub-tiles per wave
  static constexpr int KC = C / 32;                // 32-deep K chunks per tap
  // 32-deep chunks per pipeline step (one barrier each); the tall tile keeps one (its 64 x 64 wave tile already
  // holds 64 accumulator VGPRs and 8 fragments per chunk and buffer)
  static constexpr int KC2 = (KC >= 2 && !BIG) ? 2 : 1;
  static constexpr int SLOT = KC2 * C * 64;        // ring slot: KC2 sub-slices [C][32] bf16
  static constexpr int XS_BYTES = RX * LDC * 2;
  static constexpr int OSP = C + 4;                // fp32 output-tile pitch (skewed banks)
  static constexpr int OUT_BYTES = NRB2 * 16 * OSP * 4;
  static constexpr int R0_BYTES = ((XS_BYTES > OUT_BYTES ? XS_BYTES : OUT_BYTES) + 15) / 16 * 16;
  static constexpr int T1_BYTES = R1P * LDC * 2;
  // BIG: x / t1 / fp32 output alias one region, the ring behind the x tile
  static constexpr int XS16 = (XS_BYTES + 15) / 16 * 16;
  static constexpr int RING_OFF = BIG ? XS16 : R0_BYTES + T1_BYTES;
  static constexpr int LDS_BIG = (XS16 + 3 * SLOT > OUT_BYTES ? XS16 + 3 * SLOT : OUT_BYTES);
  static constexpr int LDS = BIG ? LDS_BIG : R0_BYTES + T1_BYTES + 3 * SLOT;  // + the weight-slice ring
  static constexpr int MAXRB = RPW;
  static_assert(NRB2 <= NRB1 && LDS <= 160 * 1024, "resblock tile");
  static_assert(!BIG || T1_BYTES <= XS16, "t1 aliases the x tile");
};
template <int C, int K>
using RBT = RB<C, K, 4, true>;  // the tall tile
template <int C, int K>
using RBH = RB<C, K, 4, true, 4>;  // the half tall block (two per CU)

__device__ __forceinline__ float lrelu(float v, float s) { return v >= 0.f ? v : v * s; }

// acc[r][s] = sum over (tap, 32-deep chunk) of A(src rows rb*16 + tap*row_step) * W[:, tap, chunk].
// Weight fragments are staged per step into a 3-slot LDS ring by LDS-DMA (global_load_lds: one
// 16-B chunk per lane, no VGPR round trip), three steps ahead, so the waves share one copy
// of each weight slice (NWx less L2->CU traffic than per-wave loads) and its latency is hidden.
// Slot layout: [C rows (output channel)][32 k] bf16 = 64-B rows with the 16-B chunk index XORed
// by 2 * ((row >> 2) & 1) (source-side swizzle; the DMA image is lane-linear): lane (col, quad) of a
// B-fragment ds_read_b128 then hits bank quad 4 * (row mod 4) + chunk, distinct within each of the
// instruction's four 16-lane groups ({0-3,12-15,20-27}, ...; found by exhaustive search over XOR
// swizzles -- the earlier (row >> 2) & 3 left a 2-way conflict in every group).
__device__ __forceinline__ void glds16(const void* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// DMA pieces per thread and pipeline step (vmcnt bookkeeping of conv_tile)
template <class R>
constexpr int rb_dps() {
  return R::KC2 * (R::C * 4 > R::NT ? R::C * 4 / R::NT : 1);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

// Where a tile's rows live.  Padded batches [B, Tp, C]: tile = b * tiles + i, rows [i * BM, ...) of sequence b.
// Packed batches (the length-exact vocoder path, models/hifigan.py ``Generator.infer_packed``): every sequence's
// rows are contiguous in one [R, C] buffer and the host-built tile table tt[tile] = {first row of the sequence,
// its length, t0, sequence index} -- tiles never straddle two sequences, and every conv zero-pads at the
// sequence's own ends exactly as it does at the ends of a padded row.
struct TileGeo {
  long off;  // first row of the tile's sequence
  int T;     // rows of the sequence
  int t0;    // first output row of the tile within the sequence
};

__device__ __forceinline__ TileGeo tile_geo(const int4* __restrict__ tt, int tile, int tiles, int Tp, int BM) {
  TileGeo g;
  if (tt) {
    const int4 e = tt[tile];
    g.off = e.x;
    g.T = e.y;
    g.t0 = e.z;
  } else {
    const int b = tile / tiles;
    g.off = (long)b * Tp;
    g.T = Tp;
    g.t0 = (tile - b * tiles) * BM;
  }
  return g;
}

template <class R>
__device__ __forceinline__ void stage_b(const bf16_t* __restrict__ w, int step, char* slot, int tid, int wave) {
  constexpr int C = R::C, K = R::K;
  constexpr int CHUNKS = C * 4;  // 16-B chunks per [C][32] sub-slice
  constexpr int REP = CHUNKS > R::NT ? CHUNKS / R::NT : 1;
  static_assert(CHUNKS <= R::NT || CHUNKS % R::NT == 0, "slice chunks over the block");
  if (wave * 64 < CHUNKS) {      // wave-uniform
    const int c0 = step * R::KC2, tap = c0 / R::KC, kc = c0 - tap * R::KC;
#pragma unroll
    for (int q = 0; q < REP; ++q) {
      const int t = tid + q * R::NT;
      const int n = t >> 2, p = t & 3;
      const int lc = p ^ (((n >> 2) & 1) << 1);  // logical chunk stored at physical chunk p (see conv_tile)
#pragma unroll
      for (int j = 0; j < R::KC2; ++j)
        glds16(w + (n * K + tap) * C + (kc + j) * 32 + 8 * lc, slot + j * C * 64 + (wave + q * R::NW) * 1024);
    }
  }
}

template <class R>
__device__ __forceinline__ void conv_tile(const bf16_t* __restrict__ src, int row_step, const bf16_t* __restrict__ w,
                                          char* bring, int nrb, int wave, int tid,
                                          float4v (&acc)[R::MAXRB][R::NSW]) {
  constexpr int C = R::C, K = R::K;
  constexpr int STEPS = K * R::KC / R::KC2;
  constexpr int SLOT = R::SLOT;
  const int lane = tid & 63, col = lane & 15, quad = lane >> 4;
#pragma unroll
  for (int r = 0; r < R::MAXRB; ++r)
#pragma unroll
    for (int s = 0; s < R::NSW; ++s) acc[r][s] = float4v{0.f, 0.f, 0.f, 0.f};
  const int wr = wave % R::WR, wc = wave / R::WR;
  // Ring: slot j % 3 holds step j.  DMA runs three steps ahead of the MFMAs and the fragments of
  // step+1 are read into registers while step's MFMAs run, so one barrier per step only has to
  // cover "slot step+1 landed" and "everyone is done reading slot step" (re-filled with step+3).
  stage_b<R>(w, 0, bring, tid, wave);
  if (STEPS > 1) stage_b<R>(w, 1, bring + SLOT, tid, wave);
  if (STEPS > 2) stage_b<R>(w, 2, bring + 2 * SLOT, tid, wave);
  // (vmcnt counts this thread's DMA pieces: DPS per step)
  constexpr int DPS = rb_dps<R>();
  if constexpr (STEPS > 2) wait_vm<2 * DPS>();
  else if constexpr (STEPS > 1) wait_vm<DPS>();
  else wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  const bf16_t* arow = src + (wr * 16 + col) * R::LDC + 8 * quad;  // row block wr + WR*r
  // B-fragment read offsets (bytes) within a slot, per 16-column sub-tile of this wave
  int boff[R::NSW];
#pragma unroll
  for (int s = 0; s < R::NSW; ++s) {
    const int n = (wc * R::NSW + s) * 16 + col;
    boff[s] = n * 64 + ((quad ^ (((n >> 2) & 1) << 1)) << 4);
  }
  short8 a[2][R::KC2][R::MAXRB], bf[2][R::KC2][R::NSW];
  auto load = [&](int step, int buf) {
    const int c0 = step * R::KC2, tap = c0 / R::KC, kc = c0 - tap * R::KC;
#pragma unroll
    for (int j = 0; j < R::KC2; ++j) {
      const bf16_t* ap = arow + tap * row_step * R::LDC + (kc + j) * 32;
      const char* bs = bring + (step % 3) * SLOT + j * C * 64;
#pragma unroll
      for (int s = 0; s < R::NSW; ++s) bf[buf][j][s] = *reinterpret_cast<const short8*>(bs + boff[s]);
#pragma unroll
      for (int r = 0; r < R::MAXRB; ++r)
        if (wr + R::WR * r < nrb) a[buf][j][r] = *reinterpret_cast<const short8*>(ap + r * R::WR * 16 * R::LDC);
    }
  };
  load(0, 0);
#pragma unroll
  for (int step = 0; step < STEPS; ++step) {
    const int cur = step & 1;
    if (step + 1 < STEPS) {
      if (step + 2 < STEPS) wait_vm_lgkm0<DPS>();
      else wait_vm_lgkm0<0>();
      __builtin_amdgcn_s_barrier();
      if (step + 3 < STEPS) stage_b<R>(w, step + 3, bring + (step % 3) * SLOT, tid, wave);
      load(step + 1, cur ^ 1);
    }
#pragma unroll
    for (int r = 0; r < R::MAXRB; ++r) {
      if (wr + R::WR * r < nrb) {
#pragma unroll
        for (int j = 0; j < R::KC2; ++j)
#pragma unroll
          for (int s = 0; s < R::NSW; ++s)
            acc[r][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cur][j][r], bf[cur][j][s], acc[r][s], 0, 0, 0);
      }
    }
  }
  // the caller's next phase re-uses the ring / tiles only after its own __syncthreads
}

// PROF (diagnostic instantiation, ssamd_resblock_layer_prof): wave 0 stamps s_memtime at the phase
// boundaries (start, x staged, conv1 done, t1 staged, conv2 done, output tile staged, stores issued) into
// prof[block][8]; the production instantiation compiles no stamp.
template <bool PROF>
__device__ __forceinline__ void rb_stamp(unsigned long long* st, int i) {
  if constexpr (PROF) {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    st[i] = t;
  }
}

// Persistent over tiles (tile = blockIdx.x + k * gridDim.x; the grid is the resident-block count): at C = 128
// one 150-KiB block owns a CU, so nothing hid the x tile's global round trip (12 % of a block,
// profiles/r5_resblock_phases.txt).  The next tile's x rows are fetched into registers right after conv2
// (no DMA of conv_tile is in flight any more), under the output staging and the epilogue's own loads, and
// the barriers of that span order LDS only (__syncthreads would drain the fetch: vmcnt counts it).
// Synthesis RTF -1.2..-2.8 % same-box (profiles/r5_ab_rb_persistent.txt).
template <class R, bool PROF = false>
__global__ void __launch_bounds__((R::NT)) resblock_layer_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w1,
                                                            const float* __restrict__ b1, const bf16_t* __restrict__ w2,
                                                            const float* __restrict__ b2, const bf16_t* acc_in,
                                                            bf16_t* out, int Tp, int tiles, int ntiles, int d, float slope,
                                                            float out_scale, int post_lrelu,
                                                            const int4* __restrict__ tt,
                                                            unsigned long long* __restrict__ prof = nullptr) {
  constexpr int C = R::C, K = R::K;
  unsigned long long st[8];
  constexpr int NT = R::NT;
  constexpr int CH = C / 8;                                  // 16-B chunks per row
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(lds);               // [RX][LDC]   lrelu(x) tile
  float* os = reinterpret_cast<float*>(lds);                 // [NRB2*16][OSP] conv2 + b2 (after conv1)
  // [R1P][LDC]  lrelu(conv1 + b1): its own region, or (BIG) over the dead x tile
  bf16_t* t1 = reinterpret_cast<bf16_t*>(lds + (R::BIG ? 0 : R::R0_BYTES));
  char* bring = reinterpret_cast<char*>(lds + R::RING_OFF);  // 3 x [C][32] weight slices
  const int tid0 = threadIdx.x;
  const int h1 = d * (K - 1) / 2;
  // both convs' bias columns of this lane (they depend on the sub-tile s only): loaded up front, not as
  // one exposed L2 round trip per (row block, sub-tile) between the two convolutions
  float bias1[R::NSW], bias2[R::NSW];
#pragma unroll
  for (int s = 0; s < R::NSW; ++s) {
    const int ch = ((tid0 >> 6) / R::WR * R::NSW + s) * 16 + (tid0 & 15);
    bias1[s] = b1[ch];
    bias2[s] = b2[ch];
  }
  constexpr int IX = (R::RX * CH + NT - 1) / NT;
  const int rows_x = R::R1P + (K - 1) * d;
  short8 v[IX];
  // x rows [t0 - h1 - H2, ...) of a tile into v (zero outside [0, T))
  auto fetch_x = [&](int tile, int tid) {
    const TileGeo gq = tile_geo(tt, tile, tiles, Tp, R::BM);
    const int T = gq.T, t0 = gq.t0;
    const bf16_t* xb = x + gq.off * C;
#pragma unroll
    for (int it = 0; it < IX; ++it) {
      const int q = tid + it * NT, r = q / CH, c0 = (q - r * CH) * 8;
      const int t = t0 - h1 - R::H2 + r;
      if (r < rows_x && t >= 0 && t < T) {
        v[it] = *reinterpret_cast<const short8*>(xb + (long)t * C + c0);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[it][i] = 0;
      }
    }
  };
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  fetch_x(blockIdx.x, tid0);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // the thread index re-derived opaquely per tile: otherwise both unrolled convolutions' per-lane address
    // terms are hoisted out of the tile loop and stay live across it (256 VGPRs + spills vs 152)
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, col = lane & 15, quad = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: row-block tests are scalar
    const int wr = wave % R::WR, wc = wave / R::WR;
    const TileGeo gt = tile_geo(tt, tile, tiles, Tp, R::BM);
    const int T = gt.T, t0 = gt.t0;
    const bf16_t* xb = x + gt.off * C;
    rb_stamp<PROF>(st, 0);

    // 1. lrelu(x) -> LDS
#pragma unroll
    for (int it = 0; it < IX; ++it) {
      const int q = tid + it * NT, r = q / CH, c0 = (q - r * CH) * 8;
      if (r < rows_x) {
        short8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (short)f2bf(lrelu(bf2f((bf16_t)v[it][i]), slope));
        *reinterpret_cast<short8*>(xs + r * R::LDC + c0) = o;
      }
    }
    __syncthreads();
    rb_stamp<PROF>(st, 1);

    // 2. conv1 (dilation d): t1 row i <- x rows i + tap*d
    float4v acc[R::MAXRB][R::NSW];
    conv_tile<R>(xs, d, w1, bring, R::NRB1, wave, tid, acc);
    rb_stamp<PROF>(st, 2);
    if constexpr (R::BIG) __syncthreads();  // every wave done reading x: t1 overwrites it
#pragma unroll
    for (int r = 0; r < R::MAXRB; ++r) {
      const int rb = wr + R::WR * r;
      if (rb < R::NRB1) {
#pragma unroll
        for (int s = 0; s < R::NSW; ++s) {
          const int ch = (wc * R::NSW + s) * 16 + col;
          const float bias = bias1[s];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = rb * 16 + 4 * quad + i;
            const int t = t0 - R::H2 + row;
            const float v1 = (row < R::R1 && t >= 0 && t < T) ? lrelu(acc[r][s][i] + bias, slope) : 0.f;
            t1[row * R::LDC + ch] = f2bf(v1);
          }
        }
      }
    }
    __syncthreads();  // t1 complete; the x tile is dead from here on (os aliases it)
    rb_stamp<PROF>(st, 3);

    // 3. conv2 (dilation 1): out row j <- t1 rows j + tap
    conv_tile<R>(t1, 1, w2, bring, R::NRB2, wave, tid, acc);
    rb_stamp<PROF>(st, 4);
    const int nxt = tile + gridDim.x;
    if (nxt < ntiles) fetch_x(nxt, tid);
    // BIG: the output tile overwrites t1 and the ring -- wait for every wave's last conv2 reads (LDS order only:
    // a full __syncthreads would also drain the next tile's fetch)
    if constexpr (R::BIG) lds_barrier();
    // the epilogue's residual / accumulator rows, issued before the output staging
    constexpr int BM = R::BM;
    constexpr int IE = (BM * CH + NT - 1) / NT;
    bf16_t* ob = out + gt.off * C;
    const bf16_t* ab = acc_in ? acc_in + gt.off * C : nullptr;
    // (BIG: the residual rows are read inside the store loop, after the staging -- the 64-VGPR accumulators, the
    // next tile's x and a whole tile of residual rows do not fit in 256 registers together)
    constexpr int IEP = R::BIG ? 1 : IE;
    short8 xr[IEP], ar[IEP];
    if constexpr (!R::BIG) {
#pragma unroll
      for (int it = 0; it < IE; ++it) {
        const int q = tid + it * NT, j = q / CH, c0 = (q - j * CH) * 8;
        const int t = t0 + j;
        if (j < BM && t < T) {
          xr[it] = *reinterpret_cast<const short8*>(xb + (long)t * C + c0);
          if (ab) ar[it] = *reinterpret_cast<const short8*>(ab + (long)t * C + c0);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R::MAXRB; ++r) {
      const int rb = wr + R::WR * r;
      if (rb < R::NRB2) {
#pragma unroll
        for (int s = 0; s < R::NSW; ++s) {
          const int ch = (wc * R::NSW + s) * 16 + col;
          const float bias = bias2[s];
#pragma unroll
          for (int i = 0; i < 4; ++i) os[(rb * 16 + 4 * quad + i) * R::OSP + ch] = acc[r][s][i] + bias;
        }
      }
    }
    lds_barrier();
    rb_stamp<PROF>(st, 5);

    // 4. + residual (+ MRF accumulator), scale, coalesced 16-B stores
#pragma unroll
    for (int it = 0; it < IE; ++it) {
      const int q = tid + it * NT, j = q / CH, c0 = (q - j * CH) * 8;
      const int t = t0 + j;
      if (j >= BM || t >= T) continue;
      short8 xv, av;
      if constexpr (R::BIG) {
        xv = *reinterpret_cast<const short8*>(xb + (long)t * C + c0);
        if (ab) av = *reinterpret_cast<const short8*>(ab + (long)t * C + c0);
      } else {
        xv = xr[it];
        if (ab) av = ar[it];
      }
      const float4 o0 = *reinterpret_cast<const float4*>(os + j * R::OSP + c0);
      const float4 o1 = *reinterpret_cast<const float4*>(os + j * R::OSP + c0 + 4);
      const float ov[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
      short8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float y = ov[i] + bf2f((bf16_t)xv[i]);
        if (ab) y += bf2f((bf16_t)av[i]);
        y *= out_scale;
        if (post_lrelu) y = lrelu(y, slope);  // the next upsampling conv's pre-activation
        o[i] = (short)f2bf(y);
      }
      *reinterpret_cast<short8*>(ob + (long)t * C + c0) = o;
    }
    if constexpr (PROF) {
      rb_stamp<PROF>(st, 6);
      if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < 7; ++i) prof[(long)tile * 8 + i] = st[i];
        prof[(long)tile * 8 + 7] = __builtin_amdgcn_s_memrealtime();
      }
    }
    lds_barrier();  // every os read done before the next tile's x lands in the same LDS
  }
}


// per-layer kernel variant: 1 = the tall tile (RBT) where it is instantiated, 0 = the 128-row tile (A/B switch)
static int g_rb_tall = 1;
SSAMD_API void ssamd_resblock_set_tall(int v) { g_rb_tall = v; }
template <int C, int K>
constexpr bool has_tall() {
  return (C == 128 && (K == 7 || K == 11)) || (C == 64 && (K == 7 || K == 11)) || (C == 32 && K == 11) ||
         (C == 256 && K <= 7);
}
template <int C>
constexpr bool tall_only() {  // C = 256: the 128-row tile does not fit the LDS -- the tall tile is the only one
  return C == 256;
}
template <int C, int K>
constexpr bool has_half() {
  return has_tall<C, K>() && C <= 128;
}
// the 64-row tile (one row block per wave): twice the workgroups of the 128-row tile for batch-1 utterances whose
// whole stage is a few dozen 128-row tiles (halo recompute 16-19 % instead of 8-9 %)
template <int C, int K>
using RBS = RB<C, K, 1>;

template <class R>
int launch_rb(const bf16_t* x, const bf16_t* w1, const float* b1, const bf16_t* w2, const float* b2,
              const bf16_t* acc_in, bf16_t* out, int B, int T, int d, float slope, float out_scale, int post_lrelu,
              hipStream_t s, const int4* tt = nullptr, int ntt = 0) {
  static bool lds_set = false;
  if (!lds_set) {
    allow_lds(resblock_layer_kernel<R>, R::LDS);
    lds_set = true;
  }
  static int resident = 0;  // co-resident blocks on the whole device (LDS / register limited)
  if (!resident) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, resblock_layer_kernel<R>, R::NT, R::LDS) !=
            hipSuccess || per_cu <= 0)
      per_cu = 1;
    resident = cus * per_cu;
  }
  const int tiles = tt ? 1 : (T + R::BM - 1) / R::BM;
  const long ntiles = tt ? (long)ntt : (long)B * tiles;
  if (ntiles > 0x7fffffffL) return -2;
  if (ntiles == 0) return 0;
  const int grid = (int)(ntiles < resident ? ntiles : resident);
  hipLaunchKernelGGL((resblock_layer_kernel<R>), dim3(grid), dim3(R::NT), R::LDS, s, x, w1, b1, w2, b2,
                     acc_in, out, T, tiles, (int)ntiles, d, slope, out_scale, post_lrelu, tt);
  return (int)hipGetLastError();
}

template <int C, int K>
int launch_rb_any(const bf16_t* x, const bf16_t* w1, const float* b1, const bf16_t* w2, const float* b2,
                  const bf16_t* acc_in, bf16_t* out, int B, int T, int d, float slope, float out_scale, int post_lrelu,
                  hipStream_t s, const int4* tt = nullptr, int ntt = 0) {
  if constexpr (tall_only<C>()) {
    return launch_rb<RBT<C, K>>(x, w1, b1, w2, b2, acc_in, out, B, T, d, slope, out_scale, post_lrelu, s, tt, ntt);
  } else {
    if constexpr (has_half<C, K>()) {
      if (g_rb_tall == 2)
        return launch_rb<RBH<C, K>>(x, w1, b1, w2, b2, acc_in, out, B, T, d, slope, out_scale, post_lrelu, s, tt, ntt);
    }
    if constexpr (has_tall<C, K>()) {
      if (g_rb_tall)
        return launch_rb<RBT<C, K>>(x, w1, b1, w2, b2, acc_in, out, B, T, d, slope, out_scale, post_lrelu, s, tt, ntt);
    }
    return launch_rb<RB<C, K>>(x, w1, b1, w2, b2, acc_in, out, B, T, d, slope, out_scale, post_lrelu, s, tt, ntt);
  }
}

template <int C, int K>
int rb_bm() {
  if constexpr (tall_only<C>()) {
    return RBT<C, K>::BM;
  } else {
    if constexpr (has_half<C, K>()) {
      if (g_rb_tall == 2) return RBH<C, K>::BM;
    }
    if constexpr (has_tall<C, K>()) {
      if (g_rb_tall) return RBT<C, K>::BM;
    }
    return RB<C, K>::BM;
  }
}

// ---------------------------------------------------------------------------------------------
// Square 3-tap conv (pad 1, dilation 1, N = Cin = C), y = conv(x) + b: the HiFi-GAN upsamplers whose
// 3-tap implicit-GEMM form (convT_as_conv3: N = stride * Cout) is square -- ups 3 (128 -> 2 x 64) and
// ups 4 (64 -> 2 x 32) of V1 -- over 64x / 128x the mel rate.  As a generic GEMM they are short-K
// (K = 3C = 384 / 192) tiles of N <= 128 on a 256 x 128 tile (13.9 % MFMA busy, 4.6 % of synthesis,
// profiles/r5_vocoder_pmc_summary_persistent.txt).  Here the resblock layer machinery does it: the x
// tile (128 + 2 rows) is staged once and read at the three tap offsets (no per-tap re-read of A),
// weights stream through the LDS-DMA ring (conv_tile), + bias into an fp32 LDS tile, coalesced 16-B
// stores; persistent over tiles with the next tile's x fetched under the epilogue.
template <int C>
struct C3 {
  using R = RB<C, 3>;
  static constexpr int BM = R::R1P;                               // output rows per tile (all row blocks)
  static constexpr int RXS = BM + 2;                              // staged x rows (1-row halo per side)
  static constexpr int XS_BYTES = (RXS * R::LDC * 2 + 15) / 16 * 16;
  static constexpr int OS_BYTES = BM * R::OSP * 4;
  static constexpr int LDS = XS_BYTES + OS_BYTES + 3 * R::SLOT;
  static_assert(LDS <= 160 * 1024, "conv3 tile");
};

template <int C>
__global__ void __launch_bounds__((RB<C, 3>::NT)) conv3_sq_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                                   const float* __restrict__ bias, bf16_t* __restrict__ out,
                                                                   int Tp, int tiles, int ntiles,
                                                                   const int4* __restrict__ tt) {
  using R = RB<C, 3>;
  using G = C3<C>;
  constexpr int NT = R::NT;
  constexpr int CH = C / 8;
  constexpr int BM = G::BM;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(lds);                  // [RXS][LDC]: x rows t0 - 1 ..
  float* os = reinterpret_cast<float*>(lds + G::XS_BYTES);       // [BM][OSP]
  char* bring = reinterpret_cast<char*>(lds + G::XS_BYTES + G::OS_BYTES);
  // fp32 output tile column swizzle (C = 128): the epilogue's 16-B reads of lanes 0-15 step 32 B through a row, so
  // chunks 2k and 2k + 16 shared banks (2-way); XOR-ing the chunk index with bit 4 moves the upper half by one chunk
  constexpr bool SW = C == 128;
  auto osw = [](int ch) { return SW ? ch ^ (((ch >> 6) & 1) << 2) : ch; };
  const int tid0 = threadIdx.x;
  float bv[R::NSW];
#pragma unroll
  for (int s = 0; s < R::NSW; ++s) bv[s] = bias[((tid0 >> 6) / R::WR * R::NSW + s) * 16 + (tid0 & 15)];
  constexpr int IX = (G::RXS * CH + NT - 1) / NT;
  short8 v[IX];
  auto fetch_x = [&](int tile, int tid) {
    const TileGeo gq = tile_geo(tt, tile, tiles, Tp, BM);
    const int T = gq.T, t0 = gq.t0;
    const bf16_t* xb = x + gq.off * C;
#pragma unroll
    for (int it = 0; it < IX; ++it) {
      const int q = tid + it * NT, r = q / CH, c0 = (q - r * CH) * 8;
      const int t = t0 - 1 + r;
      if (r < G::RXS && t >= 0 && t < T) {
        v[it] = *reinterpret_cast<const short8*>(xb + (long)t * C + c0);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[it][i] = 0;
      }
    }
  };
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  fetch_x(blockIdx.x, tid0);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int tid = tid0;  // opaque per tile: keeps the unrolled conv's per-lane address terms inside the loop
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, col = lane & 15, quad = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave % R::WR, wc = wave / R::WR;
    const TileGeo gt = tile_geo(tt, tile, tiles, Tp, BM);
    const int T = gt.T, t0 = gt.t0;
#pragma unroll
    for (int it = 0; it < IX; ++it) {
      const int q = tid + it * NT, r = q / CH, c0 = (q - r * CH) * 8;
      if (r < G::RXS) *reinterpret_cast<short8*>(xs + r * R::LDC + c0) = v[it];
    }
    __syncthreads();
    float4v acc[R::MAXRB][R::NSW];
    conv_tile<R>(xs, 1, w, bring, R::NRB1, wave, tid, acc);
    const int nxt = tile + gridDim.x;
    if (nxt < ntiles) fetch_x(nxt, tid);  // no DMA of conv_tile in flight any more
#pragma unroll
    for (int r = 0; r < R::MAXRB; ++r) {
      const int rb = wr + R::WR * r;
#pragma unroll
      for (int s = 0; s < R::NSW; ++s) {
        const int ch = (wc * R::NSW + s) * 16 + col;
#pragma unroll
        for (int i = 0; i < 4; ++i) os[(rb * 16 + 4 * quad + i) * R::OSP + osw(ch)] = acc[r][s][i] + bv[s];
      }
    }
    lds_barrier();
    constexpr int IE = (BM * CH + NT - 1) / NT;
    bf16_t* ob = out + gt.off * C;
#pragma unroll
    for (int it = 0; it < IE; ++it) {
      const int q = tid + it * NT, j = q / CH, c0 = (q - j * CH) * 8;
      const int t = t0 + j;
      if (j >= BM || t >= T) continue;
      const int f = SW ? (c0 >> 6) & 1 : 0;  // the pair of 16-B chunks is stored swapped when f (see osw)
      const float4 o0 = *reinterpret_cast<const float4*>(os + j * R::OSP + c0 + 4 * f);
      const float4 o1 = *reinterpret_cast<const float4*>(os + j * R::OSP + c0 + 4 - 4 * f);
      const float ov[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
      short8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (short)f2bf(ov[i]);
      *reinterpret_cast<short8*>(ob + (long)t * C + c0) = o;
    }
    lds_barrier();  // os read and xs / ring free before the next tile writes them
  }
}

template <int C>
int launch_c3(const bf16_t* x, const bf16_t* w, const float* bias, bf16_t* out, int B, int T, hipStream_t s,
              const int4* tt = nullptr, int ntt = 0) {
  using G = C3<C>;
  static int resident = 0;
  if (!resident) {
    allow_lds(conv3_sq_kernel<C>, G::LDS);
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv3_sq_kernel<C>, RB<C, 3>::NT, G::LDS) != hipSuccess ||
        per_cu <= 0)
      per_cu = 1;
    resident = cus * per_cu;
  }
  const int tiles = tt ? 1 : (T + G::BM - 1) / G::BM;
  const long ntiles = tt ? (long)ntt : (long)B * tiles;
  if (ntiles > 0x7fffffffL) return -2;
  if (ntiles == 0) return 0;
  const int grid = (int)(ntiles < resident ? ntiles : resident);
  hipLaunchKernelGGL((conv3_sq_kernel<C>), dim3(grid), dim3(RB<C, 3>::NT), G::LDS, s, x, w, bias, out, T, tiles,
                     (int)ntiles, tt);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Whole ResBlock1 in one kernel (reference hifigan/models.py:20-44, the three (c1_d, c2) layer
// pairs, dilations d0 / d1 / d2):
//
//     x_{p+1} = x_p + conv2_p( lrelu( conv1_p,d_p( lrelu(x_p) ) + b1_p ) ) + b2_p      p = 0, 1, 2
//     out = (acc_in + x_3) * out_scale  [-> lrelu]
//
// for the narrow stages (C = 32 at 256x the mel rate, C = 64 at 128x), where the per-layer kernel
// above is bound by streaming the activation through HBM three times per ResBlock (read x + halo,
// re-read x for the residual, write) at a low arithmetic intensity (C = 32: ~64 FLOP/B).  Here one
// workgroup owns R0 = 16 * NB rows of the sequence, of which the middle BM = R0 - 2 * HT are output
// rows (HT = (K-1)/2 * (d0 + d1 + d2 + 3): the summed halo of the six convs, recomputed by the
// neighbouring tiles):
//   * the residual stream x_p lives in fp32 REGISTERS in the MFMA accumulator layout (each lane owns
//     the same (row, channel) elements in every conv2 epilogue), so it never round-trips through
//     memory between layers and is not rounded to bf16 between them (the per-layer path rounds it
//     three times);
//   * two bf16 LDS tiles hold lrelu(x_p) (A) and lrelu(conv1 + b1) (T); rows are addressed in one
//     absolute frame, so every conv is "16-row block b of the output reads rows 16b - h + tap*step of
//     its input" and the valid region shrinks by h = step * (K-1)/2 per conv; rows outside it are
//     don't-care values that no valid row reads (MG margin rows keep the reads in bounds);
//   * each conv's whole weight image [C][K][C] sits in LDS (row pitch padded to 2 mod 4 16-B units:
//     conflict-free B-fragment reads), so the MFMA loop has no barrier at all; the next conv's
//     image is prefetched into registers during the current conv and written after its barrier;
//   * rows outside [0, T) are zeroed in A and T (each reference conv zero-pads its own input).
// HBM traffic per ResBlock: x (+ halo) once, acc_in once, out once -- 3x less than three layer
// launches.  Validated against the fp32 torch ResBlock (tests/test_kernels_gpu.py).
struct RFW {
  const bf16_t* w[6];  // c1_0, c2_0, c1_1, c2_1, c1_2, c2_2: bf16 [C][K][C] forward images
  const float* b[6];   // fp32 [C]
  int d[3];
};

template <int C, int K, int S = 0>  // S = 1: the short tile for tile-poor packed batches (batch-1 serving)
struct RF {
  // RING: the weights stream per (tap, 32-deep chunk) through a 3-slot LDS ring (one barrier per step)
  // instead of a whole image per conv -- the wide / long-kernel instances, whose whole image would
  // leave too few rows for the tile
  static constexpr bool RING = C >= 128 || K > 3 && C >= 64;
  static constexpr int NW = 8;
  static constexpr int NT = 64 * NW;
  static constexpr int WC = C >= 64 ? 2 : 1;       // column groups
  static constexpr int WR = NW / WC;               // row groups
  static constexpr int H2 = (K - 1) / 2;
  static constexpr int MG = MAXD * H2;             // margin rows: the widest conv's half window
  // OCC: workgroups per CU.  C = 32 / K = 3 is latency-bound at one workgroup per CU (little MFMA work
  // between the phase barriers and the HBM / L2 round trips), so it takes a smaller tile (9 % halo
  // recompute) that lets two workgroups overlap each other's phases (1.41 -> 1.18 ms per ResBlock).
  // (C = 64 / K = 3 measured: the 8-block tile at two per CU is 12 % slower than 24 blocks at one)
  static constexpr int OCC = K == 3 && C == 32 ? 2 : 1;
  // S = 1: about a third to a half of the rows (more halo recompute, 2-4x the workgroups of a batch-1 stage)
  static constexpr int NB = S ? (C == 32 ? (K == 3 ? 8 : 16) : C == 64 ? 12 : 8)
                              : (K == 3 && C == 32 ? 16 : C == 32 ? 40 : (C == 64 ? 24 : 12));
  static constexpr int R0 = NB * 16;
  static constexpr int LDC = C + 16;               // bf16 pitch: 2 (mod 4) 16-B units (see RB)
  static constexpr int ROWS = R0 + 2 * MG;
  static constexpr int BUF = (ROWS * LDC * 2 + 15) / 16 * 16;
  static constexpr int NS = C / 16;
  static constexpr int NSW = NS / WC;
  static constexpr int KC = C / 32;
  static constexpr int WROW = K * C / 8;           // 16-B chunks per weight-image row
  static constexpr int WP = (WROW + 2) * 16;       // padded row pitch (bytes): 2 (mod 4) units
  static constexpr int SLOT = C * 64;              // ring slot: [C][32] bf16
  static constexpr int WBYTES = RING ? 3 * SLOT : C * WP;
  static constexpr int WCH = C * WROW;             // 16-B chunks of one image
  static constexpr int WIT = RING ? 1 : (WCH + NT - 1) / NT;
  static constexpr int MAXRB = NB / WR;
  static constexpr int OSP = C + 4;                // fp32 output tile pitch
  static constexpr int LDS = 2 * BUF + WBYTES;
  static_assert(NB % WR == 0, "row blocks split evenly over the row groups");
  static_assert(LDS * OCC <= 160 * 1024, "fused resblock tile");
  static_assert(R0 * OSP * 4 <= 2 * BUF, "output tile aliases the A / T tiles");
};

// (Measured and lost: the epilogue tiles written as conflict-free b32 channel pairs after a DPP swap
// with the neighbour column's lane -- LDS conflicts 0.30 -> 0.16 but 6-10 % slower per ResBlock,
// profiles/r3_v7_rb_pairs_lost.jsonl; the 16-bit scattered stores stay.)
// acc[j][s] = conv over the wave's row blocks blk = wr + WR*j (all NB blocks of the tile are computed:
// straight-line MFMA code; rows outside the conv's valid region are don't-care).
template <int C, int K, int S>
__device__ __forceinline__ void conv_rf(const bf16_t* __restrict__ src, int step, const char* Ws, int wr, int wc,
                                        int col, int quad, float4v (&acc)[RF<C, K, S>::MAXRB][RF<C, K, S>::NSW]) {
  using R = RF<C, K, S>;
#pragma unroll
  for (int j = 0; j < R::MAXRB; ++j)
#pragma unroll
    for (int s = 0; s < R::NSW; ++s) acc[j][s] = float4v{0.f, 0.f, 0.f, 0.f};
  const int h = step * R::H2;
  const bf16_t* abase = src + (wr * 16 + col - h) * R::LDC + 8 * quad;
  const char* bbase = Ws + ((wc * R::NSW) * 16 + col) * R::WP + 16 * quad;
#pragma unroll
  for (int tap = 0; tap < K; ++tap) {
#pragma unroll
    for (int kc = 0; kc < R::KC; ++kc) {
      short8 bf[R::NSW], a[R::MAXRB];
#pragma unroll
      for (int s = 0; s < R::NSW; ++s)
        bf[s] = *reinterpret_cast<const short8*>(bbase + s * 16 * R::WP + (tap * C + kc * 32) * 2);
#pragma unroll
      for (int j = 0; j < R::MAXRB; ++j)
        a[j] = *reinterpret_cast<const short8*>(abase + (j * R::WR * 16 + tap * step) * R::LDC + kc * 32);
#pragma unroll
      for (int j = 0; j < R::MAXRB; ++j)
#pragma unroll
        for (int s = 0; s < R::NSW; ++s)
          acc[j][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], bf[s], acc[j][s], 0, 0, 0);
    }
  }
}

// RING form of conv_rf: weight slices [C][32] (tap, chunk) DMA'd three steps ahead into a 3-slot ring
// (same source-side chunk swizzle and pipeline as conv_tile), fragments of step+1 read while step's
// MFMAs run, one barrier per step.
template <int C, int K, int S>
__device__ __forceinline__ void stage_ring(const bf16_t* __restrict__ w, int step, char* slot, int tid, int wave) {
  if (wave * 64 < C * 4) {  // wave-uniform: C*4 16-B chunks per slice
    constexpr int KC = C / 32;
    const int tap = step / KC, kc = step - tap * KC;
    const int n = tid >> 2, p = tid & 3;
    const int lc = p ^ (((n >> 2) & 1) << 1);
    glds16(w + (n * K + tap) * C + kc * 32 + 8 * lc, slot + wave * 1024);
  }
}

template <int C, int K, int S>
__device__ __forceinline__ void conv_rf_ring(const bf16_t* __restrict__ src, int step_d, const bf16_t* __restrict__ w,
                                             char* ring, int tid, int wave, int wr, int wc, int col, int quad,
                                             float4v (&acc)[RF<C, K, S>::MAXRB][RF<C, K, S>::NSW]) {
  using R = RF<C, K, S>;
  constexpr int STEPS = K * R::KC;
  constexpr int SLOT = R::SLOT;
#pragma unroll
  for (int j = 0; j < R::MAXRB; ++j)
#pragma unroll
    for (int s = 0; s < R::NSW; ++s) acc[j][s] = float4v{0.f, 0.f, 0.f, 0.f};
  stage_ring<C, K, S>(w, 0, ring, tid, wave);
  if (STEPS > 1) stage_ring<C, K, S>(w, 1, ring + SLOT, tid, wave);
  if (STEPS > 2) stage_ring<C, K, S>(w, 2, ring + 2 * SLOT, tid, wave);
  if (STEPS > 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (STEPS > 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const int h = step_d * R::H2;
  const bf16_t* abase = src + (wr * 16 + col - h) * R::LDC + 8 * quad;
  int boff[R::NSW];
#pragma unroll
  for (int s = 0; s < R::NSW; ++s) {
    const int n = (wc * R::NSW + s) * 16 + col;
    boff[s] = n * 64 + ((quad ^ (((n >> 2) & 1) << 1)) << 4);
  }
  short8 a[2][R::MAXRB], bf[2][R::NSW];
  auto load = [&](int st, int buf) {
    const int tap = st / R::KC, kc = st - tap * R::KC;
    const char* bs = ring + (st % 3) * SLOT;
#pragma unroll
    for (int s = 0; s < R::NSW; ++s) bf[buf][s] = *reinterpret_cast<const short8*>(bs + boff[s]);
#pragma unroll
    for (int j = 0; j < R::MAXRB; ++j)
      a[buf][j] = *reinterpret_cast<const short8*>(abase + (j * R::WR * 16 + tap * step_d) * R::LDC + kc * 32);
  };
  load(0, 0);
#pragma unroll
  for (int st = 0; st < STEPS; ++st) {
    const int cur = st & 1;
    if (st + 1 < STEPS) {
      if (st + 2 < STEPS) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (st + 3 < STEPS) stage_ring<C, K, S>(w, st + 3, ring + (st % 3) * SLOT, tid, wave);
      load(st + 1, cur ^ 1);
    }
#pragma unroll
    for (int j = 0; j < R::MAXRB; ++j)
#pragma unroll
      for (int s = 0; s < R::NSW; ++s)
        acc[j][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cur][j], bf[cur][s], acc[j][s], 0, 0, 0);
  }
}

template <int C, int K, int S>
__global__ void __launch_bounds__((RF<C, K, S>::NT), (RF<C, K, S>::OCC)) resblock_fused_kernel(const bf16_t* __restrict__ x, RFW p,
                                                                        const bf16_t* acc_in, bf16_t* out, int Tp,
                                                                        int tiles, int HT, float slope,
                                                                        float out_scale, int post_lrelu,
                                                                        const int4* __restrict__ tt) {
  using R = RF<C, K, S>;
  constexpr int NT = R::NT;
  constexpr int CH = C / 8;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  bf16_t* As = reinterpret_cast<bf16_t*>(lds) + R::MG * R::LDC;           // absolute row r at As + r * LDC
  bf16_t* Ts = reinterpret_cast<bf16_t*>(lds + R::BUF) + R::MG * R::LDC;
  char* Ws = reinterpret_cast<char*>(lds + 2 * R::BUF);
  float* Os = reinterpret_cast<float*>(lds);                               // final fp32 tile (aliases A / T)
  const int BM = R::R0 - 2 * HT;
  const TileGeo gt = tile_geo(tt, blockIdx.x, tiles, Tp, BM);
  const int T = gt.T, t0 = gt.t0;
  const int tb = t0 - HT;  // sequence position of absolute row 0
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave % R::WR, wc = wave / R::WR;
  const int col = lane & 15, quad = lane >> 4;
  const bf16_t* xb = x + gt.off * C;

  // Weight images go global -> registers -> LDS.  Two register sets: the load of conv c+2's image is
  // issued at the start of conv c (two convs of latency cover), conv c+1's image is written to LDS
  // after conv c's closing barrier.
  short8 wr0[R::WIT], wr1[R::WIT];
  auto wload = [&](short8 (&wreg)[R::WIT], const bf16_t* __restrict__ w) {
#pragma unroll
    for (int it = 0; it < R::WIT; ++it) {
      const int q = tid + it * NT;
      if (q < R::WCH) wreg[it] = *reinterpret_cast<const short8*>(w + q * 8);
    }
  };
  auto wstore = [&](const short8 (&wreg)[R::WIT]) {
#pragma unroll
    for (int it = 0; it < R::WIT; ++it) {
      const int q = tid + it * NT;
      if (q < R::WCH) {
        const int n = q / R::WROW;
        *reinterpret_cast<short8*>(Ws + n * R::WP + (q - n * R::WROW) * 16) = wreg[it];
      }
    }
  };

  // 1. raw x rows [0, R0) (zero outside [0, T)) -> A; conv 0's weights -> W, conv 1's in flight
  {
    constexpr int IT = (R::R0 * CH + NT - 1) / NT;
    short8 v[IT];
    if constexpr (!R::RING) wload(wr0, p.w[0]);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int q = tid + it * NT, r = q / CH, c0 = (q - r * CH) * 8;
      const int t = tb + r;
      if (r < R::R0 && t >= 0 && t < T) {
        v[it] = *reinterpret_cast<const short8*>(xb + (long)t * C + c0);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[it][i] = 0;
      }
    }
    if constexpr (!R::RING) {
      wload(wr1, p.w[1]);
      wstore(wr0);
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int q = tid + it * NT, r = q / CH, c0 = (q - r * CH) * 8;
      if (r < R::R0) *reinterpret_cast<short8*>(As + r * R::LDC + c0) = v[it];
    }
  }
  __syncthreads();

  // 2. residual registers X (fp32, accumulator layout) and A = lrelu(x) in place (each element is
  //    read and rewritten by its owning lane only)
  float4v X[R::MAXRB][R::NSW];
#pragma unroll
  for (int j = 0; j < R::MAXRB; ++j)
#pragma unroll
    for (int s = 0; s < R::NSW; ++s) {
      const int ch = (wc * R::NSW + s) * 16 + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = (wr + R::WR * j) * 16 + 4 * quad + i;
        const float v = bf2f(As[row * R::LDC + ch]);
        X[j][s][i] = v;
        As[row * R::LDC + ch] = f2bf(lrelu(v, slope));
      }
    }
  __syncthreads();

  // the final epilogue's acc_in rows, loaded during the last conv
  constexpr int ITMAX = (R::R0 * CH + NT - 1) / NT;
  const bf16_t* ab = acc_in ? acc_in + gt.off * C : nullptr;
  short8 ar[ITMAX];

  float4v acc[R::MAXRB][R::NSW];
#pragma unroll
  for (int pp = 0; pp < 3; ++pp) {
    const int d = p.d[pp];
    // this pair's bias columns, issued before the weight prefetch: their waits (after each conv) then
    // neither stall on an exposed L2 round trip nor drain the younger weight loads still in flight
    float bb1[R::NSW], bb2[R::NSW];
#pragma unroll
    for (int s = 0; s < R::NSW; ++s) {
      const int ch = (wc * R::NSW + s) * 16 + col;
      bb1[s] = p.b[2 * pp][ch];
      bb2[s] = p.b[2 * pp + 1][ch];
    }
    // conv 2pp = conv1 (dilation d) of lrelu(x_p) -> T = lrelu(. + b1), zero outside [0, T)
    if constexpr (R::RING) {
      conv_rf_ring<C, K, S>(As, d, p.w[2 * pp], Ws, tid, wave, wr, wc, col, quad, acc);
    } else {
      if (pp < 2) wload(wr0, p.w[2 * pp + 2]);  // in flight during two convs
      conv_rf<C, K, S>(As, d, Ws, wr, wc, col, quad, acc);
    }
    {
#pragma unroll
      for (int s = 0; s < R::NSW; ++s) {
        const int ch = (wc * R::NSW + s) * 16 + col;
        const float bias = bb1[s];
#pragma unroll
        for (int j = 0; j < R::MAXRB; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = (wr + R::WR * j) * 16 + 4 * quad + i;
            const int t = tb + row;
            const float v = (t >= 0 && t < T) ? lrelu(acc[j][s][i] + bias, slope) : 0.f;
            Ts[row * R::LDC + ch] = f2bf(v);
          }
      }
    }
    __syncthreads();  // T complete; everyone is done with conv1's weights and with A
    if constexpr (!R::RING) {
      wstore(wr1);  // conv 2pp+1's image
      __syncthreads();
    }
    // conv 2pp+1 = conv2 (dilation 1) of T; X += . + b2; A = lrelu(X) for the next pair
    if (pp < 2) {
      if constexpr (!R::RING) wload(wr1, p.w[2 * pp + 3]);
    } else if (ab && !R::RING) {  // (the ring's vmcnt waits would also wait for these)
#pragma unroll
      for (int it = 0; it < ITMAX; ++it) {
        const int q = tid + it * NT, j = q / CH, c0 = (q - j * CH) * 8;
        const int t = t0 + j;
        if (j < BM && t < T) ar[it] = *reinterpret_cast<const short8*>(ab + (long)t * C + c0);
      }
    }
    if constexpr (R::RING) conv_rf_ring<C, K, S>(Ts, 1, p.w[2 * pp + 1], Ws, tid, wave, wr, wc, col, quad, acc);
    else conv_rf<C, K, S>(Ts, 1, Ws, wr, wc, col, quad, acc);
    {
#pragma unroll
      for (int s = 0; s < R::NSW; ++s) {
        const int ch = (wc * R::NSW + s) * 16 + col;
        const float bias = bb2[s];
#pragma unroll
        for (int j = 0; j < R::MAXRB; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float v = X[j][s][i] + (acc[j][s][i] + bias);
            X[j][s][i] = v;
            if (pp < 2) {
              const int row = (wr + R::WR * j) * 16 + 4 * quad + i;
              const int t = tb + row;
              As[row * R::LDC + ch] = f2bf((t >= 0 && t < T) ? lrelu(v, slope) : 0.f);
            }
          }
      }
    }
    __syncthreads();  // A complete; everyone is done with conv2's weights and with T
    if (pp < 2 && !R::RING) {
      wstore(wr0);  // conv 2pp+2's image
      __syncthreads();
    }
  }

  // 3. X -> fp32 tile (aliases A / T), then coalesced: (acc_in +) X, * out_scale [, lrelu] -> out
#pragma unroll
  for (int j = 0; j < R::MAXRB; ++j)
#pragma unroll
    for (int s = 0; s < R::NSW; ++s) {
      const int ch = (wc * R::NSW + s) * 16 + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) Os[((wr + R::WR * j) * 16 + 4 * quad + i) * R::OSP + ch] = X[j][s][i];
    }
  if constexpr (R::RING) {
    if (ab) {
#pragma unroll
      for (int it = 0; it < ITMAX; ++it) {
        const int q = tid + it * NT, j = q / CH, c0 = (q - j * CH) * 8;
        const int t = t0 + j;
        if (j < BM && t < T) ar[it] = *reinterpret_cast<const short8*>(ab + (long)t * C + c0);
      }
    }
  }
  __syncthreads();
  {
    bf16_t* ob = out + gt.off * C;
#pragma unroll
    for (int it = 0; it < ITMAX; ++it) {
      const int q = tid + it * NT, j = q / CH, c0 = (q - j * CH) * 8;
      const int t = t0 + j;
      if (j >= BM || t >= T) continue;
      const float* orow = Os + (HT + j) * R::OSP + c0;
      const float4 o0 = *reinterpret_cast<const float4*>(orow);
      const float4 o1 = *reinterpret_cast<const float4*>(orow + 4);
      const float ov[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
      short8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float v = ov[i];
        if (ab) v += bf2f((bf16_t)ar[it][i]);
        v *= out_scale;
        if (post_lrelu) v = lrelu(v, slope);
        o[i] = (short)f2bf(v);
      }
      *reinterpret_cast<short8*>(ob + (long)t * C + c0) = o;
    }
  }
}

template <int C, int K, int S>
int launch_rf(const bf16_t* x, const RFW& p, const bf16_t* acc_in, bf16_t* out, int B, int T, float slope,
              float out_scale, int post_lrelu, hipStream_t s, const int4* tt = nullptr, int ntt = 0) {
  using R = RF<C, K, S>;
  const int HT = R::H2 * (p.d[0] + p.d[1] + p.d[2] + 3);
  const int BM = R::R0 - 2 * HT;
  if (BM < 16) return -2;
  static bool lds_set = false;
  if (!lds_set) {
    allow_lds(resblock_fused_kernel<C, K, S>, R::LDS);
    lds_set = true;
  }
  const int tiles = tt ? 1 : (T + BM - 1) / BM;
  const long nblk = tt ? (long)ntt : (long)B * tiles;
  if (nblk > 0x7fffffffL) return -2;
  if (nblk == 0) return 0;
  hipLaunchKernelGGL((resblock_fused_kernel<C, K, S>), dim3(nblk), dim3(R::NT), R::LDS, s, x, p, acc_in,
                     out, T, tiles, HT, slope, out_scale, post_lrelu, tt);
  return (int)hipGetLastError();
}

// rinfo[m] = {position in its sequence, sequence length} of the packed rows at `rate` rows per frame (cu: int32
// frame offsets [B + 1]): the implicit-GEMM convs' per-row zero-padding table (ConvGeom::rinfo) for the packed
// vocoder stages that run on the generic GEMM (conv_pre, the C = 256 MRF, the first two upsamplers)
__global__ void __launch_bounds__(256) voc_rinfo_kernel(const int* __restrict__ cu, int rate, int2* __restrict__ rinfo) {
  const int b = blockIdx.y;
  const long r0 = (long)cu[b] * rate;
  const int n = (cu[b + 1] - cu[b]) * rate;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) rinfo[r0 + i] = make_int2((int)i, n);
}

// dst [R, C] bf16 <- the valid rows of src [B, M, C] (fp32 or bf16): sequence b's cu[b+1] - cu[b] rows at cu[b]
template <typename TS>
__global__ void __launch_bounds__(256) voc_pack_kernel(const TS* __restrict__ src, const int* __restrict__ cu, int M,
                                                       int C, bf16_t* __restrict__ dst) {
  const int b = blockIdx.y;
  const long n = (long)(cu[b + 1] - cu[b]) * C;
  const TS* sb = src + (long)b * M * C;
  bf16_t* db = dst + (long)cu[b] * C;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    if constexpr (sizeof(TS) == 4) db[i] = f2bf(sb[i]);
    else db[i] = sb[i];
  }
}

}  // namespace


// ------------------------------------------------------------------------------- packed (length-exact) vocoder
namespace {
template <int C, int K>
int rb_bm_kind(int kind) {  // 3: the tall per-layer tile's BM, 4: the 128-row tile's (0: no such instance)
  if constexpr (has_half<C, K>()) {
    if (kind == 3 && g_rb_tall == 2) return RBH<C, K>::BM;
  }
  if constexpr (has_tall<C, K>()) {
    if (kind == 3) return RBT<C, K>::BM;
  }
  if constexpr (!tall_only<C>()) {
    if (kind == 4) return RB<C, K>::BM;
    if (kind == 5) return RBS<C, K>::BM;
  }
  return 0;
}
}  // namespace

// Tile height (output rows per tile) of each tiled vocoder kernel, for the host-built packed tile tables:
// kind 0 = resblock_layer (C, K), 1 = resblock_fused (C, K, dilations), 2 = conv3_sq (C).  0 = no such instance.
SSAMD_API int ssamd_voc_tile_rows(int kind, int C, int K, int d0, int d1, int d2) {
#define VT_RB(CC, KK) \
  if (C == CC && K == KK) return rb_bm<CC, KK>();
#define VT_RF(CC, KK) \
  if (C == CC && K == KK) return RF<CC, KK>::R0 - 2 * (RF<CC, KK>::H2 * (d0 + d1 + d2 + 3));
  if (kind == 0) {
    VT_RB(32, 3) VT_RB(32, 7) VT_RB(32, 11) VT_RB(64, 3) VT_RB(64, 7) VT_RB(64, 11) VT_RB(128, 3) VT_RB(128, 7)
    VT_RB(128, 11) VT_RB(256, 3) VT_RB(256, 7)
  } else if (kind == 1) {
    VT_RF(32, 3) VT_RF(32, 7) VT_RF(32, 11) VT_RF(64, 3) VT_RF(64, 7) VT_RF(128, 3) VT_RF(64, 11) VT_RF(128, 7)
  } else if (kind == 6) {  // the whole-ResBlock kernel's short tile (RF S = 1)
#define VT_RFS(CC, KK) \
  if (C == CC && K == KK) return RF<CC, KK, 1>::R0 - 2 * (RF<CC, KK, 1>::H2 * (d0 + d1 + d2 + 3));
    VT_RFS(32, 3) VT_RFS(32, 7) VT_RFS(32, 11) VT_RFS(64, 3) VT_RFS(64, 7) VT_RFS(128, 3)
#undef VT_RFS
  } else if (kind == 2) {
    if (C == 128) return C3<128>::BM;
    if (C == 64) return C3<64>::BM;
  } else if (kind >= 3 && kind <= 5) {  // 3: the tall per-layer tile, 4: the 128-row one, 5: the 64-row one
#define VT_RB2(CC, KK) \
  if (C == CC && K == KK) return rb_bm_kind<CC, KK>(kind);
    VT_RB2(32, 3) VT_RB2(32, 7) VT_RB2(32, 11) VT_RB2(64, 3) VT_RB2(64, 7) VT_RB2(64, 11) VT_RB2(128, 3)
    VT_RB2(128, 7) VT_RB2(128, 11) VT_RB2(256, 3) VT_RB2(256, 7)
#undef VT_RB2
  }
#undef VT_RB
#undef VT_RF
  return 0;
}

SSAMD_API int ssamd_voc_rinfo(const int* cu, int B, int rate, int max_rows, int* rinfo, hipStream_t s) {
  if (B <= 0 || max_rows <= 0) return 0;
  const int gx = max_rows / 256 + 1 < 64 ? max_rows / 256 + 1 : 64;
  hipLaunchKernelGGL(voc_rinfo_kernel, dim3(gx, B), dim3(256), 0, s, cu, rate, reinterpret_cast<int2*>(rinfo));
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_voc_pack(const void* src, int src_f32, const int* cu, int B, int M, int C, bf16_t* dst,
                             hipStream_t s) {
  if (B <= 0 || M <= 0) return 0;
  const long n = (long)M * C;
  const int gx = (int)(n / 2048 + 1 < 32 ? n / 2048 + 1 : 32);
  if (src_f32)
    hipLaunchKernelGGL(voc_pack_kernel<float>, dim3(gx, B), dim3(256), 0, s, (const float*)src, cu, M, C, dst);
  else
    hipLaunchKernelGGL(voc_pack_kernel<bf16_t>, dim3(gx, B), dim3(256), 0, s, (const bf16_t*)src, cu, M, C, dst);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_resblock_layer_pk(const bf16_t* x, const bf16_t* w1, const float* b1, const bf16_t* w2,
                                      const float* b2, const bf16_t* acc_in, bf16_t* out, const int* tt, int ntt, int C,
                                      int K, int d, float slope, float out_scale, int post_lrelu, hipStream_t s) {
  if (d < 1 || d > MAXD || !tt) return -2;
  if (ntt <= 0) return 0;
  const int4* t4 = reinterpret_cast<const int4*>(tt);
#define RBK_CASE(CC, KK) \
  if (C == CC && K == KK) \
    return launch_rb_any<CC, KK>(x, w1, b1, w2, b2, acc_in, out, 1, 0, d, slope, out_scale, post_lrelu, s, t4, ntt);
  RBK_CASE(32, 3) RBK_CASE(32, 7) RBK_CASE(32, 11)
  RBK_CASE(64, 3) RBK_CASE(64, 7) RBK_CASE(64, 11)
  RBK_CASE(128, 3) RBK_CASE(128, 7) RBK_CASE(128, 11)
  RBK_CASE(256, 3) RBK_CASE(256, 7)  // (C = 256 / K = 11 spills at 256 VGPRs: the GEMM path)
#undef RBK_CASE
  return -2;
}

// ssamd_resblock_layer_pk with the tile chosen by the caller (tall = 1: the tall tile, 0: the 128-row tile) -- the
// packed vocoder picks per call from the tile count (ssamd_voc_tile_rows kinds 3 / 4 / 5; tall = 1 / 0 / -1): a
// batch-1 utterance gets more workgroups from the shorter tiles, a batch of 256 the tall tile's fewer LDS reads per MFMA
SSAMD_API int ssamd_resblock_layer_pk2(const bf16_t* x, const bf16_t* w1, const float* b1, const bf16_t* w2,
                                       const float* b2, const bf16_t* acc_in, bf16_t* out, const int* tt, int ntt, int C,
                                       int K, int d, float slope, float out_scale, int post_lrelu, int tall,
                                       hipStream_t s) {
  if (d < 1 || d > MAXD || !tt) return -2;
  if (ntt <= 0) return 0;
  const int4* t4 = reinterpret_cast<const int4*>(tt);
#define RBK2_CASE(CC, KK)                                                                                          \
  if (C == CC && K == KK) {                                                                                        \
    if constexpr (has_half<CC, KK>()) {                                                                            \
      if (tall > 0 && g_rb_tall == 2)                                                                                  \
        return launch_rb<RBH<CC, KK>>(x, w1, b1, w2, b2, acc_in, out, 1, 0, d, slope, out_scale, post_lrelu, s, t4, \
                                      ntt);                                                                        \
    }                                                                                                              \
    if constexpr (has_tall<CC, KK>()) {                                                                            \
      if (tall > 0)                                                                                                \
        return launch_rb<RBT<CC, KK>>(x, w1, b1, w2, b2, acc_in, out, 1, 0, d, slope, out_scale, post_lrelu, s, t4, \
                                      ntt);                                                                        \
    }                                                                                                              \
    if constexpr (!tall_only<CC>()) {                                                                              \
      if (tall == -1)                                                                                              \
        return launch_rb<RBS<CC, KK>>(x, w1, b1, w2, b2, acc_in, out, 1, 0, d, slope, out_scale, post_lrelu, s, t4, \
                                      ntt);                                                                        \
      if (!tall)                                                                                                   \
        return launch_rb<RB<CC, KK>>(x, w1, b1, w2, b2, acc_in, out, 1, 0, d, slope, out_scale, post_lrelu, s, t4,  \
                                     ntt);                                                                         \
    }                                                                                                              \
    return -2;                                                                                                     \
  }
  RBK2_CASE(32, 3) RBK2_CASE(32, 7) RBK2_CASE(32, 11) RBK2_CASE(64, 3) RBK2_CASE(64, 7) RBK2_CASE(64, 11)
  RBK2_CASE(128, 3) RBK2_CASE(128, 7) RBK2_CASE(128, 11) RBK2_CASE(256, 3) RBK2_CASE(256, 7)
#undef RBK2_CASE
  return -2;
}

SSAMD_API int ssamd_resblock_fused_pk(const bf16_t* x, const bf16_t* w0, const bf16_t* w1, const bf16_t* w2,
                                      const bf16_t* w3, const bf16_t* w4, const bf16_t* w5, const float* b0,
                                      const float* b1, const float* b2, const float* b3, const float* b4,
                                      const float* b5, const bf16_t* acc_in, bf16_t* out, const int* tt, int ntt, int C,
                                      int K, int d0, int d1, int d2, float slope, float out_scale, int post_lrelu,
                                      int short_tile, hipStream_t s) {
  const int dd[3] = {d0, d1, d2};
  for (int i = 0; i < 3; ++i)
    if (dd[i] < 1 || dd[i] > MAXD) return -2;
  if (x == out || !tt) return -2;
  if (ntt <= 0) return 0;
  const int4* t4 = reinterpret_cast<const int4*>(tt);
  RFW p = {{w0, w1, w2, w3, w4, w5}, {b0, b1, b2, b3, b4, b5}, {d0, d1, d2}};
  // short_tile: the tile table was built for the short tile (ssamd_voc_tile_rows kind 6)
#define RFK_CASE(CC, KK) \
  if (C == CC && K == KK) return launch_rf<CC, KK, 0>(x, p, acc_in, out, 1, 1, slope, out_scale, post_lrelu, s, t4, ntt);
#define RFS_CASE(CC, KK) \
  if (C == CC && K == KK) return launch_rf<CC, KK, 1>(x, p, acc_in, out, 1, 1, slope, out_scale, post_lrelu, s, t4, ntt);
  if (short_tile) {
    RFS_CASE(32, 3) RFS_CASE(32, 7) RFS_CASE(32, 11) RFS_CASE(64, 3) RFS_CASE(64, 7) RFS_CASE(128, 3)
    return -2;
  }
  RFK_CASE(32, 3) RFK_CASE(32, 7) RFK_CASE(32, 11) RFK_CASE(64, 3) RFK_CASE(64, 7) RFK_CASE(128, 3)
  RFK_CASE(64, 11) RFK_CASE(128, 7)
#undef RFK_CASE
#undef RFS_CASE
  return -2;
}

SSAMD_API int ssamd_conv3_sq_pk(const bf16_t* x, const bf16_t* w, const float* bias, bf16_t* out, const int* tt, int ntt,
                                int C, hipStream_t s) {
  if (x == out || !x || !w || !bias || !out || !tt) return -2;
  if (ntt <= 0) return 0;
  const int4* t4 = reinterpret_cast<const int4*>(tt);
  if (C == 128) return launch_c3<128>(x, w, bias, out, 1, 0, s, t4, ntt);
  if (C == 64) return launch_c3<64>(x, w, bias, out, 1, 0, s, t4, ntt);
  return -2;
}


// Whole ResBlock1 (see resblock_fused_kernel).  x / out / acc_in [B, T, C] bf16 (out must not alias x;
// acc_in may alias out, or be null); w: 6 bf16 [C][K][C] images (c1_0, c2_0, c1_1, c2_1, c1_2, c2_2);
// b: 6 fp32 [C]; dilations 1 <= d <= 5.  Returns -2 for a geometry without a fused instance
// (ssamd_resblock_fusable).
// Whole-ResBlock instances for the long-kernel geometries the per-layer kernel serves by default (C = 64 / K = 11,
// C = 128 / K = 7): the ring-fed fused kernel with their summed halo (60 / 36 rows per side on a 384 / 192-row tile,
// BM = 264 / 120 output rows) -- switched on by ssamd_resblock_set_whole_extra (A/B against the tall per-layer tile).
static int g_rf_extra = 0;
SSAMD_API void ssamd_resblock_set_whole_extra(int v) { g_rf_extra = v; }
SSAMD_API int ssamd_resblock_fusable(int C, int K) {
  return (C == 32 && (K == 3 || K == 7 || K == 11)) || (C == 64 && (K == 3 || K == 7)) || (C == 128 && K == 3) ||
         (g_rf_extra && ((C == 64 && K == 11) || (C == 128 && K == 7)));
}

SSAMD_API int ssamd_resblock_fused(const bf16_t* x, const bf16_t* w0, const bf16_t* w1, const bf16_t* w2,
                                   const bf16_t* w3, const bf16_t* w4, const bf16_t* w5, const float* b0,
                                   const float* b1, const float* b2, const float* b3, const float* b4,
                                   const float* b5, const bf16_t* acc_in, bf16_t* out, int B, int T, int C, int K,
                                   int d0, int d1, int d2, float slope, float out_scale, int post_lrelu,
                                   hipStream_t s) {
  const int dd[3] = {d0, d1, d2};
  for (int i = 0; i < 3; ++i)
    if (dd[i] < 1 || dd[i] > MAXD) return -2;
  if ((long)B * T == 0) return 0;
  if (x == out) return -2;
  RFW p = {{w0, w1, w2, w3, w4, w5}, {b0, b1, b2, b3, b4, b5}, {d0, d1, d2}};
  if (C == 32 && K == 3) return launch_rf<32, 3, 0>(x, p, acc_in, out, B, T, slope, out_scale, post_lrelu, s);
  if (C == 32 && K == 7) return launch_rf<32, 7, 0>(x, p, acc_in, out, B, T, slope, out_scale, post_lrelu, s);
  if (C == 32 && K == 11) return launch_rf<32, 11, 0>(x, p, acc_in, out, B, T, slope, out_scale, post_lrelu, s);
  if (C == 64 && K == 3) return launch_rf<64, 3, 0>(x, p, acc_in, out, B, T, slope, out_scale, post_lrelu, s);
  if (C == 64 && K == 7) return launch_rf<64, 7, 0>(x, p, acc_in, out, B, T, slope, out_scale, post_lrelu, s);
  if (C == 128 && K == 3) return launch_rf<128, 3, 0>(x, p, acc_in, out, B, T, slope, out_scale, post_lrelu, s);
  if (C == 64 && K == 11) return launch_rf<64, 11, 0>(x, p, acc_in, out, B, T, slope, out_scale, post_lrelu, s);
  if (C == 128 && K == 7) return launch_rf<128, 7, 0>(x, p, acc_in, out, B, T, slope, out_scale, post_lrelu, s);
  return -2;
}

// x / out / acc_in [B, T, C] bf16 (acc_in may alias out, or be null); w1 / w2 bf16 [C][K][C] (the
// implicit-GEMM forward image); b1 / b2 fp32 [C].  C in {32, 64, 128}, K in {3, 7, 11}, 1 <= d <= 5.
// Diagnostic: the per-layer kernel with phase stamps (see rb_stamp); prof >= 8 * B * ceil(T / BM) words.
// grid > 0 caps the workgroup count (the persistent tile loop of the production launch); 0 = one tile per block.
SSAMD_API int ssamd_resblock_layer_prof(const bf16_t* x, const bf16_t* w1, const float* b1, const bf16_t* w2,
                                        const float* b2, const bf16_t* acc_in, bf16_t* out, int B, int T, int C, int K,
                                        int d, float slope, float out_scale, int post_lrelu, unsigned long long* prof,
                                        long prof_words, int grid, hipStream_t s) {
#define RBP_CASE(CC, KK)                                                                                      \
  if (C == CC && K == KK) {                                                                                   \
    using R = RB<CC, KK>;                                                                                     \
    allow_lds(resblock_layer_kernel<R, true>, R::LDS);                                                        \
    const int tiles = (T + R::BM - 1) / R::BM;                                                                \
    if ((long)B * tiles * 8 > prof_words) return -3; /* stamp buffer too small for this tile height */       \
    const int g = grid > 0 && grid < B * tiles ? grid : B * tiles;                                            \
    hipLaunchKernelGGL((resblock_layer_kernel<R, true>), dim3(g), dim3(R::NT), R::LDS, s, x,                   \
                       w1, b1, w2, b2, acc_in, out, T, tiles, B * tiles, d, slope, out_scale, post_lrelu,      \
                       (const int4*)nullptr, prof);                                                           \
    return (int)hipGetLastError();                                                                            \
  }
  if (d < 1 || d > MAXD) return -2;
  RBP_CASE(128, 11) RBP_CASE(128, 7) RBP_CASE(64, 11)
#undef RBP_CASE
  return -2;
}

// Square 3-tap conv (pad 1): x / out [B, T, C] bf16 (out must not alias x), w bf16 [C][3][C] (implicit-GEMM
// forward image), bias fp32 [C].  C in {64, 128}.
SSAMD_API int ssamd_conv3_sq(const bf16_t* x, const bf16_t* w, const float* bias, bf16_t* out, int B, int T, int C,
                             hipStream_t s) {
  if ((long)B * T == 0) return 0;
  if (x == out || !x || !w || !bias || !out) return -2;
  if (C == 128) return launch_c3<128>(x, w, bias, out, B, T, s);
  if (C == 64) return launch_c3<64>(x, w, bias, out, B, T, s);
  return -2;
}

SSAMD_API int ssamd_resblock_layer_tile(int C, int K) {
  if (C == 128 && K == 11) return rb_bm<128, 11>();
  if (C == 128 && K == 7) return rb_bm<128, 7>();
  if (C == 64 && K == 11) return rb_bm<64, 11>();
  return 0;
}

SSAMD_API int ssamd_resblock_layer(const bf16_t* x, const bf16_t* w1, const float* b1, const bf16_t* w2,
                                   const float* b2, const bf16_t* acc_in, bf16_t* out, int B, int T, int C, int K,
                                   int d, float slope, float out_scale, int post_lrelu, hipStream_t s) {
  if (d < 1 || d > MAXD) return -2;
  if ((long)B * T == 0) return 0;
#define RB_CASE(CC, KK) \
  if (C == CC && K == KK) \
    return launch_rb_any<CC, KK>(x, w1, b1, w2, b2, acc_in, out, B, T, d, slope, out_scale, post_lrelu, s);
  RB_CASE(32, 3) RB_CASE(32, 7) RB_CASE(32, 11)
  RB_CASE(64, 3) RB_CASE(64, 7) RB_CASE(64, 11)
  RB_CASE(128, 3) RB_CASE(128, 7) RB_CASE(128, 11)
  RB_CASE(256, 3) RB_CASE(256, 7)
#undef RB_CASE
  return -2;
}
