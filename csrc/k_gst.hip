// Global-Style-Token reference encoder kernels.  The reference only declares the GST path
// (commented-out `gst:` block, config/BC2013/model.yaml:33-39; research goal README.md:7);
// SURVEY.md §2.6 scopes it in.  Model code: speakingstyle_amd/models/style.py.
//
//   * im2col / col2im for the 6 x Conv2d(3x3, stride 2, pad 1) stack in NHWC.  The
//     convolution itself is an MFMA GEMM (k_gemm.hip) over [B*Ho*Wo, 9*Cin] patch rows,
//     its weight gradient the split-M wgrad kernel; BatchNorm2d + ReLU is k_bn.hip (act 2).
//   * persistent GRU forward / BPTT: the whole recurrence is ONE launch per 16 batch rows.
//     W_hh lives in VGPRs as v_mfma_f32_16x16x32_bf16 B fragments for all steps; the
//     hidden state goes through a double-buffered LDS tile (one barrier per time step);
//     each wave owns 32 hidden units of all three gates, so the gate math is lane-local
//     on the MFMA accumulators.  The input projection (x W_ih^T) and both weight
//     gradients are big GEMMs outside the recurrence.
//   * multi-head style-token attention forward / backward, one wave per utterance; the
//     token-bank gradients are per-utterance partials reduced in a second pass (no float
//     atomics, deterministic).
#include "common.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// GRU block shape: NS 16-unit sub-tiles per wave (2, or 1 for GH = 256 so the resident W_hh
// fragments stay within the VGPR budget), GH / (16 NS) waves.
constexpr int gru_ns(int gh) { return gh >= 256 ? 1 : 2; }
constexpr int gru_threads(int gh) { return 64 * gh / (16 * gru_ns(gh)); }

// ---------------------------------------------------------------- im2col / col2im
// x [B, H, W, C] bf16; col [B*Ho*Wo, Kp] bf16 with k = (ky*3 + kx)*C + c, zero padded to Kp.
// One thread per 16-B chunk of a patch row.
__global__ void __launch_bounds__(256) im2col_s2_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ col, int H,
                                                        int W, int C, int Ho, int Wo, int Kp, long nchunks) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= nchunks) return;
  const int kc = Kp / 8;
  const long row = q / kc;
  const int k0 = (int)(q - row * kc) * 8;
  const int wo = (int)(row % Wo);
  const long t = row / Wo;
  const int ho = (int)(t % Ho);
  const long b = t / Ho;
  short8 o;
  if ((C & 7) == 0) {  // the 8 channels of one tap: one 16-B load
    const int tap = k0 / C, c = k0 - tap * C;
    const int hi = 2 * ho - 1 + tap / 3, wi = 2 * wo - 1 + tap % 3;
    if (hi >= 0 && hi < H && wi >= 0 && wi < W) {
      o = *reinterpret_cast<const short8*>(x + (((b * H + hi) * W + wi) * C + c));
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = 0;
    }
  } else {  // the first layer (C = 1): 9 taps padded to 16
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = k0 + i;
      const int tap = k / C, c = k - tap * C;
      const int hi = 2 * ho - 1 + tap / 3, wi = 2 * wo - 1 + tap % 3;
      o[i] = (tap < 9 && hi >= 0 && hi < H && wi >= 0 && wi < W) ? (short)x[((b * H + hi) * W + wi) * C + c] : (short)0;
    }
  }
  *reinterpret_cast<short8*>(col + row * Kp + k0) = o;
}

// dx[b, h, w, c] = sum over the (at most 2 x 2) taps whose stride-2 window covers (h, w):
// a gather, so no atomics.  One thread per 8 channels (C % 8 == 0).
__global__ void __launch_bounds__(256) col2im_s2_kernel(const bf16_t* __restrict__ dcol, bf16_t* __restrict__ dx,
                                                        int H, int W, int C, int Ho, int Wo, int Kp, long nchunks) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= nchunks) return;
  const int c8 = C / 8;
  const long pix = q / c8;
  const int c0 = (int)(q - pix * c8) * 8;
  const int w = (int)(pix % W);
  const long t = pix / W;
  const int h = (int)(t % H);
  const long b = t / H;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int hh = h + 1 - ky;
    if (hh < 0 || (hh & 1) || (hh >> 1) >= Ho) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ww = w + 1 - kx;
      if (ww < 0 || (ww & 1) || (ww >> 1) >= Wo) continue;
      const short8 v = *reinterpret_cast<const short8*>(
          dcol + ((b * Ho + (hh >> 1)) * Wo + (ww >> 1)) * Kp + (ky * 3 + kx) * C + c0);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += bf2f((bf16_t)v[i]);
    }
  }
  short8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (short)f2bf(acc[i]);
  *reinterpret_cast<short8*>(dx + pix * C + c0) = o;
}

// ---------------------------------------------------------------- GRU (torch gate order r, z, n)
//   r = s(gi_r + W_hr h + b_hr)   z = s(gi_z + W_hz h + b_hz)   n = tanh(gi_n + r (W_hn h + b_hn))
//   h' = (1 - z) n + z h          gi = x W_ih^T + b_ih (precomputed GEMM, fp32)
// Block = 16 batch rows.  Wave w owns hidden units j in [16 NS w, 16 NS (w + 1)) of all three
// gates: NS 16-column sub-tiles s.  MFMA C layout: col = lane & 15 (unit), row = 4*(lane>>4) + i,
// so lane (s, i) holds gate pre-activations r, z, n of the same (row, unit).
// sv [B, T, 5, GH] fp32 = (r, z, n, W_hn h + b_hn, h_prev) per step for the backward;
// hprev [B, T, GH] bf16 = the W_hh weight-gradient GEMM operand; hlast [B, GH] = h at step last[b].
template <int GH>
__global__ void __launch_bounds__(gru_threads(GH)) gru_fwd_kernel(const float* __restrict__ gi, const bf16_t* __restrict__ whh,
                                                      const float* __restrict__ bhh, const int64_t* __restrict__ last,
                                                      int B, int T, float* __restrict__ hlast, float* __restrict__ sv,
                                                      bf16_t* __restrict__ hprev) {
  __shared__ __attribute__((aligned(16))) bf16_t hb[2][16][GH + 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int r0 = blockIdx.x * 16;
  // B operand of h W_hh^T: B[k = input unit][n = gate row], lane holds k = 32 ks + 8 quad .. +8
  constexpr int KS = GH / 32, NS = gru_ns(GH);
  short8 bw[3][NS][KS];
  float bias[3][NS];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int j = 16 * (NS * w + s) + col;
      bias[g][s] = bhh[g * GH + j];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        bw[g][s][ks] = *reinterpret_cast<const short8*>(whh + (long)(g * GH + j) * GH + 32 * ks + 8 * quad);
    }
  long lastt[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = r0 + 4 * quad + i;
    lastt[i] = b < B ? last[b] : -1;
  }
  float h[NS][4];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) h[s][i] = 0.f;
  for (int i = threadIdx.x; i < 2 * 16 * (GH + 8); i += gru_threads(GH)) (&hb[0][0][0])[i] = 0;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const int cur = t & 1;
    float4v acc[3][NS];
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int s = 0; s < NS; ++s) acc[g][s] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const short8 a = *reinterpret_cast<const short8*>(&hb[cur][col][32 * ks + 8 * quad]);
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int s = 0; s < NS; ++s)
          acc[g][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[g][s][ks], acc[g][s], 0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int j = 16 * (NS * w + s) + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = 4 * quad + i, b = r0 + rr;
        float hn = 0.f;
        if (b < B) {
          const long bt = (long)b * T + t;
          const float* gp = gi + bt * 3 * GH + j;
          const float r = sigm(gp[0] + acc[0][s][i] + bias[0][s]);
          const float z = sigm(gp[GH] + acc[1][s][i] + bias[1][s]);
          const float ghn = acc[2][s][i] + bias[2][s];
          const float n = tanhf(gp[2 * GH] + r * ghn);
          hn = (1.f - z) * n + z * h[s][i];
          float* sp = sv + bt * 5 * GH + j;
          sp[0] = r;
          sp[GH] = z;
          sp[2 * GH] = n;
          sp[3 * GH] = ghn;
          sp[4 * GH] = h[s][i];
          hprev[bt * GH + j] = f2bf(h[s][i]);
          if (t == lastt[i]) hlast[(long)b * GH + j] = hn;
        }
        h[s][i] = hn;
        hb[cur ^ 1][rr][j] = f2bf(hn);
      }
    }
    __syncthreads();  // double buffer: the next step reads hb[cur ^ 1], writes hb[cur]
  }
}

// BPTT.  dh (the gradient w.r.t. the hidden state entering step t+1) lives in the same lane
// layout as the forward; d(h_prev) = dh z + dgh W_hh with dgh = (da_r, da_z, da_n r) through
// the same double-buffered LDS tile.  dgi = (da_r, da_z, da_n) feeds the W_ih / x GEMMs,
// dgh (with hprev) the W_hh / b_hh weight gradient.
template <int GH>
__global__ void __launch_bounds__(gru_threads(GH)) gru_bwd_kernel(const float* __restrict__ dhlast, const float* __restrict__ sv,
                                                      const bf16_t* __restrict__ whhT, const int64_t* __restrict__ last,
                                                      int B, int T, bf16_t* __restrict__ dgi, bf16_t* __restrict__ dgh) {
  __shared__ __attribute__((aligned(16))) bf16_t db[2][16][3 * GH + 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int r0 = blockIdx.x * 16;
  // B operand of dgh W_hh: B[k = gate row][n = unit j] = W_hh[k][j] = whhT[j][k]
  constexpr int KS = 3 * GH / 32, NS = gru_ns(GH);
  short8 bw[NS][KS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int j = 16 * (NS * w + s) + col;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      bw[s][ks] = *reinterpret_cast<const short8*>(whhT + (long)j * 3 * GH + 32 * ks + 8 * quad);
  }
  long lastt[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = r0 + 4 * quad + i;
    lastt[i] = b < B ? last[b] : -1;
  }
  float dh[NS][4];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) dh[s][i] = 0.f;
  for (int it = 0; it < T; ++it) {
    const int t = T - 1 - it, cur = it & 1;
    float dhp[NS][4];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int j = 16 * (NS * w + s) + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = 4 * quad + i, b = r0 + rr;
        float g0 = 0.f, g1 = 0.f, g2 = 0.f, g2h = 0.f, dp = 0.f;
        if (b < B) {
          float d = dh[s][i];
          if (t == lastt[i]) d += dhlast[(long)b * GH + j];
          const long bt = (long)b * T + t;
          const float* sp = sv + bt * 5 * GH + j;
          const float r = sp[0], z = sp[GH], n = sp[2 * GH], ghn = sp[3 * GH], hp = sp[4 * GH];
          const float dn = d * (1.f - z);
          const float dz = d * (hp - n);
          dp = d * z;
          const float dan = dn * (1.f - n * n);
          g0 = dan * ghn * r * (1.f - r);
          g1 = dz * z * (1.f - z);
          g2 = dan;
          g2h = dan * r;
          bf16_t* pi = dgi + bt * 3 * GH + j;
          pi[0] = f2bf(g0);
          pi[GH] = f2bf(g1);
          pi[2 * GH] = f2bf(g2);
          bf16_t* ph = dgh + bt * 3 * GH + j;
          ph[0] = f2bf(g0);
          ph[GH] = f2bf(g1);
          ph[2 * GH] = f2bf(g2h);
        }
        db[cur][rr][j] = f2bf(g0);
        db[cur][rr][GH + j] = f2bf(g1);
        db[cur][rr][2 * GH + j] = f2bf(g2h);
        dhp[s][i] = dp;
      }
    }
    __syncthreads();
    float4v acc[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) acc[s] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const short8 a = *reinterpret_cast<const short8*>(&db[cur][col][32 * ks + 8 * quad]);
#pragma unroll
      for (int s = 0; s < NS; ++s) acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[s][ks], acc[s], 0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) dh[s][i] = dhp[s][i] + acc[s][i];
  }
}

// ---------------------------------------------------------------- style-token attention
// q [B, NH*D] fp32 (query projection of the GRU state), K / V [NH, N, D] fp32 (projections of
// tanh(token bank)); o [B, NH*D] = softmax(q_h K_h^T * scale) V_h, w [B, NH, N] = the weights.
constexpr int NTOK_MAX = 32;

// one wave per (utterance, head): the head's N key / value rows are loaded up front (independent loads in
// flight together; a batch-1 synthesis is a chain of latency-bound launches), then N wave reductions
__global__ void __launch_bounds__(64) token_attn_fwd_kernel(const float* __restrict__ q, const float* __restrict__ K,
                                                            const float* __restrict__ V, int NH, int N, int D,
                                                            float scale, float* __restrict__ o,
                                                            float* __restrict__ wout) {
  const int b = blockIdx.x, hh = blockIdx.y, l = threadIdx.x;
  const bool on = l < D;
  const float qv = on ? q[((long)b * NH + hh) * D + l] : 0.f;
  float kv[NTOK_MAX], vv[NTOK_MAX], s[NTOK_MAX];
#pragma unroll
  for (int n = 0; n < NTOK_MAX; ++n) {
    const bool ok = on && n < N;
    kv[n] = ok ? K[((long)hh * N + n) * D + l] : 0.f;
    vv[n] = ok ? V[((long)hh * N + n) * D + l] : 0.f;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int n = 0; n < NTOK_MAX; ++n) {
    if (n < N) {
      s[n] = wave_sum(qv * kv[n]) * scale;
      mx = fmaxf(mx, s[n]);
    }
  }
  float den = 0.f;
#pragma unroll
  for (int n = 0; n < NTOK_MAX; ++n) {
    if (n < N) {
      s[n] = __expf(s[n] - mx);
      den += s[n];
    }
  }
  const float inv = 1.f / den;
  float acc = 0.f;
#pragma unroll
  for (int n = 0; n < NTOK_MAX; ++n) {
    if (n < N) {
      const float wn = s[n] * inv;
      acc += wn * vv[n];
      if (l == n) wout[((long)b * NH + hh) * N + n] = wn;
    }
  }
  if (on) o[((long)b * NH + hh) * D + l] = acc;
}

// dq [B, NH*D]; part [B, 2, NH, N, D] = per-utterance (dK, dV) contributions.  dwts (optional):
// gradient w.r.t. the returned attention weights (e.g. a loss on the weights themselves).
__global__ void __launch_bounds__(64) token_attn_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ q,
                                                            const float* __restrict__ K, const float* __restrict__ V,
                                                            const float* __restrict__ wts,
                                                            const float* __restrict__ dwts, int NH, int N, int D,
                                                            float scale, float* __restrict__ dq,
                                                            float* __restrict__ part) {
  const int b = blockIdx.x, l = threadIdx.x;
  const long pstride = (long)NH * N * D;
  for (int hh = 0; hh < NH; ++hh) {
    const long qo = ((long)b * NH + hh) * D + l;
    const float qv = l < D ? q[qo] : 0.f;
    const float dov = l < D ? dout[qo] : 0.f;
    float dw[NTOK_MAX], wn[NTOK_MAX];
    float sdw = 0.f;
    for (int n = 0; n < N; ++n) {
      wn[n] = wts[((long)b * NH + hh) * N + n];
      dw[n] = wave_sum(l < D ? dov * V[((long)hh * N + n) * D + l] : 0.f);
      if (dwts) dw[n] += dwts[((long)b * NH + hh) * N + n];
      sdw += wn[n] * dw[n];
    }
    float dql = 0.f;
    for (int n = 0; n < N; ++n) {
      const float ds = wn[n] * (dw[n] - sdw) * scale;
      if (l < D) {
        const long ko = ((long)hh * N + n) * D + l;
        dql += ds * K[ko];
        part[(long)b * 2 * pstride + ko] = ds * qv;
        part[(long)b * 2 * pstride + pstride + ko] = wn[n] * dov;
      }
    }
    if (l < D) dq[qo] = dql;
  }
}

// out[c] = sum_b part[b, c] (fixed order: deterministic)
__global__ void __launch_bounds__(256) colsum_f32_kernel(const float* __restrict__ part, long rows, long ncol,
                                                         float* __restrict__ out) {
  const long c = (long)blockIdx.x * 256 + threadIdx.x;
  if (c >= ncol) return;
  float acc = 0.f;
  for (long r = 0; r < rows; ++r) acc += part[r * ncol + c];
  out[c] = acc;
}

// Style-token bank (reference GST, models/style.py::token_bank): keys = tanh(E) [N][dt];
//   K[h][n][d] = sum_c keys[n][c] Wk[h*D + d][c],  V likewise with Wv  (T = NH * D outputs per token).
// Tiny (N <= 64 tokens, dt, T <= 512), fp32, fixed-order sums (bitwise reproducible).  One output element
// per thread over as many workgroups as there are outputs (one serial workgroup took ~100 us per backward).
__global__ void __launch_bounds__(256) token_bank_fwd_kernel(const float* __restrict__ E, const float* __restrict__ Wk,
                                                             const float* __restrict__ Wv, int N, int dt, int T,
                                                             int D, float* __restrict__ K, float* __restrict__ V,
                                                             float* __restrict__ tE) {
  extern __shared__ float te[];  // [N][dt], recomputed by every workgroup
  for (int i = threadIdx.x; i < N * dt; i += blockDim.x) {
    const float t = tanhf(E[i]);
    te[i] = t;
    if (blockIdx.x == 0) tE[i] = t;
  }
  __syncthreads();
  {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * T) return;
    const int n = i / T, t = i - n * T;
    float a = 0.f, b = 0.f;
    for (int c = 0; c < dt; ++c) {
      const float x = te[n * dt + c];
      a = fmaf(x, Wk[t * dt + c], a);
      b = fmaf(x, Wv[t * dt + c], b);
    }
    const int h = t / D, d = t - h * D;
    K[((long)h * N + n) * D + d] = a;
    V[((long)h * N + n) * D + d] = b;
  }
}

// dWk[t][c] = sum_n dK[n][t] tE[n][c];  dE[n][c] = (1 - tE^2) sum_t (dK[n][t] Wk[t][c] + dV[n][t] Wv[t][c])
__global__ void __launch_bounds__(256) token_bank_bwd_kernel(const float* __restrict__ dK, const float* __restrict__ dV,
                                                             const float* __restrict__ tE,
                                                             const float* __restrict__ Wk,
                                                             const float* __restrict__ Wv, int N, int dt, int T,
                                                             int D, float* __restrict__ dE, float* __restrict__ dWk,
                                                             float* __restrict__ dWv) {
  auto gk = [&](const float* g, int n, int t) {
    const int h = t / D, d = t - h * D;
    return g[((long)h * N + n) * D + d];
  };
  const int nb1 = (T * dt + blockDim.x - 1) / blockDim.x;  // workgroups [0, nb1): dWk / dWv, the rest: dE
  if ((int)blockIdx.x < nb1) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T * dt) return;
    const int t = i / dt, c = i - t * dt;
    float a = 0.f, b = 0.f;
    for (int n = 0; n < N; ++n) {
      const float x = tE[n * dt + c];
      a = fmaf(gk(dK, n, t), x, a);
      b = fmaf(gk(dV, n, t), x, b);
    }
    dWk[i] = a;
    dWv[i] = b;
    return;
  }
  {
    const int i = (blockIdx.x - nb1) * blockDim.x + threadIdx.x;
    if (i >= N * dt) return;
    const int n = i / dt, c = i - n * dt;
    float a = 0.f;
    for (int t = 0; t < T; ++t) a = fmaf(gk(dK, n, t), Wk[t * dt + c], fmaf(gk(dV, n, t), Wv[t * dt + c], a));
    const float x = tE[i];
    dE[i] = a * (1.f - x * x);
  }
}

}  // namespace

static inline int out_dim(int n) { return (n - 1) / 2 + 1; }  // k3, s2, p1

SSAMD_API int ssamd_im2col_s2(const bf16_t* x, bf16_t* col, int B, int H, int W, int C, int Kp, hipStream_t s) {
  if (Kp % 8 || Kp < 9 * C || (C % 8 && C != 1)) return -2;
  const int Ho = out_dim(H), Wo = out_dim(W);
  const long n = (long)B * Ho * Wo * (Kp / 8);
  if (n == 0) return 0;
  hipLaunchKernelGGL(im2col_s2_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, x, col, H, W, C, Ho, Wo, Kp, n);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_col2im_s2(const bf16_t* dcol, bf16_t* dx, int B, int H, int W, int C, int Kp, hipStream_t s) {
  if (C % 8 || Kp < 9 * C) return -2;
  const long n = (long)B * H * W * (C / 8);
  if (n == 0) return 0;
  hipLaunchKernelGGL(col2im_s2_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, dcol, dx, H, W, C, out_dim(H), out_dim(W),
                     Kp, n);
  return (int)hipGetLastError();
}

// Hd (gst.gru_hidden) in {64, 128, 256}
SSAMD_API int ssamd_gru_fwd(const float* gi, const bf16_t* whh, const float* bhh, const int64_t* last, int B, int T,
                            int Hd, float* hlast, float* sv, bf16_t* hprev, hipStream_t s) {
  if (Hd != 64 && Hd != 128 && Hd != 256) return -2;
  if (B == 0 || T == 0) return 0;
  auto k = Hd == 64 ? gru_fwd_kernel<64> : Hd == 128 ? gru_fwd_kernel<128> : gru_fwd_kernel<256>;
  hipLaunchKernelGGL(k, dim3(cdiv(B, 16)), dim3(gru_threads(Hd)), 0, s, gi, whh, bhh, last, B, T, hlast, sv, hprev);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_gru_bwd(const float* dhlast, const float* sv, const bf16_t* whhT, const int64_t* last, int B, int T,
                            int Hd, bf16_t* dgi, bf16_t* dgh, hipStream_t s) {
  if (Hd != 64 && Hd != 128 && Hd != 256) return -2;
  if (B == 0 || T == 0) return 0;
  auto k = Hd == 64 ? gru_bwd_kernel<64> : Hd == 128 ? gru_bwd_kernel<128> : gru_bwd_kernel<256>;
  hipLaunchKernelGGL(k, dim3(cdiv(B, 16)), dim3(gru_threads(Hd)), 0, s, dhlast, sv, whhT, last, B, T, dgi, dgh);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_token_attn_fwd(const float* q, const float* K, const float* V, int B, int NH, int N, int D,
                                   float scale, float* o, float* w, hipStream_t s) {
  if (N > NTOK_MAX || D > 64) return -2;
  if (B == 0) return 0;
  hipLaunchKernelGGL(token_attn_fwd_kernel, dim3(B, NH), dim3(64), 0, s, q, K, V, NH, N, D, scale, o, w);
  return (int)hipGetLastError();
}

// part: B * 2*NH*N*D floats of workspace; dKV [2, NH, N, D] = (dK, dV)
SSAMD_API int ssamd_token_attn_bwd(const float* dout, const float* q, const float* K, const float* V, const float* w,
                                   const float* dw, int B, int NH, int N, int D, float scale, float* dq, float* part,
                                   float* dKV, hipStream_t s) {
  if (N > NTOK_MAX || D > 64) return -2;
  const long ncol = 2L * NH * N * D;
  if (B == 0) {
    hipMemsetAsync(dKV, 0, ncol * sizeof(float), s);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(token_attn_bwd_kernel, dim3(B), dim3(64), 0, s, dout, q, K, V, w, dw, NH, N, D, scale, dq, part);
  hipLaunchKernelGGL(colsum_f32_kernel, dim3(cdiv(ncol, 256)), dim3(256), 0, s, part, (long)B, ncol, dKV);
  return (int)hipGetLastError();
}

// K / V [NH][N][D] and tanh(E) [N][dt] of the style-token bank (Wk / Wv: [T = NH*D][dt] Linear weights)
SSAMD_API int ssamd_token_bank_fwd(const float* E, const float* Wk, const float* Wv, int N, int dt, int T, int NH,
                                   float* K, float* V, float* tE, hipStream_t s) {
  if (N <= 0 || NH <= 0 || T % NH || (size_t)N * dt * 4 > 64 * 1024) return -2;
  hipLaunchKernelGGL(token_bank_fwd_kernel, dim3(cdiv((long)N * T, 256)), dim3(256), (size_t)N * dt * 4, s, E, Wk, Wv,
                     N, dt, T, T / NH, K, V, tE);
  return (int)hipGetLastError();
}

SSAMD_API int ssamd_token_bank_bwd(const float* dK, const float* dV, const float* tE, const float* Wk, const float* Wv,
                                   int N, int dt, int T, int NH, float* dE, float* dWk, float* dWv, hipStream_t s) {
  if (N <= 0 || NH <= 0 || T % NH) return -2;
  hipLaunchKernelGGL(token_bank_bwd_kernel, dim3(cdiv((long)T * dt, 256) + cdiv((long)N * dt, 256)), dim3(256), 0, s,
                     dK, dV, tE, Wk, Wv, N, dt, T, T / NH, dE, dWk, dWv);
  return (int)hipGetLastError();
}
