// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
// Wave64 everywhere: lane = threadIdx.x & 63; reductions use 64-wide shuffles.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define SSAMD_API extern "C" __attribute__((visibility("default")))

typedef unsigned short bf16_t;  // raw bf16 storage
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef float float16v __attribute__((ext_vector_type(16)));

static __device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

static __device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
  return *reinterpret_cast<bf16_t*>(&b);
}

static __device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

static __device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based uniform RNG for dropout: no state, the backward pass regenerates
// the exact forward mask from (seed, element index).  PCG-style output hash.
static __device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
// Dropout salt of this translation unit (one device global per kernel file, loaded per training step by
// the file's salt kernel -- SSAMD_DROP_SALT_LOADER -- from a device value the trainer writes): mixed into
// every dropout mask, so a step captured in a HIP graph draws the masks of the step it replays (the
// step-dependent part of the dropout seed lives here, not in the per-op seeds baked into the launches).
static __device__ unsigned long long g_drop_salt;

// Keep-scales of the N (even) consecutive elements idx0 .. idx0+N-1 (idx0 even): one 32-bit hash per element
// PAIR, its high / low 16 bits the two elements' uniforms (u = bits / 2^16, kept iff bits >= ceil(p * 2^16)).
// Half the hashing of one hash per element (the BatchNorm-backward GEMM head and the LayerNorm kernels run
// it on every element they touch), p resolved to 2^-16.  The seed half of the hash depends only on
// idx >> 32, which a chunk starting at a multiple of N (N | 2^32) shares, so it is computed once per chunk.
template <int N>
static __device__ __forceinline__ void drop_scales(uint64_t seed, uint64_t idx0, float p, float* ks) {
  static_assert(N % 2 == 0, "drop_scales: even chunks");
  if (p <= 0.f) {
#pragma unroll
    for (int i = 0; i < N; ++i) ks[i] = 1.f;
    return;
  }
  const float keep = 1.f / (1.f - p);
  seed ^= g_drop_salt * 0x9E3779B97F4A7C15ULL;
  const uint32_t S = hash_u32((uint32_t)seed ^ (uint32_t)(idx0 >> 32) * 0x9E3779B9U) ^ (uint32_t)(seed >> 32);
  const uint32_t thr = (uint32_t)ceilf(p * 65536.0f);
  const uint32_t pair0 = (uint32_t)idx0 >> 1;
#pragma unroll
  for (int i = 0; i < N / 2; ++i) {
    const uint32_t h = hash_u32((pair0 + (uint32_t)i) ^ S);
    ks[2 * i] = (h >> 16) >= thr ? keep : 0.f;
    ks[2 * i + 1] = (h & 0xFFFFu) >= thr ? keep : 0.f;
  }
}

// BatchNorm activations (k_bn.hip forward / backward and the GEMM epilogue that starts the PostNet
// BatchNorm backward, k_gemm.hip): act 0 none, 1 tanh (PostNet), 2 ReLU (GST Conv2d stack)
static __device__ __forceinline__ float bn_fast_tanh(float z) {
  // 1 - 2/(exp(2z)+1): one exp + one rcp; saturates correctly for |z| large
  const float e = __expf(2.f * z);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);  // v_rcp_f32: no IEEE division sequence
}
static __device__ __forceinline__ float bn_act_fwd(int act, float z) {
  if (act == 1) return bn_fast_tanh(z);
  if (act == 2) return fmaxf(z, 0.f);
  return z;
}
// derivative of act at the pre-activation z
static __device__ __forceinline__ float bn_act_grad(int act, float z) {
  if (act == 1) {  // 1 - tanh^2 = 4 r (1 - r), r = 1 / (exp(2z) + 1): no cancellation where |tanh| -> 1
    const float r = __builtin_amdgcn_rcpf(__expf(2.f * z) + 1.f);
    return 4.f * (r - r * r);
  }
  if (act == 2) return z > 0.f ? 1.f : 0.f;
  return 1.f;
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Allow > 64 KiB of dynamic LDS for a kernel (gfx950: 160 KiB per CU).  Once per kernel.
template <typename Kern>
static inline void allow_lds(Kern k, size_t bytes) {
  if (bytes > 65536) hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// Deterministic fixed-order reductions (csrc/k_reduce.hip), callable from every kernel file's host code.
SSAMD_API int ssamd_seg_colsum(const float* P, long ld, int nseg, int rows, int ncols, float* out, long out_ld,
                               int accumulate, int ncols1, float* out2, float* ws, long ws_floats, hipStream_t s);
SSAMD_API int ssamd_small_sum(const float* P, int rows, int k, float* out, hipStream_t s);
// scratch floats seg_colsum needs for its two-level form
static inline long seg_colsum_ws(int nseg, int ncols) { return (long)nseg * 16 * ncols; }

// The per-step dropout-salt loader of a kernel file: ssamd_<name>_salt_load(src, stream) copies the device
// value *src into this file's g_drop_salt (one lane stores it).
#define SSAMD_DROP_SALT_LOADER(NAME)                                                              \
  namespace {                                                                                     \
  __global__ void NAME##_salt_kernel(const unsigned long long* __restrict__ src) {              \
    if (threadIdx.x == 0) g_drop_salt = src[0];                                                   \
  }                                                                                               \
  }                                                                                               \
  SSAMD_API int ssamd_##NAME##_salt_load(const unsigned long long* src, hipStream_t s) {          \
    hipLaunchKernelGGL(NAME##_salt_kernel, dim3(1), dim3(64), 0, s, src);                         \
    return (int)hipGetLastError();                                                                \
  }
