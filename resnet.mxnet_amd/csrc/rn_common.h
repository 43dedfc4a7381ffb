// rn_common.h -- shared device helpers for librn (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <type_traits>

#include "../../include/rn.h"

typedef uint16_t bf16_t;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ error reporting
void rn_set_error(const std::string& msg);
#define RN_CHECK_ARG(cond, msg)                                                              \
  do {                                                                                     \
    if (!(cond)) {                                                                         \
      rn_set_error(std::string(__func__) + ": " + (msg));                                  \
      return -1;                                                                           \
    }                                                                                      \
  } while (0)
int rn_check_launch(const char* where);

// ------------------------------------------------------------------ bf16 <-> f32
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN (MI355X_MICROARCH correctness table)
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ float to_f(bf16_t v) { return bf2f(v); }
__device__ __forceinline__ float to_f(float v) { return v; }
template <typename T> __device__ __forceinline__ T from_f(float f);
template <> __device__ __forceinline__ float from_f<float>(float f) { return f; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float f) { return f2bf(f); }

// A 16-byte chunk: 8 bf16 or 4 f32. All vector memory traffic moves whole chunks.
template <typename T> struct Chunk {
  static constexpr int N = 16 / sizeof(T);
};
__device__ __forceinline__ void chunk_to_f(const uint4& u, float* f, const bf16_t*) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void chunk_to_f(const uint4& u, float* f, const float*) {
  f[0] = __uint_as_float(u.x);
  f[1] = __uint_as_float(u.y);
  f[2] = __uint_as_float(u.z);
  f[3] = __uint_as_float(u.w);
}
__device__ __forceinline__ uint4 f_to_chunk(const float* f, const bf16_t*) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint4 f_to_chunk(const float* f, const float*) {
  return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]),
                    __float_as_uint(f[3]));
}

// ------------------------------------------------------------------ fast division
// n / d for 0 <= n < 2^31 via multiply-high (Granlund-Montgomery round-up variant).
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.s = l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// ------------------------------------------------------------------ wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
static inline hipStream_t as_stream(rn_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------ int8 fake quantization
// Shared by rn_misc.hip (Quantization_int8 on a tensor) and rn_conv.hip (the quantized stem).
// State: weights t = max|w|; activations t = EMA of max|x| (initialised from the first batch),
// symbol/clip_grad_quantization_int8.py:37-54 and quant_ops.py:17-31.
__device__ __forceinline__ float quant_state_update(float curmax, float* minmax, int is_weight, int is_train,
                                                   float decay, int first) {
  if (is_weight) {
    if (is_train && minmax) *minmax = curmax;
    return curmax;
  }
  if (is_train) *minmax = first ? curmax : (*minmax) * decay + curmax * (1.f - decay);
  return *minmax;
}
// round(clip(v, -t, t) / unit) * unit, unit = t / qmax; mx.nd.round is half away from zero (= roundf)
__device__ __forceinline__ float quant_value(float v, float t, float qmax, int clip) {
  const float unit = t / qmax;
  if (clip) v = fminf(fmaxf(v, -t), t);
  return unit > 0.f ? roundf(v / unit) * unit : 0.f;
}

// ------------------------------------------------------------------ tuning knobs (rn_set_tuning)
enum { RN_TUNE_WGRAD_DMA = 0, RN_TUNE_IGEMM_DMA = 1, RN_TUNE_WGRAD_BLOCKS_PER_CU = 2, RN_TUNE_DIAG_IGEMM_L1 = 3, RN_TUNE_IGEMM_BIG = 4, RN_TUNE_WGRAD_BIG = 5, RN_TUNE_DIAG_WGRAD_NOEPI = 6, RN_TUNE_IGEMM_SCHED = 7, RN_TUNE_IGEMM_MFMA = 8, RN_TUNE_IGEMM_ROWS = 9, RN_TUNE_IGEMM_PERSIST = 10, RN_TUNE_IGEMM_W4 = 11, RN_TUNE_POOL_BLOCK_BWD = 12, RN_TUNE_IGEMM_GD = 13, RN_TUNE_WGRAD_GD = 14, RN_TUNE_GROUP_DIRECT = 15, RN_TUNE_EPI_SYNC = 16, RN_TUNE_DETERMINISTIC = 17, RN_TUNE_BN_NT = 18, RN_TUNE_WGRAD_BAND = 19, RN_TUNE_IGEMM_PRIO = 20, RN_TUNE_WGRAD_SPLIT = 21, RN_TUNE_QUANT_DIV = 22, RN_TUNE_GBAND_SPLIT = 23, RN_TUNE_BN_MERGE = 24, RN_TUNE_SLAB_FEW = 25, RN_TUNE_CONV_BAND = 26, RN_TUNE_DGRAD_STREAM = 27, RN_TUNE_COUNT = 28 };
extern int g_tune[RN_TUNE_COUNT];
// Diagnostic modes (tuning keys 3, 6, 7 and rn_sgd_mom_update_pack_checked) produce wrong results on
// purpose (they isolate one cost of a kernel): compiled only into the diagnostic build (hipcc
// -DRN_DIAG=1 -> librn_diag.so). In librn.so their branches fold away and rn_set_tuning refuses the keys.
#ifndef RN_DIAG
#define RN_DIAG 0
#endif
constexpr bool kRnDiag = RN_DIAG != 0;
