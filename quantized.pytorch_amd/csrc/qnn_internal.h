// Internal helpers shared by the qnn HIP translation units (gfx950 / CDNA4 only).
//
// Quantizer arithmetic restates models/modules/quantize.py:89-100 (the effective
// asymmetric branch) op-for-op in fp32:
//   t = fl(x + (-min)); u = fl(t / s) (IEEE division); u = clamp(u, 0, qmax);
//   q = rint(u) (round half to even);  x_hat = fl(fl(q * s) + min).
// The library is built with -ffp-contract=off so none of these is fused.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include <string>

#include "../../include/qnn.h"

namespace qnn {

void set_error(const std::string& msg);
int hip_check(hipError_t e, const char* what);
int arg_error(const char* what);

#define QNN_REQUIRE(cond, msg) \
  do {                         \
    if (!(cond)) return ::qnn::arg_error(msg); \
  } while (0)

// CU count of the calling thread's current device, queried once per device (race-free: a
// concurrent first call queries twice and stores the same value)
inline int device_cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

#define QNN_LAUNCH_CHECK(what) \
  do {                         \
    hipError_t _e = hipGetLastError(); \
    if (_e != hipSuccess) return ::qnn::hip_check(_e, what); \
  } while (0)

// -------------------------------------------------------------- device math
__device__ __forceinline__ float quant_code(float x, float neg_min, float scale, float qmax) {
  float t = x + neg_min;           // add_(-min_value)        :90
  float u = t / scale;             // div_(scale)             :90 (true fp32 division)
  u = u + 0.0f;                    // add_(qmin)              :90
  u = fminf(fmaxf(u, 0.0f), qmax); // clamp_(qmin, qmax)      :95
  return rintf(u);                 // round_()  half-to-even  :95
}

// quant_code without a per-element IEEE division, bit-identical to quant_code:
// with inv_scale = RN(1/scale) (the caller's correctly rounded 1.0f / scale) and
// q0 = RN(t * inv_scale) within 1 ulp of t/scale, the exact remainder r = t - q0*scale
// (one fma) and q = RN(q0 + r*inv_scale) give the correctly rounded quotient RN(t/scale)
// (Markstein's theorem; checked against IEEE division on 4e8 pairs concentrated at
// half-integer quotients, tests/test_quant_math.py).  Branch-free: 5 VALU.  Quotients
// beyond 2^20 (and inf) take q0: they clamp to 0 or qmax whatever their last bit.
__device__ __forceinline__ float quant_code_fast(float x, float neg_min, float scale, float inv_scale, float qmax) {
  const float t = x + neg_min;
  const float q0 = t * inv_scale;
  const float r = fmaf(-q0, scale, t);
  float q = fmaf(r, inv_scale, q0);
  q = fabsf(q0) < 1048576.0f ? q : q0;
  return rintf(fminf(fmaxf(q, 0.0f), qmax));
}

// ---- packed-pair forms for the conv epilogues (v_pk_add/mul/fma_f32: two lanes' worth of
// the same IEEE fp32 ops per VALU instruction, so results are bitwise those of the scalar
// forms above)
typedef float f2 __attribute__((ext_vector_type(2)));

#if QNN_SCALAR_FMA
// two v_fma_f32 (inline asm, so the SLP vectorizer cannot re-form a v_pk_fma_f32)
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) {
  float x, y;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(x) : "v"(a.x), "v"(b.x), "v"(c.x));
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(y) : "v"(a.y), "v"(b.y), "v"(c.y));
  return (f2){x, y};
}
#else
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
#endif

struct QParams {  // one per-tensor quantizer: x -> code
  float nm, s, inv, qmax;  // -min, scale, RN(1/scale), 2^bits-1
};

__device__ __forceinline__ QParams make_qparams(float neg_min, float scale, float qmax) {
  return {neg_min, scale, 1.0f / scale, qmax};
}

// Clamped quotient clamp(RN((x + nm) / s), 0, qmax) of quant_code_fast for a pair, before the
// final round.  q0 is clamped to [-2^20, 2^20] first (one v_med3 per element, in place of
// quant_code_fast's |q0| < 2^20 select): inside that range the corrected quotient is the
// Markstein one; beyond it the true quotient is beyond [0, qmax] on the same side as the clamped
// q0, and the correction keeps it there (|r| <= ulp(q0) s for an unclamped q0; for a clamped one
// r = t - 2^20 s has the sign of t), so it clamps to the same 0 or qmax.  Without the clamp a
// finite t with t * inv overflowing (|t| > FLT_MAX * s, a tiny scale) made r = -inf and
// q = fma(-inf, inv, inf) = NaN (tests/test_quant_math.py: the clamp-free and the clamped
// forms against IEEE division, quotients out to overflow).
__device__ __forceinline__ f2 qclamp2(f2 x, const QParams& p) {
  const f2 t = x + p.nm;
  const f2 inv = {p.inv, p.inv}, s = {p.s, p.s};
  f2 q0 = t * inv;
  q0.x = __builtin_amdgcn_fmed3f(q0.x, -1048576.0f, 1048576.0f);
  q0.y = __builtin_amdgcn_fmed3f(q0.y, -1048576.0f, 1048576.0f);
  const f2 r = pfma(-q0, s, t);
  f2 q = pfma(r, inv, q0);
  q.x = __builtin_amdgcn_fmed3f(q.x, 0.0f, p.qmax);
  q.y = __builtin_amdgcn_fmed3f(q.y, 0.0f, p.qmax);
  return q;
}

__device__ __forceinline__ f2 rint2(f2 q) { return (f2){__builtin_rintf(q.x), __builtin_rintf(q.y)}; }

// q in [0, 255] plus one of these lands in [2^23, 2^24) (ulp 1, even magic: RN-even ties
// are those of rint), so the sum's low mantissa byte is rint(q) (U8) or rint(q) - 128 mod
// 256 (S8, the int8 code' of the NHWC8 layout).
constexpr float MAGIC_U8 = 12582912.0f;  // 1.5 * 2^23
constexpr float MAGIC_S8 = 12582784.0f;  // 1.5 * 2^23 - 128

// low bytes of four magic-shifted values -> one dword (byte u = value u)
__device__ __forceinline__ int pack4(f2 a, f2 b) {
  const unsigned p01 = __builtin_amdgcn_perm(__float_as_uint(a.y), __float_as_uint(a.x), 0x0c0c0400u);
  const unsigned p23 = __builtin_amdgcn_perm(__float_as_uint(b.y), __float_as_uint(b.x), 0x0c0c0400u);
  return (int)__builtin_amdgcn_perm(p23, p01, 0x05040100u);
}

__device__ __forceinline__ float dequant(float q, float scale, float min) {
  float v = q * scale;             // add_(-qmin).mul_(scale) :100
  return v + min;                  // add_(min_value)         :100
}

__device__ __forceinline__ float fake_quant(float x, float neg_min, float min, float scale, float qmax) {
  return dequant(quant_code(x, neg_min, scale, qmax), scale, min);
}

// Wave64 reductions.
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Element (m, c) of an fp32 [M][C] map in the C-tile layout (include/qnn.h, qnn_epilogue):
// the MFMA 32x32 accumulator image, ct = ceil(C / 32) tile columns.
__device__ __forceinline__ int64_t ctile_index(int64_t m, int c, int ct) {
  return ((((m >> 5) * ct + (c >> 5)) * 4 + ((c & 31) >> 3)) << 8) + (((m & 31) + ((c & 4) << 3)) << 2) + (c & 3);
}

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace qnn
