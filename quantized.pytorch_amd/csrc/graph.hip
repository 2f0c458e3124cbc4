// Fused model-graph kernels around the int8 contraction (HBM-bound, NHWC, coalesced
// along channels, 4 channels per thread): code-domain max-pool, fused depthwise conv,
// avg-pool head.  Reference semantics cited per entry in include/qnn.h.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "qconv_common.h"

// depthwise 3x3 thread shape (MobileNet b512 depthwise, in-graph: 8 channels x 1 x 4 pixels at two
// waves per SIMD 1.08-1.09 ms; 4 channels x 2 x 4 at three 1.006-1.009, x 3 x 4 / x 4 x 4 at two
// 0.997-1.023 -- profiles/r5_dw_occupancy_ab.txt)
#ifndef QNN_DW_WPE
#define QNN_DW_WPE 3  // depthwise: waves per SIMD the register budget is sized for
#endif
#ifndef QNN_DW_P
#define QNN_DW_P 2  // depthwise: channel pairs per thread (4: 8 channels, 8-byte loads; 2: 4 channels)
#endif
#ifndef QNN_DW_RR
#define QNN_DW_RR 2  // depthwise: output rows per thread
#endif

namespace qnn {

__device__ __forceinline__ float bn_apply(float q, const qnn_bn_params& b, int c) {
  float o = dequant(q, b.scale, b.min) - b.mean[c];  // (x - mean)      quantize.py:488
  o = o * b.sq[c];                                    // * q(scale)      :488-489
  o = o * b.wq[c];                                    // * q(weight)     :495
  return o + b.bq[c];                                 // + q(bias)       :499
}

__device__ __forceinline__ void put_code4(const qnn_code_out& o, int n, int h, int w, int c, const float v[4]) {
  int8_t* p = o.ptr + (((int64_t)n * o.hp + h + o.pad) * o.wp + w + o.pad) * o.cp + c;
  int r = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) r |= (((int)quant_code(v[u], o.neg_min, o.scale, o.qmax) - 128) & 255) << (8 * u);
  *reinterpret_cast<int*>(p) = r;
}

__device__ __forceinline__ void decode_pix(int64_t i, int cg, int wo, int ho, int& g, int& ox, int& oy, int& img) {
  g = (int)(i % cg);
  int64_t t = i / cg;
  ox = (int)(t % wo);
  t /= wo;
  oy = (int)(t % ho);
  img = (int)(t / ho);
}

// ------------------------------------------------------------------ max-pool on RangeBN codes
// One thread per (output pixel, 16 channels), channel groups fastest (each window tap is
// one contiguous c-byte read per pixel).  The pool
// direction per channel (max where g_c increases, min where it decreases) is folded
// into the codes with an XOR (min q == 255 - max(255 - q)), so the window reduction is
// a plain bytewise max (two packed-u16 maxes per dword).  RangeBN params and the
// consumer code tables live in LDS.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t max_u8x4(uint32_t a, uint32_t b) {
  u16x2 alo = __builtin_bit_cast(u16x2, a & 0x00ff00ffu), ahi = __builtin_bit_cast(u16x2, (a >> 8) & 0x00ff00ffu);
  u16x2 blo = __builtin_bit_cast(u16x2, b & 0x00ff00ffu), bhi = __builtin_bit_cast(u16x2, (b >> 8) & 0x00ff00ffu);
  u16x2 lo = __builtin_elementwise_max(alo, blo), hi = __builtin_elementwise_max(ahi, bhi);
  return __builtin_bit_cast(uint32_t, lo) | (__builtin_bit_cast(uint32_t, hi) << 8);
}

__global__ __launch_bounds__(256) void maxpool_bn_kernel(const uint8_t* __restrict__ q, int n, int h, int w, int c,
                                                         int k, int stride, int pad, int ho, int wo,
                                                         qnn_bn_params bn, int relu, float* out_f32, int tiled,
                                                         uint8_t* __restrict__ out_code,
                                                         const int8_t* __restrict__ lut0, qnn_code_out c0,
                                                         const int8_t* __restrict__ lut1, qnn_code_out c1) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  float* s_mean = reinterpret_cast<float*>(smem);
  float* s_sq = s_mean + c;
  float* s_wq = s_sq + c;
  float* s_bq = s_wq + c;
  uint8_t* s_dir = reinterpret_cast<uint8_t*>(s_bq + c);  // 0xff where g_c is non-increasing
  int8_t* s_lut0 = reinterpret_cast<int8_t*>(s_dir + c);
  int8_t* s_lut1 = s_lut0 + (lut0 ? c * 256 : 0);
  for (int i = threadIdx.x; i < c; i += blockDim.x) {
    s_mean[i] = bn.mean[i];
    s_sq[i] = bn.sq[i];
    s_wq[i] = bn.wq[i];
    s_bq[i] = bn.bq[i];
    s_dir[i] = (bn.sq[i] * bn.wq[i]) < 0.f ? 0xff : 0;
  }
  for (int i = threadIdx.x; i < c * 16; i += blockDim.x) {
    if (lut0) reinterpret_cast<int4*>(s_lut0)[i] = reinterpret_cast<const int4*>(lut0)[i];
    if (lut1) reinterpret_cast<int4*>(s_lut1)[i] = reinterpret_cast<const int4*>(lut1)[i];
  }
  __syncthreads();
  const int kc = c >> 4, ct = (c + 31) >> 5;
  const int64_t M = (int64_t)n * ho * wo;
  const int64_t total = M * kc;
  // the 16-channel group is the fastest index: a pixel's c bytes are one contiguous read
  for (int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gi < total; gi += (int64_t)gridDim.x * blockDim.x) {
    const int kg = (int)(gi % kc);
    const int64_t m = gi / kc;
    const int cb = 16 * kg;
    const int ox = (int)(m % wo);
    const int64_t t = m / wo;
    const int oy = (int)(t % ho), img = (int)(t / ho);
    const uint4 dm = *reinterpret_cast<const uint4*>(s_dir + cb);
    uint4 best = make_uint4(0, 0, 0, 0);
    auto tap = [&](int r, int s2) {
      // MaxPool2d pads with -inf: an out-of-image tap reads a clamped in-image pixel and
      // is masked to 0, the identity of the folded-code max (all loads issue together)
      const int iy = oy * stride - pad + r, ix = ox * stride - pad + s2;
      const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
      const int cy = min(max(iy, 0), h - 1), cx = min(max(ix, 0), w - 1);
      const uint4 v = *reinterpret_cast<const uint4*>(q + (((int64_t)img * h + cy) * w + cx) * c + cb);
      const uint32_t msk = ok ? 0xffffffffu : 0u;
      best.x = max_u8x4(best.x, (v.x ^ dm.x) & msk);
      best.y = max_u8x4(best.y, (v.y ^ dm.y) & msk);
      best.z = max_u8x4(best.z, (v.z ^ dm.z) & msk);
      best.w = max_u8x4(best.w, (v.w ^ dm.w) & msk);
    };
    if (k == 3) {
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) tap(r, s2);
    } else {
      for (int r = 0; r < k; ++r)
        for (int s2 = 0; s2 < k; ++s2) tap(r, s2);
    }
    const uint32_t qd[4] = {best.x ^ dm.x, best.y ^ dm.y, best.z ^ dm.z, best.w ^ dm.w};
    if (out_code) {  // the pooled RangeBN input codes: a residual chain start (byte C-tile)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int ch = cb + 4 * s4;
        *reinterpret_cast<uint32_t*>(out_code + btile_off((int)(m >> 5), ch >> 5, ct, (int)(m & 31) + 32 * ((ch >> 2) & 1)) +
                                     4 * ((ch & 31) >> 3)) = qd[s4];
      }
    }
    if (out_f32) {
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ch = cb + 4 * s4 + u;
          float o = dequant((float)((qd[s4] >> (8 * u)) & 255), bn.scale, bn.min) - s_mean[ch];  // quantize.py:488
          o = o * s_sq[ch];                                                                     // :488-489
          o = o * s_wq[ch];                                                                     // :495
          o = o + s_bq[ch];                                                                     // :499
          v[u] = relu ? fmaxf(o, 0.f) : o;
        }
        const int64_t fi = tiled ? ctile_index(m, cb + 4 * s4, ct) : m * c + cb + 4 * s4;
        *reinterpret_cast<float4*>(out_f32 + fi) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      const qnn_code_out& co = o ? c1 : c0;
      const int8_t* sl = o ? s_lut1 : s_lut0;
      if (!co.ptr) continue;
      int r[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        r[s4] = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ch = cb + 4 * s4 + u;
          r[s4] |= ((int)(uint8_t)sl[ch * 256 + ((qd[s4] >> (8 * u)) & 255)]) << (8 * u);
        }
      }
      *reinterpret_cast<int4*>(co.ptr + (((int64_t)img * co.hp + oy + co.pad) * co.wp + ox + co.pad) * co.cp + cb) =
          make_int4(r[0], r[1], r[2], r[3]);
    }
  }
}

// ------------------------------------------------------------------ depthwise, fused
// x: padded NHWC8 [n][hp][wp][cp], image interior at [pad, pad+h) x [pad, pad+w).
// Taps outside the image are skipped: zero padding applies to x_hat (quantize.py:343),
// and code' 0 there is NOT x_hat = 0 for a direct fp32 sum.
__global__ void dwconv_fused_kernel(const int8_t* __restrict__ x, int n, int h, int w, int pad, int hp, int wp,
                                    int cp, int c, const float* __restrict__ wt, int kh, int kw, int sh, int sw,
                                    int ho, int wo, float x_min, float x_scale, const float* bias, qnn_bn_params bn,
                                    int has_bn, int relu, float* out_f32, qnn_code_out c0) {
  const int cg = c >> 2;
  const int64_t total = (int64_t)n * ho * wo * cg;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int g, ox, oy, img;
    decode_pix(i, cg, wo, ho, g, ox, oy, img);
    const int cbase = 4 * g;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < kh; ++r) {
      const int py = oy * sh + r;  // padded-buffer row; image row py - pad
      if (py < pad || py >= pad + h) continue;
      for (int s = 0; s < kw; ++s) {
        const int px = ox * sw + s;
        if (px < pad || px >= pad + w) continue;
        const uint32_t v = *reinterpret_cast<const uint32_t*>(x + (((int64_t)img * hp + py) * wp + px) * cp + cbase);
        const float4 w4 = *reinterpret_cast<const float4*>(wt + (int64_t)(r * kw + s) * c + cbase);
        const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int code = (int)(int8_t)((v >> (8 * u)) & 255) + 128;
          acc[u] = fmaf(dequant((float)code, x_scale, x_min), wv[u], acc[u]);
        }
      }
    }
    float val[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ch = cbase + u;
      float y = bias ? acc[u] + bias[ch] : acc[u];
      if (has_bn) y = bn_apply(quant_code(y, bn.neg_min, bn.scale, bn.qmax), bn, ch);
      val[u] = relu ? fmaxf(y, 0.f) : y;
    }
    if (out_f32)
      *reinterpret_cast<float4*>(out_f32 + (((int64_t)img * ho + oy) * wo + ox) * c + cbase) =
          make_float4(val[0], val[1], val[2], val[3]);
    if (c0.ptr) put_code4(c0, img, oy, ox, cbase, val);
  }
}

// Depthwise 3x3 (MobileNet's every depthwise layer), same arithmetic op for op as
// dwconv_fused_kernel (so bitwise equal to it and to the module path): each tap's
// x_hat = fl(fl(q*s)+min), fmaf into the accumulator in (r, s) row-major order with
// out-of-image taps skipped, + bias, RangeBN on its quantized input, ReLU, the
// consumer's codes.  Layout of the work instead: a thread owns CPT channels (4: 4-byte
// loads, coalesced along channels across the ct = cs/CPT channel threads) of an RR x R
// block of output pixels (2 rows x 4 or 2 columns), so each input pixel of the block's
// windows is dequantized once and feeds up to 9 outputs from registers; the 9 x CPT tap
// weights, the bias and the RangeBN vectors live in registers; both quantizers run
// division-free (quant_code_fast, bit-identical); 32-bit buffer offsets.
// LUT (qnn_dwconv_fused_lut): RangeBN -> ReLU -> the consumer's quantizer of each channel is
// the exact per-channel table qnn_bn_code_lut builds over the RangeBN input code (the conv
// kernels' EK_LUT), so after the RangeBN input quotient each code is one LDS byte lookup --
// half the kernel's VALU work per output was that chain.  A block then covers a slice of cs
// channels (<= 128: a 32 KiB table slice in LDS), blocks of one pixel range and every slice
// adjacent in the XCD-grouped order.
template <int S, int R, int P, bool LUT, int RR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(QNN_DW_WPE))) void dwconv3_kernel(const int8_t* __restrict__ x, int h, int w, int pad, int hp,
                                                      int wp, int cp, int c, const float* __restrict__ wt, int ho,
                                                      int wo, float x_min, float x_scale, const float* bias,
                                                      qnn_bn_params bn, int has_bn, int relu,
                                                      float* out_f32, qnn_code_out c0, int rows, const int8_t* __restrict__ lut,
                                                      int cs, int xbytes) {
  // a thread: CPT channels of an RR x R block of output pixels (RR rows, R columns), reading
  // the KR x NCOL input pixels of their windows once
  constexpr int K = 3, NCOL = (R - 1) * S + K, KR = (RR - 1) * S + K, CPT = 2 * P;
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  using LT = std::conditional_t<P == 4, u32x2, uint32_t>;    // one tap of them: 8 or 4 code bytes
  const int nsl = c / cs, ct = cs / CPT, per_blk = 256 / ct;
  const int tc = threadIdx.x % ct, tp = threadIdx.x / ct;
  const int nxg = (wo + R - 1) / R, total = rows * nxg;
  // XCD-aware block order: blocks are dealt round-robin over the 8 XCDs (b and b + 8 share
  // one), so logical block L = the bijective XCD-major index of b gives each XCD a contiguous
  // range of L -- adjacent output rows, whose 3x3 windows share input rows, are then computed
  // on one XCD and the halo rows are served by its L2 instead of being fetched once per XCD
  int blk;
  {
    const int nb = gridDim.x, bb = blockIdx.x, xcd = bb & 7, q = nb >> 3, r = nb & 7;
    blk = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bb >> 3);
  }
  const int sl = blk % nsl, pblk = blk / nsl;   // channel slice, pixel block
  const int cbl = CPT * tc, cb = sl * cs + cbl;  // this thread's channels: local, global
  extern __shared__ __attribute__((aligned(16))) int8_t s_lut[];
  if constexpr (LUT) {  // the slice's code table [cs][256], before any thread may leave
    const int8_t* src = lut + (size_t)sl * cs * 256;
    for (int i = 16 * threadIdx.x; i < cs * 256; i += 16 * 256)
      *reinterpret_cast<uint4*>(s_lut + i) = *reinterpret_cast<const uint4*>(src + i);
    __syncthreads();
  }
  if (tp >= per_blk) return;  // cs/CPT not a divisor of 256: idle tail threads
  if (pblk * per_blk + tp >= total) return;
  // every per-channel quantity as packed pairs (channels 2p, 2p+1): v_pk_fma/mul/add run the
  // same IEEE fp32 op per element as the scalar form, so the results are bitwise unchanged
  f2 wv[K * K][P];
#pragma unroll
  for (int t = 0; t < K * K; ++t) {
    const float4 a = *reinterpret_cast<const float4*>(wt + t * c + cb);
    wv[t][0] = (f2){a.x, a.y}, wv[t][1] = (f2){a.z, a.w};
    if constexpr (P == 4) {
      const float4 b = *reinterpret_cast<const float4*>(wt + t * c + cb + 4);
      wv[t][2] = (f2){b.x, b.y}, wv[t][3] = (f2){b.z, b.w};
    }
  }
  f2 bi[P], mean[P], sq[P], wq[P], bq[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    bi[p] = bias ? (f2){bias[cb + 2 * p], bias[cb + 2 * p + 1]} : (f2){0.f, 0.f};
    if (has_bn && !LUT) {
      mean[p] = (f2){bn.mean[cb + 2 * p], bn.mean[cb + 2 * p + 1]};
      sq[p] = (f2){bn.sq[cb + 2 * p], bn.sq[cb + 2 * p + 1]};
      wq[p] = (f2){bn.wq[cb + 2 * p], bn.wq[cb + 2 * p + 1]};
      bq[p] = (f2){bn.bq[cb + 2 * p], bn.bq[cb + 2 * p + 1]};
    }
  }
  const QParams bnp = make_qparams(bn.neg_min, bn.scale, bn.qmax);
  const QParams c0p = make_qparams(c0.neg_min, c0.scale, c0.qmax);
  const f2 bs2 = {bn.scale, bn.scale}, bm2 = {bn.min, bn.min};
  // (image, output row, pixel group) of group g: float reciprocals with an exact fix-up (groups
  // < 2^24 on the host), integer division otherwise -- once per thread; every later group is the
  // previous one advanced by the grid stride, in the same three coordinates
  const bool fdiv = total < (1 << 24);
  const int nyg = (ho + RR - 1) / RR;  // row groups per image (rows = n * nyg)
  const float inv_nxg = 1.0f / (float)nxg, inv_nyg = 1.0f / (float)nyg;
  auto divmod = [&](int m, int D, float invD, int& q, int& r) __attribute__((always_inline)) {
    if (fdiv) {
      q = (int)((float)m * invD);
      r = m - (int)__umul24((unsigned)q, (unsigned)D);
      if (r < 0) --q, r += D;
      if (r >= D) ++q, r -= D;
    } else {
      q = m / D, r = m - q * D;
    }
  };
  struct Pos {
    int img, oy, xg;  // oy: the group's first output row (a multiple of RR)
  };
  const int step = (gridDim.x / nsl) * per_blk;  // grid stride in groups (wave-uniform)
  const int st_row = step / nxg, st_xg = step - st_row * nxg, st_img = st_row / nyg;
  const int st_oy = (st_row - st_img * nyg) * RR, hoR = nyg * RR;
  auto advance = [&](Pos& q) __attribute__((always_inline)) {
    int dr = st_oy;
    q.xg += st_xg;
    if (q.xg >= nxg) q.xg -= nxg, dr += RR;
    q.oy += dr;
    q.img += st_img;
    if (q.oy >= hoR) q.oy -= hoR, ++q.img;
  };
  // The input as a buffer resource over its n*hp*wp*cp bytes (< 2^31 on the host): a tap load is
  // one 32-bit offset add, and a load past the end (the prefetch of the group after a thread's
  // last) returns zeros instead of faulting -- no clamping.  Every load is unconditional and all
  // K x NCOL are issued together (a load under a branch gets its own vmcnt(0) wait); the next
  // group's loads are in flight while this group computes.  Columns past a row's end read the
  // next row's bytes (or zeros): only taps outside the image read them, and those are skipped.
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, xbytes, 0x00020000);
  const int wpcp = wp * cp;
  auto load = [&](const Pos& q, LT (&v)[KR][NCOL]) __attribute__((always_inline)) {
    const uint32_t base = ((uint32_t)(q.img * hp + q.oy * S) * (uint32_t)wp + (uint32_t)(q.xg * R * S)) * (uint32_t)cp +
                          (uint32_t)cb;
#pragma unroll
    for (int r = 0; r < KR; ++r)
#pragma unroll
      for (int col = 0; col < NCOL; ++col) {
        const uint32_t o = base + (uint32_t)(r * wpcp + col * cp);
        if constexpr (P == 4) v[r][col] = __builtin_amdgcn_raw_buffer_load_b64(xrs, o, 0, 0);
        else v[r][col] = __builtin_amdgcn_raw_buffer_load_b32(xrs, o, 0, 0);
      }
  };
  // one pixel group on operands v, the next group's loads into vn (two groups per trip, the
  // buffers alternating: no register copies)
  auto group = [&](const Pos& cur, const Pos& nxt, LT (&v)[KR][NCOL], LT (&vn)[KR][NCOL]) __attribute__((always_inline)) {
    const int img = cur.img, oy0 = cur.oy;
    const int ox0 = cur.xg * R;
    load(nxt, vn);
    f2 acc[RR][R][P];
#pragma unroll
    for (int i = 0; i < RR; ++i)
#pragma unroll
      for (int j = 0; j < R; ++j)
#pragma unroll
        for (int p = 0; p < P; ++p) acc[i][j][p] = (f2){0.f, 0.f};

    // Taps outside the image (zero padding of x_hat), LUT kernels: without branches -- their
    // x_hat is made +0 exactly (q * 0 + 0), and fma(+0, w, acc) = acc for every acc the chain can
    // hold (it starts at +0 and an exact zero sum rounds to +0, so it is never -0): bitwise the
    // skipped tap, measured -4 % on MobileNet's depthwise layers.  The fp32-output kernels keep
    // the branches (the selects' registers would spill there).
    // (input row ri feeds output row i through kernel row ri - i S: each output's taps are
    // accumulated in row-major (r, s) order, as the generic kernel does)
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const bool rok = (unsigned)(oy0 * S + r - pad) < (unsigned)h;
#pragma unroll
      for (int col = 0; col < NCOL; ++col) {
        const bool ok = rok && (unsigned)(ox0 * S + col - pad) < (unsigned)w;
        if constexpr (!LUT) {
          if (!ok) continue;
        }
        const float ts = !LUT || ok ? x_scale : 0.f, tm = !LUT || ok ? x_min : 0.f;
        const f2 ts2 = {ts, ts}, tm2 = {tm, tm};
        uint32_t lo, hi = 0;  // code' ^ 0x80 = code
        if constexpr (P == 4) lo = v[r][col].x ^ 0x80808080u, hi = v[r][col].y ^ 0x80808080u;
        else lo = v[r][col] ^ 0x80808080u;
        f2 xh[P];  // dequant(q) = q * s + min (quantize.py:100), pairs
        xh[0] = (f2){(float)(lo & 255), (float)((lo >> 8) & 255)} * ts2 + tm2;
        xh[1] = (f2){(float)((lo >> 16) & 255), (float)(lo >> 24)} * ts2 + tm2;
        if constexpr (P == 4) {
          xh[2] = (f2){(float)(hi & 255), (float)((hi >> 8) & 255)} * ts2 + tm2;
          xh[3] = (f2){(float)((hi >> 16) & 255), (float)(hi >> 24)} * ts2 + tm2;
        }
        (void)hi;
#pragma unroll
        for (int i = 0; i < RR; ++i) {
          const int kr = r - i * S;
          if (kr < 0 || kr >= K) continue;  // compile-time
#pragma unroll
          for (int j = 0; j < R; ++j) {
            const int s = col - j * S;
            if (s < 0 || s >= K) continue;  // compile-time
#pragma unroll
            for (int p = 0; p < P; ++p) acc[i][j][p] = pfma(xh[p], wv[kr * K + s][p], acc[i][j][p]);
          }
        }
      }
    }

#pragma unroll
    for (int ij = 0; ij < RR * R; ++ij) {
      const int i = ij / R, j = ij % R;
      const int oy = oy0 + i, ox = ox0 + j;
      if (ox >= wo || oy >= ho) continue;
      if constexpr (LUT) {
        // RangeBN's input code per channel (the low mantissa byte of the magic-shifted clamped
        // quotient = its rint), then the consumer's code from the slice's table
        uint32_t cw[P / 2 > 0 ? P / 2 : 1];
#pragma unroll
        for (int p2 = 0; p2 < P; p2 += 2) {
          uint32_t wd = 0;
#pragma unroll
          for (int p = p2; p < p2 + 2 && p < P; ++p) {
            const f2 y = bias ? acc[i][j][p] + bi[p] : acc[i][j][p];
            const f2 m = qclamp2(y, bnp) + MAGIC_U8;
            const int ch = cbl + 2 * p;
            const uint32_t b0 = (uint8_t)s_lut[ch * 256 + (__float_as_uint(m.x) & 255u)];
            const uint32_t b1 = (uint8_t)s_lut[(ch + 1) * 256 + (__float_as_uint(m.y) & 255u)];
            wd |= (b0 | (b1 << 8)) << (16 * (p - p2));
          }
          cw[p2 / 2] = wd;
        }
        int8_t* cp0 = c0.ptr + (size_t)((img * c0.hp + oy + c0.pad) * c0.wp + ox + c0.pad) * (size_t)c0.cp + cb;
        if constexpr (P == 4) *reinterpret_cast<uint2*>(cp0) = make_uint2(cw[0], cw[1]);
        else *reinterpret_cast<uint32_t*>(cp0) = cw[0];
        continue;
      }
      f2 val[P];
#pragma unroll
      for (int p = 0; p < P; ++p) {
        f2 y = bias ? acc[i][j][p] + bi[p] : acc[i][j][p];
        if (has_bn) {  // bn_apply(quant_code(y)), quantize.py:488-499
          f2 o = rint2(qclamp2(y, bnp)) * bs2;
          o = o + bm2;
          o = o - mean[p];
          o = o * sq[p];
          o = o * wq[p];
          y = o + bq[p];
        }
        if (relu) y.x = fmaxf(y.x, 0.f), y.y = fmaxf(y.y, 0.f);
        val[p] = y;
      }
      if (out_f32) {
        float* o = out_f32 + (((size_t)img * ho + oy) * wo + ox) * c + cb;
        *reinterpret_cast<float4*>(o) = make_float4(val[0].x, val[0].y, val[1].x, val[1].y);
        if constexpr (P == 4) *reinterpret_cast<float4*>(o + 4) = make_float4(val[2].x, val[2].y, val[3].x, val[3].y);
      }
      if (c0.ptr) {
        int8_t* cp0 = c0.ptr + (size_t)((img * c0.hp + oy + c0.pad) * c0.wp + ox + c0.pad) * (size_t)c0.cp + cb;
        const int p0 = pack4(qclamp2(val[0], c0p) + MAGIC_S8, qclamp2(val[1], c0p) + MAGIC_S8);
        if constexpr (P == 4) {
          const int p1 = pack4(qclamp2(val[2], c0p) + MAGIC_S8, qclamp2(val[3], c0p) + MAGIC_S8);
          *reinterpret_cast<uint2*>(cp0) = make_uint2((uint32_t)p0, (uint32_t)p1);
        } else {
          *reinterpret_cast<uint32_t*>(cp0) = (uint32_t)p0;
        }
      }
    }
  };
  LT va[KR][NCOL], vb[KR][NCOL];
  Pos cur, nxt;
  {
    int row;
    divmod(pblk * per_blk + tp, nxg, inv_nxg, row, cur.xg);
    divmod(row, nyg, inv_nyg, cur.img, cur.oy);
    cur.oy *= RR;
  }
  nxt = cur;
  advance(nxt);
  load(cur, va);
  for (int pg = pblk * per_blk + tp; pg < total;) {
    group(cur, nxt, va, vb);
    cur = nxt;
    advance(nxt);
    pg += step;
    if (pg >= total) break;
    group(cur, nxt, vb, va);
    cur = nxt;
    advance(nxt);
    pg += step;
  }
}

// ------------------------------------------------------------------ RangeBN -> code LUT
__global__ void bn_code_lut_kernel(qnn_bn_params bn, int c, int relu, qnn_code_out nx, int8_t* lut) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c * 256) return;
  const int ch = i >> 8, q = i & 255;
  float v = bn_apply((float)q, bn, ch);
  if (relu) v = fmaxf(v, 0.f);
  lut[i] = (int8_t)((int)quant_code(v, nx.neg_min, nx.scale, nx.qmax) - 128);
}

// ------------------------------------------------------------------ avg-pool head
// Block = (image, 256 channels): lane = 4-channel group, wave w sums pixels w, w+4, ...
// (several loads in flight per lane), then wave 0 adds the four partial sums in a fixed
// order and divides by hw (adaptive_avg_pool / AvgPool2d eval; deterministic order).
// The classifier's avg-pool in the module path's summation order: torch's AvgPool2d kernel
// (aten avg_pool2d_out_cuda_frame) sums each output's window from +0 in row-major order, one
// fp32 add per tap, then divides once by the window size (count_include_pad), so one thread
// per 4 channels adds the hw pixels in order and divides: the engine's pooled features, and
// therefore its logits, are bitwise the module path's.
__global__ __launch_bounds__(64) void avgpool_quant_kernel(const float* __restrict__ x, int n, int hw, int c,
                                                           int tiled, float* out_f32, qnn_code_out c0) {
  const int img = blockIdx.y;
  const int g = blockIdx.x * 64 + threadIdx.x, cg = c >> 2, ct = (c + 31) >> 5;
  if (g >= cg) return;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 7
  for (int t = 0; t < hw; ++t) {
    const int64_t m = (int64_t)img * hw + t;
    const float4 v = *reinterpret_cast<const float4*>(x + (tiled ? ctile_index(m, 4 * g, ct) : m * c + 4 * g));
    s.x = s.x + v.x; s.y = s.y + v.y; s.z = s.z + v.z; s.w = s.w + v.w;
  }
  const float d = (float)hw;
  const float val[4] = {s.x / d, s.y / d, s.z / d, s.w / d};
  if (out_f32)
    *reinterpret_cast<float4*>(out_f32 + (int64_t)img * c + 4 * g) = make_float4(val[0], val[1], val[2], val[3]);
  if (c0.ptr) put_code4(c0, img, 0, 0, 4 * g, val);
}

// The same mean from a C-tile map, staged through LDS so the reads are coalesced: a 64-thread
// block owns one image and 64 channels; the C-tile stores 32 pixels x 8 channels contiguously
// (1 KiB, one float4 per lane), so each load instruction reads one such piece, scattered into LDS
// as [tap][64 channels] (row stride 68 floats: conflict-free 16-byte writes and reads); then thread = channel sums its taps in row-major order (s = s + v, as
// AvgPool2d), divides by hw, and the codes go out four channels per thread.  hw <= 128.
__global__ __launch_bounds__(64) void avgpool_tiled_kernel(const float* __restrict__ x, int n, int hw, int c,
                                                           float* out_f32, qnn_code_out c0) {
  extern __shared__ float s_x[];  // [hw][RS]: rows padded to 68 floats (the 32 pixels of a piece in distinct banks)
  const int img = blockIdx.y, cb = blockIdx.x * 64, lane = threadIdx.x;
  const int ct = (c + 31) >> 5;
  const int64_t mlo = (int64_t)img * hw, mhi = mlo + hw;
  const int64_t mt0 = mlo >> 5, mt1 = (mhi - 1) >> 5;
  const int mi = lane & 31, h = lane >> 5;
  for (int64_t mt = mt0; mt <= mt1; ++mt) {
    const int64_t m = mt * 32 + mi;
    const bool in = m >= mlo && m < mhi;
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // (channel tile, group of 8) pieces of this block's 64 channels
      const int ctile = (cb >> 5) + (k >> 2), g = k & 3;
      if (ctile >= ct) continue;
      const float4 v = *reinterpret_cast<const float4*>(x + (((mt * ct + ctile) * 4 + g) << 8) + lane * 4);
      const int cl = (k >> 2) * 32 + 8 * g + 4 * h;  // local channel of v.x
      if (in) *reinterpret_cast<float4*>(s_x + (m - mlo) * 68 + cl) = v;
    }
  }
  __syncthreads();
  float sum = 0.f;
#pragma unroll 8
  for (int t = 0; t < hw; ++t) sum = sum + s_x[t * 68 + lane];
  const float val = sum / (float)hw;
  const int ch = cb + lane;
  if (out_f32 && ch < c) out_f32[(int64_t)img * c + ch] = val;
  if (c0.ptr) {
    __syncthreads();
    s_x[lane] = val;
    __syncthreads();
    if (lane < 16 && cb + 4 * lane < c) {
      const float v4[4] = {s_x[4 * lane], s_x[4 * lane + 1], s_x[4 * lane + 2], s_x[4 * lane + 3]};
      put_code4(c0, img, 0, 0, cb + 4 * lane, v4);
    }
  }
}

static int grid_for(int64_t work) {
  int64_t g = cdiv(work, 256);
  if (g > 256 * 32) g = 256 * 32;
  return (int)(g < 1 ? 1 : g);
}

static qnn_code_out none_code() {
  qnn_code_out o;
  memset(&o, 0, sizeof(o));
  return o;
}

// ------------------------------------------------------------------ split chain epilogue
// The residual-chain tail of a ResNet block's last conv as its own launch (qnn_chain_epilogue):
// the conv writes only RangeBN's input codes (EK_BNCODE, byte C-tile), and this kernel -- no
// MFMA, so four waves per SIMD and packed FP32 -- evaluates everything the fused general
// epilogue did after the quotient, with the same fp32 ops in the same order (qconv.hip EK_GEN):
//   v = ((q_bn * s + min - mean) * sq * wq + bq)          RangeBN of the conv's own code
//   r = residual | chain links (qnn_res_link)             the block input, recomputed
//   v = relu(v + r); out_f32 = v; codes = quant(v)        (code1 = code0 for equal ranges)
// One thread per (32x32 tile, lane) = the lane's 16 byte-C-tile values: channels 8g + 4h + u of
// pixel 32 mt + (lane & 31), h = lane >> 5; a block stays on one channel tile (its RangeBN and
// link vectors staged once in LDS) and walks pixel tiles.
__device__ __forceinline__ int4 chain_gather16(int d0, int d1, int d2, int d3) {
  // lanes 0-31 hold channels 4h.. of groups g; two half-exchange levels leave lanes 0-31 with
  // channels 0-15 and lanes 32-63 with channels 16-31 of their pixel, in order (qconv.hip gather16)
  auto r01 = __builtin_amdgcn_permlane32_swap(d0, d1, false, false);
  auto r23 = __builtin_amdgcn_permlane32_swap(d2, d3, false, false);
  auto r02 = __builtin_amdgcn_permlane32_swap(r01[0], r23[0], false, false);
  auto r13 = __builtin_amdgcn_permlane32_swap(r01[1], r23[1], false, false);
  return make_int4((int)r02[0], (int)r13[0], (int)r02[1], (int)r13[1]);
}

// NRES links and RES (an fp32 checkpoint as the block input) are compile-time, so a launch
// carries only its chain (no runtime-branched link loop, no scalar spills); four waves per SIMD.
// FULL: c % 32 == 0, every channel of a tile exists (no per-group channel tests).
// (dx, dy, dn): a wave's pixel step between its tiles (32 * 4 * gridDim.x pixels) as columns,
// rows and images, so each lane's output coordinates advance by adds, not divisions.
template <int NRES, bool RES, bool FULL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void chain_epilogue_kernel(
    const uint8_t* __restrict__ bncode, int n, int ho, int wo, int c, int dx, int dy, int dn, const qnn_epilogue e) {
  __shared__ float4 s_v[(4 + 4 * QNN_MAX_RES) * 8];  // [vector][32 channels] as float4
  const int ct = (c + 31) >> 5, ctb = blockIdx.y;
  const int M = n * ho * wo, mts = (M + 31) >> 5;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  constexpr int nres = NRES;
  const int nvec = 4 + 4 * nres;
  float* sv = reinterpret_cast<float*>(s_v);
  for (int i = tid; i < nvec * 32; i += 256) {
    const int v = i >> 5, cc = min(ctb * 32 + (i & 31), c - 1);
    const float* src;
    if (v < 4) {
      src = v == 0 ? e.bn_mean : v == 1 ? e.bn_sq : v == 2 ? e.bn_wq : e.bn_bq;
    } else {
      const qnn_res_link& rl = e.res[(v - 4) >> 2];
      const int k = (v - 4) & 3;
      src = k == 0 ? rl.mean : k == 1 ? rl.sq : k == 2 ? rl.wq : rl.bq;
    }
    sv[i] = src[cc];
  }
  __syncthreads();
  const QParams c0p = make_qparams(e.code0_neg_min, e.code0_scale, e.code0_qmax);
  const QParams c1p = make_qparams(e.code1_neg_min, e.code1_scale, e.code1_qmax);
  const bool same01 = e.out_code0 && e.code1_neg_min == e.code0_neg_min && e.code1_scale == e.code0_scale &&
                      e.code1_qmax == e.code0_qmax;
  const f2 bn_s2 = {e.bn_scale, e.bn_scale}, bn_m2 = {e.bn_min, e.bn_min};
  const CodeDst t0 = {e.out_code0, e.code0_cp, e.code0_pad, e.code0_hp, e.code0_wp};
  const CodeDst t1 = {e.out_code1, e.code1_cp, e.code1_pad, e.code1_hp, e.code1_wp};
  const int HoWo = ho * wo;
  int nn, y, x;  // this lane's output pixel (image, row, column), advanced per tile
  {
    const int m0 = (blockIdx.x * 4 + (tid >> 6)) * 32 + (lane & 31);
    nn = m0 / HoWo;
    y = (m0 - nn * HoWo) / wo;
    x = m0 - nn * HoWo - y * wo;
  }
  // the next tile's code bytes are requested before this tile's arithmetic (one tile ahead)
  const int stride = gridDim.x * 4;
  int mt = blockIdx.x * 4 + (tid >> 6);
  uint4 qbn = make_uint4(0, 0, 0, 0), lqn[QNN_MAX_RES];
  auto fetch = [&](int t) {
    const int64_t o = ((int64_t)t * ct + ctb) * 1024 + lane * 16;
    qbn = *reinterpret_cast<const uint4*>(bncode + o);
#pragma unroll
    for (int l = 0; l < QNN_MAX_RES; ++l)
      if (l < nres) lqn[l] = *reinterpret_cast<const uint4*>(e.res[l].code + o);
  };
  if (mt < mts) fetch(mt);
  for (; mt < mts; mt += stride) {
    // the staged vectors are re-read per pixel tile: an opaque base keeps the compiler from
    // hoisting all (4 + 4 nres) x 16 of them into registers for the whole loop
    int vb = 0;
    asm volatile("" : "+v"(vb));
    const int m = mt * 32 + (lane & 31);
    const bool pok = m < M;
    const int mc = pok ? m : M - 1;
    const uint4 qb = qbn;
    uint4 lq[QNN_MAX_RES];
#pragma unroll
    for (int l = 0; l < QNN_MAX_RES; ++l)
      if (l < nres) lq[l] = lqn[l];
    if (mt + stride < mts) fetch(mt + stride);
    int k0[4], k1[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int cl = 8 * g + 4 * h;  // local channel of byte 4g (+u)
      const int cc = ctb * 32 + cl;
      const bool cok = FULL || cc < c;
      auto vec = [&](int v) { return s_v[vb + v * 8 + (cl >> 2)]; };
      auto bytes = [](unsigned wd, f2 (&q)[2]) {
        q[0] = (f2){(float)(wd & 255u), (float)((wd >> 8) & 255u)};
        q[1] = (f2){(float)((wd >> 16) & 255u), (float)(wd >> 24)};
      };
      // RangeBN of the conv's own code (the byte is the rounded quotient: rint2 is the identity)
      f2 v[2], qq[2];
      bytes(((const unsigned*)&qb)[g], qq);
      {
        const float4 mn4 = vec(0), sq4 = vec(1), wq4 = vec(2), bq4 = vec(3);
        const f2 mn[2] = {{mn4.x, mn4.y}, {mn4.z, mn4.w}}, sq[2] = {{sq4.x, sq4.y}, {sq4.z, sq4.w}};
        const f2 wq[2] = {{wq4.x, wq4.y}, {wq4.z, wq4.w}}, bq[2] = {{bq4.x, bq4.y}, {bq4.z, bq4.w}};
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          f2 o = qq[hh] * bn_s2;  // dequant: q * s
          o = o + bn_m2;          // + min
          o = o - mn[hh];         // x - mean
          o = o * sq[hh];         // * q(scale)
          o = o * wq[hh];         // * q(weight)
          v[hh] = o + bq[hh];     // + q(bias)
        }
      }
      // the block input: fp32, or recomputed from the chain exactly as its producers did
      auto link = [&](int l, f2 (&o)[2]) {
        f2 q[2];
        bytes(((const unsigned*)&lq[l])[g], q);
        const float4 mn4 = vec(4 + 4 * l), sq4 = vec(5 + 4 * l), wq4 = vec(6 + 4 * l), bq4 = vec(7 + 4 * l);
        const f2 mn[2] = {{mn4.x, mn4.y}, {mn4.z, mn4.w}}, sq[2] = {{sq4.x, sq4.y}, {sq4.z, sq4.w}};
        const f2 wq[2] = {{wq4.x, wq4.y}, {wq4.z, wq4.w}}, bq[2] = {{bq4.x, bq4.y}, {bq4.z, bq4.w}};
        const f2 s2 = {e.res[l].scale, e.res[l].scale}, m2 = {e.res[l].min, e.res[l].min};
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          f2 t = q[hh] * s2;
          t = t + m2;
          t = t - mn[hh];
          t = t * sq[hh];
          t = t * wq[hh];
          o[hh] = t + bq[hh];
        }
      };
      if (RES || nres > 0) {
        f2 r[2];
        int l0 = 0;
        if (RES) {
          const int cr = min(cc, c - 4);
          const int64_t fi = e.f32_tiled ? ctile_index(mc, cr, ct) : (int64_t)mc * c + cr;
          const float4 r4 = *reinterpret_cast<const float4*>(e.residual + fi);
          r[0] = (f2){r4.x, r4.y};
          r[1] = (f2){r4.z, r4.w};
        } else {
          link(0, r);
          if (e.res_relu0) {
            r[0].x = fmaxf(r[0].x, 0.f); r[0].y = fmaxf(r[0].y, 0.f);
            r[1].x = fmaxf(r[1].x, 0.f); r[1].y = fmaxf(r[1].y, 0.f);
          }
          l0 = 1;
        }
#pragma unroll
        for (int l = 0; l < QNN_MAX_RES; ++l) {
          if (l < l0 || l >= nres) continue;
          f2 o[2];
          link(l, o);
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const f2 t = o[hh] + r[hh];
            r[hh].x = fmaxf(t.x, 0.f);
            r[hh].y = fmaxf(t.y, 0.f);
          }
        }
        v[0] = v[0] + r[0];
        v[1] = v[1] + r[1];
      }
      if (e.relu) {
        v[0].x = fmaxf(v[0].x, 0.f); v[0].y = fmaxf(v[0].y, 0.f);
        v[1].x = fmaxf(v[1].x, 0.f); v[1].y = fmaxf(v[1].y, 0.f);
      }
      if (e.out_f32 && pok && cok) {
        const int64_t fi = e.f32_tiled ? ctile_index(m, cc, ct) : (int64_t)m * c + cc;
        *reinterpret_cast<float4*>(e.out_f32 + fi) = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
      }
      k0[g] = k1[g] = 0;
      if (e.out_code0 && cok) k0[g] = pack4(qclamp2(v[0], c0p) + MAGIC_S8, qclamp2(v[1], c0p) + MAGIC_S8);
      if (e.out_code1 && cok)
        k1[g] = same01 ? k0[g] : pack4(qclamp2(v[0], c1p) + MAGIC_S8, qclamp2(v[1], c1p) + MAGIC_S8);
    }
    const int ch = ctb * 32 + 16 * h;
    if (e.out_code0) {
      const int4 w4 = chain_gather16(k0[0], k0[1], k0[2], k0[3]);
      if (pok && ch < t0.cp)
        *reinterpret_cast<int4*>(t0.ptr + (((int64_t)nn * t0.hp + y + t0.pad) * t0.wp + x + t0.pad) * t0.cp + ch) = w4;
    }
    if (e.out_code1) {
      const int4 w4 = chain_gather16(k1[0], k1[1], k1[2], k1[3]);
      if (pok && ch < t1.cp)
        *reinterpret_cast<int4*>(t1.ptr + (((int64_t)nn * t1.hp + y + t1.pad) * t1.wp + x + t1.pad) * t1.cp + ch) = w4;
    }
    x += dx;
    y += dy;
    nn += dn;
    if (x >= wo) x -= wo, ++y;
    if (y >= ho) y -= ho, ++nn;
  }
}

static int check_code(const qnn_code_out* o, int c, const char* what) {
  if (!o || !o->ptr) return QNN_OK;
  if (o->cp < c || o->cp % 4 || o->scale <= 0.f || o->pad < 0 || (((uintptr_t)o->ptr) & 3))
    return arg_error(what);
  return QNN_OK;
}

}  // namespace qnn

using namespace qnn;

extern "C" {

int qnn_maxpool_bn(const uint8_t* q, int n, int h, int w, int c, int k, int stride, int pad, int ho, int wo,
                   const qnn_bn_params* bn, int relu, float* out_f32, int f32_tiled, uint8_t* out_code,
                   const int8_t* lut0, const qnn_code_out* code0, const int8_t* lut1, const qnn_code_out* code1,
                   qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && h > 0 && w > 0 && c > 0 && c % 16 == 0 && c <= 256 && k > 0 && stride > 0 && pad >= 0 &&
                  2 * pad <= k,
              "bad shape (c % 16 == 0, c <= 256, pad <= k/2)");
  QNN_REQUIRE(ho == (h + 2 * pad - k) / stride + 1 && wo == (w + 2 * pad - k) / stride + 1, "ho/wo inconsistent");
  QNN_REQUIRE(bn && bn->mean && bn->sq && bn->wq && bn->bq && bn->scale > 0.f, "bad RangeBN params");
  const bool has0 = code0 && code0->ptr, has1 = code1 && code1->ptr;
  QNN_REQUIRE(!has0 || (lut0 && (((uintptr_t)lut0) & 15) == 0), "code0 needs a 16-B aligned lut0");
  QNN_REQUIRE(!has1 || (lut1 && (((uintptr_t)lut1) & 15) == 0), "code1 needs a 16-B aligned lut1");
  QNN_REQUIRE(out_f32 || out_code || has0 || has1, "no output");
  QNN_REQUIRE(!out_code || (((uintptr_t)out_code) & 15) == 0, "out_code must be 16-byte aligned");
  QNN_REQUIRE(!out_f32 || (((uintptr_t)out_f32) & 15) == 0, "out_f32 must be 16-byte aligned");
  auto code16 = [&](const qnn_code_out* o) {
    return !o || !o->ptr || (o->cp >= c && o->cp % 16 == 0 && o->scale > 0.f && o->pad >= 0 &&
                             (((uintptr_t)o->ptr) & 15) == 0);
  };
  QNN_REQUIRE(code16(code0) && code16(code1), "bad code output (cp % 16, 16-B aligned)");
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(q && (((uintptr_t)q) & 15) == 0, "q must be non-null and 16-byte aligned");
  const qnn_code_out c0 = has0 ? *code0 : none_code();
  const qnn_code_out c1 = has1 ? *code1 : none_code();
  const int lds = c * 17 + ((has0 ? 1 : 0) + (has1 ? 1 : 0)) * c * 256 + 16;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)maxpool_bn_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(maxpool_bn)");
  const int64_t threads = (int64_t)n * ho * wo * (c / 16);
  hipLaunchKernelGGL(maxpool_bn_kernel, dim3(grid_for(threads)), dim3(256), lds, (hipStream_t)stream, q, n, h, w, c,
                     k, stride, pad, ho, wo, *bn, relu, out_f32, f32_tiled, out_code, has0 ? lut0 : nullptr, c0,
                     has1 ? lut1 : nullptr, c1);
  QNN_LAUNCH_CHECK("qnn_maxpool_bn");
  return QNN_OK;
}

}  // extern "C"

// The depthwise dispatcher: the 3x3 register-pipelined kernel where the shapes allow it, else
// (or when `generic`, the bitwise reference the tests compare it with) the generic kernel.
static int dwconv_fused(const int8_t* x, int n, int h, int w, int pad, int hp, int wp, int cp, int c,
                        const float* w_hat_t, int kh, int kw, int sh, int sw, int ho, int wo, float x_min,
                        float x_scale, const float* bias, const qnn_bn_params* bn, int relu, float* out_f32,
                        const qnn_code_out* code0, qnn_stream_t stream, bool generic, const int8_t* lut = nullptr) {
  QNN_REQUIRE(n >= 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0 && cp >= c && cp % 4 == 0 && kh > 0 && kw > 0 &&
                  sh > 0 && sw > 0 && pad >= 0,
              "bad shape");
  QNN_REQUIRE(hp >= h + 2 * pad && wp >= w + 2 * pad, "padded buffer smaller than image");
  QNN_REQUIRE(ho == (h + 2 * pad - kh) / sh + 1 && wo == (w + 2 * pad - kw) / sw + 1, "ho/wo inconsistent");
  QNN_REQUIRE(x_scale > 0.f, "x_scale must be > 0");
  QNN_REQUIRE(!bn || (bn->mean && bn->sq && bn->wq && bn->bq && bn->scale > 0.f), "bad RangeBN params");
  QNN_REQUIRE(out_f32 || (code0 && code0->ptr), "no output");
  if (int rc = check_code(code0, c, "bad code0")) return rc;
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(x && w_hat_t, "null pointer");
  qnn_bn_params b;
  memset(&b, 0, sizeof(b));
  if (bn) b = *bn;
  const qnn_code_out c0 = code0 ? *code0 : none_code();
  constexpr int CPT = 2 * QNN_DW_P;
  const bool fast = !generic && kh == 3 && kw == 3 && sh == sw && (sh == 1 || sh == 2) && c % CPT == 0 &&
                    c / CPT <= 256 && cp % 8 == 0 && (((uintptr_t)x) & 7) == 0 && (((uintptr_t)w_hat_t) & 15) == 0 &&
                    (!out_f32 || (((uintptr_t)out_f32) & 15) == 0) &&
                    (!c0.ptr || (c0.cp % 8 == 0 && (((uintptr_t)c0.ptr) & 7) == 0 &&
                                 (int64_t)c0.hp * c0.wp < (1LL << 31))) &&  // 32-bit pixel indices
                    (int64_t)hp * wp * cp < (1LL << 31);  // 32-bit buffer offsets within an image
  // the table path: codes only, channel slices of 128 (or all c) channels
  const int cs = lut ? (c > 128 ? 128 : c) : c;
  const bool fast_lut = fast && lut && !out_f32 && c % cs == 0 && (((uintptr_t)lut) & 15) == 0;
  if (lut && !fast_lut) return arg_error("qnn_dwconv_fused_lut: a 3x3 stride-1/2 layer with codes out only, c % 4 == 0 "
                                        "(and c % 128 == 0 above 128 channels), 16-byte aligned table");
  if (fast) {
    const int R = sh == 1 ? 4 : 2;  // stride 2: 2 pixels (5 input columns) per thread, register budget
    constexpr int RR = QNN_DW_RR;
    // the kernel addresses its input by 32-bit offsets from one buffer resource and its code
    // pixels by 32-bit indices: launched over chunks of images that keep both below 2^31
    const int64_t img_in = (int64_t)hp * wp * cp, img_px = c0.ptr ? (int64_t)c0.hp * c0.wp : 1;
    const int64_t lim = ((1LL << 31) - 1) / std::max(img_in, img_px);
    const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(n, lim));
    const int ct = cs / CPT, nsl = c / cs;
    QNN_REQUIRE((int64_t)nch * ((ho + RR - 1) / RR) * ((wo + R - 1) / R) < (1LL << 31), "depthwise too large");
    auto kern = fast_lut ? (sh == 1 ? dwconv3_kernel<1, 4, QNN_DW_P, true, RR> : dwconv3_kernel<2, 2, QNN_DW_P, true, RR>)
                         : (sh == 1 ? dwconv3_kernel<1, 4, QNN_DW_P, false, RR> : dwconv3_kernel<2, 2, QNN_DW_P, false, RR>);
    const int lds = fast_lut ? cs * 256 : 0;
    // grid-stride, sized to the resident capacity (the loop is software-pipelined); a whole
    // number of channel slices per pixel block
    const int num_cu = device_cu_count();
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds) != hipSuccess || per_cu < 1) per_cu = 1;
    for (int i0 = 0; i0 < n; i0 += nch) {
      const int ni = std::min(nch, n - i0);
      const int rows = ni * ((ho + RR - 1) / RR);  // row groups
      const int64_t groups = (int64_t)rows * ((wo + R - 1) / R);
      const int64_t pblocks =
          std::min<int64_t>(cdiv(groups, 256 / ct), std::max<int64_t>(1, (int64_t)num_cu * per_cu / nsl));
      const int blocks = (int)(pblocks * nsl);
      qnn_code_out ci = c0;
      if (ci.ptr) ci.ptr += (int64_t)i0 * ci.hp * ci.wp * ci.cp;
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, (hipStream_t)stream, x + i0 * img_in, h, w, pad, hp, wp,
                         cp, c, w_hat_t, ho, wo, x_min, x_scale, bias, b, bn ? 1 : 0, relu,
                         out_f32 ? out_f32 + (int64_t)i0 * ho * wo * c : nullptr, ci, rows, lut, cs, (int)(ni * img_in));
      QNN_LAUNCH_CHECK("qnn_dwconv_fused");
    }
    return QNN_OK;
  }
  hipLaunchKernelGGL(dwconv_fused_kernel, dim3(grid_for((int64_t)n * ho * wo * (c / 4))), dim3(256), 0,
                     (hipStream_t)stream, x, n, h, w, pad, hp, wp, cp, c, w_hat_t, kh, kw, sh, sw, ho, wo, x_min,
                     x_scale, bias, b, bn ? 1 : 0, relu, out_f32, c0);
  QNN_LAUNCH_CHECK("qnn_dwconv_fused");
  return QNN_OK;
}

extern "C" {

int qnn_dwconv_fused(const int8_t* x, int n, int h, int w, int pad, int hp, int wp, int cp, int c,
                     const float* w_hat_t, int kh, int kw, int sh, int sw, int ho, int wo, float x_min, float x_scale,
                     const float* bias, const qnn_bn_params* bn, int relu, float* out_f32, const qnn_code_out* code0,
                     qnn_stream_t stream) {
  return dwconv_fused(x, n, h, w, pad, hp, wp, cp, c, w_hat_t, kh, kw, sh, sw, ho, wo, x_min, x_scale, bias, bn, relu,
                      out_f32, code0, stream, false);
}

int qnn_dwconv_fused_generic(const int8_t* x, int n, int h, int w, int pad, int hp, int wp, int cp, int c,
                             const float* w_hat_t, int kh, int kw, int sh, int sw, int ho, int wo, float x_min,
                             float x_scale, const float* bias, const qnn_bn_params* bn, int relu, float* out_f32,
                             const qnn_code_out* code0, qnn_stream_t stream) {
  return dwconv_fused(x, n, h, w, pad, hp, wp, cp, c, w_hat_t, kh, kw, sh, sw, ho, wo, x_min, x_scale, bias, bn, relu,
                      out_f32, code0, stream, true);
}

int qnn_dwconv_fused_lut(const int8_t* x, int n, int h, int w, int pad, int hp, int wp, int cp, int c,
                         const float* w_hat_t, int kh, int kw, int sh, int sw, int ho, int wo, float x_min,
                         float x_scale, const float* bias, const qnn_bn_params* bn, const int8_t* lut,
                         const qnn_code_out* code0, qnn_stream_t stream) {
  QNN_REQUIRE(bn && lut && code0 && code0->ptr, "qnn_dwconv_fused_lut: RangeBN, its code table and a code output");
  return dwconv_fused(x, n, h, w, pad, hp, wp, cp, c, w_hat_t, kh, kw, sh, sw, ho, wo, x_min, x_scale, bias, bn, 1,
                      nullptr, code0, stream, false, lut);
}

int qnn_chain_epilogue(const uint8_t* bncode, int n, int ho, int wo, int c, const qnn_epilogue* epi,
                       qnn_stream_t stream) {
  QNN_REQUIRE(epi, "null epilogue");
  const qnn_epilogue& e = *epi;
  QNN_REQUIRE(n >= 0 && ho > 0 && wo > 0 && c > 0 && c % 16 == 0, "bad shape (c % 16 == 0)");
  QNN_REQUIRE(e.bn_mean && e.bn_sq && e.bn_wq && e.bn_bq && e.bn_scale > 0.f, "bad RangeBN params");
  QNN_REQUIRE(e.nres >= 0 && e.nres <= QNN_MAX_RES, "nres out of range");
  for (int l = 0; l < e.nres; ++l)
    QNN_REQUIRE(e.res[l].code && (((uintptr_t)e.res[l].code) & 15) == 0 && e.res[l].mean && e.res[l].sq &&
                    e.res[l].wq && e.res[l].bq,
                "bad residual link (16-byte aligned codes, all vectors)");
  QNN_REQUIRE(e.out_f32 || e.out_code0 || e.out_code1, "no output");
  QNN_REQUIRE(!e.out_f32 || (((uintptr_t)e.out_f32) & 15) == 0, "out_f32 must be 16-byte aligned");
  QNN_REQUIRE(!e.residual || (((uintptr_t)e.residual) & 15) == 0, "residual must be 16-byte aligned");
  auto code16 = [&](const int8_t* p, int cp, int pad, float scale) {
    return !p || (cp >= c && cp % 16 == 0 && pad >= 0 && scale > 0.f && (((uintptr_t)p) & 15) == 0);
  };
  QNN_REQUIRE(code16(e.out_code0, e.code0_cp, e.code0_pad, e.code0_scale) &&
                  code16(e.out_code1, e.code1_cp, e.code1_pad, e.code1_scale),
              "bad code output (cp % 16, 16-B aligned)");
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(bncode && (((uintptr_t)bncode) & 15) == 0, "bncode must be non-null and 16-byte aligned");
  const int64_t M = (int64_t)n * ho * wo;
  QNN_REQUIRE(M < ((int64_t)1 << 31), "n * ho * wo >= 2^31");
  const int64_t mts = (M + 31) / 32;
  const int ct = (c + 31) / 32;
  // one resident round: about 4 blocks per CU (<= 128 VGPRs) over the channel tiles, each
  // walking pixel tiles four at a time (a second, partial round of blocks would run at low occupancy)
  const int64_t gx = std::max<int64_t>(1, std::min<int64_t>(cdiv(mts, 4), (256 * 4) / ct));
  const dim3 grid((unsigned)gx, (unsigned)ct);
  const int64_t step = 32 * 4 * gx;  // pixels between a wave's tiles
  const int dx = (int)(step % wo), rows = (int)(step / wo), dy = rows % ho, dn = rows / ho;
  const bool full = c % 32 == 0;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, (hipStream_t)stream, bncode, n, ho, wo, c, dx, dy, dn, e);
  };
  const bool res = e.residual != nullptr;
  auto pick = [&](auto fullc) {
    constexpr bool F = decltype(fullc)::value;
    switch (e.nres * 2 + (res ? 1 : 0)) {
      case 0: go(chain_epilogue_kernel<0, false, F>); break;
      case 1: go(chain_epilogue_kernel<0, true, F>); break;
      case 2: go(chain_epilogue_kernel<1, false, F>); break;
      case 3: go(chain_epilogue_kernel<1, true, F>); break;
      case 4: go(chain_epilogue_kernel<2, false, F>); break;
      case 5: go(chain_epilogue_kernel<2, true, F>); break;
      case 6: go(chain_epilogue_kernel<3, false, F>); break;
      case 7: go(chain_epilogue_kernel<3, true, F>); break;
      case 8: go(chain_epilogue_kernel<4, false, F>); break;
      default: go(chain_epilogue_kernel<4, true, F>); break;
    }
  };
  if (full) pick(std::true_type{});
  else pick(std::false_type{});
  QNN_LAUNCH_CHECK("qnn_chain_epilogue");
  return QNN_OK;
}

int qnn_bn_code_lut(const qnn_bn_params* bn, int c, int relu, const qnn_code_out* next, int8_t* lut,
                    qnn_stream_t stream) {
  QNN_REQUIRE(c > 0 && bn && bn->mean && bn->sq && bn->wq && bn->bq && bn->scale > 0.f, "bad RangeBN params");
  QNN_REQUIRE(next && next->scale > 0.f && lut, "bad next range / null lut");
  hipLaunchKernelGGL(bn_code_lut_kernel, dim3((unsigned)cdiv((int64_t)c * 256, 256)), dim3(256), 0,
                     (hipStream_t)stream, *bn, c, relu, *next, lut);
  QNN_LAUNCH_CHECK("qnn_bn_code_lut");
  return QNN_OK;
}

int qnn_avgpool_quant(const float* x, int n, int hw, int c, int x_tiled, float* out_f32,
                      const qnn_code_out* code0, qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && hw > 0 && c > 0 && c % 4 == 0, "bad shape");
  QNN_REQUIRE(out_f32 || (code0 && code0->ptr), "no output");
  if (int rc = check_code(code0, c, "bad code0")) return rc;
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(x, "null input");
  const qnn_code_out c0 = code0 ? *code0 : none_code();
  QNN_REQUIRE(n < 65536, "batch >= 65536");
  if (x_tiled && hw <= 128 && (((uintptr_t)x) & 15) == 0)
    hipLaunchKernelGGL(avgpool_tiled_kernel, dim3((unsigned)cdiv(c, 64), (unsigned)n), dim3(64), hw * 68 * 4,
                       (hipStream_t)stream, x, n, hw, c, out_f32, c0);
  else
    hipLaunchKernelGGL(avgpool_quant_kernel, dim3((unsigned)cdiv(c / 4, 64), (unsigned)n), dim3(64), 0,
                       (hipStream_t)stream, x, n, hw, c, x_tiled, out_f32, c0);
  QNN_LAUNCH_CHECK("qnn_avgpool_quant");
  return QNN_OK;
}

}  // extern "C"
