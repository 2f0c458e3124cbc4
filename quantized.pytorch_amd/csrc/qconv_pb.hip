// Persistent-band int8 convolution on v_mfma_i32_16x16x64_i8 with the weights resident in VGPRs:
// the eval forward of QConv2d (models/modules/quantize.py:314-349) for the 3x3 layers on 64 or
// 128 input channels -- ResNet layer 1's 64@56x56 convolutions (resnet_quantized.py:52-68,
// :93-113), the stride-2 entries of layer 2 and ResNet-18's 128@28x28 pairs.  Same exact
// decomposition and epilogue (q16::epilogue_rb) as every other family, so the
// outputs are bitwise theirs.
//
// What the other families leave on the table for these layers: the ring kernel
// pulls every input byte from L2 once per tap (implicit im2col) and the weights once per pixel
// tile, the direct kernel pulls the im2col fragments through L1 at one wave per SIMD, the
// resident-band kernel runs its band, K loop and epilogue phases in series.  Here:
// * A block owns CB = 16 TM output channels and is PERSISTENT over a sequence of input BANDS
//   (R output rows of one image, or k whole images, and every padded input row they read, all
//   cp channels).  Its weights -- KS = 9 cp / 64 K steps x TM fragments -- are loaded into VGPRs
//   once per block (144 registers at TM x KS = 36).
// * Bands are double-buffered in LDS as 32-byte planes (qconv_rb.hip's layout: a tap shift is one
//   uniform add, a fragment's 16 (pixel, half) pairs hit 16 distinct bank slots).  The next band's
//   LDS-DMA is issued right after the barrier that opens the current one and lands under its
//   pixel tiles; the DMA is inline asm, invisible to the compiler's waitcnt pass, so no compiler
//   wait on the band's LDS reads stalls behind it.
// * The four waves take the band's 16-pixel tiles round-robin; per tile: KS band fragments
//   (ds_read_b128), KS x TM MFMAs, sum_valid(q'_x) as the sum of the tile pixels' nine taps of a
//   per-band-pixel channel-sum table (computed once per band), then the fused epilogue.  Two
//   blocks per CU (two waves per SIMD): one block's MFMAs run beside the other's epilogue VALU.
#include "qconv_common.h"
#include <stdlib.h>

#include <type_traits>
#include <utility>

#include "epi16.h"

#ifndef QNN_ABLATE
#define QNN_ABLATE 0  // diagnostic builds only (make pbablate): 1 no MFMA, 2 no epilogue, 3 no band DMA,
                      // 4 no code-table lookups, 5 no band fragment reads
#endif

#ifndef QNN_STAMP
#define QNN_STAMP 0  // diagnostic builds only (make pbstamp): per-wave s_memtime phase sums
#endif
#if QNN_STAMP
// [block][wave][8]: realtime start/end (100 MHz); cycles: prologue (to the first band), band
// tops (wait + barrier + channel sums + barrier), tile contraction (+ sums), epilogue; tiles, bands
__device__ unsigned long long qnn_pb_stamps[1 << 19];
#define PB_TS(v)                                                                          \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#else
#define PB_TS(v) ((void)0)
#endif

// the device error word (include/qnn.h qnn_device_errors): a global vector atomic OR, read and
// cleared by the host
__device__ unsigned qnn_dev_errors;

namespace qnn {
namespace pb {

template <int TM_, int KS_, int BPC_, int PXMAX_, int W_ = 4>
struct Cfg {
  static constexpr int WGM = 1, WGN = W_, TM = TM_, TN = 1, KS = KS_, BPC = BPC_, PXMAX = PXMAX_;
  static constexpr int W = W_, NT = 64 * W_;  // waves of the block, every one a tile worker
  static constexpr int CB = 16 * TM, BM = CB < 64 ? 64 : CB;  // BM: stage_epi's 64-float stride
  static constexpr int G = KS / 9;                            // 64-channel groups (cp = 64 G)
};

struct Geo {
  int rows;       // flattened output rows (n*ho) per band
  int nbands;     // bands of the whole batch
  int nbrows;     // padded input rows of a band
  int wb, we, s2; // band row width (= wp); stride 2: even columns first, we = (wp + 1) / 2
  int nbp;        // band pixels (nbrows * wb)
  int pl;         // bytes per 32-byte plane (1 KiB multiple)
  int npl;        // planes (cp / 32)
  int ppp;        // 1 KiB DMA pieces per plane
  int npieces;    // npl * ppp
  int buf;        // bytes of one band buffer (npl * pl)
  int sync_off;   // LDS: the band hand-off counters (4 ints)
  int rel_off;    // LDS: int source offset of every band piece lane, [npieces][64]
  int cls_off;    // LDS: hcls[ho] * nwc, then wcls[wo]
  int npt;        // 16-pixel tiles per band
  int lut;        // EK_LUT: the code table is staged (else evaluated)
  // drop-in input as fp32 NCHW (qnn_qconv2d_fwd_nchw_f32): each wave quantizes its pixels of a band
  // in registers (quant_code_fast, bitwise the IEEE quotient) into the band buffer, no code tensor
  const float* xf;  // null: the input is the padded NHWC8 codes x
  int fc, fh, fw, fpad;
  float fnm, fs, fqmax;
  int wstage;     // stage the weights through LDS (else each wave loads them from L2)
  int wsep;       // ... in a region of their own at wst_off (else in the band buffers, wst_off = 0)
  int wst_off;
  int spin_max;   // bound of every hand-off wait (SPIN_MAX; qnn_debug_set_spin_limit for tests)
};

// q = m / D, r = m % D for 0 <= m < 2^24 (checked on the host): the float quotient is off by at
// most one, fixed up exactly
__device__ __forceinline__ void fdivmod(int m, int D, float invD, int& q, int& r) {
  q = (int)((float)m * invD);
  r = m - (int)__umul24((unsigned)q, (unsigned)D);
  if (r < 0) --q, r += D;
  if (r >= D) ++q, r -= D;
}

// one 1 KiB LDS-DMA wave-instruction, invisible to the compiler's vmcnt bookkeeping (waited for
// explicitly before the barrier that publishes the band)
__device__ __forceinline__ void dma16(const int8_t* base, uint32_t off, const int8_t* lds_dst) {
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_dst);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(m), "v"(off), "s"(base) : "memory", "m0");
}

// The code-table epilogue (EK_LUT, table staged), conv -> RangeBN -> ReLU -> the consumer's
// codes: q16::epilogue_rb's arithmetic for this case (the same fp32 ops in the same order, so
// bitwise its codes), specialised -- the lane's channels lie inside the block's whole tile
// (cout % CB == 0, checked on the host), the bias add only when the layer has a bias, a table
// byte's LDS offset one AND-OR of the code with its 256-byte aligned row, and the TM = 4 code
// words transposed to one 16-byte store per lane.
template <class C, bool BIAS>
__device__ __forceinline__ void lut_epilogue(const Params& p, const v4i (&acc)[C::TM][1], int psq, int pc, int n, int ho,
                                             int wo, const int8_t* smem, int c0, int lane) {
  constexpr int TM = C::TM, BM = C::BM;
  const qnn_epilogue& e = p.e;
  const int gq = lane >> 4;
  const float* s_f = reinterpret_cast<const float*>(smem + p.epi_off);
  const uint32_t lut_off = (uint32_t)(p.epi_off + 4 * (7 + e.nclass) * BM);  // 256-byte aligned
  const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
  const f2 p2 = {(float)psq, (float)psq};
  const float* tp = s_f + (7 + pc) * BM;
  const int64_t px0 = (int64_t)(__umul24(__umul24((unsigned)n, (unsigned)e.code0_hp) + (unsigned)(ho + e.code0_pad),
                                         (unsigned)e.code0_wp) + (unsigned)(wo + e.code0_pad)) * e.code0_cp;
  // phase 1: the channel vectors and border terms; phase 2: every code's table address; phase 3:
  // the 4 TM table reads back to back; phase 4: pack
  float4 sw[TM], bw[TM], tb[TM], bi[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = 16 * i + 4 * gq;
    sw[i] = *reinterpret_cast<const float4*>(s_f + cl);
    bw[i] = *reinterpret_cast<const float4*>(s_f + BM + cl);
    tb[i] = *reinterpret_cast<const float4*>(tp + cl);
    if (BIAS) bi[i] = *reinterpret_cast<const float4*>(s_f + 2 * BM + cl);
  }
  uint32_t k[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = 16 * i + 4 * gq;
    const v4i& a = acc[i][0];
    const f2 a01 = {(float)a[0], (float)a[1]}, a23 = {(float)a[2], (float)a[3]};
    f2 v0 = pfma((f2){sw[i].x, sw[i].y}, a01, pfma((f2){bw[i].x, bw[i].y}, p2, (f2){tb[i].x, tb[i].y}));
    f2 v1 = pfma((f2){sw[i].z, sw[i].w}, a23, pfma((f2){bw[i].z, bw[i].w}, p2, (f2){tb[i].z, tb[i].w}));
    if (BIAS) {  // (without a bias the other kernels add staged zeros: v + 0 differs from v only for
                 // v = -0, and -0 and +0 quantize to the same code)
      v0 = v0 + (f2){bi[i].x, bi[i].y};
      v1 = v1 + (f2){bi[i].z, bi[i].w};
    }
    const f2 q0 = qclamp2(v0, bnp) + MAGIC_U8, q1 = qclamp2(v1, bnp) + MAGIC_U8;
    const uint32_t row = lut_off + (uint32_t)cl * 256u;  // channel cl's 256 codes; cl + u at + 256 u
    k[i][0] = (__float_as_uint(q0.x) & 255u) | row;
    k[i][1] = (__float_as_uint(q0.y) & 255u) | (row + 256u);
    k[i][2] = (__float_as_uint(q1.x) & 255u) | (row + 512u);
    k[i][3] = (__float_as_uint(q1.y) & 255u) | (row + 768u);
  }
  unsigned by[TM][4];
  const uint8_t* lb = reinterpret_cast<const uint8_t*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int u = 0; u < 4; ++u) by[i][u] = QNN_ABLATE == 4 ? (k[i][u] & 255u) : (unsigned)lb[k[i][u]];
  unsigned wrd[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) wrd[i] = by[i][0] | (by[i][1] << 8) | (by[i][2] << 16) | (by[i][3] << 24);
  if constexpr (TM == 4) {
    // M[g][i] = wrd[i] of lane group g -> register k of group g holds M[k][g] (channels 16 g + 4 k..):
    // one 16-byte store of the pixel's channels 16 g .. 16 g + 15 (q16::epilogue_rb's wide path)
    const auto s02 = __builtin_amdgcn_permlane32_swap(wrd[0], wrd[2], false, false);
    const auto s13 = __builtin_amdgcn_permlane32_swap(wrd[1], wrd[3], false, false);
    const auto t01 = __builtin_amdgcn_permlane16_swap(s02[0], s13[0], false, false);
    const auto t23 = __builtin_amdgcn_permlane16_swap(s02[1], s13[1], false, false);
    *reinterpret_cast<v4i*>(e.out_code0 + px0 + c0 + 16 * gq) = (v4i){(int)t01[0], (int)t01[1], (int)t23[0], (int)t23[1]};
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i) *reinterpret_cast<unsigned*>(e.out_code0 + px0 + c0 + 16 * i + 4 * gq) = wrd[i];
  }
}

template <class F, int... J>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, J...>) {
  (f(std::integral_constant<int, J>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// s_waitcnt lgkmcnt(N) for the hand-counted inline-asm LDS reads; the scheduling barrier keeps the
// compiler from hoisting register-only MFMAs above it
template <int N>
__device__ __forceinline__ void lds_wait() {
  static_assert(N >= 0 && N < 16, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Every wait on a counter is bounded (~0.1-0.5 s): a protocol error then yields wrong outputs, never
// a wave that spins until the process is killed -- and the wave that gave up raises
// QNN_DEVERR_PB_SPIN in the device error word (qnn_device_errors), so a production forward learns
// of it too, not only the bitwise tests
constexpr int SPIN_MAX = 1 << 21;
static int g_spin_max = SPIN_MAX;  // qnn_debug_set_spin_limit

__device__ __forceinline__ void spin_timeout(int lane) {
  if (lane == 0) atomicOr(&qnn_dev_errors, (unsigned)QNN_DEVERR_PB_SPIN);
}

// LDS counters (inline asm: the compiler's waitcnt pass must not order them behind the invisible
// band DMA, and no compiler-visible access may move across them)
__device__ __forceinline__ void lds_add(int* c, int v) {
  asm volatile("ds_add_u32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"((uint32_t)(uintptr_t)c), "v"(v) : "memory");
}
__device__ __forceinline__ int lds_get(const int* c) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)c) : "memory");
  return __builtin_amdgcn_readfirstlane(v);
}

// qconv_common.h stage_epi's layout and sources, every DMA inline asm (a compiler-visible LDS-DMA
// makes the compiler wait for vmcnt(0) -- every band piece in flight -- before its next LDS access).
// Returns the number of DMA instructions this wave issued.
__device__ __forceinline__ void dma4v(const void* src, const int8_t* ldst) {
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(m), "v"(src) : "memory", "m0");
}
__device__ __forceinline__ void dma16v(const void* src, const int8_t* ldst) {
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m), "v"(src) : "memory", "m0");
}
__device__ float qnn_pb_zero_page[64];  // zero-initialised: the bias vector of a bias-free layer, fp32 input

template <class C, int EK>
__device__ __forceinline__ void stage_epi_asm(const Params& p, const int8_t* x, int8_t* dst, int c0, int wave, int lane) {
  constexpr int BM = C::BM, W = C::W, CH = BM / 64;
  const qnn_epilogue& e = p.e;
  const int cmax = p.d.cout - 1;
  const int nvec = (EK != EK_NCHW && e.bn_mean) ? 7 : 3;
  const int nf = (nvec + e.nclass + (EK == EK_GEN ? 4 * e.nres : 0)) * CH;
  for (int jb = wave; jb < nf; jb += W) {
    const int v = jb / CH, k = jb - v * CH;
    const int arr = v < nvec ? v : 7 + (v - nvec);
    int c = c0 + 64 * k + lane;
    c = c < cmax ? c : cmax;
    const float* src;
    switch (arr) {
      case 0: src = e.sxsw; break;
      case 1: src = e.sxbw; break;
      case 2:
        if (!e.bias) {  // no bias: zeros from the input's 128-byte zero page (or the library's)
          src = x ? reinterpret_cast<const float*>(x + p.d.zero_off) : qnn_pb_zero_page;
          c = lane & 31;
        } else {
          src = e.bias;
        }
        break;
      case 3: src = e.bn_mean; break;
      case 4: src = e.bn_sq; break;
      case 5: src = e.bn_wq; break;
      case 6: src = e.bn_bq; break;
      default:
        if (arr - 7 < e.nclass) {
          src = e.table + (int64_t)(arr - 7) * p.d.cout;
        } else {  // chain link l, vector kk (mean, sq, wq, bq)
          const int lk = arr - 7 - e.nclass, l = lk >> 2, kk = lk & 3;
          const qnn_res_link& r = e.res[l];
          src = kk == 0 ? r.mean : kk == 1 ? r.sq : kk == 2 ? r.wq : r.bq;
        }
        break;
    }
    dma4v(src + c, dst + 4 * (arr * BM + 64 * k));
  }
  if constexpr (EK == EK_LUT) {
    int8_t* lut = dst + 4 * (7 + e.nclass) * BM;
    for (int jl = wave; jl < BM / 4; jl += W) {
      int c = c0 + 4 * jl + (lane >> 4);
      c = c < cmax ? c : cmax;
      dma16v(e.lut + (int64_t)c * 256 + 16 * (lane & 15), lut + 1024 * jl);
    }
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (clamped to 63: a larger count waits for more)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  n = n < 63 ? n : 63;
  static_for<64>([&](auto c) {
    if (n == decltype(c)::value) wait_vmcnt<decltype(c)::value>();
  });
}

// The general-chain epilogue (EK_GEN): q16::epilogue_rb's arithmetic in the same fp32 op order (so
// bitwise its outputs), with the residual code-chain words and the fp32 residual loaded at the
// tile's start (gen_prefetch) so their latency hides under the tile's MFMAs, not in the chain.
struct GenPre {
  unsigned cw[QNN_MAX_RES][4];  // chain link l's word of channels 16 i + 4 g .. + 3 (TM <= 4)
  float4 rf[4];                 // the fp32 residual of the same channels
};
template <class C>
__device__ __forceinline__ void gen_prefetch(const Params& p, int m, int c0, int lane, GenPre& g) {
  constexpr int TM = C::TM;
  const qnn_epilogue& e = p.e;
  const int gq = lane >> 4;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int c = c0 + 16 * i + 4 * gq;  // cout % CB == 0 for these configurations
#pragma unroll
    for (int l = 0; l < QNN_MAX_RES; ++l)
      if (l < e.nres) g.cw[l][i] = *reinterpret_cast<const unsigned*>(e.res[l].code + q16::btile_word(m, c, p.ct));
    if (e.residual) {
      const int64_t fi = e.f32_tiled ? ctile_index(m, c, p.ct) : (int64_t)m * p.d.cout + c;
      g.rf[i] = *reinterpret_cast<const float4*>(e.residual + fi);
    }
  }
}
template <class C>
__device__ __forceinline__ void gen_epilogue(const Params& p, const v4i (&acc)[C::TM][1], int psq, int pc, int m, int n,
                                             int ho, int wo, const GenPre& pre, const int8_t* smem, int c0, int lane) {
  constexpr int TM = C::TM, BM = C::BM;
  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  const int gq = lane >> 4;
  const float* s_f = reinterpret_cast<const float*>(smem + p.epi_off);
  const float* s_chain = s_f + (7 + e.nclass) * BM;
  const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
  const QParams c0p = make_qparams(e.code0_neg_min, e.code0_scale, e.code0_qmax);
  const QParams c1p = make_qparams(e.code1_neg_min, e.code1_scale, e.code1_qmax);
  const bool same01 = e.out_code0 && e.code1_neg_min == e.code0_neg_min && e.code1_scale == e.code0_scale &&
                      e.code1_qmax == e.code0_qmax;
  const f2 bn_s2 = {e.bn_scale, e.bn_scale}, bn_m2 = {e.bn_min, e.bn_min};
  const f2 p2 = {(float)psq, (float)psq};
  const float* tp = s_f + (7 + pc) * BM;
  const int64_t px0 = (int64_t)(__umul24(__umul24((unsigned)n, (unsigned)e.code0_hp) + (unsigned)(ho + e.code0_pad),
                                         (unsigned)e.code0_wp) + (unsigned)(wo + e.code0_pad)) * e.code0_cp;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = 16 * i + 4 * gq;
    const int c = c0 + cl;
    const float4 sw = *reinterpret_cast<const float4*>(s_f + cl);
    const float4 bw = *reinterpret_cast<const float4*>(s_f + BM + cl);
    const float4 bi = *reinterpret_cast<const float4*>(s_f + 2 * BM + cl);
    const float4 tb = *reinterpret_cast<const float4*>(tp + cl);
    const v4i& a = acc[i][0];
    const f2 a01 = {(float)a[0], (float)a[1]}, a23 = {(float)a[2], (float)a[3]};
    f2 v[2];
    v[0] = pfma((f2){sw.x, sw.y}, a01, pfma((f2){bw.x, bw.y}, p2, (f2){tb.x, tb.y})) + (f2){bi.x, bi.y};
    v[1] = pfma((f2){sw.z, sw.w}, a23, pfma((f2){bw.z, bw.w}, p2, (f2){tb.z, tb.w})) + (f2){bi.z, bi.w};
    if (e.bn_mean) {
      const f2 qb[2] = {qclamp2(v[0], bnp), qclamp2(v[1], bnp)};
      if (e.out_bncode) {
        const int kb = pack4(qb[0] + MAGIC_U8, qb[1] + MAGIC_U8);
        if (e.bncode_tiled) *reinterpret_cast<int*>(e.out_bncode + q16::btile_word(m, c, p.ct)) = kb;
        else *reinterpret_cast<int*>(e.out_bncode + (int64_t)m * d.cout + c) = kb;
      }
      const float4 mn4 = *reinterpret_cast<const float4*>(s_f + 3 * BM + cl);
      const float4 sq4 = *reinterpret_cast<const float4*>(s_f + 4 * BM + cl);
      const float4 wq4 = *reinterpret_cast<const float4*>(s_f + 5 * BM + cl);
      const float4 bq4 = *reinterpret_cast<const float4*>(s_f + 6 * BM + cl);
      const f2 mn[2] = {{mn4.x, mn4.y}, {mn4.z, mn4.w}}, sq[2] = {{sq4.x, sq4.y}, {sq4.z, sq4.w}};
      const f2 wq[2] = {{wq4.x, wq4.y}, {wq4.z, wq4.w}}, bq[2] = {{bq4.x, bq4.y}, {bq4.z, bq4.w}};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f2 o = rint2(qb[h]) * bn_s2;  // dequant: q * s
        o = o + bn_m2;                // + min
        o = o - mn[h];                // x - mean
        o = o * sq[h];                // * q(scale)
        o = o * wq[h];                // * q(weight)
        v[h] = o + bq[h];             // + q(bias)
      }
    }
    if (e.residual || e.nres > 0) {
      // the block input: fp32, or recomputed from the chain exactly as its producers did
      auto link = [&](int l, f2 (&o)[2]) {  // g_l(q) (quantize.py:488-499 op order)
        const unsigned wd = pre.cw[l][i];
        const float* sp = s_chain + 4 * l * BM + cl;
        const float4 lm = *reinterpret_cast<const float4*>(sp);
        const float4 ls = *reinterpret_cast<const float4*>(sp + BM);
        const float4 lw = *reinterpret_cast<const float4*>(sp + 2 * BM);
        const float4 lb = *reinterpret_cast<const float4*>(sp + 3 * BM);
        const f2 s2 = {e.res[l].scale, e.res[l].scale}, m2 = {e.res[l].min, e.res[l].min};
        const f2 q[2] = {{(float)(wd & 255u), (float)((wd >> 8) & 255u)}, {(float)((wd >> 16) & 255u), (float)(wd >> 24)}};
        const f2 lm2[2] = {{lm.x, lm.y}, {lm.z, lm.w}}, ls2[2] = {{ls.x, ls.y}, {ls.z, ls.w}};
        const f2 lw2[2] = {{lw.x, lw.y}, {lw.z, lw.w}}, lb2[2] = {{lb.x, lb.y}, {lb.z, lb.w}};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f2 t = q[h] * s2;
          t = t + m2;
          t = t - lm2[h];
          t = t * ls2[h];
          t = t * lw2[h];
          o[h] = t + lb2[h];
        }
      };
      f2 r[2];
      int l0 = 0;
      if (e.residual) {
        const float4 r4 = pre.rf[i];
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
        if (l < l0 || l >= e.nres) continue;
        f2 o[2];
        link(l, o);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f2 t2 = o[h] + r[h];
          r[h].x = fmaxf(t2.x, 0.f);
          r[h].y = fmaxf(t2.y, 0.f);
        }
      }
      v[0] = v[0] + r[0];
      v[1] = v[1] + r[1];
    }
    if (e.relu) {
      v[0].x = fmaxf(v[0].x, 0.f); v[0].y = fmaxf(v[0].y, 0.f);
      v[1].x = fmaxf(v[1].x, 0.f); v[1].y = fmaxf(v[1].y, 0.f);
    }
    if (e.out_f32) {
      const int64_t fi = e.f32_tiled ? ctile_index(m, c, p.ct) : (int64_t)m * d.cout + c;
      *reinterpret_cast<float4*>(e.out_f32 + fi) = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
    }
    int k0 = 0;
    if (e.out_code0) k0 = pack4(qclamp2(v[0], c0p) + MAGIC_S8, qclamp2(v[1], c0p) + MAGIC_S8);
    if (e.out_code0 && c < e.code0_cp) *reinterpret_cast<int*>(e.out_code0 + px0 + c) = k0;
    if (e.out_code1 && c < e.code1_cp)  // same01: two consumers with the same range, the same codes
      *reinterpret_cast<int*>(e.out_code1 + (((int64_t)n * e.code1_hp + ho + e.code1_pad) * e.code1_wp + wo + e.code1_pad) *
                                                e.code1_cp + c) =
          same01 ? k0 : pack4(qclamp2(v[0], c1p) + MAGIC_S8, qclamp2(v[1], c1p) + MAGIC_S8);
  }
}

template <class C, int EK, bool BIAS, bool F32 = false>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(C::BPC * C::W / 4))) void qconv_pb_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ w, const Params p, const Geo g) {
  constexpr int TM = C::TM, KS = C::KS, CB = C::CB, NT = C::NT;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63, gq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#if QNN_STAMP
  unsigned long long t0 = 0, ta = 0, tb = 0, c_pro = 0, c_top = 0, c_mma = 0, c_epi = 0, ntile = 0, nband = 0;
  unsigned long long tp1 = 0, tp2 = 0, tp3 = 0, tp4 = 0;
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  PB_TS(t0);
#endif

  // persistent: block b owns channel tile b % nby and bands b / nby + j * (grid / nby), j < nb
  const int nby = (d.cout + CB - 1) / CB;
  const int c0 = (blockIdx.x % nby) * CB;
  const int bstep = gridDim.x / nby;
  const int bfirst = blockIdx.x / nby;
  const int nb = bfirst < g.nbands ? (g.nbands - 1 - bfirst) / bstep + 1 : 0;
  const int nrows_all = d.n * d.ho;
  const int64_t last_px = (int64_t)d.n * d.hp * d.wp - 1;  // clamp of band rows past the batch
  // [0, 2): waves whose pieces of the band in buffer s have landed, [2, 4): tiles of it finished --
  // both cumulative over the bands that pass through the buffer (bands s, s + 2, s + 4, ...)
  int* s_sync = reinterpret_cast<int*>(smem + g.sync_off);

  // ---- the band DMA: piece r of plane v = band pixels [32r, 32r + 32), lane i pixel + (i >> 1),
  // 16-byte half i & 1 (pixels past the band re-read its last one: never used; rows past the
  // batch are clamped to its last pixel: they feed only outputs that are never stored).  Each
  // wave moves pieces k = wave + W i of every band and publishes them once they landed.  A
  // piece's per-lane source offset from the band's first padded row is the same for every band:
  // tabulated once in LDS (s_rel[k][lane]), so an issue is a read, an add and the DMA.
  const uint32_t max_off = (uint32_t)(last_px * d.cp);
  int* s_rel = reinterpret_cast<int*>(smem + g.rel_off);
  auto band_row0 = [&](int j) {  // first padded input row (batch-flat) of the block's band j
    const int r0 = (bfirst + j * bstep) * g.rows;
    return (r0 / d.ho) * d.hp + (r0 % d.ho) * d.sh;
  };
  auto fill_band_f32 = [&](int j) {  // this wave's pixels b = 64 (wave + W k) + lane of band j
    int8_t* dst = smem + (j & 1) * g.buf;
    const int R0 = band_row0(j);
    const int rows_all = d.n * d.hp;
    const float inv_wb = 1.0f / (float)g.wb, inv_hp = 1.0f / (float)d.hp;
    const QParams qp = make_qparams(g.fnm, g.fs, g.fqmax);
    const int plane_hw = g.fh * g.fw;
    for (int b = 64 * wave + lane; b < g.nbp; b += 64 * C::W) {
      int br, cc, n, hr;
      fdivmod(b, g.wb, inv_wb, br, cc);
      const int col = g.s2 ? (cc < g.we ? 2 * cc : 2 * (cc - g.we) + 1) : cc;
      const int pr = R0 + br;
      fdivmod(pr < rows_all ? pr : rows_all - 1, d.hp, inv_hp, n, hr);
      const int ih = hr - g.fpad, iw = col - g.fpad;
      const bool in = pr < rows_all && ih >= 0 && ih < g.fh && iw >= 0 && iw < g.fw;
      const float* src = g.xf + ((int64_t)n * g.fc * g.fh + (in ? ih : 0)) * g.fw + (in ? iw : 0);
      // 16 channels per step: their loads in flight together, one 16-byte LDS write (one step at a
      // time: more in flight spills the resident weights)
#pragma unroll 1
      for (int k = 0; k < 4 * C::G; ++k) {
        float f[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int ch = 16 * k + u;
          f[u] = in && ch < g.fc ? src[ch * plane_hw] : 0.f;
        }
        unsigned wd[4];
#pragma unroll
        for (int u4 = 0; u4 < 4; ++u4) {
          unsigned x4 = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int ch = 16 * k + 4 * u4 + u;
            const unsigned code = (unsigned)(int)quant_code_fast(f[4 * u4 + u], qp.nm, qp.s, qp.inv, qp.qmax) - 128u;
            x4 |= ((in && ch < g.fc ? code : 0u) & 255u) << (8 * u);
          }
          wd[u4] = x4;
        }
        *reinterpret_cast<int4*>(dst + (k >> 1) * g.pl + 32 * b + 16 * (k & 1)) =
            make_int4((int)wd[0], (int)wd[1], (int)wd[2], (int)wd[3]);
      }
    }
  };
  auto issue_band = [&](int j) {
    if (QNN_ABLATE == 3) return;
    if constexpr (F32) return fill_band_f32(j);
    const uint32_t base = (uint32_t)band_row0(j) * (uint32_t)(d.wp * d.cp);
    int8_t* dst = smem + (j & 1) * g.buf;
    int v = 0, r = wave;  // piece k = wave + W i = v * ppp + r
    while (r >= g.ppp) r -= g.ppp, ++v;
    for (int k = wave; k < g.npieces; k += C::W) {
      uint32_t off = base + (uint32_t)s_rel[64 * k + lane];
      off = off < max_off ? off : max_off & ~15u;
      dma16(x, off, dst + v * g.pl + r * 1024);
      r += C::W;
      while (r >= g.ppp) r -= g.ppp, ++v;
    }
  };

  // ---- prologue: the border classes, the counters and the piece table first (their global
  // loads then wait for nothing else), the epilogue's data (EK_LUT: with its code table when g.lut,
  // else evaluated), and the block's weights -- one copy per block by LDS-DMA into the band
  // buffers, in fragment order (fragment (s, i) = 1 KiB, lane l's 16 bytes at 16 l: conflict-free
  // ds_read_b128), instead of one copy per wave from L2
  int* s_hc = reinterpret_cast<int*>(smem + g.cls_off);
  for (int i = tid; i < d.ho + d.wo; i += NT) s_hc[i] = i < d.ho ? p.e.hcls[i] * p.e.nwc : p.e.wcls[i - d.ho];
  if (tid < 4) s_sync[tid] = 0;
  {
    const float inv_wb = 1.0f / (float)g.wb;
    for (int v = 0; v < g.npl; ++v)
      for (int i = tid; i < 64 * g.ppp; i += NT) {
        const int r = i >> 6, l = i & 63;
        int b = r * 32 + (l >> 1);
        b = b < g.nbp ? b : g.nbp - 1;
        int br, cc;
        fdivmod(b, g.wb, inv_wb, br, cc);
        const int col = g.s2 ? (cc < g.we ? 2 * cc : 2 * (cc - g.we) + 1) : cc;
        s_rel[64 * (v * g.ppp + r) + l] = (br * d.wp + col) * d.cp + 32 * v + 16 * (l & 1);
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the piece table
#if QNN_STAMP
  PB_TS(tp1);
#endif
  // the epilogue data and the weights (staged through LDS, g.wstage: in their own region when it
  // fits, g.wsep, else in the band buffers; or each wave's straight from L2), then the first two
  // bands when they have their own buffers -- every DMA inline asm, so a counted vmcnt waits for
  // the older epilogue data and weights while the band pieces stay in flight
  const bool wlds = g.wstage && (g.wsep || 1024 * KS * TM <= 2 * g.buf);
  int issued = nb < 2 ? nb : 2, published = 0;
  const int8_t* xz = F32 ? nullptr : x;  // the zero page's owner
  if (EK == EK_LUT && g.lut) stage_epi_asm<C, EK_LUT>(p, xz, smem + p.epi_off, c0, wave, lane);
  else stage_epi_asm<C, (EK == EK_LUT ? EK_BNCODE : EK)>(p, xz, smem + p.epi_off, c0, wave, lane);
  // the weights: K step s = (group s / 9, tap s % 9) is weight bytes tap * cp + 64 group of rows
  // c0 + 16 i + (lane & 15), K bytes 16 (lane >> 4)
  auto wsrc = [&](int s, int i) {
    const int gk = s / 9, t = s - 9 * gk;
    return (int64_t)(c0 + 16 * i + (lane & 15)) * d.kpad + t * d.cp + 64 * gk + 16 * gq;
  };
  if (wlds)
    for (int k = wave; k < KS * TM; k += C::W) dma16(w, (uint32_t)wsrc(k / TM, k % TM), smem + g.wst_off + 1024 * k);
  const bool early = !wlds || g.wsep;  // the bands' buffers are not the weights' staging area
  int band_dma = 0;                    // band pieces this wave has in flight
  if (early) {
    for (int j = 0; j < issued; ++j) issue_band(j);
    band_dma = F32 ? 0 : issued * ((g.npieces - wave + C::W - 1) / C::W);  // (fp32 fill: synchronous)
  }
#if QNN_STAMP
  PB_TS(tp2);
#endif
  wait_vmcnt_rt(band_dma);  // this wave's epilogue data and weights (the bands may stay in flight)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#if QNN_STAMP
  PB_TS(tp3);
#endif
  v4i fa[KS][TM];  // resident in VGPRs for the block's life
  if (wlds) {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[s][i] = *reinterpret_cast<const v4i*>(smem + g.wst_off + 1024 * (s * TM + i) + 16 * lane);
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[s][i] = *reinterpret_cast<const v4i*>(w + wsrc(s, i));
  }
  if (!early) {
    // every wave holds its weights before the bands overwrite the staging area (a raw barrier:
    // the fragments are compiler-visible LDS reads, waited for by lgkmcnt(0))
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int j = 0; j < issued; ++j) issue_band(j);
  }
#if QNN_STAMP
  PB_TS(tp4);
#endif

  // the code-table epilogue stores once per tile (TM = 4: one 16-byte word; else TM words); the
  // pieces issued before a tile are then waited for with the tile's stores left in flight
  constexpr int STORES = TM == 4 ? 1 : TM;
  const bool counted = EK == EK_LUT && g.lut && QNN_ABLATE != 2;
  bool tile_since_issue = false;
  // EK_GEN: the vector-memory instructions a tile issues after its band DMA -- the residual
  // chain's prefetch (gen_prefetch) and the epilogue's stores, only those every tile issues
  // (at most the true count: vector memory completes in issue order, so waiting until no more
  // than these are in flight still covers the older band pieces)
  int gen_young = 0;
  if constexpr (EK == EK_GEN) {
    const qnn_epilogue& e = p.e;
    gen_young = TM * (e.nres + (e.residual ? 1 : 0) + (e.bn_mean && e.out_bncode ? 1 : 0) + (e.out_f32 ? 1 : 0) +
                      (e.out_code0 && e.code0_cp >= d.cout ? 1 : 0) + (e.out_code1 && e.code1_cp >= d.cout ? 1 : 0));
  }
  auto publish = [&] {  // this wave's pieces of the bands it issued have landed
    if (published < issued) {
      if (counted && tile_since_issue) wait_vmcnt<STORES>();
      else if (EK == EK_GEN && tile_since_issue) wait_vmcnt_rt(gen_young);
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        for (int j = published; j < issued; ++j) lds_add(&s_sync[j & 1], 1);
      published = issued;
    }
  };
  // the next band's buffer is free once every tile of the band two before it is finished
  auto can_issue = [&] {
    const int k = issued;
    return k < nb && lds_get(&s_sync[2 + (k & 1)]) >= g.npt * ((k - 2) / 2 + 1);
  };

  // band pixel offset of tap t (row-major 3x3); stride 2: even input columns first
  auto tap_px = [&](int t) {
    const int tr = t / 3, tc = t - 3 * tr;
    return tr * g.wb + (g.s2 ? (tc & 1) * g.we + (tc >> 1) : tc);
  };
  const float inv_wo = 1.0f / (float)d.wo, inv_ho = 1.0f / (float)d.ho;
  const int half = 16 * ((lane >> 4) & 1), pl_sel = (lane >> 5) * g.pl;
  const v4i ones = {0x01010101, 0x01010101, 0x01010101, 0x01010101};
#if QNN_STAMP
  PB_TS(tb);
  c_pro = tb - t0;
#endif

  // ---- the wave's tiles T = wave + W i of the block's band sequence (npt tiles per band), no
  // workgroup barrier: each tile start publishes this wave's landed pieces of earlier issues,
  // issues the next band's pieces when its buffer is free, and waits for its own band
  int j = 0, t = wave;
  while (t >= g.npt && j < nb) t -= g.npt, ++j;
  for (; j < nb;) {
#if QNN_STAMP
    PB_TS(ta);
    ++ntile;
#endif
    publish();
    if (can_issue()) issue_band(issued++), tile_since_issue = false;
    while (issued <= j) {  // this band's buffer waits for another wave's last tile of band j - 2
      publish();             // (never wait while holding unpublished pieces another wave may wait for)
      int guard = 0;
      for (; !can_issue() && guard < g.spin_max; ++guard) __builtin_amdgcn_s_sleep(2);
      if (guard >= g.spin_max && !can_issue()) spin_timeout(lane);
      issue_band(issued++);
      tile_since_issue = false;
    }
    // this wave's own pieces of band j must be published before it waits for the band; younger
    // bands' pieces just issued stay in flight (published at the next tile start: no wave can be
    // waiting for them before band j is complete, so holding them cannot deadlock)
    if (published <= j) publish();
    {
      const int target = C::W * (j / 2 + 1);
      int guard = 0;
      for (; lds_get(&s_sync[j & 1]) < target && guard < g.spin_max; ++guard) __builtin_amdgcn_s_sleep(1);
      if (guard >= g.spin_max && lds_get(&s_sync[j & 1]) < target) spin_timeout(lane);
    }
#if QNN_STAMP
    PB_TS(tb);
    c_top += tb - ta;
    ta = tb;
#endif
    const int buf = j & 1;
    const int r0 = (bfirst + j * bstep) * g.rows;
    const int R0 = band_row0(j);
    const int npx_blk = ((r0 + g.rows <= nrows_all) ? g.rows : nrows_all - r0) * d.wo;
    int q = 16 * t + (lane & 15);
    const bool ok = q < npx_blk;
    q = ok ? q : npx_blk - 1;
    int rr, col, n, hh;
    fdivmod(q, d.wo, inv_wo, rr, col);
    fdivmod(r0 + rr, d.ho, inv_ho, n, hh);
    const int b0 = (n * d.hp + hh * d.sh - R0) * g.wb + col;  // band pixel of tap (0, 0)
    const int pbase = buf * g.buf + 32 * b0 + pl_sel + half;
    GenPre pre;
    if constexpr (EK == EK_GEN) gen_prefetch<C>(p, r0 * d.wo + q, c0, lane, pre);
    v4i acc[TM][1], sacc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[i][0] = (v4i){0, 0, 0, 0};
    // the nine band fragments of a 64-channel group read up front (inline asm: the compiler
    // would otherwise read one, wait, compute, read the next), each step's MFMAs waiting only for
    // its own fragment (LDS returns in order: lgkmcnt(8 - u); tools/asm_lgkm_check.py)
#pragma unroll
    for (int c = 0; c < KS / 9; ++c) {
      v4i fb[9];
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        if (QNN_ABLATE == 5) {
          fb[u] = (v4i){pbase, u, lane, c};
        } else {
          const uint32_t a = (uint32_t)(uintptr_t)(smem + pbase + 2 * c * g.pl + 32 * tap_px(u));
          asm volatile("ds_read_b128 %0, %1" : "=v"(fb[u]) : "v"(a));
        }
      }
      static_for<9>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if (QNN_ABLATE != 5) lds_wait<8 - u>();
        // sum_valid(q'_x): an all-ones A row sums the fragment's codes (padding codes are 0)
        sacc = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, fb[u], sacc, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if (QNN_ABLATE == 1) {
            asm volatile("" ::"v"(fa[9 * c + u][i]), "v"(fb[u]));
            acc[i][0][0] ^= fb[u].x + fa[9 * c + u][i].y;
          } else {
            acc[i][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[9 * c + u][i], fb[u], acc[i][0], 0, 0, 0);
          }
        }
      });
    }
    __builtin_amdgcn_sched_barrier(0);
    int sumq[1] = {sacc[0]};
    auto pixel = [&](int, q16::Pix& P, int& pc) {
      P.ok = ok;
      P.m = r0 * d.wo + q;
      P.n = n, P.ho = hh, P.wo = col;
      pc = s_hc[hh] + s_hc[d.ho + col];
    };
#if QNN_STAMP
    PB_TS(tb);
    c_mma += tb - ta;
    ta = tb;
#endif
    if (QNN_ABLATE == 2) {
      int z = sumq[0] ^ n;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) z ^= acc[i][0][r];
      if (z == 0x7fffffff) p.e.out_code0[0] = 1;  // keeps every MFMA live, (almost) never stores
    } else if (EK == EK_LUT && g.lut) {
      lut_epilogue<C, BIAS>(p, acc, sumq[0], s_hc[hh] + s_hc[d.ho + col], n, hh, col, smem, c0, lane);
    } else if (EK == EK_GEN) {
      gen_epilogue<C>(p, acc, sumq[0], s_hc[hh] + s_hc[d.ho + col], r0 * d.wo + q, n, hh, col, pre, smem, c0, lane);
    } else {
      q16::epilogue_rb<C, EK>(p, acc, sumq, pixel, smem, c0, 0, lane, g.lut);
    }
    // the tile's band fragments were consumed by its MFMAs: count it finished
    __builtin_amdgcn_sched_barrier(0);
    if (lane == 0) lds_add(&s_sync[2 + buf], 1);
    tile_since_issue = true;
#if QNN_STAMP
    PB_TS(tb);
    c_epi += tb - ta;
#endif
    t += C::W;
    while (t >= g.npt && j < nb) t -= g.npt, ++j;
  }
  // the bands other waves still need from this one
  while (issued < nb) {
    publish();
    int guard = 0;
    for (; !can_issue() && guard < g.spin_max; ++guard) __builtin_amdgcn_s_sleep(2);
    if (guard >= g.spin_max && !can_issue()) spin_timeout(lane);
    issue_band(issued++);
    tile_since_issue = false;
  }
  publish();
#if QNN_STAMP
  nband = nb;
  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && blockIdx.x < (1 << 19) / (16 * C::W)) {
    unsigned long long* o = qnn_pb_stamps + ((size_t)blockIdx.x * C::W + wave) * 16;
    o[0] = rt0; o[1] = rt1; o[2] = c_pro; o[3] = c_top; o[4] = c_mma; o[5] = c_epi; o[6] = ntile; o[7] = nband;
    o[8] = tp1 - t0; o[9] = tp2 - t0; o[10] = tp3 - t0; o[11] = tp4 - t0;
  }
#endif
}

// ---------------------------------------------------------------- host side
static int epi_bytes(const Params& p, int BM, bool lut) {
  const int k = epi_kind(p.e);
  return 4 * (7 + p.e.nclass) * BM + (k == EK_GEN ? 16 * p.e.nres * BM : 0) + (lut ? 256 * BM : 0);
}

// Band rows: k whole images when they fit PXMAX pixels, else the largest divisor of ho that does,
// whose double buffer + tables fit LDS / BPC (with the code table if EK_LUT allows, else without);
// the first candidate with at least BPC * 256 bands per channel tile... else the first that fits.
// Returns the LDS bytes (and q.epi_off) or -1.
template <class C>
static int geometry(const Params& p, Geo& g, Params& q) {
  const qnn_conv_desc& d = p.d;
  const int ek = epi_kind(p.e);
  if (d.kh != 3 || d.kw != 3 || d.kmask || d.cp != 64 * C::G || d.kpad < 9 * d.cp) return -1;
  if (d.sh != d.sw || (d.sh != 1 && d.sh != 2)) return -1;
  if ((int64_t)d.n * d.ho * d.wo >= (1 << 24) || (int64_t)d.n * d.hp * d.wp * d.cp >= (1LL << 31)) return -1;
  if (ek != EK_NCHW && d.cout % 16) return -1;
  if (ek == EK_GEN && d.cout % C::CB) return -1;  // gen_epilogue: whole channel tiles
  g.s2 = d.sh == 2;
  g.wb = d.wp;
  g.we = (d.wp + 1) / 2;
  g.npl = d.cp / 32;
  const int img = d.ho * d.wo;
  const int nby = (int)cdiv(d.cout, C::CB);
  const int budget = LDS_MAX / C::BPC;
  auto fit = [&](int rows, int nbrows, bool lut) {
    g.rows = rows;
    g.nbrows = nbrows;
    g.nbp = nbrows * g.wb;
    g.pl = (int)cdiv((int64_t)g.nbp * 32, 1024) * 1024;
    g.ppp = g.pl / 1024;
    g.npieces = g.npl * g.ppp;
    g.buf = g.npl * g.pl;
    g.wst_off = 0;
    g.wsep = 0;
    if (2 * g.buf + 1024 * C::KS * C::TM + 256 * g.npieces + 4 * (d.ho + d.wo) + epi_bytes(p, C::BM, lut) + 512 <= budget) {
      g.wst_off = 2 * g.buf;  // the weights' own staging area (the first bands load beside it)
      g.wsep = 1;
    }
    g.sync_off = 2 * g.buf + (g.wsep ? 1024 * C::KS * C::TM : 0);
    g.rel_off = g.sync_off + 16;
    g.cls_off = g.rel_off + 256 * g.npieces;
    // 256-byte aligned (dynamic LDS starts at address 0): the code table after the 64-float
    // vectors then is too, so a table byte's offset is its row's offset OR-ed with the code
    const int epi_off = (g.cls_off + 4 * (d.ho + d.wo) + 255) & ~255;
    g.npt = (int)cdiv((int64_t)rows * d.wo, 16);
    g.lut = lut ? 1 : 0;
    const int lds = epi_off + epi_bytes(p, C::BM, lut);
    if (lds > budget) return -1;
    q.epi_off = epi_off;
    return lds;
  };
  struct Cand {
    int rows, nbrows;
  };
  Cand cands[64];
  int nc = 0;
  if (img <= C::PXMAX)
    for (int k = C::PXMAX / img < d.n ? C::PXMAX / img : d.n; k >= 1 && nc < 32; --k)
      cands[nc++] = {k * d.ho, (k - 1) * d.hp + (d.ho - 1) * d.sh + 3};
  for (int rows = d.ho - 1; rows >= 1 && nc < 64; --rows)
    if (d.ho % rows == 0 && rows * d.wo <= C::PXMAX) cands[nc++] = {rows, (rows - 1) * d.sh + 3};
  // the candidate whose busiest block slot has the least work (ceil(bands / slots) x a band's
  // tiles and overhead), the taller band on a tie (less halo); the code table whenever it fits
  const int64_t slots = (int64_t)NUM_CU * C::BPC;
  int best = -1, best_lut = 0;
  int64_t best_cost = 0;
  for (int i = 0; i < nc; ++i) {
    const bool want_lut = ek == EK_LUT && d.cout % C::CB == 0 && p.e.code0_cp >= d.cout;
    int lut = want_lut ? 1 : 0;
    if (fit(cands[i].rows, cands[i].nbrows, lut) < 0) {
      if (!lut || fit(cands[i].rows, cands[i].nbrows, false) < 0) continue;
      lut = 0;
    }
    const int64_t nb = cdiv((int64_t)d.n * d.ho, cands[i].rows) * nby;
    // a band costs its tiles plus ~2/3 of a tile per wave of hand-off overhead (its DMA issue and
    // publication; measured, tools/pb_stamps.py): taller bands win unless they unbalance the slots
    const int64_t cost = cdiv(nb, slots) * (3 * cdiv((int64_t)cands[i].rows * d.wo, 16) + 2 * C::W) * 1024 +
                         (1023 - (lut ? 0 : 512));
    if (best < 0 || cost < best_cost) best = i, best_cost = cost, best_lut = lut;
  }
  if (best >= 0) {
    const int lds = fit(cands[best].rows, cands[best].nbrows, best_lut);
    g.nbands = (int)cdiv((int64_t)d.n * d.ho, cands[best].rows);
    q.epi_early = 1;
    q.scr_off = 0;
    return lds;
  }
  return -1;
}

// co-resident blocks per CU at `lds` bytes (hipOccupancy..., cached per kernel and LDS size)
static int blocks_per_cu(const void* kern, int nt, int lds) {
  static std::atomic<long long> cache[8];  // (kernel slot hash, lds) -> n: tiny direct-mapped cache
  const long long key = ((long long)(uintptr_t)kern << 20) ^ lds;
  const int slot = (int)((((uintptr_t)kern) >> 4) ^ lds) & 7;
  const long long v = cache[slot].load(std::memory_order_relaxed);
  if (v != 0 && (v >> 8) == (key & ((1LL << 55) - 1))) return (int)(v & 255);
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, nt, lds) != hipSuccess || n < 1) n = 1;
  cache[slot].store(((key & ((1LL << 55) - 1)) << 8) | (n & 255), std::memory_order_relaxed);
  return n;
}

// F32: the fp32-input instantiation (qnn_qconv2d_fwd_nchw_f32; its own register allocation, so the
// band fill's registers never touch the code-input kernels')
template <class C, int EK, bool BIAS = false, bool F32 = false>
static int launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ, const F32In* fin) {
  auto kern = qconv_pb_kernel<C, EK, BIAS, F32>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  Geo g;
  Params q = p;
  const int lds = geometry<C>(p, g, q);
  if (lds < 0) return arg_error("tile configuration not built for this layer / epilogue kind");
  static const int wstage = [] {  // (diagnostic switch while the two prologues are compared)
    const char* v = getenv("QNN_PB_WSTAGE");
    return v ? atoi(v) : 1;
  }();
  g.wstage = wstage;
  g.spin_max = g_spin_max;
  g.xf = nullptr;
  if (fin) {
    g.xf = fin->x;
    g.fc = fin->c, g.fh = fin->h, g.fw = fin->w, g.fpad = fin->pad;
    g.fnm = fin->neg_min, g.fs = fin->scale, g.fqmax = fin->qmax;
  }
  const int nby = (int)cdiv(p.d.cout, C::CB);
  const int per_cu = blocks_per_cu((const void*)kern, C::NT, lds);
  int64_t nblk = ((int64_t)NUM_CU * per_cu / nby) * nby;
  nblk = nblk < nby ? nby : nblk;
  const int64_t tiles = (int64_t)g.nbands * nby;
  nblk = nblk < tiles ? nblk : tiles;
  if (occ) {
    occ->blocks_per_cu = per_cu, occ->lds = lds, occ->grid = (int)nblk;
    return QNN_OK;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(C::NT), lds, s, x, w, q, g);
  return QNN_OK;
}

template <class C>
static int launch_ek(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ, const F32In* fin) {
  if (fin) {  // the drop-in's fp32 input: built for its fp32 NCHW output only
    if (epi_kind(p.e) != EK_NCHW) return arg_error("fp32-input convolution: fp32 NCHW output only");
    return launch<C, EK_NCHW, false, true>(x, w, p, s, occ, fin);
  }
  switch (epi_kind(p.e)) {
    case EK_NCHW: return launch<C, EK_NCHW>(x, w, p, s, occ, fin);
    case EK_LUT:
      return p.e.bias ? launch<C, EK_LUT, true>(x, w, p, s, occ, fin) : launch<C, EK_LUT, false>(x, w, p, s, occ, fin);
    case EK_BNCODE: return launch<C, EK_BNCODE>(x, w, p, s, occ, fin);
    default:  // the general chain beside 144 resident weight registers spills at two waves per SIMD: not built
      if constexpr (C::TM * C::KS > 18 && C::BPC * C::W / 4 > 1) return arg_error("tile configuration not built for this layer / epilogue kind");
      else return launch<C, EK_GEN>(x, w, p, s, occ, fin);
  }
}

//   id  block (cout)  waves  weights resident  blocks/CU  band pixels  fits
//   0   64            4      36 fragments      2          <= 256       3x3 on 64 channels (ResNet layer 1, layer-2 entry)
//   1   64            8      36 fragments      1          <= 512       the same, one block per CU (one weight staging)
//   2   32            4      18 fragments      2          <= 256       the same at half the registers (general chains)
//   3   32            4      36 fragments      2          <= 256       3x3 on 128 channels (ResNet-18 layer 2)
//   4   32            8      36 fragments      1          <= 512       the same, one block per CU
using P0 = Cfg<4, 9, 2, 256>;
using P1 = Cfg<4, 9, 1, 512, 8>;
using P2 = Cfg<2, 9, 2, 256>;
using P3 = Cfg<2, 18, 2, 256>;
using P4 = Cfg<2, 18, 1, 512, 8>;
constexpr int NP = 5;
struct Info {
  int cb;
  float rate;
};
static const Info INFO[NP] = {{64, 1.5f}, {64, 1.5f}, {32, 1.4f}, {32, 1.5f}, {32, 1.5f}};

template <int K>
using CfgK = std::conditional_t<K == 0, P0, std::conditional_t<K == 1, P1, std::conditional_t<K == 2, P2,
             std::conditional_t<K == 3, P3, P4>>>>;

template <int K>
static bool ok_k(const Params& p) {
  using C = CfgK<K>;
  if (epi_kind(p.e) == EK_GEN && C::TM * C::KS > 18 && C::BPC * C::W / 4 > 1) return false;
  Geo g;
  Params q = p;
  return geometry<CfgK<K>>(p, g, q) >= 0;
}

}  // namespace pb

int pb_count() { return pb::NP; }

extern "C" int qnn_device_errors(uint32_t* flags, int clear) {
  unsigned v = 0;
  if (int rc = hip_check(hipDeviceSynchronize(), "qnn_device_errors: synchronize")) return rc;
  if (int rc = hip_check(hipMemcpyFromSymbol(&v, HIP_SYMBOL(::qnn_dev_errors), sizeof(v)), "qnn_device_errors"))
    return rc;
  if (clear && v) {
    const unsigned z = 0;
    if (int rc = hip_check(hipMemcpyToSymbol(HIP_SYMBOL(::qnn_dev_errors), &z, sizeof(z)), "qnn_device_errors: clear"))
      return rc;
  }
  if (flags) *flags = v;
  return QNN_OK;
}

extern "C" int qnn_debug_set_spin_limit(int limit) {
  pb::g_spin_max = limit < 0 ? pb::SPIN_MAX : limit;
  return QNN_OK;
}

#if QNN_STAMP
extern "C" int qnn_debug_stamps_pb(void* dst, size_t bytes) {
  if (bytes > sizeof(::qnn_pb_stamps)) bytes = sizeof(::qnn_pb_stamps);
  return hip_check(hipMemcpyFromSymbol(dst, HIP_SYMBOL(::qnn_pb_stamps), bytes), "stamps");
}
#endif

void pb_tile(int k, int* bm, int* bn) {
  *bm = pb::INFO[k].cb;
  *bn = 16;
}

bool pb_ok(int k, const Params& p) {
  switch (k) {
    case 0: return pb::ok_k<0>(p);
    case 1: return pb::ok_k<1>(p);
    case 2: return pb::ok_k<2>(p);
    case 3: return pb::ok_k<3>(p);
    case 4: return pb::ok_k<4>(p);
    default: return false;
  }
}

int64_t pb_blocks(int k, const Params& p) { return cdiv(p.M, 16) * cdiv(p.d.cout, pb::INFO[k].cb); }

// the cost model's units (qconv.hip cfg_cost): padded MFMA work of a CU's share / rate
double pb_cost(int k, const Params& p) {
  if (!pb_ok(k, p)) return 1e30;
  const pb::Info& f = pb::INFO[k];
  const double work = (double)cdiv(p.M, 16) * 16 * cdiv(p.d.cout, f.cb) * f.cb * (p.taps * p.d.cp);
  return work / NUM_CU / f.rate;
}

int pb_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ, const F32In* fin) {
  switch (k) {
    case 0: return pb::launch_ek<pb::P0>(x, w, p, s, occ, fin);
    case 1: return pb::launch_ek<pb::P1>(x, w, p, s, occ, fin);
    case 2: return pb::launch_ek<pb::P2>(x, w, p, s, occ, fin);
    case 3: return pb::launch_ek<pb::P3>(x, w, p, s, occ, fin);
    case 4: return pb::launch_ek<pb::P4>(x, w, p, s, occ, fin);
    default: return arg_error("tile configuration not built for this layer / epilogue kind");
  }
}

}  // namespace qnn
