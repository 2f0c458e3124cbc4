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
#include <type_traits>

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

namespace qnn {
namespace pb {

template <int TM_, int KS_, int BPC_, int PXMAX_>
struct Cfg {
  static constexpr int WGM = 1, WGN = 4, TM = TM_, TN = 1, KS = KS_, BPC = BPC_, PXMAX = PXMAX_;
  static constexpr int W = 4, NT = 256;
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
  int cls_off;    // LDS: hcls[ho] * nwc, then wcls[wo]
  int npt;        // 16-pixel tiles per band
  int lut;        // EK_LUT: the code table is staged (else evaluated)
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
template <class C>
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
  const bool has_bias = e.bias != nullptr;
  unsigned wrd[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = 16 * i + 4 * gq;
    const float4 sw = *reinterpret_cast<const float4*>(s_f + cl);
    const float4 bw = *reinterpret_cast<const float4*>(s_f + BM + cl);
    const float4 tb = *reinterpret_cast<const float4*>(tp + cl);
    const v4i& a = acc[i][0];
    const f2 a01 = {(float)a[0], (float)a[1]}, a23 = {(float)a[2], (float)a[3]};
    f2 v0 = pfma((f2){sw.x, sw.y}, a01, pfma((f2){bw.x, bw.y}, p2, (f2){tb.x, tb.y}));
    f2 v1 = pfma((f2){sw.z, sw.w}, a23, pfma((f2){bw.z, bw.w}, p2, (f2){tb.z, tb.w}));
    if (has_bias) {  // (the other kernels add staged zeros: v + 0 differs from v only for v = -0,
                     // and -0 and +0 quantize to the same code)
      const float4 bi = *reinterpret_cast<const float4*>(s_f + 2 * BM + cl);
      v0 = v0 + (f2){bi.x, bi.y};
      v1 = v1 + (f2){bi.z, bi.w};
    }
    const f2 q0 = qclamp2(v0, bnp) + MAGIC_U8, q1 = qclamp2(v1, bnp) + MAGIC_U8;
    const uint32_t row = lut_off + (uint32_t)cl * 256u;  // channel cl's 256 codes; cl + u at + 256 u
    const uint32_t k0 = (__float_as_uint(q0.x) & 255u) | row;
    const uint32_t k1 = (__float_as_uint(q0.y) & 255u) | (row + 256u);
    const uint32_t k2 = (__float_as_uint(q1.x) & 255u) | (row + 512u);
    const uint32_t k3 = (__float_as_uint(q1.y) & 255u) | (row + 768u);
    const uint8_t* lb = reinterpret_cast<const uint8_t*>(smem);
    if (QNN_ABLATE == 4) wrd[i] = (k0 & 255u) | ((k1 & 255u) << 8) | ((k2 & 255u) << 16) | ((k3 & 255u) << 24);
    else wrd[i] = (unsigned)lb[k0] | ((unsigned)lb[k1] << 8) | ((unsigned)lb[k2] << 16) | ((unsigned)lb[k3] << 24);
  }
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

// Every wait on a counter is bounded (~0.1-0.5 s): a protocol error then yields wrong outputs that
// the bitwise tests catch, never a wave that spins until the process is killed
constexpr int SPIN_MAX = 1 << 21;

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

template <class C, int EK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(C::BPC))) void qconv_pb_kernel(
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
  // wave moves pieces k = wave + 4 i of every band and publishes them once they landed.
  const uint32_t max_off = (uint32_t)(last_px * d.cp);
  const float inv_wb = 1.0f / (float)g.wb;
  auto band_row0 = [&](int j) {  // first padded input row (batch-flat) of the block's band j
    const int r0 = (bfirst + j * bstep) * g.rows;
    return (r0 / d.ho) * d.hp + (r0 % d.ho) * d.sh;
  };
  auto issue_band = [&](int j) {
    if (QNN_ABLATE == 3) return;
    const uint32_t base = (uint32_t)band_row0(j) * (uint32_t)(d.wp * d.cp);
    int8_t* dst = smem + (j & 1) * g.buf;
    for (int k = wave; k < g.npieces; k += 4) {
      const int v = k / g.ppp, r = k - v * g.ppp;  // wave-uniform
      int b = r * 32 + (lane >> 1);
      b = b < g.nbp ? b : g.nbp - 1;
      int br, cc;
      fdivmod(b, g.wb, inv_wb, br, cc);
      const int col = g.s2 ? (cc < g.we ? 2 * cc : 2 * (cc - g.we) + 1) : cc;
      uint32_t off = base + (uint32_t)((br * d.wp + col) * d.cp + 32 * v + 16 * (lane & 1));
      off = off < max_off ? off : max_off & ~15u;
      dma16(x, off, dst + v * g.pl + r * 1024);
    }
  };

  // ---- prologue: the epilogue's data (EK_LUT: with its code table when g.lut, else evaluated),
  // the border classes, the counters, and the block's weights -- staged once through the band
  // buffers (one copy per block instead of one per wave from L2) when they fit there
  if (EK == EK_LUT && g.lut) stage_epi<C, EK_LUT>(p, x, smem + p.epi_off, c0, wave, lane);
  else stage_epi<C, (EK == EK_LUT ? EK_BNCODE : EK)>(p, x, smem + p.epi_off, c0, wave, lane);
  int* s_hc = reinterpret_cast<int*>(smem + g.cls_off);
  for (int i = tid; i < d.ho + d.wo; i += NT) s_hc[i] = i < d.ho ? p.e.hcls[i] * p.e.nwc : p.e.wcls[i - d.ho];
  if (tid < 4) s_sync[tid] = 0;
#if QNN_STAMP
  PB_TS(tp1);
#endif
  const int wbytes = CB * d.kpad;  // rows c0 .. c0 + CB - 1 of the packed weights, contiguous
  const bool wlds = wbytes <= 2 * g.buf;
  if (wlds)
    for (int k = wave; 1024 * k < wbytes; k += 4) {
      int off = 1024 * k + 16 * lane;
      off = off < wbytes ? off : wbytes - 16;
      dma16(w, (uint32_t)((int64_t)c0 * d.kpad + off), smem + 1024 * k);
    }
#if QNN_STAMP
  PB_TS(tp2);
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#if QNN_STAMP
  PB_TS(tp3);
#endif
  // the weights, resident in VGPRs for the block's life: K step s = (group s / 9, tap s % 9) is
  // weight bytes tap * cp + 64 group of rows c0 + 16 i + (lane & 15), K bytes 16 (lane >> 4)
  v4i fa[KS][TM];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int gk = s / 9, t = s - 9 * gk;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = 16 * i + (lane & 15);
      const int kb = t * d.cp + 64 * gk + 16 * gq;
      if (wlds) fa[s][i] = *reinterpret_cast<const v4i*>(smem + row * d.kpad + kb);
      else fa[s][i] = *reinterpret_cast<const v4i*>(w + (int64_t)(c0 + row) * d.kpad + kb);
    }
  }
  // every wave holds its weights before the bands overwrite the staging area (a raw barrier:
  // the fragments are compiler-visible LDS reads, waited for by lgkmcnt(0))
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#if QNN_STAMP
  PB_TS(tp4);
#endif
  int issued = nb < 2 ? nb : 2, published = 0;
  for (int j = 0; j < issued; ++j) issue_band(j);

  auto publish = [&] {  // this wave's pieces of the bands it issued have landed
    if (published < issued) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

  // ---- the wave's tiles T = wave + 4 i of the block's band sequence (npt tiles per band), no
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
    if (can_issue()) issue_band(issued++);
    while (issued <= j) {  // this band's buffer waits for another wave's last tile of band j - 2
      publish();             // (never wait while holding unpublished pieces another wave may wait for)
      for (int guard = 0; !can_issue() && guard < SPIN_MAX; ++guard) __builtin_amdgcn_s_sleep(2);
      issue_band(issued++);
    }
    publish();
    {
      const int target = 4 * (j / 2 + 1);
      for (int guard = 0; lds_get(&s_sync[j & 1]) < target && guard < SPIN_MAX; ++guard) __builtin_amdgcn_s_sleep(1);
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
    v4i acc[TM][1], sacc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[i][0] = (v4i){0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int gk = s / 9, tp = s - 9 * gk;
      v4i fb;
      if (QNN_ABLATE == 5) fb = (v4i){pbase, s, lane, 1};
      else fb = *reinterpret_cast<const v4i*>(smem + pbase + 2 * gk * g.pl + 32 * tap_px(tp));
      // sum_valid(q'_x): an all-ones A row sums the fragment's codes (padding codes are 0)
      sacc = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, fb, sacc, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (QNN_ABLATE == 1) {
          asm volatile("" ::"v"(fa[s][i]), "v"(fb));
          acc[i][0][0] ^= fb.x + fa[s][i].y;
        } else {
          acc[i][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s][i], fb, acc[i][0], 0, 0, 0);
        }
      }
    }
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
      lut_epilogue<C>(p, acc, sumq[0], s_hc[hh] + s_hc[d.ho + col], n, hh, col, smem, c0, lane);
    } else {
      q16::epilogue_rb<C, EK>(p, acc, sumq, pixel, smem, c0, 0, lane, g.lut);
    }
    // the tile's band fragments were consumed by its MFMAs: count it finished
    __builtin_amdgcn_sched_barrier(0);
    if (lane == 0) lds_add(&s_sync[2 + buf], 1);
#if QNN_STAMP
    PB_TS(tb);
    c_epi += tb - ta;
#endif
    t += 4;
    while (t >= g.npt && j < nb) t -= g.npt, ++j;
  }
  // the bands other waves still need from this one
  while (issued < nb) {
    publish();
    for (int guard = 0; !can_issue() && guard < SPIN_MAX; ++guard) __builtin_amdgcn_s_sleep(2);
    issue_band(issued++);
  }
  publish();
#if QNN_STAMP
  nband = nb;
  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && blockIdx.x < (1 << 19) / 64) {
    unsigned long long* o = qnn_pb_stamps + ((size_t)blockIdx.x * 4 + wave) * 16;
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
    g.sync_off = 2 * g.buf;
    g.cls_off = g.sync_off + 16;
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
  for (int pass = 0; pass < 2; ++pass) {  // pass 0: enough bands for every block slot; pass 1: any
    for (int i = 0; i < nc; ++i) {
      const int64_t nb = cdiv((int64_t)d.n * d.ho, cands[i].rows);
      if (pass == 0 && nb * nby < (int64_t)NUM_CU * C::BPC) continue;
      int lds = -1;
      // the staged code table (lut_epilogue) when the block's channel tile is whole
      if (ek == EK_LUT && d.cout % C::CB == 0 && p.e.code0_cp >= d.cout) lds = fit(cands[i].rows, cands[i].nbrows, true);
      if (lds < 0) lds = fit(cands[i].rows, cands[i].nbrows, false);
      if (lds < 0) continue;
      g.nbands = (int)nb;
      q.epi_early = 1;
      q.scr_off = 0;
      return lds;
    }
  }
  return -1;
}

// co-resident blocks per CU at `lds` bytes (hipOccupancy..., cached per kernel and LDS size)
static int blocks_per_cu(const void* kern, int lds) {
  static std::atomic<long long> cache[8];  // (kernel slot hash, lds) -> n: tiny direct-mapped cache
  const long long key = ((long long)(uintptr_t)kern << 20) ^ lds;
  const int slot = (int)((((uintptr_t)kern) >> 4) ^ lds) & 7;
  const long long v = cache[slot].load(std::memory_order_relaxed);
  if (v != 0 && (v >> 8) == (key & ((1LL << 55) - 1))) return (int)(v & 255);
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, 256, lds) != hipSuccess || n < 1) n = 1;
  cache[slot].store(((key & ((1LL << 55) - 1)) << 8) | (n & 255), std::memory_order_relaxed);
  return n;
}

template <class C, int EK>
static int launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  auto kern = qconv_pb_kernel<C, EK>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  Geo g;
  Params q = p;
  const int lds = geometry<C>(p, g, q);
  if (lds < 0) return arg_error("tile configuration not built for this layer / epilogue kind");
  const int nby = (int)cdiv(p.d.cout, C::CB);
  const int per_cu = blocks_per_cu((const void*)kern, lds);
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
static int launch_ek(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  switch (epi_kind(p.e)) {
    case EK_NCHW: return launch<C, EK_NCHW>(x, w, p, s, occ);
    case EK_LUT: return launch<C, EK_LUT>(x, w, p, s, occ);
    case EK_BNCODE: return launch<C, EK_BNCODE>(x, w, p, s, occ);
    default:  // the general chain beside 144 resident weight registers spills at two waves per SIMD: not built
      if constexpr (C::TM * C::KS > 18 && C::BPC > 1) return arg_error("tile configuration not built for this layer / epilogue kind");
      else return launch<C, EK_GEN>(x, w, p, s, occ);
  }
}

//   id  block (cout)  weights resident  blocks/CU  band pixels  fits
//   0   64            36 fragments      2          <= 256       3x3 on 64 channels (ResNet layer 1, layer-2 entry)
//   1   64            36 fragments      1          <= 512       the same, taller bands
//   2   32            18 fragments      2          <= 256       the same at half the registers (general chains)
//   3   32            36 fragments      2          <= 256       3x3 on 128 channels (ResNet-18 layer 2)
//   4   32            36 fragments      1          <= 512       the same, taller bands
using P0 = Cfg<4, 9, 2, 256>;
using P1 = Cfg<4, 9, 1, 512>;
using P2 = Cfg<2, 9, 2, 256>;
using P3 = Cfg<2, 18, 2, 256>;
using P4 = Cfg<2, 18, 1, 512>;
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
  if (epi_kind(p.e) == EK_GEN && C::TM * C::KS > 18 && C::BPC > 1) return false;
  Geo g;
  Params q = p;
  return geometry<CfgK<K>>(p, g, q) >= 0;
}

}  // namespace pb

int pb_count() { return pb::NP; }

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

int pb_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  switch (k) {
    case 0: return pb::launch_ek<pb::P0>(x, w, p, s, occ);
    case 1: return pb::launch_ek<pb::P1>(x, w, p, s, occ);
    case 2: return pb::launch_ek<pb::P2>(x, w, p, s, occ);
    case 3: return pb::launch_ek<pb::P3>(x, w, p, s, occ);
    case 4: return pb::launch_ek<pb::P4>(x, w, p, s, occ);
    default: return arg_error("tile configuration not built for this layer / epilogue kind");
  }
}

}  // namespace qnn
