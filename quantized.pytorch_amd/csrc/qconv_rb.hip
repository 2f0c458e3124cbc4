// Resident-band int8 convolution on v_mfma_i32_16x16x64_i8: the eval forward of QConv2d
// (models/modules/quantize.py:314-349) for kh x kw > 1, same exact decomposition and
// epilogue arithmetic as qconv.hip / qconv16.hip, so every configuration
// of every kernel family computes bitwise identical outputs.
//
// A block owns whole output rows -- one or more images, or a divisor of an image's rows --
// and BM output channels.  Its input BAND (every padded input row those output rows read,
// ALL Cp channels) is loaded into LDS once, at kernel start, by LDS-DMA; every tap of every
// K step then reads its B fragment at a tap-shifted LDS address.  No input byte crosses L2
// more than once per block (qconv.hip's implicit im2col pulls it once per tap), and the
// main loop has no barrier at all:
//
// * B = the band, 32-byte PLANES (plane v = bytes [32v, 32v + 32) of every band pixel,
//   planes 1 KiB aligned).  A 16x16x64 fragment lane (pixel l&15, K bytes 16*(l>>4)..) reads
//   plane 2g + (l>>5), half (l>>4)&1, of its pixel: within each ds_read_b128 lane group the
//   16 (pixel, half) pairs land on 16 distinct bank slots (2*pixel + half mod 16) -- no
//   swizzle, no padding; a tap shift is one uniform add.  Tiles that straddle an output row
//   end see at most 2-way conflicts.
// * A = the weights straight from the packed rows ([cout_pad][kpad], tap-major) into VGPRs,
//   one global_load_dwordx4 per 16-channel tile per K step, prefetched DA - 1 steps ahead.  Each
//   wave owns its own output channels, so nothing is shared and nothing synchronises.  K
//   steps run plane-pair major (g = 2gp, 2gp+1 for each tap), so the two loads of a pair
//   consume each 128-byte weight line whole, back to back.
// * sum_valid(q'_x): per band pixel channel sums after the loop, then the taps' sum per
//   output pixel (padding codes are 0, so the receptive-field sum is exact).
#include <stdlib.h>

#include <type_traits>
#include <utility>

#include "rb_common.h"

#ifndef QNN_ABLATE
#define QNN_ABLATE 0  // diagnostic builds only: 1 no weight loads, 2 no MFMA, 3 no epilogue
#endif
#ifndef QNN_RB_ASM
#define QNN_RB_ASM 1  // 1: band reads as inline asm with hand-counted lgkmcnt; 0: compiler-scheduled
#endif
#ifndef QNN_RB_AGPR
#define QNN_RB_AGPR 0  // 1: accumulators in AGPRs (an 'a'-constrained asm operand makes the
                       // compiler select the AGPR form of the MFMAs)
#endif
#if QNN_STAMP
// [block][wave][8]: realtime start/end, cycles: band landed, K loop, sums, late staging, epilogue
// code, store drain
__device__ unsigned long long qnn_rb_stamps[1 << 18];
#endif

namespace qnn {
namespace rb {

// ---------------------------------------------------------------- kernel
// The whole band lands before the K loop (one vmcnt(0) + barrier); the weights are plain
// compiler-scheduled loads, so every VMEM wait in the loop is the compiler's own.
template <class C, int EK, int H>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(C::BPC * C::W / 4))) void qconv_rb_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ w, const Params p, const Geo g) {
  constexpr int BM = C::BM, W = C::W, TM = C::TM, TN = C::TN, DA = C::DA, NT = C::NT;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];

  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WGN, wn = wave % C::WGN;
#if QNN_STAMP
  unsigned long long ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0, ts4 = 0, ts5 = 0, ts6 = 0;
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  RB_TS(ts0);
#endif

  // ---- XCD-aware bijective block -> (band, channel tile) map, channel tiles fastest
  const int nby = (d.cout + BM - 1) / BM;
  const int nblk = g.nbands * nby;
  int t;
  {
    const int bb = blockIdx.x, xcd = bb & 7, q = nblk >> 3, r = nblk & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bb >> 3);
  }
  const int band = t / nby;
  const int c0 = (t - band * nby) * BM;
  const int r0 = band * g.rows;              // first flattened output row
  const int nrows_all = d.n * d.ho;
  const int R0 = (r0 / d.ho) * d.hp + (r0 % d.ho) * d.sh;  // first padded input row (batch-flat)
  const int rows_in = d.n * d.hp;

  // ---- band DMA: a piece is 1 KiB of plane v = band pixels [32r, 32r + 32) (range r), lane i
  // pixel + (i >> 1), 16-byte half i & 1.  A wave issues every plane of a range back to back
  // (ranges r = wave + W*j), so the 4 pieces reading one 128-byte pixel line hit L1 after the
  // first.  Ranges past the band re-read the last one (identical bytes to the same place).
  auto band_src = [&](int r, int v) -> uint32_t {
    int b = r * 32 + (lane >> 1);
    b = b < g.nbp ? b : g.nbp - 1;
    const int br = b / g.wb, cc = b - br * g.wb;
    const int col = g.s2 ? (cc < g.we ? 2 * cc : 2 * (cc - g.we) + 1) : cc;
    int row = R0 + br;
    row = row < rows_in ? row : rows_in - 1;  // past the batch: feeds only pixels never stored
    if (cc >= d.wp) return (uint32_t)d.zero_off;  // row padding of the band (never read)
    return (uint32_t)((row * d.wp + col) * d.cp + 32 * v + 16 * (lane & 1));
  };
  auto band_dst = [&](int r, int v) -> int8_t* { return smem + v * g.pl + r * 1024; };
  auto issue_piece = [&](int r, int v) {
    r = r < g.ppp ? r : g.ppp - 1;
    uint32_t off = band_src(r, v);
    asm volatile("" : "+v"(off));
    __builtin_amdgcn_global_load_lds((const void*)(x + off), (lds_ptr_t)band_dst(r, v), 16, 0, 0);
  };
  for (int k = 0; k < g.nbw; ++k) issue_piece(wave + W * (k / g.npl), k % g.npl);
  // the epilogue's data next (EK_LUT: with its code table when g.lut, else evaluated)
  auto stage = [&] {
    if (EK == EK_LUT && g.lut) stage_epi<C, EK_LUT>(p, x, smem + p.epi_off, c0, wave, lane);
    else stage_epi<C, (EK == EK_LUT ? EK_BNCODE : EK)>(p, x, smem + p.epi_off, c0, wave, lane);
  };
  if (p.epi_early) stage();

  // ---- this lane's pixels: block pixel q = (wn*TN + j)*16 + (lane & 15); past the block
  // (or the batch) they stand in for the block's last pixel and are never stored
  const int npx_blk = __builtin_amdgcn_readfirstlane(
      (r0 + g.rows <= nrows_all ? g.rows : nrows_all - r0) * d.wo);
  int pb[TN];  // band pixel of tap (0, 0), in bytes of a plane (x32)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int q = (wn * TN + j) * 16 + (lane & 15);
    q = q < npx_blk ? q : npx_blk - 1;
    const int rr = q / d.wo, col = q - rr * d.wo;
    const int r = r0 + rr, n = r / d.ho, ho = r - n * d.ho;
    pb[j] = ((n * d.hp + ho * d.sh - R0) * g.wb + col) * 32 + (lane >> 5) * g.pl + 16 * ((lane >> 4) & 1);
  }

  // ---- weights: rows c0 + wm*16*TM + 16*i + (lane & 15), K bytes 16*(lane >> 4) of each step
  const int8_t* wblk = w + (int64_t)c0 * d.kpad;
  uint32_t aoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int row = wm * 16 * TM + 16 * i + (lane & 15);
    row = c0 + row < d.cout_pad ? row : d.cout_pad - 1 - c0;
    aoff[i] = (uint32_t)(row * d.kpad + 16 * (lane >> 4));
  }

  // K steps: plane pairs gp (H = 2 64-byte channel groups each; H = 1 when cp == 64), taps t,
  // h in the pair: step (g = H*gp + h, t) is weight bytes t*cp + 64g and band planes 2g, 2g+1
  const int KS = (d.cp / 64) * p.taps;
  struct Cur {
    int t, tr, tc, gp, h;
  };
  auto advance = [&](Cur& c) {
    if (++c.h == H) {
      c.h = 0;
      if (++c.tc == d.kw) c.tc = 0, ++c.tr;
      if (++c.t == p.taps) c.t = 0, c.tr = 0, c.tc = 0, ++c.gp;
    }
  };
  auto kbytes = [&](const Cur& c) { return c.t * d.cp + 64 * (H * c.gp + c.h); };

  // DA register slots, DA - 1 K steps of weights in flight: step s computes from slot s % DA and
  // then refills slot (s - 1) % DA, whose last reader (step s - 1's MFMAs) issued a whole step of
  // MFMAs earlier.  Refilling the slot the step has just read lets a load's asynchronous return
  // overwrite an A operand the matrix core has not finished reading when another workgroup's
  // MFMAs hold the XDL pipe (the two-blocks-per-CU corruption of row 12 of an A fragment,
  // DESIGN.md §4; tools/asm_mfma_war_check.py finds such loads in the ISA).
  v4i fa[DA][TM];
  Cur cl = {0, 0, 0, 0, 0};  // the next step to load
  auto load_a = [&](v4i (&dst)[TM]) {
    if (QNN_ABLATE == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i) dst[i] = (v4i){i, 1, 2, 3};
      return;
    }
    const int8_t* base = wblk + kbytes(cl);
#pragma unroll
    for (int i = 0; i < TM; ++i) dst[i] = *reinterpret_cast<const v4i*>(base + aoff[i]);
    if (H * cl.gp + cl.h < d.cp / 64 - 1 || cl.t < p.taps - 1 || cl.h < H - 1) advance(cl);  // clamp at the last step
  };
#pragma unroll
  for (int s = 0; s < DA - 1; ++s) load_a(fa[s]);
  // LDS constants and the epilogue's data (their loads wait behind the band and the weights)
  int* s_tap = reinterpret_cast<int*>(smem + g.tap_off);
  int* s_hc = reinterpret_cast<int*>(smem + g.cls_off);  // border classes: hcls[ho] * nwc, wcls[wo]
  if (tid < p.taps) {
    const int tr = tid / d.kw, tc = tid - tr * d.kw;
    s_tap[tid] = tr * g.wb + (g.s2 ? (tc & 1) * g.we + (tc >> 1) : tc);
  }
  for (int i = tid; i < d.ho + d.wo; i += NT)
    s_hc[i] = i < d.ho ? p.e.hcls[i] * p.e.nwc : p.e.wcls[i - d.ho];

  v4i acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4i){0, 0, 0, 0};
#if QNN_RB_AGPR
  {
    int z = 0;
    asm volatile("; agpr form" : "+a"(z));
    if (z == 0x7fffffff) p.e.out_f32[0] = 1.f;
  }
#endif

  // the band's group 0, the weights and the epilogue data have landed for this wave
  wait_vmcnt<0>();
  __syncthreads();
#if QNN_STAMP
  RB_TS(ts1);
#endif

  Cur cc = {0, 0, 0, 0, 0};
  // One K step: the TN band fragments are read up front (inline asm, so the compiler
  // cannot interleave each read with its first use), then each fragment's TM MFMAs wait
  // only for that fragment (LDS returns in order: lgkmcnt(TN-1-j)).  The partner wave on
  // the SIMD runs its MFMAs while this one waits for its reads.
  auto step = [&](auto slotc) {
    constexpr int SL = decltype(slotc)::value;
    const int dt = cc.tr * g.wb + (g.s2 ? (cc.tc & 1) * g.we + (cc.tc >> 1) : cc.tc);
    const int boff = (2 * (H * cc.gp + cc.h)) * g.pl + 32 * dt;
    v4i fb[TN];
#if QNN_RB_ASM
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      v4i r;
      asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(pb[j] + boff));
      fb[j] = r;
    }
#else
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const v4i*>(smem + pb[j] + boff);
    __builtin_amdgcn_sched_group_barrier(0x100, TN, 0);       // the TN band reads first
    __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);  // then the MFMAs
#endif
    static_for<TN>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
#if QNN_RB_ASM
      lds_wait<TN - 1 - j>();
#endif
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (QNN_ABLATE == 2) {
          asm volatile("" ::"v"(fa[SL][i]), "v"(fb[j]));
          acc[i][j][0] += fa[SL][i].x;
        } else {
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[SL][i], fb[j], acc[i][j], 0, 0, 0);
        }
      }
    });
    // the refill goes after this step's MFMAs (the asm path's last lds_wait already fences all
    // but the last fragment's): slot (SL + DA - 1) % DA was last read one step earlier
    __builtin_amdgcn_sched_barrier(0);
    load_a(fa[(SL + DA - 1) % DA]);
    advance(cc);
  };
  static_assert(DA >= 1 && DA <= 4, "the K loop unrolls at most four weight slots per pass");
#pragma nounroll
  for (int k0 = 0; k0 < KS; k0 += DA) {
    step(std::integral_constant<int, 0>{});
    if constexpr (DA > 1) step(std::integral_constant<int, 1>{});
    if constexpr (DA > 2) step(std::integral_constant<int, 2>{});
    if constexpr (DA > 3) step(std::integral_constant<int, 3>{});
  }

#if QNN_STAMP
  RB_TS(ts2);
#endif
  // ---- sum_valid(q'_x): channel sums of every band pixel, then each output pixel's taps
  int* s_ps = reinterpret_cast<int*>(smem + g.psum_off);
  for (int b = tid; b < g.nbp; b += NT) {
    int sm[4] = {0, 0, 0, 0};  // independent chains (exact integer sums in any order)
#pragma unroll 2
    for (int v = 0; v < g.npl; ++v) {
      const v4i a = *reinterpret_cast<const v4i*>(smem + v * g.pl + 32 * b);
      const v4i c = *reinterpret_cast<const v4i*>(smem + v * g.pl + 32 * b + 16);
      sm[0] = __builtin_amdgcn_sdot4(a.x, 0x01010101, sm[0], false);
      sm[1] = __builtin_amdgcn_sdot4(a.y, 0x01010101, sm[1], false);
      sm[2] = __builtin_amdgcn_sdot4(a.z, 0x01010101, sm[2], false);
      sm[3] = __builtin_amdgcn_sdot4(a.w, 0x01010101, sm[3], false);
      sm[0] = __builtin_amdgcn_sdot4(c.x, 0x01010101, sm[0], false);
      sm[1] = __builtin_amdgcn_sdot4(c.y, 0x01010101, sm[1], false);
      sm[2] = __builtin_amdgcn_sdot4(c.z, 0x01010101, sm[2], false);
      sm[3] = __builtin_amdgcn_sdot4(c.w, 0x01010101, sm[3], false);
    }
    s_ps[b] = (sm[0] + sm[1]) + (sm[2] + sm[3]);
  }
  __syncthreads();
  int sumq[TN], b0[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    sumq[j] = 0;
    b0[j] = (pb[j] - (lane >> 5) * g.pl) >> 5;  // band pixel of tap (0, 0)
  }
  {
    int tr = 0, tc = 0;
    for (int tt = 0; tt < p.taps; ++tt) {  // per tap: TN independent reads
      const int dt = tr * g.wb + (g.s2 ? (tc & 1) * g.we + (tc >> 1) : tc);
#pragma unroll
      for (int j = 0; j < TN; ++j) sumq[j] += s_ps[b0[j] + dt];
      if (++tc == d.kw) tc = 0, ++tr;
    }
  }
  wait_vmcnt<0>();  // the clamped tail weight loads
  __syncthreads();  // the band and sums are dead: the epilogue may stage over them
#if QNN_STAMP
  RB_TS(ts3);
#endif
  if (QNN_ABLATE == 3) {
    int z = sumq[0];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) z ^= acc[i][j][r];
    if (z == 0x7fffffff) p.e.out_f32[0] = 1.f;
    return;
  }
  if (!p.epi_early) {
    stage();
    wait_vmcnt<0>();
    __syncthreads();
  }
#if QNN_STAMP
  RB_TS(ts5);
#endif
  {
    const int HoWo = d.ho * d.wo;
    // this lane's pixel of tile j, stepped from tile j-1 (the epilogue visits j in order):
    // one division for tile 0, then +16 with carries; pixels past the block take its last
    int cq = (wn * TN) * 16 + (lane & 15);
    int cm = r0 * d.wo + (cq < npx_blk ? cq : npx_blk - 1);
    int cn = cm / HoWo, cho = (cm - cn * HoWo) / d.wo, cwo = cm - cn * HoWo - cho * d.wo;
    const int lm = r0 * d.wo + npx_blk - 1;
    const int ln = lm / HoWo, lho = (lm - ln * HoWo) / d.wo, lwo = lm - ln * HoWo - lho * d.wo;
    auto pixel = [&](int j, q16::Pix& P, int& pc) {
      if (j > 0) {
        cq += 16;
        cwo += 16;
        while (cwo >= d.wo) {
          cwo -= d.wo;
          if (++cho == d.ho) cho = 0, ++cn;
        }
      }
      P.ok = cq < npx_blk;
      P.m = P.ok ? r0 * d.wo + cq : lm;
      P.n = P.ok ? cn : ln;
      P.ho = P.ok ? cho : lho;
      P.wo = P.ok ? cwo : lwo;
      pc = s_hc[P.ho] + s_hc[d.ho + P.wo];
    };
    const qnn_epilogue& e = p.e;
    if (EK == EK_LUT && g.lut && c0 + BM <= d.cout && c0 + BM <= e.code0_cp) {
      // fast path of the common case (a full channel tile, the code table staged): the
      // epilogue_rb EK_LUT arithmetic with no per-group branch
      const float* s_f = reinterpret_cast<const float*>(smem + p.epi_off);
      const int8_t* s_lut = smem + p.epi_off + 4 * (7 + e.nclass) * BM;
      const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
      const int gq = lane >> 4;
      float4 sw[TM], bw[TM], bi[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int cl = wm * 16 * TM + 16 * i + 4 * gq;
        sw[i] = *reinterpret_cast<const float4*>(s_f + cl);
        bw[i] = *reinterpret_cast<const float4*>(s_f + BM + cl);
        bi[i] = *reinterpret_cast<const float4*>(s_f + 2 * BM + cl);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        q16::Pix P;
        int pc;
        pixel(j, P, pc);
        int8_t* op = e.out_code0 + (((int64_t)P.n * e.code0_hp + P.ho + e.code0_pad) * e.code0_wp + P.wo + e.code0_pad) *
                                       e.code0_cp + c0 + wm * 16 * TM + 4 * gq;
        const float* tp = s_f + (7 + pc) * BM + wm * 16 * TM + 4 * gq;
        const f2 p2 = {(float)sumq[j], (float)sumq[j]};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float4 tb = *reinterpret_cast<const float4*>(tp + 16 * i);
          const v4i& a = acc[i][j];
          const f2 a01 = {(float)a[0], (float)a[1]}, a23 = {(float)a[2], (float)a[3]};
          const f2 v0 = pfma((f2){sw[i].x, sw[i].y}, a01, pfma((f2){bw[i].x, bw[i].y}, p2, (f2){tb.x, tb.y})) +
                        (f2){bi[i].x, bi[i].y};
          const f2 v1 = pfma((f2){sw[i].z, sw[i].w}, a23, pfma((f2){bw[i].z, bw[i].w}, p2, (f2){tb.z, tb.w})) +
                        (f2){bi[i].z, bi[i].w};
          const f2 q0 = qclamp2(v0, bnp) + MAGIC_U8, q1 = qclamp2(v1, bnp) + MAGIC_U8;
          const int8_t* lp = s_lut + (wm * 16 * TM + 16 * i + 4 * gq) * 256;
          const int b0 = (uint8_t)lp[__float_as_uint(q0.x) & 255u];
          const int b1 = (uint8_t)lp[256 + (__float_as_uint(q0.y) & 255u)];
          const int b2 = (uint8_t)lp[512 + (__float_as_uint(q1.x) & 255u)];
          const int b3 = (uint8_t)lp[768 + (__float_as_uint(q1.y) & 255u)];
          *reinterpret_cast<int*>(op + 16 * i) = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
        }
      }
    } else {
      q16::epilogue_rb<C, EK>(p, acc, sumq, pixel, smem, c0, wm, lane, g.lut);
    }
  }
#if QNN_STAMP
  RB_TS(ts6);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  RB_TS(ts4);
  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && blockIdx.x < (1 << 18) / (8 * W)) {
    unsigned long long* o = qnn_rb_stamps + ((size_t)blockIdx.x * W + wave) * 8;
    o[0] = rt0; o[1] = rt1; o[2] = ts1 - ts0; o[3] = ts2 - ts1; o[4] = ts3 - ts2; o[5] = ts5 - ts3;
    o[6] = ts6 - ts5; o[7] = ts4 - ts6;
  }
#endif
}

// ---------------------------------------------------------------- host side
template <class C, int EK>
static int plan_lds(const Params& p, Params& q, Geo& g) {
  const int main = geometry(p, C::BM, C::BN, C::W, C::BPC, 0, g);
  if (main < 0) return arg_error("tile configuration not built for this layer / epilogue kind"), -1;
  q = p;
  int epi = epi_bytes(p, C::BM);
  // EK_LUT: the 256-byte-per-channel code table beside the band when it fits (else evaluated)
  g.lut = 0;
  if (EK == EK_LUT && main + epi + 256 * C::BM <= LDS_MAX / C::BPC) g.lut = 1, epi += 256 * C::BM;
  int lds;
  if (main + epi <= LDS_MAX / C::BPC) {
    q.epi_early = 1, q.epi_off = main;
    lds = main + epi;
  } else {  // staged after the loop over the band (the border classes past it stay)
    if (epi > g.psum_off) return arg_error("conv tile needs more than 160 KiB of LDS (too many border classes)"), -1;
    q.epi_early = 0, q.epi_off = 0;
    lds = main;
  }
  q.scr_off = 0;
  if (lds > LDS_MAX) return arg_error("conv tile needs more than 160 KiB of LDS (too many border classes)"), -1;
  return lds;
}

template <class C, int EK, int H>
static int launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  auto kern = qconv_rb_kernel<C, EK, H>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  Geo g;
  Params q;
  const int lds = plan_lds<C, EK>(p, q, g);
  if (lds < 0) return QNN_ERR_ARG;  // (plan_lds set the message)
  // natural occupancy: as many blocks per CU as registers and LDS allow
  const int nblk = g.nbands * (int)cdiv(p.d.cout, C::BM);
  if (occ) {
    int n = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, C::NT, lds);
    if (e != hipSuccess) return hip_check(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    occ->blocks_per_cu = n, occ->lds = lds, occ->grid = nblk;
    return QNN_OK;
  }
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(C::NT), lds, s, x, w, q, g);
  return QNN_OK;
}

template <class C, int EK>
static int launch_h(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  if (p.d.cp == 64) {  // 28 accumulator tiles spill beside the 64-channel (H = 1) loop: not built
    if constexpr (C::TM * C::TN > 26) return arg_error("tile configuration not built for this layer / epilogue kind");
    else return launch<C, EK, 1>(x, w, p, s, occ);
  }
  return launch<C, EK, 2>(x, w, p, s, occ);
}

template <class C>
static int launch_ek(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  switch (epi_kind(p.e)) {
    case EK_NCHW: return launch_h<C, EK_NCHW>(x, w, p, s, occ);
    case EK_LUT: return launch_h<C, EK_LUT>(x, w, p, s, occ);
    case EK_BNCODE: return launch_h<C, EK_BNCODE>(x, w, p, s, occ);
    default:  // 26 accumulator tiles + the general chain spill registers: not built
      if constexpr (C::TM * C::TN > 16) return arg_error("tile configuration not built for this layer / epilogue kind");
      else return launch_h<C, EK_GEN>(x, w, p, s, occ);
  }
}

//   id  block (cout x px cols)  waves (each)      blocks/CU  fits
//   0   256 x 208               8 (32 x 208)      1          14x14 images (ResNet-50 layer 3, b256)
//   1   128 x 224               8 (32 x 112)      1          128-channel tiles of 14x14 / 28x28 / 56x56 rows
//   2   256 x 224               8 (64 x 112)      1          14x14 images, each band fragment feeds 4 MFMAs
//   3   128 x 256               8 (64 x 64)       1          128-channel tiles, 4 MFMAs per fragment
//   4   128 x 128               8 (32 x 64)       2          two co-resident blocks (<= 128 VGPRs, <= 80 KiB LDS)
//   5   64 x 224                4 (32 x 112)      3          64-channel layers: 4 rows of 56, 7 rows of 28
//   6   64 x 128                4 (32 x 64)       4          64-channel layers: 2 rows of 56, many small blocks
//   7   64 x 448                8 (32 x 112)      1          64-channel layers: 8 rows of 56
//   8   256 x 112               8 (32 x 112)      1          half 14x14 images (7 rows): 2 blocks per image
using R0 = Cfg<8, 1, 2, 13, 3, 1>;
using R1 = Cfg<4, 2, 2, 7, 3, 1>;
using R3 = Cfg<4, 2, 4, 7, 3, 1>;
using R4 = Cfg<2, 4, 4, 4, 3, 1>;
using R5 = Cfg<4, 2, 2, 4, 3, 2>;
using R6 = Cfg<2, 2, 2, 7, 3, 3>;
using R7 = Cfg<2, 2, 2, 4, 3, 4>;
using R8 = Cfg<2, 4, 2, 7, 3, 1>;
using R9 = Cfg<8, 1, 2, 7, 3, 1>;
constexpr int NR = 9;
static const Info INFO[NR] = {
    {256, 208, 8, 1, 26, 1.40f},
    {128, 224, 8, 1, 14, 1.25f},
    {256, 224, 8, 1, 28, 1.45f},
    {128, 256, 8, 1, 16, 1.25f},
    {128, 128, 8, 2, 8, 0.60f},
    {64, 224, 4, 3, 14, 0.60f},
    {64, 128, 4, 4, 8, 0.50f},
    {64, 448, 8, 1, 14, 0.60f},
    {256, 112, 8, 1, 14, 1.00f},
};

}  // namespace rb

int rb_count() { return rb::NR + direct_count(); }

#if QNN_STAMP
extern "C" int qnn_debug_stamps_rb(void* dst, size_t bytes) {
  if (bytes > sizeof(::qnn_rb_stamps)) bytes = sizeof(::qnn_rb_stamps);
  return hip_check(hipMemcpyFromSymbol(dst, HIP_SYMBOL(::qnn_rb_stamps), bytes), "stamps");
}
#endif

void rb_tile(int k, int* bm, int* bn) {
  if (k >= rb::NR) return direct_tile(k - rb::NR, bm, bn);
  *bm = rb::INFO[k].bm;
  *bn = rb::INFO[k].bn;
}

bool rb_ok(int k, const Params& p) {
  using namespace rb;
  if (k >= NR) return direct_ok(k - NR, p);
  if (k < 0) return false;
  const Info& f = INFO[k];
  if (epi_kind(p.e) == EK_GEN && f.acc_tiles > 16) return false;  // the general chain spills beside the accumulators
  if (p.d.cp == 64 && f.acc_tiles > 26) return false;              // spills beside the H = 1 loop
  Geo g;
  return geometry(p, f.bm, f.bn, f.w, f.bpc, 0, g) >= 0;
}

int64_t rb_blocks(int k, const Params& p) {
  if (k >= rb::NR) return direct_blocks(k - rb::NR, p);
  const rb::Info& f = rb::INFO[k];
  rb::Geo g;
  if (rb::geometry(p, f.bm, f.bn, f.w, f.bpc, 0, g) < 0) return 0;
  return (int64_t)g.nbands * cdiv(p.d.cout, f.bm);
}

double rb_cost(int k, const Params& p) {
  if (k >= rb::NR) return direct_cost(k - rb::NR, p);
  const rb::Info& f = rb::INFO[k];
  rb::Geo g;
  if (rb::geometry(p, f.bm, f.bn, f.w, f.bpc, 0, g) < 0) return 1e30;
  const int64_t tiles = (int64_t)g.nbands * cdiv(p.d.cout, f.bm);
  const int64_t slots = (int64_t)NUM_CU * f.bpc;
  const int64_t rounds = cdiv(tiles, slots);
  const double share = tiles < slots ? (double)cdiv(tiles, NUM_CU) : (double)f.bpc;
  return (double)rounds * share * f.bm * f.bn * (p.taps * p.d.cp) / f.rate;  // dummy tiles cost MFMA time too
}

int rb_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  using namespace rb;
  if (k >= NR) return direct_launch(k - NR, x, w, p, s, occ);
  switch (k) {
    case 0: return launch_ek<R0>(x, w, p, s, occ);
    case 1: return launch_ek<R1>(x, w, p, s, occ);
    case 2: return launch_ek<R3>(x, w, p, s, occ);
    case 3: return launch_ek<R4>(x, w, p, s, occ);
    case 4: return launch_ek<R5>(x, w, p, s, occ);
    case 5: return launch_ek<R6>(x, w, p, s, occ);
    case 6: return launch_ek<R7>(x, w, p, s, occ);
    case 7: return launch_ek<R8>(x, w, p, s, occ);
    default: return launch_ek<R9>(x, w, p, s, occ);
  }
}

}  // namespace qnn
