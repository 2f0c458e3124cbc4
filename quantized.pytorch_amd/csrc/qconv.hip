// int8 MFMA implicit-GEMM convolution: the eval forward of QConv2d / QLinear
// (models/modules/quantize.py:314-349, :398-428; biprecision's out1+out2-out1
// is one contraction).  CDNA4 / gfx950: v_mfma_i32_32x32x32_i8.
//
// GEMM view  D[c][m] = sum_k Wq'[c][k] * Xq'[k][m]
//   c: output channel  -> MFMA rows    (operand A: packed weights [cout_pad][kpad])
//   m: output pixel    -> MFMA columns (operand B: implicit im2col of the NHWC8 codes)
//   k: (kh, kw, ci) tap-major, ci padded to Cp = 16 * 2^j
// The input is SPATIALLY PRE-PADDED ([n][hp][wp][cp], border code' = 0): zero
// padding of x_hat contributes nothing to any term of the exact decomposition
// (SURVEY.md §0.5), so the gather has no bounds checks at all and goes straight
// HBM -> LDS with global_load_lds_dwordx4.  Chunks past K read a zero page.
//
// Epilogue: y = s_x*s_w[c]*acc + s_x*b_w[c]*sum_valid(q'_x) + b_x*sum_valid(w_hat[c]) (+ bias)
//   sum_valid(q'_x): v_dot4 of the B fragments against 1s (exact, in-loop);
//   border term: per (row class, col class, c) table staged in LDS.
// Then either the drop-in output (fp32 NCHW, the reference module boundary), or
// the fused chain of the model graph: RangeBN eval (quantize.py:461-499, exact
// fp32 op order) -> + residual -> ReLU -> fp32 (C-tile or NHWC) and/or requantized
// NHWC8 codes for up to two consumer convs (their QuantMeasure ranges).
//
// Kernel v5 (tile configurations below): 4- or 8-wave blocks, each wave a
// (32*TM) x (32*TN) tile of 32x32x32 MFMAs.  The main loop is bound by how many
// bytes the CU can pull from L2 into LDS per MFMA (measured ~40 B/clk/CU with
// LDS-DMA), so blocks are as large as LDS allows: 256x256 moves 1 byte per 256
// int8 ops (v4's 128x128: 1 per 128).  K advances in 64-byte stages through a
// 4-slot LDS ring filled by global_load_lds_dwordx4 three stages ahead, with
// ONE s_barrier per stage (the slot a wave refills was consumed two barriers
// ago).  LDS rows are XOR-swizzled on the DMA source side so ds_read_b128
// fragment reads are conflict-free.  Epilogue: per-channel parameters, border
// table and code LUT staged in LDS; drop-in NCHW fp32 goes through a per-wave
// LDS transpose so every global store is 16 bytes of 4 consecutive pixels.
#include <stdlib.h>

#include <type_traits>

#include "qconv_common.h"

namespace qnn {

#ifndef QNN_ABLATE
#define QNN_ABLATE 0  // diagnostic builds only (make ablate): 1 no loads, 2 no MFMA, 3 no epilogue
#endif

#ifndef QNN_STAMP
#define QNN_STAMP 0  // diagnostic builds only (make stamp): per-wave s_memtime phase sums
#endif
#if QNN_STAMP
// [block][wave][10]: realtime start/end, cycles in prologue / issue / wait+barrier /
// compute / 0 / epilogue, HW_ID, stages
__device__ unsigned long long qnn_dbg_stamps[1 << 20];
__device__ unsigned long long qnn_dbg_epi[1 << 18];  // [block][wave][4]: staging, pixel state, body
#define QNN_TSV(v)                                                                        \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#define QNN_TS(v)                                                                         \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#else
#define QNN_TS(v) ((void)0)
#define QNN_TSV(v) ((void)0)
#endif


// Tile configuration: WGM x WGN waves, each (32*TM) x (32*TN) (cout x pixels), K stage
// BK bytes, NS-slot LDS ring.  KSP > 1 (the ring kernel only): KSP such wave grids in one block,
// K group g taking stages g, g + KSP, ... through a ring of its own; the groups' accumulators
// are summed through LDS before one group's epilogue (more waves on a tile without a global
// split-K hand-off: the deep-K layers whose tiles leave CUs half empty).
template <int WGM_, int WGN_, int TM_, int TN_, int BK_, int NS_, int BPC_ = (WGM_ * WGN_ == 4 ? 2 : 1), int KSP_ = 1>
struct Cfg {
  static constexpr int WGM = WGM_, WGN = WGN_, TM = TM_, TN = TN_, BK = BK_, NS = NS_, KSP = KSP_;
  static constexpr int WG = WGM * WGN;  // waves of one K group (the tile's wave grid)
  static constexpr int W = WG * KSP, NT = 64 * W;
  static constexpr int BM = WGM * TM * 32, BN = WGN * TN * 32;
  static constexpr int CPR = BK / 16;    // 16-B chunks per LDS row
  static constexpr int RPI = 1024 / BK;  // rows per 1 KiB LDS-DMA wave-instruction
  static constexpr int NA = BM / RPI / WG, NB = BN / RPI / WG;  // DMA per wave per stage
  static constexpr int STAGE = (BM + BN) * BK;
  static constexpr int KS = BK / 32;  // MFMA k-steps per stage
  static constexpr int P = NA + NB;
  static constexpr int BPC = BPC_;  // resident blocks per CU the LDS budget must allow
  static_assert((BM / RPI) % WG == 0 && (BN / RPI) % WG == 0, "DMA rows must split evenly over the waves");
  static_assert(KSP == 1 || KSP == 2, "K groups");
  static_assert(BK == 64 || BK == 128, "BK");
  static_assert(NS >= 3 && NS <= 4, "ring depth");
};

// Byte offset of 16-byte chunk `chunk` of LDS row `row` (rows of BK bytes): XOR swizzle so
// that the 16-lane groups of a ds_read_b128 fragment read (16 rows, one chunk) hit 16
// distinct 16-B bank slots: BK=128 (2 rows per 256-B bank row) xor (row>>1)&7,
// BK=64 (4 rows per bank row) xor (row>>2)&3.
template <int BK>
__device__ __forceinline__ int swz(int row, int chunk) {
  if constexpr (BK == 128) return row * BK + ((chunk ^ ((row >> 1) & 7)) << 4);
  else return row * BK + ((chunk ^ ((row >> 2) & 3)) << 4);
}


// Byte offset of tap t (row-major over kh x kw) from a pixel's tap (0, 0); uniform.
__device__ __forceinline__ int tap_offset(const Params& p, int t) {
  const int r = (t * p.kw_magic) >> 16;
  return (r * p.d.wp + (t - r * p.d.kw)) * p.d.cp;
}

__device__ __forceinline__ int code_byte(float v, float nm, float s, float inv, float qmax) {
  return ((int)quant_code_fast(v, nm, s, inv, qmax) - 128) & 255;
}

// Lane holds dwords g = 0..3 = channels [8g + 4h, 8g + 4h + 4) of a 32-channel group
// (h = lane / 32).  Two half-exchange levels leave lanes 0-31 with channels 0-15 and
// lanes 32-63 with channels 16-31 in order; returns them as one 16-byte vector.
__device__ __forceinline__ v4i gather16(int d0, int d1, int d2, int d3) {
  auto r01 = __builtin_amdgcn_permlane32_swap(d0, d1, false, false);
  auto r23 = __builtin_amdgcn_permlane32_swap(d2, d3, false, false);
  auto r02 = __builtin_amdgcn_permlane32_swap(r01[0], r23[0], false, false);
  auto r13 = __builtin_amdgcn_permlane32_swap(r01[1], r23[1], false, false);
  return (v4i){(int)r02[0], (int)r13[0], (int)r02[1], (int)r13[1]};
}



// y for channels cl..cl+3 (register group g of an accumulator): the exact decomposition
// s_x*s_w*acc + s_x*b_w*sum_valid(q'_x) + border term, + bias; parameters read as float4.
// Packed pairs: v[0] = channels cl, cl+1; v[1] = cl+2, cl+3 (fma(sw, acc, fma(bw, psq, tb)) + bias).
__device__ __forceinline__ void conv_out4p(const float* s_f, int BM, int cl, int ptab, float psq, const v16i& a, int g,
                                           f2 (&v)[2]) {
  const float4 sw = *reinterpret_cast<const float4*>(s_f + cl);
  const float4 bw = *reinterpret_cast<const float4*>(s_f + BM + cl);
  const float4 tb = *reinterpret_cast<const float4*>(s_f + ptab + cl);
  const float4 bi = *reinterpret_cast<const float4*>(s_f + 2 * BM + cl);
  const f2 p2 = {psq, psq};
  const f2 a01 = {(float)a[4 * g + 0], (float)a[4 * g + 1]}, a23 = {(float)a[4 * g + 2], (float)a[4 * g + 3]};
  v[0] = pfma((f2){sw.x, sw.y}, a01, pfma((f2){bw.x, bw.y}, p2, (f2){tb.x, tb.y})) + (f2){bi.x, bi.y};
  v[1] = pfma((f2){sw.z, sw.w}, a23, pfma((f2){bw.z, bw.w}, p2, (f2){tb.z, tb.w})) + (f2){bi.z, bi.w};
}

__device__ __forceinline__ void conv_out4(const float* s_f, int BM, int cl, int ptab, float psq, const v16i& a, int g,
                                          float (&v)[4]) {
  f2 p[2];
  conv_out4p(s_f, BM, cl, ptab, psq, a, g, p);
  v[0] = p[0].x, v[1] = p[0].y, v[2] = p[1].x, v[3] = p[1].y;
}


// Border-table class of each of this lane's TN pixels (computed before the main loop so
// the hcls / wcls loads complete under it).
template <class C>
__device__ __forceinline__ void pixel_classes(const Params& p, int m0, int wn, int lane, int (&pcls)[C::TN]) {
  const int HoWo = p.d.ho * p.d.wo;
#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    int m = m0 + wn * 32 * C::TN + j * 32 + (lane & 31);
    m = m < p.M ? m : p.M - 1;
    const int n = m / HoWo, hw = m - n * HoWo, ho = hw / p.d.wo, wo = hw - ho * p.d.wo;
    pcls[j] = p.e.hcls[ho] * p.e.nwc + p.e.wcls[wo];
  }
}

// sumq[j]: full receptive-field sum of q'_x for this lane's pixel of column tile j.
// The epilogue data is staged (stage_epi) and visible (barrier) on entry.
template <class C, int EK>
__device__ __forceinline__ void epilogue(const Params& p, v16i (&acc)[C::TM][C::TN], const int (&sumq)[C::TN],
                                         const int (&pcls)[C::TN], int8_t* smem, int m0, int c0, int wm, int wn,
                                         int lane, int tid, int wave) {
  constexpr int BM = C::BM, TM = C::TM, TN = C::TN;
  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  const int frow = lane & 31, fh = lane >> 5;
  const int HoWo = d.ho * d.wo;
#if QNN_STAMP
  unsigned long long e0 = 0, e1 = 0, e2 = 0, e3 = 0;
#endif
  QNN_TSV(e0);
  const float* s_f = reinterpret_cast<const float*>(smem + p.epi_off);
  const int nparam = 7 * BM;
  const int8_t* s_tail = smem + p.epi_off + 4 * (7 + e.nclass) * BM;  // LUT [BM][256] (EK_LUT)
  QNN_TSV(e1);

  // per-pixel (lane) state for the TN 32-pixel column tiles of this wave
  int pm[TN], pn[TN], pho[TN], pwo[TN], ptab[TN];
  float psq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int m = m0 + wn * 32 * TN + j * 32 + frow;
    pm[j] = m;
    const int mm = m < p.M ? m : p.M - 1;
    pn[j] = mm / HoWo;
    const int hw = mm - pn[j] * HoWo;
    pho[j] = hw / d.wo;
    pwo[j] = hw - pho[j] * d.wo;
    ptab[j] = nparam + pcls[j] * BM;
    psq[j] = (float)sumq[j];
  }
  QNN_TSV(e2);

  if constexpr (EK == EK_NCHW) {
    // drop-in output: NCHW fp32.  Each 32x32 sub-tile goes through this wave's LDS
    // scratch ([32 channels][32 pixels], conflict-free both ways) so that a lane then
    // holds 4 consecutive pixels of one channel: one 16-byte store (needs HoWo % 4 == 0,
    // so 4 consecutive pixels never straddle images; else one scalar store per value).
    float* scr = reinterpret_cast<float*>(smem + p.scr_off) + wave * 1024;
    const bool vec = (HoWo & 3) == 0;
    const int q4 = lane & 7, rsub = lane >> 3;  // read phase: pixel quad, row within 8
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int mq = m0 + wn * 32 * TN + j * 32 + 4 * q4;  // first pixel of this lane's quad
      const int mqc = mq < p.M ? mq : p.M - 1;
      const int nq = mqc / HoWo, hwq = mqc - nq * HoWo;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int clb = wm * 32 * TM + i * 32;  // local channel base of this sub-tile
        float y[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int cl = clb + 8 * g + 4 * fh;
          float yg[4];
          conv_out4(s_f, BM, cl, ptab[j], psq[j], acc[i][j], g, yg);
#pragma unroll
          for (int u = 0; u < 4; ++u) y[4 * g + u] = yg[u];
        }
        if (vec) {
#pragma unroll
          for (int r = 0; r < 16; ++r) scr[(8 * (r >> 2) + 4 * fh + (r & 3)) * 32 + frow] = y[r];
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int row = 8 * k + rsub;
            const float4 v = *reinterpret_cast<const float4*>(scr + row * 32 + 4 * q4);
            const int c = c0 + clb + row;
            if (mq < p.M && c < d.cout)
              *reinterpret_cast<float4*>(e.out_f32 + ((int64_t)nq * d.cout + c) * HoWo + hwq) = v;
          }
          __builtin_amdgcn_wave_barrier();
        } else if (pm[j] < p.M) {
          float* yp = e.out_f32 + (int64_t)pn[j] * d.cout * HoWo + (pm[j] - pn[j] * HoWo);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int c = c0 + clb + 8 * (r >> 2) + 4 * fh + (r & 3);
            if (c < d.cout) yp[(int64_t)c * HoWo] = y[r];
          }
        }
      }
    }
  } else {
    const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
    const QParams c0p = make_qparams(e.code0_neg_min, e.code0_scale, e.code0_qmax);
    const QParams c1p = make_qparams(e.code1_neg_min, e.code1_scale, e.code1_qmax);
    // two consumers calibrated on the same tensor hold the same range: their codes are equal
    const bool same01 = e.out_code0 && e.code1_neg_min == e.code0_neg_min && e.code1_scale == e.code0_scale &&
                        e.code1_qmax == e.code0_qmax;
    const f2 bn_s2 = {e.bn_scale, e.bn_scale}, bn_m2 = {e.bn_min, e.bn_min};
    const CodeDst t0 = {e.out_code0, e.code0_cp, e.code0_pad, e.code0_hp, e.code0_wp};
    const CodeDst t1 = {e.out_code1, e.code1_cp, e.code1_pad, e.code1_hp, e.code1_wp};
    const CodeDst tb = {reinterpret_cast<int8_t*>(e.out_bncode), d.cout, 0, d.ho, d.wo};
    const bool has_res = EK == EK_GEN && e.residual != nullptr;
    const int nres = EK == EK_GEN ? e.nres : 0;
    const bool want_bn = EK == EK_BNCODE || (EK == EK_GEN && e.out_bncode);
    // residual code chain (qnn_res_link): one 16-byte byte-C-tile load per link per sub-tile
    const float* s_chain = s_f + (7 + e.nclass) * BM;
    auto load_chain = [&](v4i (&rc)[QNN_MAX_RES], int i, int j) {
      int mt = (m0 + wn * 32 * TN + j * 32) >> 5;
      mt = mt < (p.M + 31) >> 5 ? mt : ((p.M + 31) >> 5) - 1;  // the map holds ceil(M/32) pixel tiles
      int ctb = (c0 + wm * 32 * TM + i * 32) >> 5;
      ctb = ctb < p.ct ? ctb : p.ct - 1;  // channel tiles past cout: any in-bounds bytes (unused)
      const int64_t off = btile_off(mt, ctb, p.ct, lane);
#pragma unroll
      for (int l = 0; l < QNN_MAX_RES; ++l)
        if (l < nres) rc[l] = *reinterpret_cast<const v4i*>(e.res[l].code + off);
    };
    // g_l(q) for the 4 channels cl..cl+3 of register group g (quantize.py:488-499 op order)
    auto link = [&](const v4i (&rc)[QNN_MAX_RES], int l, int g, int cl, f2 (&o)[2]) {
      const unsigned wd = (unsigned)rc[l][g];
      const float* sp = s_chain + 4 * l * BM + cl;
      const float4 mn4 = *reinterpret_cast<const float4*>(sp);
      const float4 sq4 = *reinterpret_cast<const float4*>(sp + BM);
      const float4 wq4 = *reinterpret_cast<const float4*>(sp + 2 * BM);
      const float4 bq4 = *reinterpret_cast<const float4*>(sp + 3 * BM);
      const f2 s2 = {e.res[l].scale, e.res[l].scale}, m2 = {e.res[l].min, e.res[l].min};
      const f2 q[2] = {{(float)(wd & 255u), (float)((wd >> 8) & 255u)},
                       {(float)((wd >> 16) & 255u), (float)(wd >> 24)}};
      const f2 mn[2] = {{mn4.x, mn4.y}, {mn4.z, mn4.w}}, sq[2] = {{sq4.x, sq4.y}, {sq4.z, sq4.w}};
      const f2 wq[2] = {{wq4.x, wq4.y}, {wq4.z, wq4.w}}, bq[2] = {{bq4.x, bq4.y}, {bq4.z, bq4.w}};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f2 t = q[h] * s2;
        t = t + m2;
        t = t - mn[h];
        t = t * sq[h];
        t = t * wq[h];
        o[h] = t + bq[h];
      }
    };
    // fetched one sub-tile ahead, except under the 128-VGPR budget of 4 blocks per CU
    constexpr bool CAHEAD = C::BPC < 4;
    v4i ccur[QNN_MAX_RES], cnxt[CAHEAD ? QNN_MAX_RES : 1][QNN_MAX_RES];
    if (CAHEAD && EK == EK_GEN && nres > 0) load_chain(ccur, 0, 0);
    // fp32 residual of sub-tile (i, j): 4 float4 per lane
    auto load_res = [&](float4 (&r)[4], int i, int j) {
      const int m = pm[j] < p.M ? pm[j] : p.M - 1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int c = c0 + wm * 32 * TM + i * 32 + 8 * g + 4 * fh;
        if (c > d.cout - 4) c = d.cout - 4;
        const int64_t fi = e.f32_tiled ? ctile_index(m, c, p.ct) : (int64_t)m * d.cout + c;
        r[g] = *reinterpret_cast<const float4*>(e.residual + fi);
      }
    };
    float4 rcur[4];  // fp32 residual (a chain checkpoint): loaded per sub-tile
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cb = c0 + wm * 32 * TM + i * 32;  // first channel of this lane's 32-channel group
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (EK == EK_GEN && has_res) load_res(rcur, i, j);
        if (EK == EK_GEN && nres > 0) {
          if constexpr (CAHEAD) {
            if (j + 1 < TN) load_chain(cnxt[0], i, j + 1);
            else if (i + 1 < TM) load_chain(cnxt[0], i + 1, 0);
          } else {
            load_chain(ccur, i, j);
          }
        }
        const bool pok = pm[j] < p.M;
        int k0[4], k1[4], kb[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int cl = cb - c0 + 8 * g + 4 * fh;  // local channel of reg 4g (+u)
          const int c = c0 + cl;
          const bool cok = c < d.cout;  // cout % 16 == 0: a 4-channel group is all in or all out
          f2 v[2];
          conv_out4p(s_f, BM, cl, ptab[j], psq[j], acc[i][j], g, v);
          k0[g] = k1[g] = 0;
          if constexpr (EK == EK_LUT) {  // conv -> RangeBN -> ReLU -> next quantizer, tabulated (exact)
            const f2 m0 = qclamp2(v[0], bnp) + MAGIC_U8, m1 = qclamp2(v[1], bnp) + MAGIC_U8;
            const unsigned qq[4] = {__float_as_uint(m0.x) & 255u, __float_as_uint(m0.y) & 255u,
                                    __float_as_uint(m1.x) & 255u, __float_as_uint(m1.y) & 255u};
            int r = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) r |= ((int)(uint8_t)s_tail[(cl + u) * 256 + qq[u]]) << (8 * u);
            k0[g] = cok ? r : 0;
            continue;
          }
          f2 qb[2];  // RangeBN input: clamped quotient (rounded below)
          if (EK == EK_BNCODE || e.bn_mean) {
            qb[0] = qclamp2(v[0], bnp);
            qb[1] = qclamp2(v[1], bnp);
          }
          kb[g] = 0;
          if (want_bn && cok) kb[g] = pack4(qb[0] + MAGIC_U8, qb[1] + MAGIC_U8);
          if constexpr (EK == EK_BNCODE) {
            continue;
          } else {
            if (e.bn_mean) {
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
            if (has_res || nres > 0) {
              // the block input: fp32, or recomputed from the chain exactly as its producers did
              f2 r[2];
              int l0 = 0;
              if (has_res) {
                const float4 r4 = rcur[g];
                r[0] = (f2){r4.x, r4.y};
                r[1] = (f2){r4.z, r4.w};
              } else {
                link(ccur, 0, g, cl, r);
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
                link(ccur, l, g, cl, o);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                  const f2 t = o[h] + r[h];
                  r[h].x = fmaxf(t.x, 0.f);
                  r[h].y = fmaxf(t.y, 0.f);
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
              const int64_t fi = e.f32_tiled ? ctile_index(pm[j], c, p.ct) : (int64_t)pm[j] * d.cout + c;
              *reinterpret_cast<float4*>(e.out_f32 + fi) = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
            }
            if (e.out_code0 && cok)
              k0[g] = pack4(qclamp2(v[0], c0p) + MAGIC_S8, qclamp2(v[1], c0p) + MAGIC_S8);
            if (e.out_code1 && cok)
              k1[g] = same01 ? k0[g] : pack4(qclamp2(v[0], c1p) + MAGIC_S8, qclamp2(v[1], c1p) + MAGIC_S8);
          }
        }
        const int ch = cb + 16 * fh;
        if (want_bn) {
          if (e.bncode_tiled) {  // chain link: lane-linear 16 bytes of the sub-tile
            if (cb < d.cout && m0 + wn * 32 * TN + j * 32 < p.M)  // sub-tiles inside the ceil(M/32)*32 map
              *reinterpret_cast<v4i*>(e.out_bncode + btile_off((m0 + wn * 32 * TN + j * 32) >> 5, cb >> 5, p.ct, lane)) =
                  (v4i){kb[0], kb[1], kb[2], kb[3]};
          } else {
            store_codes(tb, pn[j], pho[j], pwo[j], ch, pok, gather16(kb[0], kb[1], kb[2], kb[3]));
          }
        }
        if constexpr (EK == EK_BNCODE) {
        } else {
          if (EK == EK_LUT || e.out_code0)
            store_codes(t0, pn[j], pho[j], pwo[j], ch, pok, gather16(k0[0], k0[1], k0[2], k0[3]));
          if (EK == EK_GEN && e.out_code1)
            store_codes(t1, pn[j], pho[j], pwo[j], ch, pok, gather16(k1[0], k1[1], k1[2], k1[3]));
        }
        if (CAHEAD && EK == EK_GEN && nres > 0) {
#pragma unroll
          for (int l = 0; l < QNN_MAX_RES; ++l) ccur[l] = cnxt[0][l];
        }
      }
    }
  }
#if QNN_STAMP
  QNN_TSV(e3);
  if (lane == 0 && blockIdx.x < (1 << 18) / (4 * C::W)) {
    unsigned long long* o = qnn_dbg_epi + ((size_t)blockIdx.x * C::W + wave) * 4;
    o[0] = e1 - e0; o[1] = e2 - e1; o[2] = e3 - e2; o[3] = 0;
  }
#endif
}

template <class C, int EK, int TAPM, bool MASKED>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(C::BPC * C::W / 4))) void qconv_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ w,
                                                      const Params p) {
  constexpr int BM = C::BM, BN = C::BN, BK = C::BK, NS = C::NS, W = C::W, TM = C::TM, TN = C::TN;
  constexpr int CPR = C::CPR, RPI = C::RPI, NA = C::NA, NB = C::NB, STAGE = C::STAGE, KS = C::KS, P = C::P;
  constexpr int WG = C::WG, KSP = C::KSP;
  static_assert(!MASKED || TAPM == TAP_LDS, "masked (space-to-depth) stems use the LDS tap table");
  // one dynamic LDS object (a second __shared__ array can make hipcc drain vmcnt before ds_reads)
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  int* s_tap = reinterpret_cast<int*>(smem + KSP * NS * STAGE);
  int8_t* s_mask = smem + KSP * NS * STAGE + 4 * MAX_TAPS;

  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // K group kg (its own ring at kg * NS * STAGE) and the wave's place wg in the tile's wave grid
  const int kg = wave / WG, wg = wave - kg * WG;
  const int wm = wg / C::WGN, wn = wg % C::WGN;

  // ---- XCD-aware, bijective block -> tile map: each XCD gets a contiguous run of
  // tiles, output-channel tiles fastest so blocks sharing an activation tile share L2
  const int nby = (d.cout + BM - 1) / BM;
  const int nbx = (p.M + BN - 1) / BN;
  const int nblk = nbx * nby;
  int t;
  {
    const int b = blockIdx.x, xcd = b & 7, q = nblk >> 3, r = nblk & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int m0 = (t / nby) * BN;
  const int c0 = (t % nby) * BM;
  const int HoWo = d.ho * d.wo;

  if constexpr (TAPM == TAP_LDS) {
    if (tid < p.taps) s_tap[tid] = ((tid / d.kw) * d.wp + (tid % d.kw)) * d.cp;
  }
  if constexpr (MASKED) {
    for (int i = tid; i < d.kpad / 16; i += C::NT)
      *reinterpret_cast<v4i*>(s_mask + 16 * i) = *reinterpret_cast<const v4i*>(d.kmask + 16 * i);
  }

  // ---- per-lane gather state: B chunk (row, slot) -> pixel base + chunk-in-tap offset,
  // and which of the stage's taps the chunk belongs to.  DMA instruction i of the B
  // (A) image covers rows [i*RPI, (i+1)*RPI); wave w issues i = w, w + W, ...
  const int cpt_mask = (1 << p.lgcpt) - 1;
  uint32_t bbase[NB];
  int bdelta[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int row = RPI * (wg + WG * j) + lane / CPR;
    int m = m0 + row;
    if (m > p.M - 1) m = p.M - 1;
    const int n = m / HoWo, rem = m - n * HoWo, ho = rem / d.wo, wo = rem - ho * d.wo;
    const int bch = (swz<BK>(row, lane % CPR) - row * BK) >> 4;  // the chunk that lands in this lane's slot
    bbase[j] = (uint32_t)(((n * d.hp + ho * d.sh) * d.wp + wo * d.sw) * d.cp) + ((bch & cpt_mask) << 4);
    bdelta[j] = bch >> p.lgcpt;
  }
  const int8_t* wblk = w + (int64_t)c0 * d.kpad;
  uint32_t aoff[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int row = RPI * (wg + WG * j) + lane / CPR;
    const int crow = (c0 + row < d.cout_pad ? row : d.cout_pad - 1 - c0);  // never past the packed rows
    aoff[j] = (uint32_t)(crow * d.kpad + (swz<BK>(row, lane % CPR) - row * BK));
  }
  int pcls[TN];
  pixel_classes<C>(p, m0, wn, lane, pcls);
  if (p.epi_early) stage_epi<C, EK>(p, x, smem + p.epi_off, c0, wave, lane);  // oldest DMAs: land under the loop
  if constexpr (TAPM == TAP_LDS || MASKED) __syncthreads();  // s_tap / s_mask

  int8_t* const ring = smem + kg * NS * STAGE;  // this K group's ring
  // local stage ls of this K group = K stage kg + KSP ls
  auto issue = [&](int ls, int slot) {
    if (QNN_ABLATE == 1) return;
    const int st = kg + KSP * ls;
    int8_t* sa = ring + slot * STAGE;
    int8_t* sb = sa + BM * BK;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      uint32_t off = aoff[j] + (uint32_t)(st * BK);
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_global_load_lds((const void*)(wblk + off), (lds_ptr_t)(sa + (wg + WG * j) * 1024), 16, 0, 0);
    }
    const int t0 = (st * CPR) >> p.lgcpt;                           // first tap of this stage
    const uint32_t uin = (uint32_t)(((st * CPR) & cpt_mask) << 4);  // chunk-in-tap part (cp > 16*CPR)
    const uint32_t zoff = (uint32_t)d.zero_off;
    uint32_t T0 = 0, T1 = 0;
    bool v0 = false, v1 = false;
    if constexpr (TAPM != TAP_LDS) {
      v0 = t0 < p.taps;
      T0 = (uint32_t)tap_offset(p, t0) + uin;
      if constexpr (TAPM == TAP_TWO) {
        v1 = t0 + 1 < p.taps;
        T1 = (uint32_t)tap_offset(p, t0 + 1);
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      uint32_t off;
      if constexpr (TAPM == TAP_ONE) {
        off = v0 ? bbase[j] + T0 : zoff;
      } else if constexpr (TAPM == TAP_TWO) {
        off = bdelta[j] ? (v1 ? bbase[j] + T1 : zoff) : (v0 ? bbase[j] + T0 : zoff);
      } else {
        const int tap = t0 + bdelta[j];
        const uint32_t to = (uint32_t)s_tap[tap < MAX_TAPS ? tap : MAX_TAPS - 1];
        off = tap < p.taps ? bbase[j] + uin + to : zoff;
      }
      asm volatile("" : "+v"(off));  // keep ONE per-lane-address load (no saddr/vaddr branch split)
      __builtin_amdgcn_global_load_lds((const void*)(x + off), (lds_ptr_t)(sb + (wg + WG * j) * 1024), 16, 0, 0);
    }
  };

  v16i acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v16i){0};
  int sumq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] = 0;

  // per-lane fragment offsets of each k-step (the XOR swizzle depends only on frow)
  const int frow = lane & 31, fh = lane >> 5;
  int offa[KS], offb[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int xo = swz<BK>(frow, 2 * ks + fh) - frow * BK;
    offa[ks] = (wm * 32 * TM + frow) * BK + xo;
    offb[ks] = BM * BK + (wn * 32 * TN + frow) * BK + xo;
  }

  auto compute = [&](auto slotc, int ls) {
    constexpr int BO = decltype(slotc)::value * STAGE;
    const int st = kg + KSP * ls;
    v4i fa[2][TM], fb[2][TN];
    auto load = [&](int ks, int sl) {
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[sl][i] = *reinterpret_cast<const v4i*>(ring + BO + offa[ks] + i * 32 * BK);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[sl][j] = *reinterpret_cast<const v4i*>(ring + BO + offb[ks] + j * 32 * BK);
    };
    load(0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < KS) load(ks + 1, cur ^ 1);
      v4i ones = {0x01010101, 0x01010101, 0x01010101, 0x01010101};
      if constexpr (MASKED) ones = *reinterpret_cast<const v4i*>(s_mask + st * BK + 16 * (2 * ks + fh));
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int s = __builtin_amdgcn_sdot4(fb[cur][j].x, ones.x, sumq[j], false);
        s = __builtin_amdgcn_sdot4(fb[cur][j].y, ones.y, s, false);
        s = __builtin_amdgcn_sdot4(fb[cur][j].z, ones.z, s, false);
        sumq[j] = __builtin_amdgcn_sdot4(fb[cur][j].w, ones.w, s, false);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (QNN_ABLATE == 2) {
            asm volatile("" ::"v"(fa[cur][i]), "v"(fb[cur][j]));
            acc[i][j][0] += fa[cur][i].x;
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[cur][i], fb[cur][j], acc[i][j], 0, 0, 0);
          }
        }
    }
  };

  const int nstage = d.kpad / BK / KSP;  // this K group's stages (the host checks KSP divides them)
  const bool late = p.stagger && wave >= 4;
#if QNN_STAMP
  unsigned long long ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0, c_iss = 0, c_wait = 0, c_comp = 0;
  const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const unsigned long long t_begin = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
#endif
  // prologue: NS-1 stages in flight
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nstage) issue(s, s);

  // stage st lives in slot st % NS.  Before the barrier of step st every wave waits for
  // its own DMA of stage st (the younger stages st+1 .. st+NS-2 may stay in flight);
  // after it, all of stage st is in LDS and every wave has finished stage st-1, whose
  // slot (st+NS-1) % NS is refilled with stage st+NS-1.
  auto step = [&](auto slotc, int st) {
    constexpr int SL = decltype(slotc)::value;
    QNN_TS(ts0);
    const int ahead = nstage - 1 - st;  // stages issued after st (capped at NS-2)
    if (ahead >= NS - 2) wait_vmcnt<(NS - 2) * P>();
    else if (NS == 4 && ahead == 1) wait_vmcnt<P>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    QNN_TS(ts1);
    // stagger: the two waves sharing a SIMD (w, w + 4) split roles within the stage — the
    // low half issues its DMA first while the high half's MFMAs keep the matrix pipe busy,
    // then the high half issues while the low half computes
    const bool refill = st + NS - 1 < nstage;
    if (!late && refill) issue(st + NS - 1, (SL + NS - 1) % NS);
    QNN_TS(ts2);
    compute(slotc, st);
    if (late && refill) issue(st + NS - 1, (SL + NS - 1) % NS);
    QNN_TS(ts3);
#if QNN_STAMP
    c_wait += ts1 - ts0;
    c_iss += ts2 - ts1;
    c_comp += ts3 - ts2;
#endif
  };
#if QNN_STAMP
  QNN_TS(ts0);
  const unsigned long long c_pro = ts0 - t_begin;
#endif
  for (int st = 0; st < nstage; st += NS) {
    step(std::integral_constant<int, 0>{}, st);
    if (st + 1 < nstage) step(std::integral_constant<int, 1>{}, st + 1);
    if (st + 2 < nstage) step(std::integral_constant<int, 2>{}, st + 2);
    if constexpr (NS == 4)
      if (st + 3 < nstage) step(std::integral_constant<int, 3>{}, st + 3);
  }

#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] += __shfl_xor(sumq[j], 32, 64);
  __syncthreads();  // main-loop LDS is reused by the epilogue
  if constexpr (KSP > 1) {
    // K group 1's partial sums to group 0 through the free rings: per wave of the grid, its
    // (TM TN 16 + TN) ints lane-linear (conflict-free), then group 0 adds them
    constexpr int NR = TM * TN * 16 + TN;
    int* red = reinterpret_cast<int*>(smem) + wg * NR * 64 + lane;
    if (kg == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) red[((i * TN + j) * 16 + r) * 64] = acc[i][j][r];
#pragma unroll
      for (int j = 0; j < TN; ++j) red[(TM * TN * 16 + j) * 64] = sumq[j];
    }
    __syncthreads();
    if (kg == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] += red[((i * TN + j) * 16 + r) * 64];
#pragma unroll
      for (int j = 0; j < TN; ++j) sumq[j] += red[(TM * TN * 16 + j) * 64];
    }
    __syncthreads();  // the epilogue's LDS (staging, scratch) may overlap the hand-off area
  }
  if (QNN_ABLATE == 3) {
    int z = sumq[0];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) z ^= acc[i][j][r];
    if (z == 0x7fffffff) p.e.out_f32[0] = 1.f;  // keeps every MFMA live, (almost) never stores
    return;
  }
#if QNN_STAMP
  QNN_TS(ts0);
#endif
  if (!p.epi_early) {  // no room beside the ring: stage into it now
    stage_epi<C, EK>(p, x, smem + p.epi_off, c0, wave, lane);
    wait_vmcnt<0>();
    __syncthreads();
  }
  if (KSP > 1 && kg != 0) return;  // group 0 runs the epilogue (no barrier follows)
  epilogue<C, EK>(p, acc, sumq, pcls, smem, m0, c0, wm, wn, lane, tid, wave);
#if QNN_STAMP
  QNN_TS(ts1);
  const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  unsigned hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  if (lane == 0 && blockIdx.x < (1 << 20) / (10 * W)) {
    unsigned long long* o = qnn_dbg_stamps + ((size_t)blockIdx.x * W + wave) * 10;
    o[0] = rt_start; o[1] = rt_end; o[2] = c_pro; o[3] = c_iss; o[4] = c_wait; o[5] = c_comp; o[6] = 0;
    o[7] = ts1 - ts0; o[8] = hwid; o[9] = nstage;
  }
#endif
}

// ---------------------------------------------------------------- ping-pong main loop
// 8-wave blocks (waves w and w + 4 share a SIMD).  The K loop runs in PHASES of KPP
// k-steps; each phase is [load segment: ds_read this phase's fragments, issue part of
// the LDS-DMA of K-tile t+2] s_barrier [MFMA segment: the phase's MFMAs] s_barrier.
// Waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave is in its MFMA
// segment while its partner loads: the matrix pipe never waits for ds_read / DMA issue.
// LDS ring of 4 K-tiles; K-tile t+2 is written into the slot of t-2, whose last ds_read
// retired (lgkmcnt) two phases earlier.  Before the last phase's barrier of K-tile t each
// wave waits (vmcnt) for its own DMA of K-tile t+1, which is first read a phase later.
template <class C, int KPP, int EK, int TAPM, bool MASKED>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(2))) void qconv_pp_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ w, const Params p) {
  constexpr int BM = C::BM, BN = C::BN, BK = C::BK, NS = C::NS, W = C::W, TM = C::TM, TN = C::TN;
  constexpr int CPR = C::CPR, RPI = C::RPI, NA = C::NA, NB = C::NB, STAGE = C::STAGE, KS = C::KS, P = C::P;
  constexpr int PPT = KS / KPP;  // phases per K-tile
  static_assert(W == 8 && NS == 4 && KS % KPP == 0, "ping-pong: 8 waves, 4-slot ring");
  static_assert(!MASKED || TAPM == TAP_LDS, "masked (space-to-depth) stems use the LDS tap table");
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  int* s_tap = reinterpret_cast<int*>(smem + NS * STAGE);
  int8_t* s_mask = smem + NS * STAGE + 4 * MAX_TAPS;

  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  const bool late = wave >= 4;

  const int nby = (d.cout + BM - 1) / BM;
  const int nbx = (p.M + BN - 1) / BN;
  const int nblk = nbx * nby;
  int t;
  {
    const int b = blockIdx.x, xcd = b & 7, q = nblk >> 3, r = nblk & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int m0 = (t / nby) * BN;
  const int c0 = (t % nby) * BM;
  const int HoWo = d.ho * d.wo;

  if constexpr (TAPM == TAP_LDS) {
    if (tid < p.taps) s_tap[tid] = ((tid / d.kw) * d.wp + (tid % d.kw)) * d.cp;
  }
  if constexpr (MASKED) {
    for (int i = tid; i < d.kpad / 16; i += C::NT)
      *reinterpret_cast<v4i*>(s_mask + 16 * i) = *reinterpret_cast<const v4i*>(d.kmask + 16 * i);
  }
  const int cpt_mask = (1 << p.lgcpt) - 1;
  uint32_t bbase[NB];
  int bdelta[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int row = RPI * (wave + W * j) + lane / CPR;
    int m = m0 + row;
    if (m > p.M - 1) m = p.M - 1;
    const int n = m / HoWo, rem = m - n * HoWo, ho = rem / d.wo, wo = rem - ho * d.wo;
    const int bch = (swz<BK>(row, lane % CPR) - row * BK) >> 4;
    bbase[j] = (uint32_t)(((n * d.hp + ho * d.sh) * d.wp + wo * d.sw) * d.cp) + ((bch & cpt_mask) << 4);
    bdelta[j] = bch >> p.lgcpt;
  }
  const int8_t* wblk = w + (int64_t)c0 * d.kpad;
  uint32_t aoff[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int row = RPI * (wave + W * j) + lane / CPR;
    const int crow = (c0 + row < d.cout_pad ? row : d.cout_pad - 1 - c0);
    aoff[j] = (uint32_t)(crow * d.kpad + (swz<BK>(row, lane % CPR) - row * BK));
  }
  int pcls[TN];
  pixel_classes<C>(p, m0, wn, lane, pcls);
  if (p.epi_early) stage_epi<C, EK>(p, x, smem + p.epi_off, c0, wave, lane);  // oldest DMAs: land under the loop
  if constexpr (TAPM == TAP_LDS || MASKED) __syncthreads();

  const int nstage = d.kpad / BK;
  // DMA of K-tile st (clamped to the last tile: the ring slots past the end are free, so
  // re-reading valid bytes into them keeps every wave's DMA count uniform) into `slot`;
  // part q of PPT: the A rows and B rows are split over the phases of a K-tile.
  auto issue = [&](int st, int slot, int q) {
    if (QNN_ABLATE == 1) return;
    if (st > nstage - 1) st = nstage - 1;
    int8_t* sa = smem + slot * STAGE;
    int8_t* sb = sa + BM * BK;
    if (PPT == 1 || q == 0) {
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        uint32_t off = aoff[j] + (uint32_t)(st * BK);
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_global_load_lds((const void*)(wblk + off), (lds_ptr_t)(sa + (wave + W * j) * 1024), 16, 0, 0);
      }
    }
    if (PPT == 1 || q == PPT - 1) {
      const int t0 = (st * CPR) >> p.lgcpt;
      const uint32_t uin = (uint32_t)(((st * CPR) & cpt_mask) << 4);
      const uint32_t zoff = (uint32_t)d.zero_off;
      uint32_t T0 = 0, T1 = 0;
      bool v0 = false, v1 = false;
      if constexpr (TAPM != TAP_LDS) {
        v0 = t0 < p.taps;
        T0 = (uint32_t)tap_offset(p, t0) + uin;
        if constexpr (TAPM == TAP_TWO) {
          v1 = t0 + 1 < p.taps;
          T1 = (uint32_t)tap_offset(p, t0 + 1);
        }
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        uint32_t off;
        if constexpr (TAPM == TAP_ONE) {
          off = v0 ? bbase[j] + T0 : zoff;
        } else if constexpr (TAPM == TAP_TWO) {
          off = bdelta[j] ? (v1 ? bbase[j] + T1 : zoff) : (v0 ? bbase[j] + T0 : zoff);
        } else {
          const int tap = t0 + bdelta[j];
          const uint32_t to = (uint32_t)s_tap[tap < MAX_TAPS ? tap : MAX_TAPS - 1];
          off = tap < p.taps ? bbase[j] + uin + to : zoff;
        }
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_global_load_lds((const void*)(x + off), (lds_ptr_t)(sb + (wave + W * j) * 1024), 16, 0, 0);
      }
    }
  };

  v16i acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v16i){0};
  int sumq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] = 0;

  const int frow = lane & 31, fh = lane >> 5;
  int offa[KS], offb[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int xo = swz<BK>(frow, 2 * ks + fh) - frow * BK;
    offa[ks] = (wm * 32 * TM + frow) * BK + xo;
    offb[ks] = BM * BK + (wn * 32 * TN + frow) * BK + xo;
  }

  v4i fa[KPP][TM], fb[KPP][TN];
  auto read_frags = [&](auto slotc, int q) {
    constexpr int BO = decltype(slotc)::value * STAGE;
#pragma unroll
    for (int kk = 0; kk < KPP; ++kk) {
      const int ks = q * KPP + kk;
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[kk][j] = *reinterpret_cast<const v4i*>(smem + BO + offb[ks] + j * 32 * BK);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[kk][i] = *reinterpret_cast<const v4i*>(smem + BO + offa[ks] + i * 32 * BK);
    }
  };
  auto mfma_seg = [&](int st, int q) {
#pragma unroll
    for (int kk = 0; kk < KPP; ++kk) {
      v4i ones = {0x01010101, 0x01010101, 0x01010101, 0x01010101};
      if constexpr (MASKED) ones = *reinterpret_cast<const v4i*>(s_mask + st * BK + 16 * (2 * (q * KPP + kk) + fh));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (QNN_ABLATE == 2) {
            asm volatile("" ::"v"(fa[kk][i]), "v"(fb[kk][j]));
            acc[i][j][0] += fa[kk][i].x;
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[kk][i], fb[kk][j], acc[i][j], 0, 0, 0);
          }
          if (i == 0) {  // sum_valid(q'_x) of this column tile: one v_dot4 per MFMA gap
            int s = __builtin_amdgcn_sdot4(fb[kk][j].x, ones.x, sumq[j], false);
            s = __builtin_amdgcn_sdot4(fb[kk][j].y, ones.y, s, false);
            s = __builtin_amdgcn_sdot4(fb[kk][j].z, ones.z, s, false);
            sumq[j] = __builtin_amdgcn_sdot4(fb[kk][j].w, ones.w, s, false);
          }
        }
    }
  };
  auto bar = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

#if QNN_STAMP
  const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const unsigned long long t_begin = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  unsigned long long ts0 = 0, ts1 = 0;
#endif
  // prologue: K-tiles 0 and 1 in flight, K-tile 0 landed for every wave; waves 4-7
  // then take one extra barrier (the stagger)
#pragma unroll
  for (int q = 0; q < PPT; ++q) issue(0, 0, q);
#pragma unroll
  for (int q = 0; q < PPT; ++q) issue(1, 1, q);
  wait_vmcnt<P>();
  bar();
  if (late) bar();
#if QNN_STAMP
  QNN_TS(ts0);
  const unsigned long long c_pro = ts0 - t_begin;
#endif

  auto ktile = [&](auto slotc, int st) {
    constexpr int SL = decltype(slotc)::value;
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      read_frags(slotc, q);
      issue(st + 2, (SL + 2) % NS, q);
      if (q == PPT - 1) wait_vmcnt<P>();  // own DMA of K-tile st+1 landed (st+2 in flight)
      bar();
      __builtin_amdgcn_s_setprio(1);
      mfma_seg(st, q);
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
  };
  for (int st = 0; st < nstage; st += NS) {
    ktile(std::integral_constant<int, 0>{}, st);
    if (st + 1 < nstage) ktile(std::integral_constant<int, 1>{}, st + 1);
    if (st + 2 < nstage) ktile(std::integral_constant<int, 2>{}, st + 2);
    if (st + 3 < nstage) ktile(std::integral_constant<int, 3>{}, st + 3);
  }
  if (!late) bar();  // equal barrier counts
  wait_vmcnt<0>();   // the clamped tail DMAs still write LDS
#if QNN_STAMP
  QNN_TS(ts1);
  const unsigned long long c_loop = ts1 - ts0;
#endif

#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] += __shfl_xor(sumq[j], 32, 64);
  __syncthreads();
  if (QNN_ABLATE == 3) {
    int z = sumq[0];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) z ^= acc[i][j][r];
    if (z == 0x7fffffff) p.e.out_f32[0] = 1.f;
    return;
  }
#if QNN_STAMP
  QNN_TS(ts0);
#endif
  if (!p.epi_early) {  // no room beside the ring: stage into it now
    stage_epi<C, EK>(p, x, smem + p.epi_off, c0, wave, lane);
    wait_vmcnt<0>();
    __syncthreads();
  }
  epilogue<C, EK>(p, acc, sumq, pcls, smem, m0, c0, wm, wn, lane, tid, wave);
#if QNN_STAMP
  QNN_TS(ts1);
  const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  unsigned hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  if (lane == 0 && blockIdx.x < (1 << 20) / (10 * W)) {
    unsigned long long* o = qnn_dbg_stamps + ((size_t)blockIdx.x * W + wave) * 10;
    o[0] = rt_start; o[1] = rt_end; o[2] = c_pro; o[3] = 0; o[4] = 0; o[5] = c_loop; o[6] = 0;
    o[7] = ts1 - ts0; o[8] = hwid; o[9] = nstage;
  }
#endif
}

// ---------------------------------------------------------------- halo-band main loop
// For kh x kw > 1 the implicit im2col of qconv_kernel pulls every input byte through
// L2 -> LDS once per tap (9x for 3x3, 16x for the space-to-depth 7x7 stem): on CDNA4
// the per-CU L2 -> LDS rate (~30 B/clk), not the MFMA pipe, bounds those layers.  Here
// a block loads the BAND of input rows its BN output pixels read -- once per K chunk --
// into LDS, and every tap's B fragment is an LDS read at a tap-shifted band address.
// Only the weights stream per K stage (through the D-slot LDS ring, as before).
//
// K order: chunk c of Cp (16 << LW bytes of channels per band pixel, LW = 2 for
// Cp >= 64), then taps (row-major), then the chunk's 16-byte slots -- which is the
// tap-major packed weight row read at column t*Cp + 64c (LW = 2) or 64s (one chunk).
// A 64-byte stage is one tap (LW 2), two taps (LW 1, Cp 32) or four (LW 0, Cp 16).
//
// Band layout: pixel q of the band (padded input rows [R0, R1), stride-2 convs with
// each row's even columns first) holds its chunk at q * (16 << LW), the 16-byte slots
// XOR-swizzled by q's bits [4-LW, 4) so that the 32 consecutive pixels of a 32x32x32
// B fragment hit 16 distinct bank slots per ds_read_b128 lane group.  The swizzle is
// applied on the DMA source side (LDS-DMA destinations are lane-linear).
struct Band {
  int nc, ns, kt;                   // K chunks, 64-B stages per chunk, stages in all
  int s2, we;                       // stride 2: deinterleaved columns, even count (wp + 1) / 2
  uint32_t wp_magic;                // ceil(2^32 / wp): q / wp == umulhi(q, wp_magic)
  int nbw;                          // band DMA pieces (1 KiB) per wave per chunk
  int band_off, band_bytes, nbuf;   // LDS: band buffers (2 when nc > 1)
  int zero_off, mask_off;           // LDS: 64 zero bytes (padded taps), K mask (MASKED)
};

// vmcnt(n) for a run-time n (uniform): the exact count or a smaller one (waits longer)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  if (n >= 24) wait_vmcnt<24>();
  else if (n >= 16) wait_vmcnt<16>();
  else switch (n) {
      case 15: wait_vmcnt<15>(); break;
      case 14: wait_vmcnt<14>(); break;
      case 13: wait_vmcnt<13>(); break;
      case 12: wait_vmcnt<12>(); break;
      case 11: wait_vmcnt<11>(); break;
      case 10: wait_vmcnt<10>(); break;
      case 9: wait_vmcnt<9>(); break;
      case 8: wait_vmcnt<8>(); break;
      case 7: wait_vmcnt<7>(); break;
      case 6: wait_vmcnt<6>(); break;
      case 5: wait_vmcnt<5>(); break;
      case 4: wait_vmcnt<4>(); break;
      case 3: wait_vmcnt<3>(); break;
      case 2: wait_vmcnt<2>(); break;
      case 1: wait_vmcnt<1>(); break;
      default: wait_vmcnt<0>(); break;
    }
}

template <int LW>
__device__ __forceinline__ int band_slot_xor(int q) {  // swizzle of band pixel q's 16-byte slots
  if constexpr (LW == 0) return 0;
  else return (q >> (4 - LW)) & ((1 << LW) - 1);
}

template <class C, int EK, int LW, bool MASKED>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(C::BPC * C::W / 4))) void qconv_band_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ w, const Params p, const Band bd) {
  constexpr int BM = C::BM, BN = C::BN, W = C::W, TM = C::TM, TN = C::TN, D = C::NS, NA = C::NA;
  constexpr int PS = 16 << LW;     // band pixel bytes (one K chunk)
  constexpr int STAGE_A = BM * 64;
  static_assert(C::BK == 64, "band kernel: 64-byte weight stages");
  static_assert(!MASKED || LW == 0, "masked (space-to-depth) stems have 16-channel band pixels");
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];

  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WGN, wn = wave % C::WGN;

  const int nby = (d.cout + BM - 1) / BM;
  const int nbx = (p.M + BN - 1) / BN;
  const int nblk = nbx * nby;
  int t;
  {
    const int bb = blockIdx.x, xcd = bb & 7, q = nblk >> 3, r = nblk & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bb >> 3);
  }
  const int m0 = (t / nby) * BN;
  const int c0 = (t % nby) * BM;
  const int HoWo = d.ho * d.wo;
  auto grow = [&](int m) {  // padded input row (over the whole batch) of output pixel m's tap row 0
    const int n = m / HoWo, r = m - n * HoWo, ho = r / d.wo;
    return n * d.hp + ho * d.sh;
  };
  const int R0 = __builtin_amdgcn_readfirstlane(grow(m0));
  const int mlast = (m0 + BN < p.M ? m0 + BN : p.M) - 1;
  const int NBP = __builtin_amdgcn_readfirstlane((grow(mlast) + d.kh - R0) * d.wp);

  if (tid < 4) *reinterpret_cast<v4i*>(smem + bd.zero_off + 16 * tid) = (v4i){0, 0, 0, 0};
  if constexpr (MASKED) {
    for (int i = tid; i < d.kpad / 16; i += C::NT)
      *reinterpret_cast<v4i*>(smem + bd.mask_off + 16 * i) = *reinterpret_cast<const v4i*>(d.kmask + 16 * i);
  }
  __syncthreads();  // before any LDS-DMA is in flight (a barrier then would drain it)

  // ---- per-lane state: this lane's pixel of each column tile j as a band pixel (tap 0,0)
  const int frow = lane & 31, fh = lane >> 5;
  int pb[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int m = m0 + wn * 32 * TN + j * 32 + frow;
    m = m < p.M ? m : p.M - 1;
    const int n = m / HoWo, r = m - n * HoWo, ho = r / d.wo, wo = r - ho * d.wo;
    pb[j] = (n * d.hp + ho * d.sh - R0) * d.wp + wo;  // input column wo*sw: wo itself (s2: even half)
  }
  const int8_t* wblk = w + (int64_t)c0 * d.kpad;
  uint32_t aoff[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int row = 16 * (wave + W * j) + lane / 4;
    const int crow = (c0 + row < d.cout_pad ? row : d.cout_pad - 1 - c0);
    aoff[j] = (uint32_t)(crow * d.kpad + (swz<64>(row, lane % 4) - row * 64));
  }
  int pcls[TN];
  pixel_classes<C>(p, m0, wn, lane, pcls);
  if (p.epi_early) stage_epi<C, EK>(p, x, smem + p.epi_off, c0, wave, lane);  // oldest DMAs: land under the loop

  // ---- DMA issue
  auto issue_band = [&](int c, int bi) {
    int8_t* dst = smem + bd.band_off + bi * bd.band_bytes;
    for (int k = 0; k < bd.nbw; ++k) {
      const int piece = wave + W * k;
      const int byte = piece * 1024 + 16 * lane;
      int q = byte >> (4 + LW);
      q = q < NBP ? q : NBP - 1;
      const int u = ((byte >> 4) & ((1 << LW) - 1)) ^ band_slot_xor<LW>(q);
      const int r = (int)__umulhi((uint32_t)q, bd.wp_magic);
      const int ci = q - r * d.wp;
      const int col = bd.s2 ? (ci < bd.we ? 2 * ci : 2 * (ci - bd.we) + 1) : ci;
      uint32_t off = (uint32_t)(((R0 + r) * d.wp + col) * d.cp + c * PS + 16 * u);
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_global_load_lds((const void*)(x + off), (lds_ptr_t)(dst + piece * 1024), 16, 0, 0);
    }
  };
  auto koff = [&](int c, int s) -> uint32_t {  // packed weight column of stage (c, s)
    if constexpr (LW == 2) return (uint32_t)(s * d.cp + 64 * c);
    else return (uint32_t)(64 * s);
  };
  auto issue_w = [&](int c, int s, int slot) {
    if (QNN_ABLATE == 1) return;
    const uint32_t ko = koff(c, s);
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      uint32_t off = aoff[j] + ko;
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_global_load_lds((const void*)(wblk + off), (lds_ptr_t)(smem + slot * STAGE_A + (wave + W * j) * 1024),
                                       16, 0, 0);
    }
  };
  // band offset of tap t (uniform)
  auto tap_delta = [&](int tt) {
    const int tr = (tt * p.kw_magic) >> 16, tc = tt - tr * d.kw;
    return tr * d.wp + (bd.s2 ? (tc & 1) * bd.we + (tc >> 1) : tc);
  };

  v16i acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v16i){0};
  int sumq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] = 0;
  int offa[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) offa[ks] = (wm * 32 * TM + frow) * 64 + (swz<64>(frow, 2 * ks + fh) - frow * 64);

  // one 64-byte stage: 2 k-steps of 32x32x32; B fragments read from the band at tap-shifted
  // addresses (padded taps of LW < 2 read the zero bytes)
  auto compute = [&](auto slotc, int bi, int s) {
    constexpr int AO = decltype(slotc)::value * STAGE_A;
    const int bbase = bd.band_off + bi * bd.band_bytes;
    v4i fa[2][TM], fb[2][TN];
    auto load = [&](int ks, int sl) {
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[sl][i] = *reinterpret_cast<const v4i*>(smem + AO + offa[ks] + i * 32 * 64);
      int tt, u;
      if constexpr (LW == 2) tt = s, u = 2 * ks + fh;
      else if constexpr (LW == 1) tt = 2 * s + ks, u = fh;
      else tt = 4 * s + 2 * ks + fh, u = 0;
      int dl;
      if constexpr (LW == 0) {
        const int t0 = 4 * s + 2 * ks;
        const int d0 = tap_delta(t0), d1 = tap_delta(t0 + 1);
        dl = fh ? d1 : d0;
      } else {
        dl = tap_delta(tt);
      }
      const bool pad = tt >= p.taps;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int q = pb[j] + dl;
        int addr = bbase + q * PS + ((u ^ band_slot_xor<LW>(q)) << 4);
        if (LW < 2) addr = pad ? bd.zero_off : addr;
        fb[sl][j] = *reinterpret_cast<const v4i*>(smem + addr);
      }
    };
    load(0, 0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < 2) load(ks + 1, cur ^ 1);
      v4i ones = {0x01010101, 0x01010101, 0x01010101, 0x01010101};
      if constexpr (MASKED) ones = *reinterpret_cast<const v4i*>(smem + bd.mask_off + s * 64 + 16 * (2 * ks + fh));
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int sm = __builtin_amdgcn_sdot4(fb[cur][j].x, ones.x, sumq[j], false);
        sm = __builtin_amdgcn_sdot4(fb[cur][j].y, ones.y, sm, false);
        sm = __builtin_amdgcn_sdot4(fb[cur][j].z, ones.z, sm, false);
        sumq[j] = __builtin_amdgcn_sdot4(fb[cur][j].w, ones.w, sm, false);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (QNN_ABLATE == 2) {
            asm volatile("" ::"v"(fa[cur][i]), "v"(fb[cur][j]));
            acc[i][j][0] += fa[cur][i].x;
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[cur][i], fb[cur][j], acc[i][j], 0, 0, 0);
          }
        }
    }
  };

  // ---- prologue: band chunk 0, weight stages 0 .. D-2 (clamped: counts stay uniform)
  const int KT = bd.kt;
  issue_band(0, 0);
  {
    int c = 0, s = 0;
#pragma unroll
    for (int k = 0; k < D - 1; ++k) {
      issue_w(c, s, k);
      if (k + 1 < KT) {
        if (++s == bd.ns) s = 0, ++c;
      }
    }
  }
  // stage k = (c, s) lives in weight slot k % D and band buffer c & 1.  Before the barrier
  // of stage k each wave waits for its own DMA of stage k (issued D-1 stages earlier; the
  // band chunk it reads is older still); the younger DMAs may stay in flight: D-2 weight
  // stages, plus the next band chunk when it was issued within them.
  int c = 0, s = 0;    // current stage
  int ca = 0, sa = 0;  // the newest issued weight stage: D-2 (clamped to the last one)
  for (int k = 0; k < D - 2 && k + 1 < KT; ++k)
    if (++sa == bd.ns) sa = 0, ++ca;
  auto step = [&](auto slotc) {
    constexpr int SL = decltype(slotc)::value;
    const bool band_young = s >= 1 && s <= D - 2 && c + 1 < bd.nc;
    wait_vmcnt_rt((D - 2) * NA + (band_young ? bd.nbw : 0));
    __builtin_amdgcn_s_barrier();
    if (s == 0 && c + 1 < bd.nc) issue_band(c + 1, (c + 1) & 1);
    // advance the issue-ahead stage (clamped at the last stage) and refill the freed slot
    if (ca * bd.ns + sa + 1 < KT) {
      if (++sa == bd.ns) sa = 0, ++ca;
    }
    issue_w(ca, sa, (SL + D - 1) % D);
    compute(slotc, c & 1, s);
    if (++s == bd.ns) s = 0, ++c;
  };
  for (int k = 0; k < KT; k += D) {
    step(std::integral_constant<int, 0>{});
    if (k + 1 < KT) step(std::integral_constant<int, 1>{});
    if (k + 2 < KT) step(std::integral_constant<int, 2>{});
    if constexpr (D == 4)
      if (k + 3 < KT) step(std::integral_constant<int, 3>{});
  }
  wait_vmcnt<0>();  // the clamped tail DMAs still write LDS

#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] += __shfl_xor(sumq[j], 32, 64);
  __syncthreads();  // main-loop LDS is reused by the epilogue
  if (QNN_ABLATE == 3) {
    int z = sumq[0];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) z ^= acc[i][j][r];
    if (z == 0x7fffffff) p.e.out_f32[0] = 1.f;
    return;
  }
  if (!p.epi_early) {
    stage_epi<C, EK>(p, x, smem + p.epi_off, c0, wave, lane);
    wait_vmcnt<0>();
    __syncthreads();
  }
  epilogue<C, EK>(p, acc, sumq, pcls, smem, m0, c0, wm, wn, lane, tid, wave);
}

template <class C>
static int main_lds_bytes(int tapm, bool masked) {
  const int red = C::KSP > 1 ? (C::TM * C::TN * 16 + C::TN) * 64 * 4 * C::WG : 0;  // K-group hand-off
  const int ring = C::KSP * C::NS * C::STAGE;
  return (ring > red ? ring : red) + ((tapm == TAP_LDS) ? 4 * MAX_TAPS : 0) + (masked ? MAX_MASK : 0);
}

// LDS of a launch: main loop (lds_main bytes at 0), epilogue data (early: beside the main
// loop's LDS, DMA'd at kernel start; late: at 0 once the main loop is done), NCHW transpose
// scratch (after the loop).  Returns the dynamic LDS bytes, or -1 if over 160 KiB.
template <class C>
static int plan_epi_lds(int lds_main, Params& q) {
  lds_main = (lds_main + 15) & ~15;
  const int k = epi_kind(q.e);
  const int epi = 4 * (7 + q.e.nclass) * C::BM + (k == EK_LUT ? 256 * C::BM : 0) +
                  (k == EK_GEN ? 16 * q.e.nres * C::BM : 0);
  const int scr = k == EK_NCHW ? 4096 * C::W : 0;
  int lds;
  if (lds_main + epi <= LDS_MAX / C::BPC && scr <= lds_main) {
    q.epi_early = 1, q.epi_off = lds_main, q.scr_off = 0;
    lds = lds_main + epi;
  } else {
    q.epi_early = 0, q.epi_off = 0, q.scr_off = (epi + 15) & ~15;
    lds = q.scr_off + scr > lds_main ? q.scr_off + scr : lds_main;
  }
  return lds > LDS_MAX ? -1 : lds;
}

template <class C, int PP, int EK, int TAPM, bool MASKED>
static int launch_kernel(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  auto kern = [] {
    if constexpr (PP > 0) return qconv_pp_kernel<C, PP, EK, TAPM, MASKED>;
    else return qconv_kernel<C, EK, TAPM, MASKED>;
  }();
  static const hipError_t attr =  // allow > 64 KiB of dynamic LDS (gfx950: 160 KiB per CU)
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  Params q = p;
  const int lds = plan_epi_lds<C>(main_lds_bytes<C>(TAPM, MASKED), q);
  if (lds < 0) return arg_error("conv tile needs more than 160 KiB of LDS (too many border classes)");
  const int nblk = (int)(cdiv(p.M, C::BN) * cdiv(p.d.cout, C::BM));
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(C::NT), lds, s, x, w, q);
  return QNN_OK;
}

// ---- halo-band kernel: geometry and LDS of a layer for a (BM, BN, waves, ring depth)
static int band_lw(const qnn_conv_desc& d) { return d.cp >= 64 ? 2 : (d.cp == 32 ? 1 : 0); }

// Fills the K schedule and band sizing; returns the main-loop LDS bytes, or -1 when the
// layer is not a band layer (1x1, unsupported stride) or the band does not fit.
static int band_geometry(const Params& p, int BM, int BN, int nwaves, int D, int bpc, Band& b) {
  const qnn_conv_desc& d = p.d;
  if (p.taps <= 1 || d.sh != d.sw || (d.sh != 1 && d.sh != 2)) return -1;
  const int lw = band_lw(d), W = 1 << lw, tps = 4 / W;
  if (d.kmask && lw != 0) return -1;
  const int taps_pad = (p.taps + tps - 1) / tps * tps;
  b.nc = lw == 2 ? d.cp / 64 : 1;
  b.ns = taps_pad / tps;
  b.kt = b.nc * b.ns;
  if (b.nc > 1 && b.ns < D - 1) return -1;
  if ((lw < 2 ? b.ns * 64 : p.taps * d.cp) > d.kpad) return -1;
  b.s2 = d.sh == 2;
  b.we = (d.wp + 1) / 2;
  b.wp_magic = (uint32_t)((0x100000000ULL + (uint64_t)d.wp - 1) / (uint64_t)d.wp);
  // largest band over the tiles: BN consecutive output pixels span at most RO + 1 output
  // rows and ceil-many image crossings, each adding hp - ho*sh padded rows
  const int RO = (BN + d.wo - 2) / d.wo;
  const int cross = (d.ho - 1 + RO) / d.ho;
  const int nrows = RO * d.sh + cross * (d.hp - d.ho * d.sh) + d.kh;
  const int64_t nbp = (int64_t)nrows * d.wp;
  const int64_t pieces = cdiv(nbp * (16 << lw), 1024);
  b.nbw = (int)cdiv(pieces, nwaves);
  b.band_bytes = b.nbw * nwaves * 1024;
  b.nbuf = b.nc > 1 ? 2 : 1;
  b.band_off = D * BM * 64;
  b.zero_off = b.band_off + b.nbuf * b.band_bytes;
  b.mask_off = b.zero_off + 64;
  const int lds = b.mask_off + (d.kmask ? d.kpad : 0);
  if (b.nbw > 16 || lds > LDS_MAX / bpc) return -1;
  return lds;
}

template <class C, int EK, int LW, bool MASKED>
static int launch_band(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  auto kern = qconv_band_kernel<C, EK, LW, MASKED>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  Band b;
  const int main = band_geometry(p, C::BM, C::BN, C::W, C::NS, C::BPC, b);
  if (main < 0) return arg_error("band tile does not fit this layer");
  Params q = p;
  const int lds = plan_epi_lds<C>(main, q);
  if (lds < 0) return arg_error("conv tile needs more than 160 KiB of LDS (too many border classes)");
  const int nblk = (int)(cdiv(p.M, C::BN) * cdiv(p.d.cout, C::BM));
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(C::NT), lds, s, x, w, q, b);
  return QNN_OK;
}

template <class C, int EK>
static int launch_band_lw(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  const int lw = band_lw(p.d);
  if (lw == 2) return launch_band<C, EK, 2, false>(x, w, p, s);
  if constexpr (C::BM == 64) {  // few-channel layers (stems, CIFAR) have few output channels
    if (p.d.kmask) return launch_band<C, EK, 0, true>(x, w, p, s);
    if (lw == 1) return launch_band<C, EK, 1, false>(x, w, p, s);
    return launch_band<C, EK, 0, false>(x, w, p, s);
  }
  return arg_error("band tile not built for this channel count");
}

template <class C>
static int launch_band_ek(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  switch (epi_kind(p.e)) {
    case EK_NCHW: return launch_band_lw<C, EK_NCHW>(x, w, p, s);
    case EK_LUT: return launch_band_lw<C, EK_LUT>(x, w, p, s);
    case EK_BNCODE: return launch_band_lw<C, EK_BNCODE>(x, w, p, s);
    default:
      if constexpr (C::TM * C::TN >= 8) return arg_error("general fused epilogue not built for this tile");
      else return launch_band_lw<C, EK_GEN>(x, w, p, s);
  }
}

template <class C, int PP, int EK>
static int launch_tap(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  constexpr int CPR = C::CPR;
  const int cpt = 1 << p.lgcpt;
  if (p.d.kmask) return launch_kernel<C, PP, EK, TAP_LDS, true>(x, w, p, s);
  if (cpt >= CPR) return launch_kernel<C, PP, EK, TAP_ONE, false>(x, w, p, s);
  if (2 * cpt == CPR) return launch_kernel<C, PP, EK, TAP_TWO, false>(x, w, p, s);
  return launch_kernel<C, PP, EK, TAP_LDS, false>(x, w, p, s);
}

// PP = k-steps per ping-pong phase (qconv_pp_kernel), 0 = the plain ring loop (qconv_kernel)
template <class C, int PP = 0>
static int launch_ek(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  switch (epi_kind(p.e)) {
    case EK_NCHW: return launch_tap<C, PP, EK_NCHW>(x, w, p, s);
    case EK_LUT: return launch_tap<C, PP, EK_LUT>(x, w, p, s);
    case EK_BNCODE: return launch_tap<C, PP, EK_BNCODE>(x, w, p, s);
    default:
      // 256x256 blocks + the general chain spill registers: never picked, not built
      if constexpr (C::TM * C::TN >= 8) return arg_error("general fused epilogue not built for this tile");
      else return launch_tap<C, PP, EK_GEN>(x, w, p, s);
  }
}

// ---- tile configurations and the per-layer choice
//   id  block (cout x px)  waves  LDS ring        blocks/CU  note
//   0   256 x 256          8      4 x 32 KiB      1          1 byte from L2 per 256 ops
//   1   128 x 256          8      4 x 24 KiB      1
//   2   256 x 128          8      4 x 24 KiB      1
//   3    64 x 256          4      4 x 20 KiB      2          64-channel layers
//   4   128 x 128          4      4 x 16 KiB      2          small layers (more tiles)
//   5    64 x 128          4      4 x 12 KiB      2          tiny layers / fc
using C0 = Cfg<4, 2, 2, 4, 64, 4>;
using C1 = Cfg<2, 4, 2, 2, 64, 4>;
using C2 = Cfg<4, 2, 2, 2, 64, 4>;
using C3 = Cfg<1, 4, 2, 2, 64, 4>;
using C4 = Cfg<2, 2, 2, 2, 64, 4>;
using C5 = Cfg<1, 2, 2, 2, 64, 4>;
using C6 = Cfg<2, 4, 4, 2, 64, 4>;  // 256 x 256 ping-pong, waves 128 x 64, 1 k-step per phase
using C7 = Cfg<2, 4, 2, 2, 64, 4>;  // 128 x 256 ping-pong, waves 64 x 64, 2 k-steps per phase
using C8 = Cfg<4, 2, 2, 2, 64, 4>;  // 256 x 128 ping-pong
using C10 = Cfg<1, 4, 2, 2, 64, 3, 2>;  // 64 x 256, 3-slot ring: 2 blocks/CU with a stem's K mask
using C11 = Cfg<1, 4, 2, 1, 64, 3, 4>;  // 64 x 128, 3-slot ring: 4 blocks/CU (short-K, epilogue-bound layers)
// halo-band configurations (qconv_band_kernel; kh x kw > 1 only), 3-slot weight ring
//   12  256 x 256   8 waves (128 x 64)   1 block/CU
//   13  128 x 256   8 waves (64 x 64)    1
//   14  256 x 128   8 waves (64 x 64)    1
//   15   64 x 256   4 waves (64 x 64)    2   (also stems and 16/32-channel inputs)
//   16  128 x 128   4 waves (64 x 64)    2
//   17   64 x 128   2 waves (64 x 64)    4   (also stems and 16/32-channel inputs)
using B12 = Cfg<2, 4, 4, 2, 64, 3, 1>;
using B13 = Cfg<2, 4, 2, 2, 64, 3, 1>;
using B14 = Cfg<4, 2, 2, 2, 64, 3, 1>;
using B15 = Cfg<1, 4, 2, 2, 64, 3, 2>;
using B16 = Cfg<2, 2, 2, 2, 64, 3, 2>;
using B17 = Cfg<1, 2, 2, 2, 64, 3, 4>;
// ring-loop configurations after the persistent band (ids 50-53): deeper K stages (BK 128: half
// the barriers per K) and smaller blocks (more resident blocks on the small-spatial deep-K
// layers, ResNet layer 4's 392 tiles of 64 x 128 leave ~1.5 blocks per CU)
//   50   64 x 128   4 waves (64 x 32)   BK 128, 3 x 24 KiB   2 blocks/CU
//   51   64 x  64   2 waves (64 x 32)   BK 64,  3 x 8 KiB    4
//   52   64 x 128   4 waves (32 x 64)   BK 64,  3 x 12 KiB   4
//   53   64 x  64   2 waves (64 x 32)   BK 128, 3 x 16 KiB   2
//   54   64 x 128   8 waves: 2 K groups x 4 (64 x 32), BK 64, 2 x 3 x 12 KiB   2   (even stage count)
//   55   64 x 128   8 waves: 2 K groups x 4 (64 x 32), BK 128, 2 x 3 x 24 KiB  1   (even stage count)
using X0 = Cfg<1, 4, 2, 1, 128, 3, 2>;
using X1 = Cfg<1, 2, 2, 1, 64, 3, 4>;
using X2 = Cfg<2, 2, 1, 2, 64, 3, 4>;
using X3 = Cfg<1, 2, 2, 1, 128, 3, 2>;
using X4 = Cfg<1, 4, 2, 1, 64, 3, 2, 2>;
using X5 = Cfg<1, 4, 2, 1, 128, 3, 1, 2>;
constexpr int NCFG = 18;  // qconv.hip configurations (9: C6 with 2 k-steps per phase); then qconv16.hip's
struct CfgInfo {
  int bm, bn, per_cu, waves;
  float rate;  // relative throughput per CU, fitted to tools/sweep_tiles.py (profiles/r2_sweep_tiles_q16.jsonl)
  bool band;
};
static const CfgInfo CFG[NCFG] = {
    {256, 256, 1, 8, 1.00f, false}, {128, 256, 1, 8, 0.85f, false}, {256, 128, 1, 8, 0.85f, false},
    {64, 256, 2, 4, 0.70f, false},  {128, 128, 2, 4, 0.70f, false}, {64, 128, 2, 2, 0.50f, false},
    {256, 256, 1, 8, 1.20f, false}, {128, 256, 1, 8, 0.95f, false}, {256, 128, 1, 8, 0.95f, false},
    {256, 256, 1, 8, 1.15f, false}, {64, 256, 2, 4, 0.70f, false},  {64, 128, 4, 4, 0.45f, false},
    {256, 256, 1, 8, 0.98f, true},  {128, 256, 1, 8, 0.72f, true},  {256, 128, 1, 8, 0.72f, true},
    {64, 256, 2, 4, 0.70f, true},   {128, 128, 2, 4, 0.67f, true},  {64, 128, 4, 2, 0.45f, true},
};

constexpr int NX = 6;
static const CfgInfo XCFG[NX] = {
    {64, 128, 2, 4, 0.40f, false}, {64, 64, 4, 2, 0.40f, false}, {64, 128, 4, 4, 0.40f, false}, {64, 64, 2, 2, 0.40f, false},
    {64, 128, 2, 8, 0.40f, false}, {64, 128, 1, 8, 0.40f, false},
};
static const int XKSP_BK[NX] = {0, 0, 0, 0, 64, 128};  // K-group configurations: their stage size

// Whether configuration k is built for (and fits) this layer and epilogue kind
static int ncfg_all() { return NCFG + q16_count() + rb_count() + rbp_count() + dtab_count() + 1 + pb_count() + NX + rs_count(); }
static int rb_first() { return NCFG + q16_count(); }
static int rbp_first() { return NCFG + q16_count() + rb_count(); }
static int dtab_first() { return rbp_first() + rbp_count(); }
static int dhead_id() { return dtab_first() + dtab_count(); }  // configuration 44: the classifier head
static int pb_first() { return dhead_id() + 1; }                 // configurations 45-49: persistent band
static int xr_first() { return pb_first() + pb_count(); }         // configurations 50-55: extra ring tiles
static int rs_first() { return xr_first() + NX; }                 // configurations 56-63: streamed resident band

static bool cfg_ok(int k, const Params& p) {
  if (k >= ncfg_all()) return false;
  if (k >= rs_first()) return rs_ok(k - rs_first(), p);
  if (k >= xr_first()) {
    const int x = k - xr_first();
    if (XKSP_BK[x] && (p.d.kpad / XKSP_BK[x]) % 2) return false;  // two K groups: an even stage count
    return epi_kind(p.e) != EK_GEN || XCFG[x].bm * XCFG[x].bn < 65536;
  }
  if (k >= pb_first()) return pb_ok(k - pb_first(), p);
  if (k == dhead_id()) return dhead_ok(p);
  if (k >= dtab_first()) return dtab_ok(k - dtab_first(), p);
  if (k >= rbp_first()) return rbp_ok(k - rbp_first(), p);
  if (k >= rb_first()) return rb_ok(k - rb_first(), p);
  if (k >= NCFG) return q16_ok(k - NCFG, p);
  if (k < 0) return false;
  const int ek = epi_kind(p.e);
  const CfgInfo& c = CFG[k];
  if (ek == EK_GEN && (k == 0 || k == 6 || k == 9 || k == 12)) return false;  // 256x256 + general chain
  if (!c.band) return true;
  if (band_lw(p.d) < 2 && c.bm != 64) return false;
  Band b;
  return band_geometry(p, c.bm, c.bn, c.waves, 3, c.per_cu, b) >= 0;
}

// Estimated time (arbitrary units) of config k: rounds of resident blocks over the CUs,
// each round as long as one block's padded MFMA work at that config's rate.
static double cfg_cost(int k, const Params& p) {
  if (k >= rs_first()) return rs_cost(k - rs_first(), p);
  const bool xr = k >= xr_first();  // the extra ring tiles: the ring's cost model below
  if (!xr && k >= pb_first()) return pb_cost(k - pb_first(), p);
  if (k == dhead_id()) return p.M <= 256 ? 0.0 : 1e30;  // measured: ahead of cfg 11 at b128 (6.4 vs 11.2 us), behind at b512
  if (!xr && k >= dtab_first()) return dtab_cost(k - dtab_first(), p);
  if (!xr && k >= rbp_first()) return rbp_cost(k - rbp_first(), p);
  if (!xr && k >= rb_first()) return rb_cost(k - rb_first(), p);
  if (!xr && k >= NCFG) return q16_cost(k - NCFG, p);
  const CfgInfo& c = xr ? XCFG[k - xr_first()] : CFG[k];
  const int64_t tiles = cdiv(p.M, c.bn) * cdiv(p.d.cout, c.bm);
  const int64_t slots = (int64_t)NUM_CU * c.per_cu;
  const int64_t rounds = cdiv(tiles, slots);
  // with fewer tiles than slots the blocks of a round do not share a CU
  const double share = tiles < slots ? (double)cdiv(tiles, NUM_CU) : (double)c.per_cu;
  return (double)rounds * share * c.bm * c.bn * p.d.kpad / c.rate;
}

static int pick_cfg(const Params& p) {
  auto ok = [&](int k) { return cfg_ok(k, p); };
#if QNN_STAMP || QNN_ABLATE
  static int forced = [] {  // diagnostic builds only: QNN_CONV_CFG overrides every caller
    const char* v = getenv("QNN_CONV_CFG");
    return v ? atoi(v) : -1;
  }();
  if (ok(forced)) return forced;
#endif
  if (p.d.tile > 0) return ok(p.d.tile - 1) ? p.d.tile - 1 : -1;  // explicit: built, or an argument error
  int best = -1;
  double bc = 0;
  for (int k = 0; k < ncfg_all(); ++k) {
    if (!ok(k)) continue;  // 256x256 + the general chain spills registers
    const double c = cfg_cost(k, p);
    if (best < 0 || c < bc) best = k, bc = c;
  }
  return best;
}

static int launch_cfg(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  if (k >= rs_first()) return rs_launch(k - rs_first(), x, w, p, s);
  if (k >= xr_first()) {
    switch (k - xr_first()) {
      case 0: return launch_ek<X0>(x, w, p, s);
      case 1: return launch_ek<X1>(x, w, p, s);
      case 2: return launch_ek<X2>(x, w, p, s);
      case 3: return launch_ek<X3>(x, w, p, s);
      case 4: return launch_ek<X4>(x, w, p, s);
      default: return launch_ek<X5>(x, w, p, s);
    }
  }
  if (k >= pb_first()) return pb_launch(k - pb_first(), x, w, p, s);
  if (k == dhead_id()) return dhead_launch(x, w, p, s);
  if (k >= dtab_first()) return dtab_launch(k - dtab_first(), x, w, p, s);
  if (k >= rbp_first()) return rbp_launch(k - rbp_first(), x, w, p, s);
  if (k >= rb_first()) return rb_launch(k - rb_first(), x, w, p, s);
  if (k >= NCFG) return q16_launch(k - NCFG, x, w, p, s);
  switch (k) {
    case 0: return launch_ek<C0>(x, w, p, s);
    case 1: return launch_ek<C1>(x, w, p, s);
    case 2: return launch_ek<C2>(x, w, p, s);
    case 3: return launch_ek<C3>(x, w, p, s);
    case 4: return launch_ek<C4>(x, w, p, s);
    case 5: return launch_ek<C5>(x, w, p, s);
    case 6: return launch_ek<C6, 1>(x, w, p, s);
    case 7: return launch_ek<C7, 2>(x, w, p, s);
    case 8: return launch_ek<C8, 2>(x, w, p, s);
    case 9: return launch_ek<C6, 2>(x, w, p, s);
    case 10: return launch_ek<C10>(x, w, p, s);
    case 11: return launch_ek<C11>(x, w, p, s);
    case 12: return launch_band_ek<B12>(x, w, p, s);
    case 13: return launch_band_ek<B13>(x, w, p, s);
    case 14: return launch_band_ek<B14>(x, w, p, s);
    case 15: return launch_band_ek<B15>(x, w, p, s);
    case 16: return launch_band_ek<B16>(x, w, p, s);
    default: return launch_band_ek<B17>(x, w, p, s);
  }
}

}  // namespace qnn

using namespace qnn;

#if QNN_STAMP
extern "C" int qnn_debug_stamps(void* dst, size_t bytes) {
  if (bytes > sizeof(qnn_dbg_stamps)) bytes = sizeof(qnn_dbg_stamps);
  return hip_check(hipMemcpyFromSymbol(dst, HIP_SYMBOL(qnn_dbg_stamps), bytes), "stamps");
}
extern "C" int qnn_debug_epi(void* dst, size_t bytes) {
  if (bytes > sizeof(qnn_dbg_epi)) bytes = sizeof(qnn_dbg_epi);
  return hip_check(hipMemcpyFromSymbol(dst, HIP_SYMBOL(qnn_dbg_epi), bytes), "stamps");
}
#endif

static int conv_params(const qnn_conv_desc& d, const qnn_epilogue& e, Params& p) {
  QNN_REQUIRE(d.n >= 0 && d.hp > 0 && d.wp > 0 && d.cout > 0 && d.kh > 0 && d.kw > 0 && d.sh > 0 && d.sw > 0,
              "bad shape");
  QNN_REQUIRE(d.cp >= 16 && (d.cp & (d.cp - 1)) == 0, "cp must be 16 * 2^j");
  QNN_REQUIRE(d.kh * d.kw <= MAX_TAPS && d.kw <= 64, "at most 64 taps");
  QNN_REQUIRE(d.ho > 0 && d.wo > 0 && (d.ho - 1) * d.sh + d.kh <= d.hp && (d.wo - 1) * d.sw + d.kw <= d.wp,
              "ho/wo exceed the padded input");
  QNN_REQUIRE(d.kpad % KPAD_ALIGN == 0 && d.kpad >= d.kh * d.kw * d.cp, "kpad must be a multiple of 128 covering K");
  QNN_REQUIRE(d.cout_pad >= d.cout, "cout_pad < cout");
  QNN_REQUIRE((int64_t)d.n * d.hp * d.wp * d.cp < (1LL << 31) && d.zero_off >= 0 && d.zero_off % 16 == 0,
              "input too large or bad zero_off");
  QNN_REQUIRE(!d.kmask || (d.kpad <= MAX_MASK && (((uintptr_t)d.kmask) & 15) == 0), "kmask: kpad <= 1024, 16-B aligned");
  QNN_REQUIRE(e.nclass > 0 && e.nclass <= MAX_CLASSES && e.nwc > 0, "border classes out of range");
  QNN_REQUIRE(e.mode == 0 || e.mode == 1, "mode must be 0 (drop-in NCHW) or 1 (fused NHWC)");
  p.d = d;
  p.e = e;
  const int64_t M = (int64_t)d.n * d.ho * d.wo;
  QNN_REQUIRE(M < (1LL << 31), "too many output pixels");
  p.M = (int)M;
  p.taps = d.kh * d.kw;
  p.lgcpt = __builtin_ctz(d.cp / 16);
  p.kw_magic = (65536 + d.kw - 1) / d.kw;
  p.ct = (int)cdiv(d.cout, 32);
#if QNN_STAMP || QNN_ABLATE
  static const int stagger = [] {  // diagnostic builds only: QNN_CONV_STAGGER=0 disables
    const char* v = getenv("QNN_CONV_STAGGER");
    return v ? atoi(v) : 1;
  }();
  p.stagger = stagger;
#else
  p.stagger = 1;
#endif
  return QNN_OK;
}

extern "C" int qnn_conv_tile_count(void) { return ncfg_all(); }

extern "C" const char* qnn_conv_tile_kernel(int k) {
  if (k < 0 || k >= ncfg_all()) return nullptr;
  if (k >= rs_first()) return "qconv_rs_kernel";
  if (k >= xr_first()) return "qconv_kernel";
  if (k >= pb_first()) return "qconv_pb_kernel";
  if (k == dhead_id()) return "qconv_direct_kernel";
  if (k >= dtab_first()) return "qconv_dtab_kernel";
  if (k >= rbp_first()) return "qconv_rbp_kernel";
  if (k >= rb_first()) return k - rb_first() < rb_count() - direct_count() ? "qconv_rb_kernel" : "qconv_direct_kernel";
  if (k >= NCFG) return "qconv16_kernel";
  if (k >= 12) return "qconv_band_kernel";
  if (k >= 6 && k <= 9) return "qconv_pp_kernel";
  return "qconv_kernel";
}

extern "C" int qnn_conv_plan(const qnn_conv_desc* desc, const qnn_epilogue* epi, int* cfg, int* bm, int* bn,
                             int* nblk) {
  QNN_REQUIRE(desc && epi, "null descriptor");
  Params p;
  const int rc = conv_params(*desc, *epi, p);
  if (rc != QNN_OK) return rc;
  const int k = pick_cfg(p);
  QNN_REQUIRE(k >= 0, "tile configuration not built for this layer / epilogue kind");
  if (cfg) *cfg = k;
  int tbm, tbn;
  if (k >= rs_first()) rs_tile(k - rs_first(), &tbm, &tbn);
  else if (k >= xr_first()) tbm = XCFG[k - xr_first()].bm, tbn = XCFG[k - xr_first()].bn;
  else if (k >= pb_first()) pb_tile(k - pb_first(), &tbm, &tbn);
  else if (k == dhead_id()) tbm = 16, tbn = 64;
  else if (k >= dtab_first()) dtab_tile(k - dtab_first(), &tbm, &tbn);
  else if (k >= rbp_first()) rbp_tile(k - rbp_first(), &tbm, &tbn);
  else if (k >= rb_first()) rb_tile(k - rb_first(), &tbm, &tbn);
  else if (k >= NCFG) q16_tile(k - NCFG, &tbm, &tbn);
  else tbm = CFG[k].bm, tbn = CFG[k].bn;
  if (bm) *bm = tbm;
  if (bn) *bn = tbn;
  if (nblk)
    *nblk = k >= rs_first() ? (int)rs_blocks(k - rs_first(), p)
            : k >= xr_first() ? (int)(cdiv(p.M, tbn) * cdiv(p.d.cout, tbm))
            : k >= pb_first() ? (int)pb_blocks(k - pb_first(), p)
            : k == dhead_id() ? (int)dhead_blocks(p)
            : k >= dtab_first() ? (int)dtab_blocks(k - dtab_first(), p)
            : k >= rbp_first() ? (int)rbp_blocks(k - rbp_first(), p)
            : k >= rb_first() ? (int)rb_blocks(k - rb_first(), p)
                              : (int)(cdiv(p.M, tbn) * cdiv(p.d.cout, tbm));
  return QNN_OK;
}

extern "C" int qnn_qconv2d_maxpool_fwd(const int8_t* x, const int8_t* wq, const qnn_conv_desc* desc,
                                      const qnn_epilogue* epi, int pool_ho, int pool_wo, uint8_t* out_code,
                                      const int8_t* lut0, const qnn_code_out* code0, const int8_t* lut1,
                                      const qnn_code_out* code1, qnn_stream_t stream) {
  QNN_REQUIRE(desc && epi, "null descriptor");
  Params p;
  const int rc0 = conv_params(*desc, *epi, p);
  if (rc0 != QNN_OK) return rc0;
  const qnn_epilogue& e = *epi;
  QNN_REQUIRE(e.mode == 1 && e.bn_mean && e.bn_sq && e.bn_wq && e.bn_bq && e.bn_scale > 0.f,
              "stem max-pool: mode 1 with the stem's RangeBN");
  const bool has0 = code0 && code0->ptr, has1 = code1 && code1->ptr;
  QNN_REQUIRE(!has0 || (lut0 && (((uintptr_t)lut0) & 15) == 0), "code0 needs a 16-B aligned lut0");
  QNN_REQUIRE(!has1 || (lut1 && (((uintptr_t)lut1) & 15) == 0), "code1 needs a 16-B aligned lut1");
  QNN_REQUIRE(out_code || has0 || has1, "no output");
  QNN_REQUIRE(!out_code || (((uintptr_t)out_code) & 15) == 0, "out_code must be 16-byte aligned");
  auto code16 = [&](const qnn_code_out* o) {
    return !o || !o->ptr || (o->cp >= desc->cout && o->cp % 16 == 0 && o->scale > 0.f && o->pad >= 0 &&
                             (((uintptr_t)o->ptr) & 15) == 0);
  };
  QNN_REQUIRE(code16(code0) && code16(code1), "bad code output (cp % 16, 16-B aligned)");
  if (desc->n == 0) return QNN_OK;
  QNN_REQUIRE(x && wq && e.sxsw && e.sxbw && e.table && e.hcls && e.wcls, "null pointer");
  QNN_REQUIRE((((uintptr_t)x) & 15) == 0 && (((uintptr_t)wq) & 15) == 0, "x/wq must be 16-byte aligned");
  qnn_code_out none{};
  const int rc = stem_pool_launch(x, wq, p, pool_ho, pool_wo, out_code, has0 ? lut0 : nullptr, has0 ? *code0 : none,
                                  has1 ? lut1 : nullptr, has1 ? *code1 : none, (hipStream_t)stream);
  if (rc != QNN_OK) return rc;
  QNN_LAUNCH_CHECK("qnn_qconv2d_maxpool_fwd");
  return QNN_OK;
}

extern "C" int qnn_conv_occupancy(const qnn_conv_desc* desc, const qnn_epilogue* epi, int* cfg, int* blocks_per_cu,
                                  int* lds_bytes, int* grid) {
  QNN_REQUIRE(desc && epi, "null descriptor");
  Params p;
  const int rc = conv_params(*desc, *epi, p);
  if (rc != QNN_OK) return rc;
  const int k = pick_cfg(p);
  QNN_REQUIRE(k >= 0, "tile configuration not built for this layer / epilogue kind");
  QNN_REQUIRE(k >= rb_first() && (k < xr_first() || k >= rs_first()),
              "occupancy is reported for the resident-band, direct-fragment and persistent-band configurations");
  Occ o{0, 0, 0};
  const int r = k >= rs_first()    ? rs_launch(k - rs_first(), nullptr, nullptr, p, nullptr, &o)
                : k >= pb_first()    ? pb_launch(k - pb_first(), nullptr, nullptr, p, nullptr, &o)
                : k == dhead_id()    ? dhead_launch(nullptr, nullptr, p, nullptr, &o)
                : k >= dtab_first()  ? dtab_launch(k - dtab_first(), nullptr, nullptr, p, nullptr, &o)
                : k >= rbp_first() ? rbp_launch(k - rbp_first(), nullptr, nullptr, p, nullptr, &o)
                                   : rb_launch(k - rb_first(), nullptr, nullptr, p, nullptr, &o);
  if (r != QNN_OK) return r;
  if (cfg) *cfg = k;
  if (blocks_per_cu) *blocks_per_cu = o.blocks_per_cu;
  if (lds_bytes) *lds_bytes = o.lds;
  if (grid) *grid = o.grid;
  return QNN_OK;
}

// the arguments of a forward launch (x: the code tensor, or the fp32 input of the _nchw_f32 entry);
// QNN_OK with p filled, -1 for an empty batch (nothing to launch), else the error status
static int fwd_args(const void* x, const int8_t* wq, const qnn_conv_desc* desc, const qnn_epilogue* epi, Params& p) {
  QNN_REQUIRE(desc && epi, "null descriptor");
  const qnn_conv_desc& d = *desc;
  const qnn_epilogue& e = *epi;
  const int rc0 = conv_params(d, e, p);
  if (rc0 != QNN_OK) return rc0;
  if (d.n == 0) return -1;
  QNN_REQUIRE(x && wq && e.sxsw && e.sxbw && e.table && e.hcls && e.wcls, "null pointer");
  QNN_REQUIRE((((uintptr_t)x) & 15) == 0 && (((uintptr_t)wq) & 15) == 0, "x/wq must be 16-byte aligned");
  if (e.mode == 0) {
    QNN_REQUIRE(e.out_f32 != nullptr, "mode 0 needs out_f32");
    QNN_REQUIRE((((uintptr_t)e.out_f32) & 15) == 0, "out_f32 must be 16-byte aligned");
  } else {
    QNN_REQUIRE(d.cout % 16 == 0, "fused mode needs cout % 16 == 0");
    QNN_REQUIRE(!e.bn_mean || (e.bn_sq && e.bn_wq && e.bn_bq && e.bn_scale > 0.f), "incomplete RangeBN");
    auto code_ok = [](const int8_t* ptr, int cp, float scale) {
      return cp % 16 == 0 && scale > 0.f && (((uintptr_t)ptr) & 15) == 0;
    };
    QNN_REQUIRE(!e.out_code0 || code_ok(e.out_code0, e.code0_cp, e.code0_scale), "bad code0 (cp % 16, 16-B aligned)");
    QNN_REQUIRE(!e.out_code1 || code_ok(e.out_code1, e.code1_cp, e.code1_scale), "bad code1 (cp % 16, 16-B aligned)");
    QNN_REQUIRE(!e.out_bncode || (e.bn_mean && (((uintptr_t)e.out_bncode) & 15) == 0), "bncode needs RangeBN, 16-B aligned");
    QNN_REQUIRE(e.out_f32 || e.out_code0 || e.out_code1 || e.out_bncode, "fused mode without an output");
    QNN_REQUIRE(!e.lut || (e.bn_mean && e.out_code0 && !e.residual && !e.out_f32 && !e.out_code1 && !e.out_bncode &&
                           (((uintptr_t)e.lut) & 15) == 0),
                "lut needs RangeBN, exactly one code output, no residual/fp32/bncode, 16-B aligned");
    QNN_REQUIRE(!e.f32_tiled || ((((uintptr_t)e.out_f32) & 15) == 0 && (((uintptr_t)e.residual) & 15) == 0),
                "C-tile fp32 maps must be 16-byte aligned");
    QNN_REQUIRE(e.nres >= 0 && e.nres <= QNN_MAX_RES && (e.nres == 0 || (!e.lut && e.bn_mean)) &&
                    (!e.res_relu0 || (e.nres > 0 && !e.residual)),
                "residual chain: 0..4 links, needs RangeBN, no lut; res_relu0 only for a code-started chain");
    for (int l = 0; l < e.nres; ++l) {
      const qnn_res_link& r = e.res[l];
      QNN_REQUIRE(r.code && (((uintptr_t)r.code) & 15) == 0 && r.mean && r.sq && r.wq && r.bq && r.scale > 0.f,
                  "bad residual chain link (16-B aligned codes, RangeBN params, scale > 0)");
    }
  }
  return QNN_OK;
}

extern "C" int qnn_qconv2d_fwd(const int8_t* x, const int8_t* wq, const qnn_conv_desc* desc, const qnn_epilogue* epi,
                               qnn_stream_t stream) {
  Params p;
  const int rc0 = fwd_args(x, wq, desc, epi, p);
  if (rc0 != QNN_OK) return rc0 == -1 ? QNN_OK : rc0;
  hipStream_t s = (hipStream_t)stream;
  const int k = pick_cfg(p);
  QNN_REQUIRE(k >= 0, "tile configuration not built for this layer / epilogue kind");
  const int rc = launch_cfg(k, x, wq, p, s);
  if (rc != QNN_OK) return rc;
  QNN_LAUNCH_CHECK("qnn_qconv2d_fwd");
  return QNN_OK;
}

// The drop-in forward from the module's fp32 NCHW input: one persistent-band launch quantizes the
// input into its band buffers (quant_code_fast: bitwise the codes qnn_quantize_nchw_to_nhwc8 writes)
// and convolves, instead of the quantize launch + qnn_qconv2d_fwd.  desc describes the code tensor
// that quantize would write (hp = h + 2 pad, wp = w + 2 pad, cp >= c); tile: 0 for the cheapest
// persistent-band configuration that fits, k + 1 for configuration k (45-49).  QNN_ERR_UNSUPPORTED when none does (the
// caller then takes the two-launch path).
extern "C" int qnn_qconv2d_fwd_nchw_f32(const float* x, int c, int h, int w, int pad, float neg_min, float scale,
                                        float qmax, const int8_t* wq, const qnn_conv_desc* desc,
                                        const qnn_epilogue* epi, int tile, qnn_stream_t stream) {
  if (x && (((uintptr_t)x) & 15) != 0) {
    // the band fill reads the fp32 input with scalar loads, but the launch checks share
    // qnn_qconv2d_fwd's 16-byte rule: a misaligned view takes the caller's two-launch path
    set_error("fp32 input not 16-byte aligned (two-launch path)");
    return QNN_ERR_UNSUPPORTED;
  }
  Params p;
  const int rc0 = fwd_args(x, wq, desc, epi, p);
  if (rc0 != QNN_OK) return rc0 == -1 ? QNN_OK : rc0;
  const qnn_conv_desc& d = *desc;
  QNN_REQUIRE(c >= 1 && c <= d.cp && h >= 1 && w >= 1 && pad >= 0 && d.hp == h + 2 * pad && d.wp == w + 2 * pad,
              "fp32 input geometry must match the padded code tensor (hp = h + 2 pad, wp = w + 2 pad, c <= cp)");
  QNN_REQUIRE(scale > 0.f && qmax >= 1.f && qmax <= 255.f, "bad input quantizer");
  QNN_REQUIRE((int64_t)d.n * c * h * w < (1LL << 31), "input too large");
  int k = -1;
  if (tile > 0) {
    QNN_REQUIRE(tile - 1 >= pb_first() && tile - 1 < ncfg_all(), "tile must be a persistent-band configuration");
    if (pb_ok(tile - 1 - pb_first(), p)) k = tile - 1;
  } else {
    double best = 0;
    for (int i = 0; i < pb_count(); ++i)
      if (pb_ok(i, p) && (k < 0 || pb_cost(i, p) < best)) k = pb_first() + i, best = pb_cost(i, p);
  }
  if (k < 0) {
    set_error("no persistent-band configuration for this layer (fp32 input)");
    return QNN_ERR_UNSUPPORTED;
  }
  const F32In fin = {x, c, h, w, pad, neg_min, scale, qmax};
  const int rc = pb_launch(k - pb_first(), nullptr, wq, p, (hipStream_t)stream, nullptr, &fin);
  if (rc != QNN_OK) return rc;
  QNN_LAUNCH_CHECK("qnn_qconv2d_fwd_nchw_f32");
  return QNN_OK;
}
