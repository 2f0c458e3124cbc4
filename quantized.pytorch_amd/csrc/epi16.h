// The 16x16-accumulator epilogue shared by the v_mfma_i32_16x16x64_i8 kernels
// (qconv16.hip's band kernel, qconv_rb.hip's resident-band kernel): the exact decomposition
//  with the op order of qconv.hip's conv_out4p, then the fused output kinds.
#pragma once
#include "qconv_common.h"

namespace qnn {
namespace q16 {

// y of 4 consecutive channels cl..cl+3 (local) of one pixel: the exact decomposition with the
// op order of qconv.hip's conv_out4p (fma(sw, acc, fma(bw, psq, tb)) + bias), packed pairs.
__device__ __forceinline__ void conv_out4(const float* s_f, int BM, int cl, int ptab, float psq, const v4i& a,
                                          f2 (&v)[2]) {
  const float4 sw = *reinterpret_cast<const float4*>(s_f + cl);
  const float4 bw = *reinterpret_cast<const float4*>(s_f + BM + cl);
  const float4 tb = *reinterpret_cast<const float4*>(s_f + ptab + cl);
  const float4 bi = *reinterpret_cast<const float4*>(s_f + 2 * BM + cl);
  const f2 p2 = {psq, psq};
  const f2 a01 = {(float)a[0], (float)a[1]}, a23 = {(float)a[2], (float)a[3]};
  v[0] = pfma((f2){sw.x, sw.y}, a01, pfma((f2){bw.x, bw.y}, p2, (f2){tb.x, tb.y})) + (f2){bi.x, bi.y};
  v[1] = pfma((f2){sw.z, sw.w}, a23, pfma((f2){bw.z, bw.w}, p2, (f2){tb.z, tb.w})) + (f2){bi.z, bi.w};
}

struct Pix {  // one output pixel of a lane
  int m, n, ho, wo;
  bool ok;
};

// Epilogue over the 16x16 accumulator layout: acc[i][j] lane l holds channels
// c0 + wm*16*TM + 16i + 4(l>>4) + r (r = 0..3) of pixel m0 + wn*16*TN + 16j + (l&15).
template <class C, int EK>
__device__ __forceinline__ void epilogue16(const Params& p, const v4i (&acc)[C::TM][C::TN], const int (&sumq)[C::TN],
                                           const int (&pcls)[C::TN], const Pix (&pix)[C::TN], const int8_t* smem,
                                           int c0, int wm, int lane) {
  constexpr int BM = C::BM, TM = C::TM, TN = C::TN;
  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  const int g = lane >> 4;
  const int HoWo = d.ho * d.wo;
  const float* s_f = reinterpret_cast<const float*>(smem + p.epi_off);
  const int nparam = 7 * BM;
  const int8_t* s_lut = smem + p.epi_off + 4 * (7 + e.nclass) * BM;
  const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
  const QParams c0p = make_qparams(e.code0_neg_min, e.code0_scale, e.code0_qmax);
  const QParams c1p = make_qparams(e.code1_neg_min, e.code1_scale, e.code1_qmax);
  // two consumers calibrated on the same tensor hold the same range: their codes are equal
  const bool same01 = e.out_code0 && e.code1_neg_min == e.code0_neg_min && e.code1_scale == e.code0_scale &&
                      e.code1_qmax == e.code0_qmax;
  const f2 bn_s2 = {e.bn_scale, e.bn_scale}, bn_m2 = {e.bn_min, e.bn_min};
  const bool has_res = EK == EK_GEN && e.residual != nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const Pix& P = pix[j];
    const int ptab = nparam + pcls[j] * BM;
    const float psq = (float)sumq[j];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cl = wm * 16 * TM + 16 * i + 4 * g;  // local channel of register 0
      const int c = c0 + cl;
      const bool cok = c < d.cout;                   // fused modes: cout % 16 == 0 (4-channel groups all in)
      f2 v[2];
      conv_out4(s_f, BM, cl, ptab, psq, acc[i][j], v);
      if constexpr (EK == EK_NCHW) {  // drop-in QConv2d output, NCHW fp32
        if (P.ok) {
          float* yp = e.out_f32 + ((int64_t)P.n * d.cout + c) * HoWo + P.ho * d.wo + P.wo;
          const float y4[4] = {v[0].x, v[0].y, v[1].x, v[1].y};
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (c + r < d.cout) yp[(int64_t)r * HoWo] = y4[r];
        }
      } else if constexpr (EK == EK_LUT) {  // conv -> RangeBN -> ReLU -> consumer quantizer, tabulated
        const f2 q0 = qclamp2(v[0], bnp) + MAGIC_U8, q1 = qclamp2(v[1], bnp) + MAGIC_U8;
        const unsigned qq[4] = {__float_as_uint(q0.x) & 255u, __float_as_uint(q0.y) & 255u,
                                __float_as_uint(q1.x) & 255u, __float_as_uint(q1.y) & 255u};
        int rr = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) rr |= ((int)(uint8_t)s_lut[(cl + u) * 256 + qq[u]]) << (8 * u);
        if (P.ok && c < e.code0_cp)
          *reinterpret_cast<int*>(e.out_code0 + (((int64_t)P.n * e.code0_hp + P.ho + e.code0_pad) * e.code0_wp +
                                                 P.wo + e.code0_pad) * e.code0_cp + c) = cok ? rr : 0;
      } else if constexpr (EK == EK_BNCODE) {
        const int rr = pack4(qclamp2(v[0], bnp) + MAGIC_U8, qclamp2(v[1], bnp) + MAGIC_U8);
        if (P.ok && cok) *reinterpret_cast<int*>(e.out_bncode + (int64_t)P.m * d.cout + c) = rr;
      } else {  // EK_GEN: [RangeBN] [+ residual] [ReLU] -> fp32 and/or codes x2
        if (e.bn_mean) {
          const f2 qb[2] = {qclamp2(v[0], bnp), qclamp2(v[1], bnp)};
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
        const int mc = P.ok ? P.m : p.M - 1;
        const int cc = cok ? c : d.cout - 4;
        if (has_res) {
          const int64_t fi = e.f32_tiled ? ctile_index(mc, cc, p.ct) : (int64_t)mc * d.cout + cc;
          const float4 r4 = *reinterpret_cast<const float4*>(e.residual + fi);
          v[0] = v[0] + (f2){r4.x, r4.y};
          v[1] = v[1] + (f2){r4.z, r4.w};
        }
        if (e.relu) {
          v[0].x = fmaxf(v[0].x, 0.f); v[0].y = fmaxf(v[0].y, 0.f);
          v[1].x = fmaxf(v[1].x, 0.f); v[1].y = fmaxf(v[1].y, 0.f);
        }
        if (e.out_f32 && P.ok && cok) {
          const int64_t fi = e.f32_tiled ? ctile_index(P.m, c, p.ct) : (int64_t)P.m * d.cout + c;
          *reinterpret_cast<float4*>(e.out_f32 + fi) = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
        }
        int k0 = 0;
        if (e.out_code0 && cok) k0 = pack4(qclamp2(v[0], c0p) + MAGIC_S8, qclamp2(v[1], c0p) + MAGIC_S8);
        if (e.out_code0 && P.ok && c < e.code0_cp)
          *reinterpret_cast<int*>(e.out_code0 + (((int64_t)P.n * e.code0_hp + P.ho + e.code0_pad) * e.code0_wp +
                                                 P.wo + e.code0_pad) * e.code0_cp + c) = k0;
        if (e.out_code1 && P.ok && c < e.code1_cp) {
          const int k1 = !cok ? 0 : same01 ? k0 : pack4(qclamp2(v[0], c1p) + MAGIC_S8, qclamp2(v[1], c1p) + MAGIC_S8);
          *reinterpret_cast<int*>(e.out_code1 + (((int64_t)P.n * e.code1_hp + P.ho + e.code1_pad) * e.code1_wp +
                                                 P.wo + e.code1_pad) * e.code1_cp + c) = k1;
        }
      }
    }
  }
}

// Byte offset of the 4-byte word holding channels c..c+3 (c % 4 == 0) of pixel m in a byte
// C-tile code map (include/qnn.h, qnn_res_link): the 32x32 accumulator image's lane
// (m & 31) + 32*((c >> 2) & 1), bytes 4*((c & 31) >> 3) .. +3 of its 16.
__device__ __forceinline__ int64_t btile_word(int m, int c, int ct) {
  return btile_off(m >> 5, c >> 5, ct, (m & 31) + 32 * ((c >> 2) & 1)) + 4 * ((c & 31) >> 3);
}

// The resident-band kernels' epilogue: epilogue16's arithmetic (bitwise the same op order as
// qconv.hip's epilogue) with the per-channel parameters of the lane's TM channel groups held
// in registers across the TN pixel tiles, and the residual code chains (qnn_res_link) read
// as one 4-byte word per link per 4 channels of a pixel.
// pixel(j, P, pcls) fills this lane's pixel of column tile j and its border class (computed
// per tile, not held across the loop).  A lane whose tile slot lies past the block's pixels
// stands in for the block's last pixel -- the same accumulator, sums and border class -- so
// its stores write that pixel's own values again: every store is unconditional on P.ok.
template <class C, int EK, class PixF>
__device__ __forceinline__ void epilogue_rb(const Params& p, const v4i (&acc)[C::TM][C::TN], const int (&sumq)[C::TN],
                                            PixF&& pixel, const int8_t* smem, int c0, int wm, int lane, int use_lut) {
  constexpr int BM = C::BM, TM = C::TM, TN = C::TN;
  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  const int g = lane >> 4;
  const int HoWo = d.ho * d.wo;
  const float* s_f = reinterpret_cast<const float*>(smem + p.epi_off);
  const int nparam = 7 * BM;
  const float* s_chain = s_f + (7 + e.nclass) * BM;
  const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
  const QParams c0p = make_qparams(e.code0_neg_min, e.code0_scale, e.code0_qmax);
  const QParams c1p = make_qparams(e.code1_neg_min, e.code1_scale, e.code1_qmax);
  // two consumers calibrated on the same tensor hold the same range: their codes are equal
  const bool same01 = e.out_code0 && e.code1_neg_min == e.code0_neg_min && e.code1_scale == e.code0_scale &&
                      e.code1_qmax == e.code0_qmax;
  const f2 bn_s2 = {e.bn_scale, e.bn_scale}, bn_m2 = {e.bn_min, e.bn_min};
  const bool has_res = EK == EK_GEN && e.residual != nullptr;
  const int nres = EK == EK_GEN ? e.nres : 0;
  const bool want_bn = EK == EK_BNCODE || (EK == EK_GEN && e.out_bncode);
  // EK_LUT is evaluated, not looked up: RangeBN -> ReLU -> the consumer's quantizer with
  // the ops qnn_bn_code_lut tabulates (graph.hip bn_apply + quant_code), so the codes are the
  // table's bitwise and no 256-byte-per-channel table is staged
  const bool bn_gen = (EK == EK_GEN || (EK == EK_LUT && !use_lut)) && e.bn_mean;
  const int8_t* s_lut = smem + p.epi_off + 4 * (7 + e.nclass) * BM;  // EK_LUT with use_lut: [BM][256]
  constexpr bool CACHE_BN = TM * TN <= 16 && TM <= 2;  // the RangeBN vectors stay in registers beside few accumulators
  // one pixel tile per lane (TN == 1): nothing to reuse, the channel vectors are read where used
  constexpr bool CACHE_W = TN > 1;

  float4 sw[TM], bw[TM], bi[TM], mn[TM], sq[TM], wq[TM], bq[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cl = wm * 16 * TM + 16 * i + 4 * g;
    if (CACHE_W) {
      sw[i] = *reinterpret_cast<const float4*>(s_f + cl);
      bw[i] = *reinterpret_cast<const float4*>(s_f + BM + cl);
      bi[i] = *reinterpret_cast<const float4*>(s_f + 2 * BM + cl);
    }
    if (CACHE_BN && bn_gen) {
      mn[i] = *reinterpret_cast<const float4*>(s_f + 3 * BM + cl);
      sq[i] = *reinterpret_cast<const float4*>(s_f + 4 * BM + cl);
      wq[i] = *reinterpret_cast<const float4*>(s_f + 5 * BM + cl);
      bq[i] = *reinterpret_cast<const float4*>(s_f + 6 * BM + cl);
    }
  }
  // EK_LUT, 64 channels per wave: the four 4-byte code words of a pixel (channels 16i + 4g..)
  // are transposed across the lane groups (two v_permlane32_swap + two v_permlane16_swap), so
  // lane group g holds the pixel's channels 16g..16g+15 and stores them as one 16-byte word
  const bool wide = EK == EK_LUT && TM == 4 && use_lut && c0 + wm * 64 + 64 <= d.cout &&
                    c0 + wm * 64 + 64 <= e.code0_cp;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    Pix P;
    int pc;
    pixel(j, P, pc);
    const int ptab = nparam + pc * BM;
    unsigned wrd[TM];  // the wide path's code words
    const f2 p2 = {(float)sumq[j], (float)sumq[j]};
    const int mc = P.m;  // a valid pixel (past-the-block slots hold the last one)
    // padded pixel index (its factors < 2^24: full-rate 24-bit multiplies) x cp, 64-bit
    const int64_t px0 = (int64_t)(__umul24(__umul24((unsigned)P.n, (unsigned)e.code0_hp) + (unsigned)(P.ho + e.code0_pad),
                                           (unsigned)e.code0_wp) + (unsigned)(P.wo + e.code0_pad)) * e.code0_cp;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cl = wm * 16 * TM + 16 * i + 4 * g;  // local channel of register 0
      const int c = c0 + cl;
      const bool cok = c < d.cout;                   // fused modes: cout % 16 == 0 (4-channel groups all in)
      const int cc = cok ? c : d.cout - 4;
      const float4 tb = *reinterpret_cast<const float4*>(s_f + ptab + cl);
      if (!CACHE_W) {
        sw[i] = *reinterpret_cast<const float4*>(s_f + cl);
        bw[i] = *reinterpret_cast<const float4*>(s_f + BM + cl);
        bi[i] = *reinterpret_cast<const float4*>(s_f + 2 * BM + cl);
      }
      const v4i& a = acc[i][j];
      const f2 a01 = {(float)a[0], (float)a[1]}, a23 = {(float)a[2], (float)a[3]};
      f2 v[2];
      v[0] = pfma((f2){sw[i].x, sw[i].y}, a01, pfma((f2){bw[i].x, bw[i].y}, p2, (f2){tb.x, tb.y})) + (f2){bi[i].x, bi[i].y};
      v[1] = pfma((f2){sw[i].z, sw[i].w}, a23, pfma((f2){bw[i].z, bw[i].w}, p2, (f2){tb.z, tb.w})) + (f2){bi[i].z, bi[i].w};
      if constexpr (EK == EK_NCHW) {  // drop-in QConv2d output, NCHW fp32
        {
          float* yp = e.out_f32 + ((int64_t)P.n * d.cout + c) * HoWo + P.ho * d.wo + P.wo;
          const float y4[4] = {v[0].x, v[0].y, v[1].x, v[1].y};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (c + r < d.cout) yp[(int64_t)r * HoWo] = y4[r];
#if QNN_RB_STORE_WAIT  // diagnostic build: every store has read its operands before the next instruction
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
          }
        }
        continue;
      }
      if (EK == EK_LUT && use_lut) {  // conv -> RangeBN -> ReLU -> consumer quantizer, tabulated
        const f2 q0 = qclamp2(v[0], bnp) + MAGIC_U8, q1 = qclamp2(v[1], bnp) + MAGIC_U8;
        const unsigned qq[4] = {__float_as_uint(q0.x) & 255u, __float_as_uint(q0.y) & 255u,
                                __float_as_uint(q1.x) & 255u, __float_as_uint(q1.y) & 255u};
        int rr = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) rr |= ((int)(uint8_t)s_lut[(cl + u) * 256 + qq[u]]) << (8 * u);
        if (wide) wrd[i] = (unsigned)rr;
        else if (c < e.code0_cp) *reinterpret_cast<int*>(e.out_code0 + px0 + c) = cok ? rr : 0;
        continue;
      }
      f2 qb[2];  // RangeBN input: clamped quotient (rounded below)
      if (EK == EK_BNCODE || bn_gen) {  // (EK_LUT: bn_gen)
        qb[0] = qclamp2(v[0], bnp);
        qb[1] = qclamp2(v[1], bnp);
      }
      if (want_bn && cok) {
        const int kb = pack4(qb[0] + MAGIC_U8, qb[1] + MAGIC_U8);
        if (e.bncode_tiled) *reinterpret_cast<int*>(e.out_bncode + btile_word(P.m, c, p.ct)) = kb;
        else *reinterpret_cast<int*>(e.out_bncode + (int64_t)P.m * d.cout + c) = kb;
      }
      if constexpr (EK == EK_GEN || EK == EK_LUT) {
        if (bn_gen) {
          float4 m4 = mn[i], s4 = sq[i], w4 = wq[i], b4 = bq[i];
          if constexpr (!CACHE_BN) {
            m4 = *reinterpret_cast<const float4*>(s_f + 3 * BM + cl);
            s4 = *reinterpret_cast<const float4*>(s_f + 4 * BM + cl);
            w4 = *reinterpret_cast<const float4*>(s_f + 5 * BM + cl);
            b4 = *reinterpret_cast<const float4*>(s_f + 6 * BM + cl);
          }
          const f2 mn2[2] = {{m4.x, m4.y}, {m4.z, m4.w}}, sq2[2] = {{s4.x, s4.y}, {s4.z, s4.w}};
          const f2 wq2[2] = {{w4.x, w4.y}, {w4.z, w4.w}}, bq2[2] = {{b4.x, b4.y}, {b4.z, b4.w}};
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            f2 o = rint2(qb[h]) * bn_s2;  // dequant: q * s
            o = o + bn_m2;                // + min
            o = o - mn2[h];               // x - mean
            o = o * sq2[h];               // * q(scale)
            o = o * wq2[h];               // * q(weight)
            v[h] = o + bq2[h];            // + q(bias)
          }
        }
        if (EK == EK_GEN && (has_res || nres > 0)) {
          // the block input: fp32, or recomputed from the chain exactly as its producers did
          auto link = [&](int l, f2 (&o)[2]) {  // g_l(q) (quantize.py:488-499 op order)
            const unsigned wd = *reinterpret_cast<const unsigned*>(e.res[l].code + btile_word(mc, cc, p.ct));
            const float* sp = s_chain + 4 * l * BM + cl;
            const float4 lm = *reinterpret_cast<const float4*>(sp);
            const float4 ls = *reinterpret_cast<const float4*>(sp + BM);
            const float4 lw = *reinterpret_cast<const float4*>(sp + 2 * BM);
            const float4 lb = *reinterpret_cast<const float4*>(sp + 3 * BM);
            const f2 s2 = {e.res[l].scale, e.res[l].scale}, m2 = {e.res[l].min, e.res[l].min};
            const f2 q[2] = {{(float)(wd & 255u), (float)((wd >> 8) & 255u)},
                             {(float)((wd >> 16) & 255u), (float)(wd >> 24)}};
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
          if (has_res) {
            const int64_t fi = e.f32_tiled ? ctile_index(mc, cc, p.ct) : (int64_t)mc * d.cout + cc;
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
        if (EK == EK_GEN && e.out_f32 && cok) {
          const int64_t fi = e.f32_tiled ? ctile_index(P.m, c, p.ct) : (int64_t)P.m * d.cout + c;
          *reinterpret_cast<float4*>(e.out_f32 + fi) = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
        }
        int k0 = 0;
        if (e.out_code0 && cok) k0 = pack4(qclamp2(v[0], c0p) + MAGIC_S8, qclamp2(v[1], c0p) + MAGIC_S8);
        if (e.out_code0 && c < e.code0_cp) *reinterpret_cast<int*>(e.out_code0 + px0 + c) = k0;
        if (EK == EK_GEN && e.out_code1 && c < e.code1_cp) {
          const int k1 = !cok ? 0 : same01 ? k0 : pack4(qclamp2(v[0], c1p) + MAGIC_S8, qclamp2(v[1], c1p) + MAGIC_S8);
          *reinterpret_cast<int*>(e.out_code1 + (((int64_t)P.n * e.code1_hp + P.ho + e.code1_pad) * e.code1_wp +
                                                 P.wo + e.code1_pad) * e.code1_cp + c) = k1;
        }
      }
    }
    if constexpr (EK == EK_LUT && TM == 4) {
      if (wide) {
        // M[g][i] = wrd[i] of lane group g.  permlane32_swap(r0, r2), (r1, r3) exchange the
        // upper groups of r0/r1 with the lower groups of r2/r3; permlane16_swap(r0, r1),
        // (r2, r3) then the odd groups of the first with the even groups of the second:
        // afterwards register k of group g holds M[k][g], i.e. channels 16g + 4k..
        const auto s02 = __builtin_amdgcn_permlane32_swap(wrd[0], wrd[2], false, false);
        const auto s13 = __builtin_amdgcn_permlane32_swap(wrd[1], wrd[3], false, false);
        const auto t01 = __builtin_amdgcn_permlane16_swap(s02[0], s13[0], false, false);
        const auto t23 = __builtin_amdgcn_permlane16_swap(s02[1], s13[1], false, false);
        *reinterpret_cast<v4i*>(e.out_code0 + px0 + c0 + wm * 64 + 16 * g) =
            (v4i){(int)t01[0], (int)t01[1], (int)t23[0], (int)t23[1]};
      }
    }
  }
}

}  // namespace q16
}  // namespace qnn
