// Depthwise QConv2d (groups == c, mobilenet_quantized.py:38-40) on v_mfma_i32_16x16x64_i8, with
// the exact decomposition every contraction kernel uses:
//   conv(x_hat, w_hat)[c, p] = s_x s_w[c] sum_t q'_t q'_w[c,t] + s_x b_w[c] sum_valid q'_t
//                              + b_x sum_valid w_hat[c, t]
// (the last term a per-(border class, channel) table, qnn_conv_border_table over the depthwise
// tap sums).  The reference evaluates F.conv2d(x_hat, w_hat, groups=c) in fp32; the exact
// integer sum is within the per-layer bar of it like every other conv (tests/test_gpu_parity.py
// depthwise cases), and the engine and the drop-in module both run this kernel, so they agree
// bitwise.
//
// The contraction as an MFMA: a block owns 16 channels c0..c0+15 and K = taps x 16 channels,
// tap-major, so a B-fragment lane (pixel l & 15, K bytes 16 (l >> 4)..+16 of a step) is one
// 16-byte load of one tap's 16 channels of one input pixel -- the padded NHWC8 codes as they lie
// -- and A is block-diagonal: row r holds q'_w[c0 + r, t] at K byte 16 t + r and zeros
// elsewhere (built in registers from the packed depthwise rows, one byte per tap).  A second
// MFMA against the block-diagonal of ones gives sum_valid q' per (channel, pixel).  One
// 16x16 tile is 3 + 3 MFMAs for 256 outputs (15/16 of the A operand is zeros: the MFMA pipe
// still does it in a fraction of the time the per-output VALU needed for the nine fp32 FMAs
// and their dequantisations, csrc/graph.hip dwconv3_kernel).
// Epilogues: EK_NCHW (the drop-in module's fp32 NCHW output) and EK_LUT (RangeBN -> ReLU ->
// the pointwise consumer's quantizer as the per-channel code table, codes out: the engine).
#include <map>
#include <mutex>
#include <utility>

#include "qconv_common.h"

namespace qnn {
namespace dwm {

constexpr int W = 4, NT = 64 * W, CB = 16;
constexpr int KS_MAX = 4;  // taps <= 16 (3x3: 3 K steps)

// FDIV: output pixels < 2^24, decoded by float reciprocals with an exact fix-up; else integer
// division (ResNet-scale batches of the 112x112 layers)
template <int TN, int KS, int EK, bool FDIV>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2))) void qconv_dw_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ wq, const Params p) {
  constexpr int BN = W * TN * 16;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // block -> (channel tile, first pixel tile), persistent over pixel tiles; with the grid a
  // multiple of 8 * nby the blocks of one pixel slot share an XCD (its input rows' L2)
  const int nby = d.cout / CB, G = gridDim.x, b = blockIdx.x;
  const int pstep = G / nby, npt = (p.M + BN - 1) / BN;
  int cty, pt;
  if (G % (8 * nby) == 0) {
    const int q = b >> 3;
    cty = q % nby;
    pt = (q / nby) * 8 + (b & 7);
  } else {
    cty = b % nby;
    pt = b / nby;
  }
  const int c0 = cty * CB, c = c0 + 4 * g;  // this lane's accumulator channels c..c+3

  // LDS: border table rows of the block's channels [nclass][16] f32, the classes of each row /
  // column, (EK_LUT) the code table [16][256]
  float* s_tab = reinterpret_cast<float*>(smem);
  int* s_hc = reinterpret_cast<int*>(smem + 4 * CB * e.nclass);
  int8_t* s_lut = smem + 4 * CB * e.nclass + 4 * ((d.ho + d.wo + 3) & ~3);
  for (int i = tid; i < CB * e.nclass; i += NT) s_tab[i] = e.table[(int64_t)(i >> 4) * d.cout + c0 + (i & 15)];
  for (int i = tid; i < d.ho + d.wo; i += NT) s_hc[i] = i < d.ho ? e.hcls[i] * e.nwc : e.wcls[i - d.ho];
  if constexpr (EK == EK_LUT)
    for (int i = 16 * tid; i < CB * 256; i += 16 * NT)
      *reinterpret_cast<uint4*>(s_lut + i) = *reinterpret_cast<const uint4*>(e.lut + (int64_t)c0 * 256 + i);

  // A (block-diagonal weights, ones) and the B tap offsets of this lane's K chunks: step s,
  // chunk g = tap 4s + g (taps past kh*kw: zero weights, the zero page)
  v4i fa[KS], fo[KS];
  int doff[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int t = 4 * s + g;
    const bool real = t < p.taps;
    const int tr = t / d.kw, tc = t - tr * d.kw;
    doff[s] = real ? (tr * d.wp + tc) * d.cp + c0 : -1;
    const uint32_t wb = real ? (uint32_t)(uint8_t)wq[(int64_t)(c0 + r) * d.kpad + 16 * t] : 0u;
    v4i a = {0, 0, 0, 0}, o = {0, 0, 0, 0};
    a[r >> 2] = (int)(wb << (8 * (r & 3)));
    o[r >> 2] = real ? (int)(1u << (8 * (r & 3))) : 0;
    fa[s] = a, fo[s] = o;
  }
  const float4 sw = *reinterpret_cast<const float4*>(e.sxsw + c);
  const float4 bw = *reinterpret_cast<const float4*>(e.sxbw + c);
  const float4 bi = e.bias ? *reinterpret_cast<const float4*>(e.bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
  const int HoWo = d.ho * d.wo;
  const float inv_hw = 1.0f / (float)HoWo, inv_wo = 1.0f / (float)d.wo;
  auto divmod = [&](int m, int D, float invD, int& q, int& rm) __attribute__((always_inline)) {
    if constexpr (FDIV) {  // m < 2^24: the float quotient is off by at most one, fixed up exactly
      q = (int)((float)m * invD);
      rm = m - (int)__umul24((unsigned)q, (unsigned)D);
      if (rm < 0) --q, rm += D;
      if (rm >= D) ++q, rm -= D;
    } else {
      q = m / D, rm = m - q * D;
    }
  };
  struct Tile {
    v4i fb[KS][TN];
    int pn[TN], pho[TN], pwo[TN];
  };
  auto load_t = [&](int t, Tile& T) __attribute__((always_inline)) {
    t = t < npt ? t : npt - 1;  // a prefetch past the last tile re-reads it
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int m = t * BN + (wave * TN + j) * 16 + r;
      m = m < p.M ? m : p.M - 1;  // past the batch: the last pixel (its values re-stored)
      int n, hw, ho, wo;
      divmod(m, HoWo, inv_hw, n, hw);
      divmod(hw, d.wo, inv_wo, ho, wo);
      T.pn[j] = n, T.pho[j] = ho, T.pwo[j] = wo;
      // padded pixel index x cp < 2^31 and its factors < 2^24 (host): 24-bit multiplies
      const int base = (int)__umul24(__umul24(__umul24((unsigned)n, (unsigned)d.hp) + __umul24((unsigned)ho, (unsigned)d.sh),
                                              (unsigned)d.wp) +
                                         __umul24((unsigned)wo, (unsigned)d.sw),
                                     (unsigned)d.cp);
#pragma unroll
      for (int s = 0; s < KS; ++s)
        T.fb[s][j] = *reinterpret_cast<const v4i*>(x + (doff[s] >= 0 ? base + doff[s] : d.zero_off));
    }
  };
  Tile ta, tb;
  load_t(pt, ta);
  __syncthreads();

  auto step = [&](Tile& C, Tile& N) __attribute__((always_inline)) {
    load_t(pt + pstep, N);  // lands under this tile's epilogue
    v4i acc[TN], sacc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = sacc[j] = (v4i){0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s], C.fb[s][j], acc[j], 0, 0, 0);
        sacc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fo[s], C.fb[s][j], sacc[j], 0, 0, 0);
      }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int m = pt * BN + (wave * TN + j) * 16 + r;
      const int n = C.pn[j], ho = C.pho[j], wo = C.pwo[j];
      const int pc = s_hc[ho] + s_hc[d.ho + wo];
      const float4 tb4 = *reinterpret_cast<const float4*>(s_tab + pc * CB + 4 * g);
      // the exact decomposition, conv_out4's op order, sum_valid q' per channel
      float v[4];
      const float sw_[4] = {sw.x, sw.y, sw.z, sw.w}, bw_[4] = {bw.x, bw.y, bw.z, bw.w};
      const float tb_[4] = {tb4.x, tb4.y, tb4.z, tb4.w}, bi_[4] = {bi.x, bi.y, bi.z, bi.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = fmaf(sw_[u], (float)acc[j][u], fmaf(bw_[u], (float)sacc[j][u], tb_[u])) + bi_[u];
      if constexpr (EK == EK_NCHW) {
        if (m < p.M) {
          float* yp = e.out_f32 + ((int64_t)n * d.cout + c) * HoWo + ho * d.wo + wo;
#pragma unroll
          for (int u = 0; u < 4; ++u) yp[(int64_t)u * HoWo] = v[u];
        }
      } else {  // EK_LUT: RangeBN's input code (low byte of the magic-shifted quotient), the table
        const f2 q0 = qclamp2((f2){v[0], v[1]}, bnp) + MAGIC_U8, q1 = qclamp2((f2){v[2], v[3]}, bnp) + MAGIC_U8;
        const int8_t* lp = s_lut + 4 * g * 256;
        const uint32_t k0 = (uint8_t)lp[__float_as_uint(q0.x) & 255u];
        const uint32_t k1 = (uint8_t)lp[256 + (__float_as_uint(q0.y) & 255u)];
        const uint32_t k2 = (uint8_t)lp[512 + (__float_as_uint(q1.x) & 255u)];
        const uint32_t k3 = (uint8_t)lp[768 + (__float_as_uint(q1.y) & 255u)];
        const unsigned px = __umul24(__umul24((unsigned)n, (unsigned)e.code0_hp) + (unsigned)(ho + e.code0_pad),
                                     (unsigned)e.code0_wp) + (unsigned)(wo + e.code0_pad);
        *reinterpret_cast<uint32_t*>(e.out_code0 + (int)(px * (unsigned)e.code0_cp) + c) = k0 | (k1 << 8) | (k2 << 16) | (k3 << 24);
      }
    }
    pt += pstep;
  };
  while (pt < npt) {
    step(ta, tb);
    if (pt >= npt) break;
    step(tb, ta);
  }
}

static int lds_bytes(const Params& p, int ek) {
  return 4 * CB * p.e.nclass + 4 * ((p.d.ho + p.d.wo + 3) & ~3) + (ek == EK_LUT ? CB * 256 : 0);
}

static int blocks_per_cu(const void* kern, int lds) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_pair(kern, lds);
  const auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, NT, lds) != hipSuccess || n < 1) n = 1;
  cache.emplace(key, n);
  return n;
}

template <int TN, int KS, int EK>
static int launch(const int8_t* x, const int8_t* wq, const Params& p, hipStream_t s) {
  auto kern = p.M < (1 << 24) ? qconv_dw_kernel<TN, KS, EK, true> : qconv_dw_kernel<TN, KS, EK, false>;
  const int lds = lds_bytes(p, EK);
  if (lds > 64 * 1024) return arg_error("depthwise: too many border classes");
  const int per_cu = blocks_per_cu((const void*)kern, lds);
  const int64_t nby = p.d.cout / CB, tiles = cdiv(p.M, W * TN * 16) * nby;
  int64_t nblk = (int64_t)device_cu_count() * per_cu;
  nblk = nblk % (8 * nby) == 0 ? nblk : (nblk / nby) * nby;  // XCD-grouped when it divides
  nblk = nblk < nby ? nby : nblk;
  if (nblk > tiles) nblk = tiles;
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(NT), lds, s, x, wq, p);
  return QNN_OK;
}

template <int EK>
static int launch_k(const int8_t* x, const int8_t* wq, const Params& p, hipStream_t s) {
  switch ((p.taps + 3) >> 2) {
    case 1: return launch<4, 1, EK>(x, wq, p, s);
    case 2: return launch<4, 2, EK>(x, wq, p, s);
    case 3: return launch<4, 3, EK>(x, wq, p, s);
    default: return launch<2, 4, EK>(x, wq, p, s);
  }
}

}  // namespace dwm
}  // namespace qnn

using namespace qnn;

extern "C" int qnn_dwconv_mfma_fwd(const int8_t* x, const int8_t* wq, const qnn_conv_desc* desc,
                                   const qnn_epilogue* epi, qnn_stream_t stream) {
  QNN_REQUIRE(desc && epi, "null descriptor");
  const qnn_conv_desc& d = *desc;
  const qnn_epilogue& e = *epi;
  QNN_REQUIRE(d.n >= 0 && d.cout > 0 && d.cout % dwm::CB == 0 && d.cp >= d.cout && d.cp % 16 == 0 && d.kh > 0 &&
                  d.kw > 0 && d.kh * d.kw <= 4 * dwm::KS_MAX && d.sh > 0 && d.sw > 0 && d.ho > 0 && d.wo > 0,
              "depthwise: 16-channel groups, cp % 16 == 0, at most 16 taps");
  QNN_REQUIRE((d.ho - 1) * d.sh + d.kh <= d.hp && (d.wo - 1) * d.sw + d.kw <= d.wp, "ho/wo exceed the padded input");
  QNN_REQUIRE(d.kpad >= 16 * d.kh * d.kw && d.cout_pad >= d.cout && d.zero_off >= 0 && d.zero_off % 16 == 0,
              "depthwise weights: rows of kpad >= 16 * taps bytes (qnn_pack_weight_i8, cin 1)");
  QNN_REQUIRE(!d.kmask, "depthwise: no K mask");
  QNN_REQUIRE(e.nclass > 0 && e.nclass <= MAX_CLASSES && e.nwc > 0, "border classes out of range");
  const int64_t M = (int64_t)d.n * d.ho * d.wo;
  QNN_REQUIRE(M < (1LL << 31) && (int64_t)d.n * d.hp * d.wp * d.cp < (1LL << 31) && (int64_t)d.n * d.hp < (1 << 24) &&
                  (int64_t)d.n * d.hp * d.wp < (1 << 24) && d.cp < (1 << 24),
              "depthwise too large");
  const bool lut = e.mode == 1;
  if (lut)
    QNN_REQUIRE(e.lut && e.out_code0 && e.bn_scale > 0.f && !e.out_f32 && !e.out_code1 && !e.out_bncode && !e.residual &&
                    e.nres == 0 && e.code0_cp >= d.cout && e.code0_cp % 4 == 0 &&
                    (int64_t)d.n * e.code0_hp * e.code0_wp * e.code0_cp < (1LL << 31) && (int64_t)d.n * e.code0_hp < (1 << 24) &&
                    (((uintptr_t)e.lut) & 15) == 0,
                "depthwise mode 1: the RangeBN -> ReLU -> consumer code table (lut) and one code output only");
  else
    QNN_REQUIRE(e.mode == 0 && e.out_f32, "depthwise: mode 0 (NCHW fp32 out) or mode 1 (lut codes)");
  if (d.n == 0) return QNN_OK;
  QNN_REQUIRE(x && wq && e.sxsw && e.sxbw && e.table && e.hcls && e.wcls, "null pointer");
  QNN_REQUIRE((((uintptr_t)x) & 15) == 0 && (((uintptr_t)e.sxsw) & 15) == 0 && (((uintptr_t)e.sxbw) & 15) == 0 &&
                  (!e.bias || (((uintptr_t)e.bias) & 15) == 0),
              "depthwise: 16-byte aligned codes and channel vectors");
  Params p{};
  p.d = d;
  p.e = e;
  p.M = (int)M;
  p.taps = d.kh * d.kw;
  p.ct = (int)cdiv(d.cout, 32);
  const int rc = lut ? dwm::launch_k<EK_LUT>(x, wq, p, (hipStream_t)stream)
                     : dwm::launch_k<EK_NCHW>(x, wq, p, (hipStream_t)stream);
  if (rc != QNN_OK) return rc;
  QNN_LAUNCH_CHECK("qnn_dwconv_mfma_fwd");
  return QNN_OK;
}
