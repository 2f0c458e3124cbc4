// Depthwise QConv2d (groups == c, mobilenet_quantized.py:38-40) on v_mfma_i32_16x16x64_i8 over
// an LDS-staged band of input rows, with the exact decomposition every contraction kernel uses
// (SURVEY.md §0.5):
//   conv(x_hat, w_hat)[c, p] = s_x s_w[c] sum_t q'_t q'_w[c,t] + s_x b_w[c] sum_valid q'_t
//                              + b_x sum_valid w_hat[c, t]
// (the last term a per-(border class, channel) table, qnn_conv_border_table over the depthwise
// tap sums).  The reference evaluates F.conv2d(x_hat, w_hat, groups=c) in fp32; the exact
// integer sum is within the per-layer bar of it like every other conv, and the engine and the
// drop-in module both run this kernel, so they agree bitwise.
//
// A block owns 16 channels c0..c0+15 and walks bands of R output rows of one image: the band's
// padded input rows ((R-1) S + kh of them, every column, the block's 16 channels: 16 bytes per
// pixel) are staged in LDS once, then every output pixel's taps are read from there.  The
// contraction is an MFMA with K = taps x 16 channels, tap-major: a B-fragment lane (pixel l & 15,
// K chunk l >> 4 of a step = one tap) is one ds_read_b128 of that tap's 16 channels, and A is
// block-diagonal -- row r holds q'_w[c0 + r, t] at K byte 16 t + r, zeros elsewhere, built in
// registers once per block -- with a second MFMA against the block-diagonal of ones for
// sum_valid q' per (channel, pixel).  A 16x16 tile is 2 KS MFMAs for 256 outputs.
// (Round 4 first fetched each tap's 16 bytes from global memory per output pixel: every input
// byte crossed L1/L2 nine times and the layer ran 1.4x slower than the fp32 kernel; the band
// reads each input byte from HBM once per (R - 1) S + kh rows / R S.)
// Epilogues: EK_NCHW (the drop-in module's fp32 NCHW output) and EK_LUT (RangeBN -> ReLU ->
// the pointwise consumer's quantizer as the per-channel code table, codes out: the engine).
#include <map>
#include <mutex>
#include <utility>

#include "qconv_common.h"

namespace qnn {
namespace dwb {

constexpr int W = 4, NT = 64 * W, CB = 16;
constexpr int KS_MAX = 4;  // taps <= 16 (3x3: 3 K steps)

template <int KS, int EK>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2))) void qconv_dwb_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ wq, const Params p, int R) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int nby = d.cout / CB;
  const int cg = blockIdx.x % nby, c0 = cg * CB, c = c0 + 4 * g;  // this lane's channels c..c+3
  const int bstep = gridDim.x / nby;
  const int nbr = (d.ho + R - 1) / R, nbands = d.n * nbr;
  const int rows_in = (R - 1) * d.sh + d.kh;      // padded input rows of a band
  const int npx = R * d.wo, ntile = (npx + 15) >> 4;  // output pixels / 16-pixel tiles of a band

  // LDS: the band [rows_in][wp][16] bytes, the border table rows of the block's channels
  // [nclass][16] f32, the classes of each output row / column, (EK_LUT) the code table [16][256]
  int8_t* s_band = smem;
  const int band_bytes = rows_in * d.wp * 16;
  float* s_tab = reinterpret_cast<float*>(smem + band_bytes);
  int* s_hc = reinterpret_cast<int*>(smem + band_bytes + 4 * CB * e.nclass);
  int8_t* s_lut = smem + band_bytes + 4 * CB * e.nclass + 4 * ((d.ho + d.wo + 3) & ~3);
  for (int i = tid; i < CB * e.nclass; i += NT) s_tab[i] = e.table[(int64_t)(i >> 4) * d.cout + c0 + (i & 15)];
  for (int i = tid; i < d.ho + d.wo; i += NT) s_hc[i] = i < d.ho ? e.hcls[i] * e.nwc : e.wcls[i - d.ho];
  if constexpr (EK == EK_LUT)
    for (int i = 16 * tid; i < CB * 256; i += 16 * NT)
      *reinterpret_cast<uint4*>(s_lut + i) = *reinterpret_cast<const uint4*>(e.lut + (int64_t)c0 * 256 + i);

  // A (block-diagonal weights, ones) and this lane's tap offsets in the band: step s, chunk g =
  // tap 4s + g (taps past kh*kw: zero weights, any in-band bytes)
  v4i fa[KS], fo[KS];
  int toff[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int t = 4 * s + g;
    const bool real = t < p.taps;
    const int tr = t / d.kw, tc = t - tr * d.kw;
    toff[s] = real ? (tr * d.wp + tc) * 16 : 0;
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
  const float inv_wo = 1.0f / (float)d.wo;

  for (int bd = blockIdx.x / nby; bd < nbands; bd += bstep) {
    const int n = bd / nbr, r0 = (bd - n * nbr) * R;  // image, first output row
    // ---- stage the band: padded input rows r0 S .. r0 S + rows_in - 1 of image n (clamped to
    // the buffer: rows past ho feed only pixels never stored), 16 bytes per pixel
    __syncthreads();  // the previous band's readers are done
    const int8_t* src0 = x + (int64_t)n * d.hp * d.wp * d.cp + c0;
    for (int i = tid; i < rows_in * d.wp; i += NT) {
      const int br = i / d.wp, col = i - br * d.wp;
      int row = r0 * d.sh + br;
      row = row < d.hp ? row : d.hp - 1;
      *reinterpret_cast<v4i*>(s_band + 16 * i) = *reinterpret_cast<const v4i*>(src0 + ((int64_t)row * d.wp + col) * d.cp);
    }
    __syncthreads();
    const int rows_out = d.ho - r0 < R ? d.ho - r0 : R;
    const int npx_b = rows_out * d.wo;
    for (int t = wave; t < ntile; t += W) {
      int q = 16 * t + r;
      const bool ok = q < npx_b;
      q = ok ? q : npx_b - 1;  // past the band: its last pixel (not stored)
      int rr = (int)((float)q * inv_wo), oc = q - rr * d.wo;  // q < 2^24: exact after the fix-up
      if (oc < 0) --rr, oc += d.wo;
      if (oc >= d.wo) ++rr, oc -= d.wo;
      const int base = ((rr * d.sh) * d.wp + oc * d.sw) * 16;
      v4i acc = {0, 0, 0, 0}, sacc = {0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const v4i fb = *reinterpret_cast<const v4i*>(s_band + base + toff[s]);
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s], fb, acc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_i32_16x16x64_i8(fo[s], fb, sacc, 0, 0, 0);
      }
      const int ho = r0 + rr, wo = oc;
      const int pc = s_hc[ho] + s_hc[d.ho + wo];
      const float4 tb4 = *reinterpret_cast<const float4*>(s_tab + pc * CB + 4 * g);
      // the exact decomposition, conv_out4's op order, sum_valid q' per channel
      float v[4];
      const float sw_[4] = {sw.x, sw.y, sw.z, sw.w}, bw_[4] = {bw.x, bw.y, bw.z, bw.w};
      const float tb_[4] = {tb4.x, tb4.y, tb4.z, tb4.w}, bi_[4] = {bi.x, bi.y, bi.z, bi.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = fmaf(sw_[u], (float)acc[u], fmaf(bw_[u], (float)sacc[u], tb_[u])) + bi_[u];
      if (!ok) continue;
      if constexpr (EK == EK_NCHW) {
        float* yp = e.out_f32 + ((int64_t)n * d.cout + c) * HoWo + ho * d.wo + wo;
#pragma unroll
        for (int u = 0; u < 4; ++u) yp[(int64_t)u * HoWo] = v[u];
      } else {  // EK_LUT: RangeBN's input code (low byte of the magic-shifted quotient), the table
        const f2 q0 = qclamp2((f2){v[0], v[1]}, bnp) + MAGIC_U8, q1 = qclamp2((f2){v[2], v[3]}, bnp) + MAGIC_U8;
        const int8_t* lp = s_lut + 4 * g * 256;
        const uint32_t k0 = (uint8_t)lp[__float_as_uint(q0.x) & 255u];
        const uint32_t k1 = (uint8_t)lp[256 + (__float_as_uint(q0.y) & 255u)];
        const uint32_t k2 = (uint8_t)lp[512 + (__float_as_uint(q1.x) & 255u)];
        const uint32_t k3 = (uint8_t)lp[768 + (__float_as_uint(q1.y) & 255u)];
        const int px = ((n * e.code0_hp + ho + e.code0_pad) * e.code0_wp + wo + e.code0_pad);
        *reinterpret_cast<uint32_t*>(e.out_code0 + (int64_t)px * e.code0_cp + c) = k0 | (k1 << 8) | (k2 << 16) | (k3 << 24);
      }
    }
  }
}

// output rows per band: about 512 output pixels (32 tiles, 8 per wave), at most the image
static int band_rows(const qnn_conv_desc& d) {
  int R = 512 / d.wo;
  R = R < 1 ? 1 : R;
  return R > d.ho ? d.ho : R;
}

static int lds_bytes(const Params& p, int ek, int R) {
  const int rows_in = (R - 1) * p.d.sh + p.d.kh;
  return rows_in * p.d.wp * 16 + 4 * CB * p.e.nclass + 4 * ((p.d.ho + p.d.wo + 3) & ~3) + (ek == EK_LUT ? CB * 256 : 0);
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

template <int KS, int EK>
static int launch(const int8_t* x, const int8_t* wq, const Params& p, hipStream_t s) {
  auto kern = qconv_dwb_kernel<KS, EK>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  int R = band_rows(p.d);
  while (R > 1 && lds_bytes(p, EK, R) > 64 * 1024) --R;
  const int lds = lds_bytes(p, EK, R);
  if (lds > LDS_MAX) return arg_error("depthwise: the input band does not fit LDS");
  const int per_cu = blocks_per_cu((const void*)kern, lds);
  const int64_t nby = p.d.cout / CB, nbands = (int64_t)p.d.n * cdiv(p.d.ho, R);
  int64_t slots = (int64_t)device_cu_count() * per_cu / nby;  // persistent: band slots per channel group
  slots = slots < 1 ? 1 : slots;
  slots = slots < nbands ? slots : nbands;
  hipLaunchKernelGGL(kern, dim3((unsigned)(slots * nby)), dim3(NT), lds, s, x, wq, p, R);
  return QNN_OK;
}

template <int EK>
static int launch_k(const int8_t* x, const int8_t* wq, const Params& p, hipStream_t s) {
  switch ((p.taps + 3) >> 2) {
    case 1: return launch<1, EK>(x, wq, p, s);
    case 2: return launch<2, EK>(x, wq, p, s);
    case 3: return launch<3, EK>(x, wq, p, s);
    default: return launch<4, EK>(x, wq, p, s);
  }
}

}  // namespace dwb
}  // namespace qnn

using namespace qnn;

extern "C" int qnn_dwconv_mfma_fwd(const int8_t* x, const int8_t* wq, const qnn_conv_desc* desc,
                                   const qnn_epilogue* epi, qnn_stream_t stream) {
  QNN_REQUIRE(desc && epi, "null descriptor");
  const qnn_conv_desc& d = *desc;
  const qnn_epilogue& e = *epi;
  QNN_REQUIRE(d.n >= 0 && d.cout > 0 && d.cout % dwb::CB == 0 && d.cp >= d.cout && d.cp % 16 == 0 && d.kh > 0 &&
                  d.kw > 0 && d.kh * d.kw <= 4 * dwb::KS_MAX && d.sh > 0 && d.sw > 0 && d.ho > 0 && d.wo > 0,
              "depthwise: 16-channel groups, cp % 16 == 0, at most 16 taps");
  QNN_REQUIRE((d.ho - 1) * d.sh + d.kh <= d.hp && (d.wo - 1) * d.sw + d.kw <= d.wp, "ho/wo exceed the padded input");
  QNN_REQUIRE(d.kpad >= 16 * d.kh * d.kw && d.cout_pad >= d.cout && d.zero_off >= 0 && d.zero_off % 16 == 0,
              "depthwise weights: rows of kpad >= 16 * taps bytes (qnn_pack_weight_i8, cin 1)");
  QNN_REQUIRE(!d.kmask, "depthwise: no K mask");
  QNN_REQUIRE(e.nclass > 0 && e.nclass <= MAX_CLASSES && e.nwc > 0, "border classes out of range");
  const int64_t M = (int64_t)d.n * d.ho * d.wo;
  QNN_REQUIRE(M < (1LL << 31) && (int64_t)d.hp * d.wp * d.cp < (1LL << 31), "depthwise too large");
  const bool lut = e.mode == 1;
  if (lut)
    QNN_REQUIRE(e.lut && e.out_code0 && e.bn_scale > 0.f && !e.out_f32 && !e.out_code1 && !e.out_bncode && !e.residual &&
                    e.nres == 0 && e.code0_cp >= d.cout && e.code0_cp % 4 == 0 &&
                    (int64_t)d.n * e.code0_hp * e.code0_wp < (1LL << 31) &&
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
  const int rc = lut ? dwb::launch_k<EK_LUT>(x, wq, p, (hipStream_t)stream)
                     : dwb::launch_k<EK_NCHW>(x, wq, p, (hipStream_t)stream);
  if (rc != QNN_OK) return rc;
  QNN_LAUNCH_CHECK("qnn_dwconv_mfma_fwd");
  return QNN_OK;
}
