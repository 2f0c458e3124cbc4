// Direct-fragment int8 convolution on v_mfma_i32_16x16x64_i8 for SHORT reductions (kpad <=
// 256: the space-to-depth stems -- ResNet 7x7/s2 = 4x4 taps x 16 channels, MobileNet 3x3/s2 =
// 2x2 taps x 16 channels -- and the narrow 1x1s), the eval forward of QConv2d
// (models/modules/quantize.py:314-349) with the exact decomposition and epilogue arithmetic
// of every other kernel family, so its outputs are bitwise theirs.
//
// With K this short there is nothing to stage: the work is the epilogue and the output
// bytes.  So no LDS ring, no band and no K-loop barrier:
// * B: a 16x16x64 fragment lane (pixel l&15, K bytes 16*(l>>4)..+16) IS one 16-byte chunk of
//   one tap of one input pixel (K is tap-major, cp bytes per tap): a single global load per
//   fragment, straight from the padded NHWC codes (the taps' overlap hits L1/L2).
// * A: the packed weight rows, one 16-byte load per 16-channel tile per K step (a few KiB
//   shared by every block: L2/L1-resident).
// * sum_valid(q'_x): one more MFMA per fragment against an all-ones A (the K mask's bytes for
//   the space-to-depth stems), so every lane gets its pixel's sum in int32, exactly.
// * The block's CB channels are all of a small cout (32 or 64): no wasted MFMA rows, and the
//   epilogue (q16::epilogue_rb: registers-resident channel parameters, LDS code table) is
//   spread over 4 waves x TN 16-pixel tiles with several blocks resident per CU.
#include <map>
#include <mutex>
#include <utility>

#include "qconv_common.h"
#include "epi16.h"

#ifndef QNN_ABLATE
#define QNN_ABLATE 0  // diagnostic builds only: 1 no B loads, 2 no MFMA, 3 no epilogue
#endif

namespace qnn {
namespace dk {

// 4 waves side by side along the pixels; each owns all TM 16-channel tiles of its TN
// 16-pixel tiles.  CB channels per block; BM = max(CB, 64) is the stride of the staged epilogue
// vectors (stage_epi moves 64 floats per DMA; channels past the block's CB are staged, unused).
// (WGM, BPC: the members stage_epi / epilogue_rb expect.)
template <int TM_, int TN_, bool K576_ = false, bool PF_ = true>
struct Cfg {
  static constexpr int WGM = 1, WGN = 4, TM = TM_, TN = TN_, BPC = 1;
  static constexpr bool K576 = K576_;  // built for exactly nine K steps (3x3 on 64 channels)
  static constexpr bool PF = PF_;      // prefetch the next tile's fragments under this one's work
  static constexpr int W = WGM * WGN, NT = 64 * W;
  static constexpr int CB = TM * 16, BM = CB < 64 ? 64 : CB, BN = WGN * TN * 16;
  static_assert(CB <= BM, "channel tile wider than the staging stride");
};

constexpr int KPAD_MAX = 256;  // configurations 0-2
constexpr int KS_3X3 = 9;      // configurations 3-4: the 3x3 layers on 64 input channels (K = 576)

// q = m / D, r = m % D for 0 <= m < 2^24 (checked on the host): the float quotient is off by
// at most one, fixed up exactly -- a few VALU ops where an integer division costs ~40
__device__ __forceinline__ void fdivmod(int m, int D, float invD, int& q, int& r) {
  q = (int)((float)m * invD);
  r = m - (int)__umul24((unsigned)q, (unsigned)D);  // q, D < 2^24: the full-rate 24-bit multiply
  if (r < 0) --q, r += D;
  if (r >= D) ++q, r -= D;
}

// the register budget: two waves per SIMD (256 VGPRs).  With one (the budget of the prefetching
// configurations until round 5) the 1x1 code-table launches took 180 VGPRs + 32 AGPRs -- two
// waves resident anyway -- where two fit them in 147, three resident: MobileNet b512 in-graph
// contractions 1.474-1.476 -> 1.41-1.44 ms, ResNet-18 b128 unchanged (gpurun_out/dkw A/B).
#ifndef QNN_DK_WPE
#define QNN_DK_WPE 2
#endif
template <class C, int EK, bool MASKED, int KS>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(QNN_DK_WPE))) void qconv_direct_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ w,
                                                            const Params p) {
  constexpr int TM = C::TM, TN = C::TN, CB = C::CB, BN = C::BN;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // persistent: block b owns one channel tile and pixel tiles pt0 + k * (grid / nby).  With the
  // grid a multiple of 8 * nby, block b sits on XCD b % 8 and the nby blocks of each pixel tile
  // stream (b = 8 (q nby + cty) + x) share one XCD, so a pixel tile's input codes are fetched into
  // one L2 once for all its channel tiles (qconv_dtab_kernel's mapping); else b % nby, b / nby
  const int nby = (d.cout + CB - 1) / CB;
  const int pstep = gridDim.x / nby, npt = (p.M + BN - 1) / BN;
  int cty, pt0;
  {
    const int G = gridDim.x, b = blockIdx.x;
    if (G % (8 * nby) == 0) {
      const int r = b >> 3;
      cty = r % nby;
      pt0 = (r / nby) * 8 + (b & 7);
    } else {
      cty = b % nby;
      pt0 = b / nby;
    }
  }
  const int c0 = cty * CB;

  // the epilogue's data by LDS-DMA, once per block
  stage_epi<C, EK>(p, x, smem, c0, wave, lane);

  // this lane's 16-byte K chunk of step s: tap u / cpg, channels 16 * (u % cpg), u = 4s + g;
  // chunks past the taps read the zero page (their weights are zero)
  const int cpg = d.cp >> 4, kreal = p.taps * cpg;
  int doff[KS];
  v4i fa[KS][TM], ones[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int u = 4 * s + g;
    const int tap = u / cpg, tr = tap / d.kw, tc = tap - tr * d.kw;
    doff[s] = u < kreal ? (tr * d.wp + tc) * d.cp + 16 * (u - tap * cpg) : -1;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int row = c0 + 16 * i + (lane & 15);
      row = row < d.cout_pad ? row : d.cout_pad - 1;
      fa[s][i] = *reinterpret_cast<const v4i*>(w + (int64_t)row * d.kpad + 64 * s + 16 * g);
    }
    if constexpr (MASKED) ones[s] = *reinterpret_cast<const v4i*>(d.kmask + 64 * s + 16 * g);
    else ones[s] = (v4i){0x01010101, 0x01010101, 0x01010101, 0x01010101};
  }

  const int HoWo = d.ho * d.wo;
  const float inv_hw = 1.0f / (float)HoWo, inv_wo = 1.0f / (float)d.wo;
  auto decode = [&](int m, int& n, int& ho, int& wo) {
    int hw;
    fdivmod(m, HoWo, inv_hw, n, hw);
    fdivmod(hw, d.wo, inv_wo, ho, wo);
  };
  // B fragments of pixel tile pt (clamped: a prefetch past the last tile re-reads it;
  // pixels past the batch stand in for the last one, whose values they re-store)
  // (also keeps each pixel's (n, ho, wo) for the epilogue of that tile)
  const int lgcp = 4 + p.lgcpt;  // cp = 16 << lgcpt
  auto load_b = [&](int pt, v4i (&fb)[KS][TN], int (&pn)[TN], int (&pho)[TN], int (&pwo)[TN]) {
    pt = pt < npt ? pt : npt - 1;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int m = pt * BN + (wave * TN + j) * 16 + (lane & 15);
      m = m < p.M ? m : p.M - 1;
      int n, ho, wo;
      decode(m, n, ho, wo);
      pn[j] = n, pho[j] = ho, pwo[j] = wo;
      // padded pixel index < 2^31 / cp, its factors < 2^24: 24-bit multiplies, then the cp shift
      const int base = (int)(__umul24(__umul24((unsigned)n, (unsigned)d.hp) + (unsigned)(ho * d.sh), (unsigned)d.wp) +
                             (unsigned)(wo * d.sw)) << lgcp;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (QNN_ABLATE == 1) fb[s][j] = (v4i){base, s, 1, 2};
        else fb[s][j] = *reinterpret_cast<const v4i*>(x + (doff[s] >= 0 ? base + doff[s] : d.zero_off));
      }
    }
  };
  v4i fnx[KS][TN];
  int nn[TN], nho[TN], nwo[TN];
  int pt = pt0;
  if constexpr (C::PF) load_b(pt, fnx, nn, nho, nwo);
  // border classes in LDS past the epilogue data: hcls[ho] * nwc, then wcls[wo]
  int* s_hc = reinterpret_cast<int*>(smem + p.scr_off);
  for (int i = tid; i < d.ho + d.wo; i += C::NT)
    s_hc[i] = i < d.ho ? p.e.hcls[i] * p.e.nwc : p.e.wcls[i - d.ho];
  wait_vmcnt<0>();  // the staged epilogue data (and the first tile)
  __syncthreads();

  for (; pt < npt; pt += pstep) {
    v4i fb[KS][TN];
    int cn[TN], cho[TN], cwo[TN];
    if constexpr (C::PF) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        cn[j] = nn[j], cho[j] = nho[j], cwo[j] = nwo[j];
#pragma unroll
        for (int s = 0; s < KS; ++s) fb[s][j] = fnx[s][j];
      }
      load_b(pt + pstep, fnx, nn, nho, nwo);  // the next tile's fragments land under this one's epilogue
    } else {
      load_b(pt, fb, cn, cho, cwo);  // (no prefetch: the co-resident waves hide the latency)
    }
    v4i acc[TM][TN], sacc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      sacc[j] = (v4i){0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[i][j] = (v4i){0, 0, 0, 0};
    }
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (QNN_ABLATE == 2) {
          sacc[j][0] += fb[s][j].x;
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[i][j][i & 3] ^= fa[s][i].y + fb[s][j].z;
          continue;
        }
        sacc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones[s], fb[s][j], sacc[j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s][i], fb[s][j], acc[i][j], 0, 0, 0);
      }
    int sumq[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) sumq[j] = sacc[j][0];
    auto pixel = [&](int j, q16::Pix& P, int& pc) {
      const int m = pt * BN + (wave * TN + j) * 16 + (lane & 15);
      P.ok = m < p.M;
      P.m = P.ok ? m : p.M - 1;
      P.n = cn[j], P.ho = cho[j], P.wo = cwo[j];
      pc = s_hc[P.ho] + s_hc[d.ho + P.wo];
    };
    if (QNN_ABLATE == 3) {
      int z = sumq[0] ^ cn[0];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) z ^= acc[i][j][r];
      if (z == 0x7fffffff) p.e.out_code0[0] = 1;
      continue;
    }
    q16::epilogue_rb<C, EK>(p, acc, sumq, pixel, smem, c0, 0, lane, 1);
  }
}

static int epi_bytes(const Params& p, int BM) {
  const int k = epi_kind(p.e);
  return 4 * (7 + p.e.nclass) * BM + (k == EK_GEN ? 16 * p.e.nres * BM : 0) + (k == EK_LUT ? 256 * BM : 0);
}

// Co-resident blocks per CU of one kernel at `lds` bytes, queried once per (kernel, lds).  The
// cache is shared by every layer and caller thread (the ABI is re-entrant per stream; the
// reference's DataParallel runs replica forwards from threads, main.py:345), so it is locked.
static int blocks_per_cu(const void* kern, int nt, int lds) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_pair(kern, lds);
  const auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, nt, lds) != hipSuccess || n < 1) n = 1;
  cache.emplace(key, n);
  return n;
}

// The persistent grid: as many blocks as fit at once, a whole number per channel tile
template <class C>
static int64_t persistent_grid(const Params& p, int per_cu) {
  const int64_t nby = cdiv(p.d.cout, C::CB), tiles = cdiv(p.M, C::BN) * nby;
  int64_t nblk = ((int64_t)NUM_CU * per_cu / nby) * nby;
  nblk = nblk < nby ? nby : nblk;
  return nblk < tiles ? nblk : tiles;
}

template <class C, int EK, bool MASKED, int KS>
static int launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  auto kern = qconv_direct_kernel<C, EK, MASKED, KS>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  const int epi = (epi_bytes(p, C::BM) + 15) & ~15;
  const int lds = epi + 4 * (p.d.ho + p.d.wo);
  if (lds > LDS_MAX) return arg_error("conv tile needs more than 160 KiB of LDS (too many border classes)");
  Params q = p;
  q.epi_off = 0, q.epi_early = 1, q.scr_off = epi;
  const int per_cu = blocks_per_cu((const void*)kern, C::NT, lds);
  const int64_t nblk = persistent_grid<C>(p, per_cu);
  if (occ) {
    occ->blocks_per_cu = per_cu, occ->lds = lds, occ->grid = (int)nblk;
    return QNN_OK;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(C::NT), lds, s, x, w, q);
  return QNN_OK;
}

template <class C, int EK, bool MASKED>
static int launch_k(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  if constexpr (C::K576) {  // the K = 576 configurations: nine K steps, weights resident in VGPRs
    if constexpr (MASKED) return arg_error("tile configuration not built for this layer / epilogue kind");
    else return launch<C, EK, false, KS_3X3>(x, w, p, s, occ);
  } else {
    switch ((p.taps * (p.d.cp >> 4) + 3) >> 2) {  // K steps holding real chunks
      case 1: return launch<C, EK, MASKED, 1>(x, w, p, s, occ);
      case 2: return launch<C, EK, MASKED, 2>(x, w, p, s, occ);
      case 3: return launch<C, EK, MASKED, 3>(x, w, p, s, occ);
      default: return launch<C, EK, MASKED, 4>(x, w, p, s, occ);
    }
  }
}

template <class C, int EK>
static int launch_m(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  return p.d.kmask ? launch_k<C, EK, true>(x, w, p, s, occ) : launch_k<C, EK, false>(x, w, p, s, occ);
}

template <class C>
static int launch_ek(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  switch (epi_kind(p.e)) {
    case EK_NCHW: return launch_m<C, EK_NCHW>(x, w, p, s, occ);
    case EK_LUT: return launch_m<C, EK_LUT>(x, w, p, s, occ);
    case EK_BNCODE: return launch_m<C, EK_BNCODE>(x, w, p, s, occ);
    default:  // the general chain spills beside more than 16 accumulator tiles: not built
      if constexpr (C::TM * C::TN > 16) return arg_error("tile configuration not built for this layer / epilogue kind");
      else return launch_m<C, EK_GEN>(x, w, p, s, occ);
  }
}

//   id  block (cout x px)   waves (each)       fits
//   0   32 x 256            4 (32 x 64)        MobileNet's 32-channel stem, 32-channel 1x1s
//   1   64 x 128            4 (64 x 32)        ResNet's 64-channel stem, 64-channel 1x1s
//   2   128 x 64            4 (128 x 16)       128-channel 1x1s (MobileNet's pointwise layers)
//   3   64 x 64             4 (64 x 16)        3x3 on 64 input channels (K = 576: ResNet layer 1):
//                                              36 weight fragments resident per lane
//   4   64 x 64             4 (64 x 16)        the same without the next-tile prefetch (<= 256 registers:
//                                              two waves/SIMD hide each other's loads)
// (two pixel tiles per wave, with or without the prefetch -- 400 / 256+spill registers, one wave per
// SIMD -- measured 42-44 us on the ResNet-18 b128 layer-1 LUT launches: not kept)
using D0 = Cfg<2, 4>;
using D1 = Cfg<4, 2>;
using D2 = Cfg<8, 1>;
using D3 = Cfg<4, 1, true>;
using D4 = Cfg<4, 1, true, false>;
constexpr int ND = 5;
struct Info {
  int bm, bn, acc_tiles;
  float rate;
};
static const Info INFO[ND] = {{32, 256, 8, 1.0f}, {64, 128, 8, 1.0f}, {128, 64, 8, 1.0f}, {64, 64, 4, 1.0f}, {64, 64, 4, 1.0f}};

}  // namespace dk

int direct_count() { return dk::ND; }

void direct_tile(int k, int* bm, int* bn) {
  *bm = dk::INFO[k].bm;
  *bn = dk::INFO[k].bn;
}

bool direct_ok(int k, const Params& p) {
  if (k < 0 || k >= dk::ND) return false;
  const qnn_conv_desc& d = p.d;
  if (d.cp % 16 || d.cout % 16 || p.taps * d.cp > d.kpad || p.M >= (1 << 24)) return false;  // fdivmod's range
  if (k >= 3) {  // exactly nine K steps of real chunks, no K mask
    if (d.kmask || p.taps * d.cp != 64 * dk::KS_3X3) return false;
  } else if (d.kpad > dk::KPAD_MAX || d.kpad % 64) {
    return false;
  }
  const int bm = dk::INFO[k].bm < 64 ? 64 : dk::INFO[k].bm;
  return dk::epi_bytes(p, bm) + 16 + 4 * (d.ho + d.wo) <= LDS_MAX;
}

// pixel tiles x channel tiles (the persistent grid loops over them: qnn_conv_occupancy.grid)
int64_t direct_blocks(int k, const Params& p) {
  const dk::Info& f = dk::INFO[k];
  return cdiv(p.M, f.bn) * cdiv(p.d.cout, f.bm);
}

// the cost model's units (qconv.hip cfg_cost): rounds of resident blocks x one block's
// padded MFMA work / rate, four blocks resident per CU
double direct_cost(int k, const Params& p) {
  const dk::Info& f = dk::INFO[k];
  const int64_t tiles = direct_blocks(k, p);
  const int64_t slots = (int64_t)NUM_CU * 4;
  const int64_t rounds = cdiv(tiles, slots);
  const double share = tiles < slots ? (double)cdiv(tiles, NUM_CU) : 4.0;
  return (double)rounds * share * f.bm * f.bn * p.d.kpad / f.rate;
}

int direct_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  if (!direct_ok(k, p)) return arg_error("tile configuration not built for this layer / epilogue kind");
  switch (k) {
    case 0: return dk::launch_ek<dk::D0>(x, w, p, s, occ);
    case 1: return dk::launch_ek<dk::D1>(x, w, p, s, occ);
    case 2: return dk::launch_ek<dk::D2>(x, w, p, s, occ);
    case 3: return dk::launch_ek<dk::D3>(x, w, p, s, occ);
    default: return dk::launch_ek<dk::D4>(x, w, p, s, occ);
  }
}

// ---------------------------------------------------------------------------------------------
// The classifier head (configuration 44, round 4): QLinear / 1x1 on few pixels -- the batch --
// with K = 512 or 1024 (ResNet-18 / MobileNet fc, resnet_quantized.py:154, mobilenet_quantized.py
// :158) and the drop-in fp32 output.  The ring configurations tile it 64 channels x 128 pixels:
// 16 blocks for a 128-image batch, each walking 8-16 K stages -- 16 of 256 CUs busy.  Here a
// block is 16 channels x 64 pixels (4 waves x one 16-pixel tile), every K fragment one global
// load straight into VGPRs (the direct kernel, all KS steps resident): 126 blocks at b128, each a
// few microseconds.  cout need not be a multiple of 16 (the NCHW stores are masked per channel).
namespace dh {
using DH = dk::Cfg<1, 1>;
constexpr int BN = 64, CB = 16;
}  // namespace dh

bool dhead_ok(const Params& p) {
  const qnn_conv_desc& d = p.d;
  if (epi_kind(p.e) != EK_NCHW || p.taps != 1 || d.kmask || d.cp % 16 || p.M >= (1 << 24)) return false;
  if (d.kpad != 512 && d.kpad != 1024) return false;
  if (p.taps * d.cp > d.kpad || d.cout_pad < (int)cdiv(d.cout, dh::CB) * dh::CB) return false;
  return dk::epi_bytes(p, 64) + 16 + 4 * (d.ho + d.wo) <= LDS_MAX;
}

int64_t dhead_blocks(const Params& p) { return cdiv(p.M, dh::BN) * cdiv(p.d.cout, dh::CB); }

int dhead_launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  if (!dhead_ok(p)) return arg_error("tile configuration not built for this layer / epilogue kind");
  return p.d.kpad == 512 ? dk::launch<dh::DH, EK_NCHW, false, 8>(x, w, p, s, occ)
                         : dk::launch<dh::DH, EK_NCHW, false, 16>(x, w, p, s, occ);
}

// ---------------------------------------------------------------------------------------------
// Table-epilogue configurations (ids after the two-team ones, qnn_conv_tile_kernel
// "qconv_dtab_kernel"): the general chain -- RangeBN, the residual (fp32 and/or a code chain of
// up to four links), ReLU, codes / fp32 out -- of the short-K 1x1 layers, ResNet-50's expand
// convolutions above all, where the contraction is a few MFMAs per output and the epilogue
// is the launch (profiles/r4_pmc_valu_wait_resnet50_b256.json: ~80 VALU per output value on
// layer 1's third expand, the chip's whole VALU issue rate for the launch's 406 us).
//
// Every float the chain computes from a one-byte code is a function of (channel, code): the
// RangeBN of the output, g(q) = fl(fl(fl(fl(rint(q)*s) + min) - mean[c]) * sq[c]) * wq[c]) +
// bq[c] of the clamped quotient, and each chain link's g_l of its stored byte
// (quantize.py:488-499 op order, qnn_res_link).  A block owns 16 channels, so those functions
// are 16 x 256 floats each: the block evaluates them once into LDS with the same fp32 ops
// and the epilogue looks them up -- two VALU (byte -> address) and one ds_read_b32 for what
// took seven VALU per value per link, bitwise the same floats.  What stays per value is what
// depends on the accumulator: the exact decomposition, the RangeBN input quotient, the sums
// and max of the chain, and the consumer's quantizer.
// Rows are 257 floats apart, so the two channels a 32-lane group reads for one register land
// on different banks for equal codes.
// The rest is the direct kernel's: B fragments straight from the padded NHWC codes, one tile
// ahead, with the next tile's chain words / fp32 residual; weights and the lane's per-channel
// constants in registers for the whole persistent loop; blocks of one pixel tile's channel
// tiles placed on one XCD (the tile's codes are read from that XCD's L2 once per 16 channels).
//
// Measured (profiles/r4_dtab_resnet50_b256.txt): the tables cut the launch's VALU instructions by
// a third (layer 1's expand, one chain link: 1.15e8 vs 1.72e8), but the launches are still slower
// than configuration 11 (322 vs 297 us; three links 522 vs 417 us): 16-channel blocks with up to
// 82 KiB of tables hold one or two blocks per CU, two waves per SIMD do not cover the lookups'
// latency, and random codes make 60 % of the table reads' LDS cycles bank conflicts.  The cost
// model never picks these configurations; the autotuner times them beside the others.
namespace dt {

constexpr int W = 4, NT = 64 * W, CB = 16, TSTR = 257;
struct Stage {  // what stage_epi reads: 64-float staging stride, 4 waves
  static constexpr int BM = 64, W = dt::W;
};
constexpr int BM = Stage::BM;

// Byte offset of the 4-byte word of channels c..c+3 of pixel m in a byte C-tile code map
// (q16::btile_word) in 32-bit arithmetic: dtab_ok bounds the map below 2^31 bytes, and
// (m >> 5) * ct < 2^24 takes the full-rate 24-bit multiply.
__device__ __forceinline__ int btile_word32(int m, int c, int ct) {
  return ((int)__umul24((unsigned)(m >> 5), (unsigned)ct) + (c >> 5)) * 1024 + ((m & 31) + 32 * ((c >> 2) & 1)) * 16 +
         4 * ((c & 31) >> 3);
}

// One pixel tile's prefetched operands: B fragments, pixel coordinates (general geometry), the
// byte C-tile word offset of each pixel (chain links and the RangeBN code output share it),
// the chain words and the fp32 residual of this lane's channels
template <int TN, int KS>
struct Tile {
  v4i fb[KS][TN];
  int pn[TN], pho[TN], pwo[TN], woff[TN];
  unsigned cw[QNN_MAX_RES][TN];
  float4 rf[TN];
};

// DENSE: 1x1, stride 1, no input padding and unpadded code outputs (ResNet-50's expand convs):
// pixel m of the output is pixel m of the input and of every consumer buffer, so no pixel
// decode and no padded-index arithmetic.
template <int TN, int KS, bool DENSE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2))) void qconv_dtab_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ w, const Params p) {
  constexpr int BN = W * TN * 16;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // block -> (channel tile, first pixel tile); persistent over pixel tiles pt += pstep.  With
  // the grid a multiple of 8 * nby, block b sits on XCD b % 8 and the nby blocks of each pixel
  // slot share it.
  const int nby = d.cout / CB, G = gridDim.x, b = blockIdx.x;
  const int pstep = G / nby, npt = (p.M + BN - 1) / BN;
  int cty, pt;
  if (G % (8 * nby) == 0) {
    const int r = b >> 3;
    cty = r % nby;
    pt = (r / nby) * 8 + (b & 7);
  } else {
    cty = b % nby;
    pt = b / nby;
  }
  const int c0 = cty * CB, cl = 4 * g, c = c0 + cl;  // this lane's four channels c..c+3

  stage_epi<Stage, EK_GEN>(p, x, smem, c0, wave, lane);
  const float* s_f = reinterpret_cast<const float*>(smem);
  const float* s_chain = s_f + (7 + e.nclass) * BM;
  int* s_hc = reinterpret_cast<int*>(smem + p.scr_off);
  float* s_tab = reinterpret_cast<float*>(smem + p.scr_off + 4 * ((d.ho + d.wo + 3) & ~3));
  for (int i = tid; i < d.ho + d.wo; i += NT) s_hc[i] = i < d.ho ? e.hcls[i] * e.nwc : e.wcls[i - d.ho];

  const int cpg = d.cp >> 4, kreal = p.taps * cpg;
  int doff[KS];
  v4i fa[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int u = 4 * s + g;
    const int tap = u / cpg, tr = tap / d.kw, tc = tap - tr * d.kw;
    doff[s] = u < kreal ? (tr * d.wp + tc) * d.cp + 16 * (u - tap * cpg) : -1;
    fa[s] = *reinterpret_cast<const v4i*>(w + (int64_t)(c0 + (lane & 15)) * d.kpad + 64 * s + 16 * g);
  }
  const v4i ones = {0x01010101, 0x01010101, 0x01010101, 0x01010101};

  const int nres = e.nres;
  const bool has_res = e.residual != nullptr, bn = e.bn_mean != nullptr;
  const int HoWo = d.ho * d.wo;
  const float inv_hw = 1.0f / (float)HoWo, inv_wo = 1.0f / (float)d.wo;
  const int lgcp = 4 + p.lgcpt;
  auto pixel = [&](int t, int j) __attribute__((always_inline)) {
    const int m = t * BN + (wave * TN + j) * 16 + (lane & 15);
    return m < p.M ? m : p.M - 1;  // past the batch: the last pixel again (same values re-stored)
  };
  // tile t's operands (clamped: a prefetch past the last tile re-reads it)
  auto load_t = [&](int t, Tile<TN, KS>& T) __attribute__((always_inline)) {
    t = t < npt ? t : npt - 1;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int m = pixel(t, j);
      int base;
      if constexpr (DENSE) {
        base = m << lgcp;
      } else {
        int n, hw, ho, wo;
        dk::fdivmod(m, HoWo, inv_hw, n, hw);
        dk::fdivmod(hw, d.wo, inv_wo, ho, wo);
        T.pn[j] = n, T.pho[j] = ho, T.pwo[j] = wo;
        base = (int)(__umul24(__umul24((unsigned)n, (unsigned)d.hp) + (unsigned)(ho * d.sh), (unsigned)d.wp) +
                     (unsigned)(wo * d.sw)) << lgcp;
      }
#pragma unroll
      for (int s = 0; s < KS; ++s)
        T.fb[s][j] = *reinterpret_cast<const v4i*>(x + (doff[s] >= 0 ? base + doff[s] : d.zero_off));
      T.woff[j] = btile_word32(m, c, p.ct);
      if (has_res) {
        const int64_t fi = e.f32_tiled ? ctile_index(m, c, p.ct) : (int64_t)m * d.cout + c;
        T.rf[j] = *reinterpret_cast<const float4*>(e.residual + fi);
      }
#pragma unroll
      for (int l = 0; l < QNN_MAX_RES; ++l)
        if (l < nres) T.cw[l][j] = *reinterpret_cast<const unsigned*>(e.res[l].code + T.woff[j]);
    }
  };
  Tile<TN, KS> ta, tb_;
  load_t(pt, ta);
  wait_vmcnt<0>();  // the staged epilogue data (and the first tile)
  __syncthreads();

  // the tables: [RangeBN] then the chain links, [16 channels][TSTR] each
  const int ntab = (bn ? 1 : 0) + nres;
  for (int i = tid; i < ntab * CB * 256; i += NT) {
    const int t = i >> 12, ch = (i >> 8) & 15, q = i & 255;
    const float fq = (float)q;
    float o;
    if (bn && t == 0) {
      o = fq * e.bn_scale;       // dequant: q * s
      o = o + e.bn_min;          // + min
      o = o - s_f[3 * BM + ch];  // x - mean
      o = o * s_f[4 * BM + ch];  // * q(scale)
      o = o * s_f[5 * BM + ch];  // * q(weight)
      o = o + s_f[6 * BM + ch];  // + q(bias)
    } else {
      const int l = t - (bn ? 1 : 0);
      const float* sp = s_chain + 4 * l * BM + ch;
      o = fq * e.res[l].scale;
      o = o + e.res[l].min;
      o = o - sp[0];
      o = o * sp[BM];
      o = o * sp[2 * BM];
      o = o + sp[3 * BM];
    }
    s_tab[(t * CB + ch) * TSTR + q] = o;
  }
  const float4 sw = *reinterpret_cast<const float4*>(s_f + cl);
  const float4 bw = *reinterpret_cast<const float4*>(s_f + BM + cl);
  const float4 bi = *reinterpret_cast<const float4*>(s_f + 2 * BM + cl);
  const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
  const QParams c0p = make_qparams(e.code0_neg_min, e.code0_scale, e.code0_qmax);
  const QParams c1p = make_qparams(e.code1_neg_min, e.code1_scale, e.code1_qmax);
  const bool same01 = e.out_code0 && e.code1_neg_min == e.code0_neg_min && e.code1_scale == e.code0_scale &&
                      e.code1_qmax == e.code0_qmax;
  const bool want_bn = e.out_bncode != nullptr;
  const float* tab_l = s_tab + ((bn ? 1 : 0) * CB + cl) * TSTR;  // this lane's rows of link 0
  const float* tab_b = s_tab + cl * TSTR;                           // ... of the RangeBN table
  // one border class (the unpadded 1x1s): its table row stays in registers
  const bool one_class = DENSE || e.nclass == 1;
  const float4 tb1 = *reinterpret_cast<const float4*>(s_f + 7 * BM + cl);
  // element offset of pixel m (coordinates of tile T, column j) in a consumer's NHWC8 buffer:
  // general geometry by 24-bit products of factors < 2^24 (conv_params bounds every buffer) and
  // one 32 x 32 -> 64 multiply by cp
  auto code_off = [&](const Tile<TN, KS>& T, int j, int m, int hp, int wp, int pad, int cp) __attribute__((always_inline)) {
    if constexpr (DENSE) {
      return (int64_t)(unsigned)m * cp + c;
    } else {
      const unsigned px = __umul24(__umul24((unsigned)T.pn[j], (unsigned)hp) + (unsigned)(T.pho[j] + pad), (unsigned)wp) +
                          (unsigned)(T.pwo[j] + pad);
      return (int64_t)px * cp + c;
    }
  };
  __syncthreads();

  // one tile: prefetch the next one into N, contract and finish C
  auto step = [&](Tile<TN, KS>& C, Tile<TN, KS>& N) __attribute__((always_inline)) {
    load_t(pt + pstep, N);  // lands under this tile's epilogue
    v4i acc[TN], sacc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = sacc[j] = (v4i){0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        sacc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, C.fb[s][j], sacc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s], C.fb[s][j], acc[j], 0, 0, 0);
      }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int m = pixel(pt, j);
      const float4 tb = one_class ? tb1
                                  : *reinterpret_cast<const float4*>(s_f + (7 + s_hc[C.pho[j]] + s_hc[d.ho + C.pwo[j]]) * BM + cl);
      const f2 p2 = {(float)sacc[j][0], (float)sacc[j][0]};
      const v4i& a = acc[j];
      f2 v[2];  // the exact decomposition, conv_out4's op order
      v[0] = pfma((f2){sw.x, sw.y}, (f2){(float)a[0], (float)a[1]}, pfma((f2){bw.x, bw.y}, p2, (f2){tb.x, tb.y})) +
             (f2){bi.x, bi.y};
      v[1] = pfma((f2){sw.z, sw.w}, (f2){(float)a[2], (float)a[3]}, pfma((f2){bw.z, bw.w}, p2, (f2){tb.z, tb.w})) +
             (f2){bi.z, bi.w};
      if (bn || want_bn) {
        // RangeBN's input code: its low mantissa byte is rint of the clamped quotient
        const f2 mb[2] = {qclamp2(v[0], bnp) + MAGIC_U8, qclamp2(v[1], bnp) + MAGIC_U8};
        if (want_bn) {
          const int kb = pack4(mb[0], mb[1]);
          if (e.bncode_tiled) *reinterpret_cast<int*>(e.out_bncode + C.woff[j]) = kb;
          else *reinterpret_cast<int*>(e.out_bncode + (int64_t)m * d.cout + c) = kb;
        }
        if (bn) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            v[h].x = tab_b[(2 * h) * TSTR + (__float_as_uint(mb[h].x) & 255u)];
            v[h].y = tab_b[(2 * h + 1) * TSTR + (__float_as_uint(mb[h].y) & 255u)];
          }
        }
      }
      if (has_res || nres > 0) {
        f2 r[2];
        int l0 = 0;
        if (has_res) {
          r[0] = (f2){C.rf[j].x, C.rf[j].y};
          r[1] = (f2){C.rf[j].z, C.rf[j].w};
        } else {
          const unsigned wd = C.cw[0][j];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            r[h].x = tab_l[(2 * h) * TSTR + ((wd >> (16 * h)) & 255u)];
            r[h].y = tab_l[(2 * h + 1) * TSTR + ((wd >> (16 * h + 8)) & 255u)];
          }
          if (e.res_relu0) {
            r[0].x = fmaxf(r[0].x, 0.f); r[0].y = fmaxf(r[0].y, 0.f);
            r[1].x = fmaxf(r[1].x, 0.f); r[1].y = fmaxf(r[1].y, 0.f);
          }
          l0 = 1;
        }
#pragma unroll
        for (int l = 0; l < QNN_MAX_RES; ++l) {
          if (l < l0 || l >= nres) continue;
          const unsigned wd = C.cw[l][j];
          const float* tl = tab_l + l * CB * TSTR;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f2 o = {tl[(2 * h) * TSTR + ((wd >> (16 * h)) & 255u)], tl[(2 * h + 1) * TSTR + ((wd >> (16 * h + 8)) & 255u)]};
            const f2 t2 = o + r[h];
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
      if (e.out_code0 && c < e.code0_cp)
        *reinterpret_cast<int*>(e.out_code0 + code_off(C, j, m, e.code0_hp, e.code0_wp, e.code0_pad, e.code0_cp)) = k0;
      if (e.out_code1 && c < e.code1_cp) {
        // two consumers calibrated on the same tensor hold the same range: their codes are equal
        const int k1 = same01 ? k0 : pack4(qclamp2(v[0], c1p) + MAGIC_S8, qclamp2(v[1], c1p) + MAGIC_S8);
        *reinterpret_cast<int*>(e.out_code1 + code_off(C, j, m, e.code1_hp, e.code1_wp, e.code1_pad, e.code1_cp)) = k1;
      }
    }
    pt += pstep;
  };
  // two tiles per trip, the operand sets alternating (no register copies between tiles)
  while (pt < npt) {
    step(ta, tb_);
    if (pt >= npt) break;
    step(tb_, ta);
  }
}

// LDS bytes: the staged vectors, the border classes, the tables
static int lds_bytes(const Params& p) {
  const int epi = (dk::epi_bytes(p, BM) + 15) & ~15;
  const int ntab = (p.e.bn_mean ? 1 : 0) + p.e.nres;
  return epi + 4 * ((p.d.ho + p.d.wo + 3) & ~3) + 4 * ntab * CB * TSTR;
}

//   id  block (cout x px)   waves (each)          K steps
//   0   16 x 256            4 (16 x 64)           1-2 (K <= 128: ResNet-50 layers 1-2 expand)
//   1   16 x 128            4 (16 x 32)           1-4 (K <= 256: layer 3 expand)
constexpr int NDT = 2;
static const int TNS[NDT] = {4, 2};

// DENSE's geometry (qconv_dtab_kernel)
static bool dense(const Params& p) {
  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  auto flat = [&](const int8_t* ptr, int hp, int wp, int pad) { return !ptr || (pad == 0 && hp == d.ho && wp == d.wo); };
  return p.taps == 1 && d.sh == 1 && d.sw == 1 && d.hp == d.ho && d.wp == d.wo && e.nclass == 1 &&
         flat(e.out_code0, e.code0_hp, e.code0_wp, e.code0_pad) && flat(e.out_code1, e.code1_hp, e.code1_wp, e.code1_pad);
}

template <int TN, int KS, bool DENSE>
static int launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  auto kern = qconv_dtab_kernel<TN, KS, DENSE>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  const int lds = lds_bytes(p);
  if (lds > LDS_MAX) return arg_error("conv tile needs more than 160 KiB of LDS (too many border classes)");
  Params q = p;
  q.epi_off = 0, q.epi_early = 1, q.scr_off = (dk::epi_bytes(p, BM) + 15) & ~15;
  const int per_cu = dk::blocks_per_cu((const void*)kern, NT, lds);
  const int64_t nby = p.d.cout / CB, tiles = cdiv(p.M, W * TN * 16) * nby;
  int64_t nblk = (int64_t)NUM_CU * per_cu;
  nblk = nblk % (8 * nby) == 0 ? nblk : (nblk / nby) * nby;  // XCD-grouped when it divides
  nblk = nblk < nby ? nby : nblk;
  if (nblk > tiles) nblk = tiles;
  if (occ) {
    occ->blocks_per_cu = per_cu, occ->lds = lds, occ->grid = (int)nblk;
    return QNN_OK;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(NT), lds, s, x, w, q);
  return QNN_OK;
}

template <int TN, bool DENSE>
static int launch_d(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  switch ((p.taps * (p.d.cp >> 4) + 3) >> 2) {  // K steps holding real chunks
    case 1: return launch<TN, 1, DENSE>(x, w, p, s, occ);
    case 2: return launch<TN, 2, DENSE>(x, w, p, s, occ);
    case 3: if constexpr (TN <= 2) return launch<TN, 3, DENSE>(x, w, p, s, occ); else break;
    case 4: if constexpr (TN <= 2) return launch<TN, 4, DENSE>(x, w, p, s, occ); else break;
    default: break;
  }
  return arg_error("tile configuration not built for this layer / epilogue kind");
}

template <int TN>
static int launch_k(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  return dense(p) ? launch_d<TN, true>(x, w, p, s, occ) : launch_d<TN, false>(x, w, p, s, occ);
}

}  // namespace dt

int dtab_count() { return dt::NDT; }

void dtab_tile(int k, int* bm, int* bn) {
  *bm = dt::CB;
  *bn = dt::W * dt::TNS[k] * 16;
}

bool dtab_ok(int k, const Params& p) {
  if (k < 0 || k >= dt::NDT) return false;
  const qnn_conv_desc& d = p.d;
  if (epi_kind(p.e) != EK_GEN || p.e.mode != 1) return false;
  if (d.cp % 16 || d.cout % dt::CB || d.kmask || p.M >= (1 << 24)) return false;  // fdivmod's range
  if (d.kpad > dk::KPAD_MAX || d.kpad % 64) return false;
  const int ks = (p.taps * (d.cp >> 4) + 3) >> 2;
  if (ks > (dt::TNS[k] <= 2 ? 4 : 2)) return false;
  if (cdiv(p.M, 32) * p.ct * 1024 >= (1LL << 31)) return false;  // btile_word32's range
  return dt::lds_bytes(p) <= LDS_MAX;
}

int64_t dtab_blocks(int k, const Params& p) { return cdiv(p.M, dt::W * dt::TNS[k] * 16) * (p.d.cout / dt::CB); }

// the cost model's units (qconv.hip cfg_cost).  Measured slower than the ring kernel's
// configuration 11 on every ResNet-50 expand launch (profiles/r4_dtab_*), so the
// cost model never picks these; the autotuner times them with the rest.
double dtab_cost(int k, const Params& p) {
  const int64_t tiles = dtab_blocks(k, p);
  return (double)tiles * dt::CB * dt::W * dt::TNS[k] * 16 * p.d.kpad * 64.0;
}

int dtab_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  if (!dtab_ok(k, p)) return arg_error("tile configuration not built for this layer / epilogue kind");
  return k == 0 ? dt::launch_k<4>(x, w, p, s, occ) : dt::launch_k<2>(x, w, p, s, occ);
}

}  // namespace qnn
