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

template <class C, int EK, bool MASKED, int KS>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu((C::PF || C::TN > 1) ? 1 : 2))) void qconv_direct_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ w,
                                                            const Params p) {
  constexpr int TM = C::TM, TN = C::TN, CB = C::CB, BN = C::BN;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // persistent: block b owns channel tile b % nby and pixel tiles b / nby + k * (grid / nby)
  const int nby = (d.cout + CB - 1) / CB;
  const int c0 = (blockIdx.x % nby) * CB;
  const int pstep = gridDim.x / nby, npt = (p.M + BN - 1) / BN;

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
  int pt = blockIdx.x / nby;
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

}  // namespace qnn
