// int8 implicit-GEMM convolution on v_mfma_i32_16x16x64_i8 with LDS-staged input bands:
// the eval forward of QConv2d / QLinear (models/modules/quantize.py:314-349, :398-428),
// same exact decomposition and epilogue arithmetic as qconv.hip, so every
// configuration of either file computes bitwise identical outputs.
//
// Why a second kernel family (measured on MI355X, profiles/r2_mfma_peak.jsonl): a stream of
// v_mfma_i32_32x32x32_i8 holds the chip at 1.4-1.7 GHz (3.40 POPS at best), the same work as
// v_mfma_i32_16x16x64_i8 at ~2.0 GHz (3.94 POPS); and qconv.hip's implicit im2col pulls each
// input byte through L2 -> LDS once per tap.  Here:
//
// * B operand = a BAND in LDS, loaded once per K chunk (Cp up to 64 channels = one 64-byte
//   K stage per tap): for kh x kw > 1 the padded input rows [R0, R1) the block's BN output
//   pixels read (stride-2 rows with even columns first), for 1x1 the block's pixels
//   themselves (any stride).  Every tap's B fragment is an LDS read at a shifted address.
// * Band layout: PLANAR, plane g = bytes [16g, 16g+16) of every band pixel's chunk, planes
//   1 KiB aligned.  A 16x16x64 B fragment (lane: pixel lane&15, K bytes 16*(lane>>4)..)
//   reads plane lane>>4 at 16 consecutive band pixels: 16 distinct bank slots per
//   ds_read_b128 lane group, no swizzle, one VALU (the tap offset add) per fragment.
// * A operand = weights through a D-slot LDS ring, one 64-byte K stage per slot, LDS-DMA
//   D-1 stages ahead, one s_barrier per stage.  Rows XOR-swizzled on the DMA source side
//   (slot ^ ((row >> 2) & 1) << 1) so A fragment reads are conflict-free.
// * sum_valid(q'_x) (the s_x*b_w term): per band pixel channel sums accumulated once per
//   chunk, then summed over the taps per output pixel after the loop; space-to-depth stems
//   (per-tap channel masks) accumulate masked v_dot4 of their fragments instead.
#include <type_traits>

#include "qconv_common.h"
#include "epi16.h"

#ifndef QNN_ABLATE
#define QNN_ABLATE 0  // diagnostic builds only (make ablate): 1 no weight loads, 2 no MFMA, 3 no epilogue
#endif

namespace qnn {
namespace q16 {

template <int WGM_, int WGN_, int TM_, int TN_, int D_, int BPC_>
struct Cfg {
  static constexpr int WGM = WGM_, WGN = WGN_, TM = TM_, TN = TN_, D = D_, BPC = BPC_;
  static constexpr int W = WGM * WGN, NT = 64 * W;
  static constexpr int BM = WGM * TM * 16, BN = WGN * TN * 16;
  static constexpr int STAGE_A = BM * 64;
  static constexpr int AP = BM / 16;                 // weight DMA pieces (16 rows x 64 B) per stage
  static constexpr int NA = AP >= W ? AP / W : 1;     // per wave (fewer pieces than waves: duplicated)
  static_assert(AP % W == 0 || W % AP == 0, "weight DMA pieces must split evenly over the waves");
  static_assert(BM % 64 == 0, "epilogue staging moves 64-channel groups");
};

constexpr int NBWMAX = 12;  // band DMA pieces per wave per chunk
constexpr int PPTMAX = 4;  // band pixels per thread (channel sums)
constexpr int NBS = 2;     // band DMA pieces per wave in every stage's DMA group

struct Band16 {
  int list;            // 1: band pixel q = output pixel m0 + q (1x1); 0: padded input rows [R0, R1)
  int npl, tps;        // 16-byte planes per band pixel, taps per 64-byte stage (4 / npl)
  int nc, ns, kt;      // K chunks, stages per chunk, stages in all
  int s2, we;          // row band of a stride-2 conv: even columns first, we = (wp + 1) / 2
  uint32_t wp_magic;   // ceil(2^32 / wp)
  int plane, ppp;      // LDS bytes per plane (multiple of 1 KiB), 1 KiB pieces per plane
  int nbw;             // band DMA pieces per wave per chunk (<= NBWMAX)
  int nbuf, bufsz;     // band buffers and their size
  int band_off, dummy_off, zero_off, tap_off, s_off, mask_off;
};

// s_waitcnt lgkmcnt(N) for hand-counted inline-asm LDS reads; the scheduling barrier keeps the
// compiler from hoisting register-only MFMAs above it (cdna_hip_programming.md rule 18)
template <int N>
__device__ __forceinline__ void lds_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void wait_rt(int n) {
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


template <class C, int EK, int NPL, bool MASKED>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(C::BPC * C::W / 4))) void qconv16_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ w, const Params p, const Band16 b) {
  constexpr int BM = C::BM, BN = C::BN, W = C::W, TM = C::TM, TN = C::TN, D = C::D, NA = C::NA, NT = C::NT;
  constexpr int STAGE_A = C::STAGE_A;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];

  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  const int px = lane & 15, g = lane >> 4;

  // ---- XCD-aware bijective block -> tile map (channel tiles fastest: blocks sharing a band share L2)
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
  auto decode = [&](int m, Pix& P) {
    P.m = m;
    P.n = m / HoWo;
    const int r = m - P.n * HoWo;
    P.ho = r / d.wo;
    P.wo = r - P.ho * d.wo;
  };
  const int mlast = (m0 + BN < p.M ? m0 + BN : p.M) - 1;
  int R0 = 0, NBP;
  {
    Pix a, z;
    decode(m0, a);
    decode(mlast, z);
    if (b.list) {
      NBP = mlast - m0 + 1;
    } else {
      R0 = a.n * d.hp + a.ho * d.sh;
      NBP = (z.n * d.hp + z.ho * d.sh + d.kh - R0) * d.wp;
    }
  }
  R0 = __builtin_amdgcn_readfirstlane(R0);
  NBP = __builtin_amdgcn_readfirstlane(NBP);

  // ---- LDS constants: zero bytes, tap offsets (band pixels; padded taps -> tap 0), K mask
  int* s_tap = reinterpret_cast<int*>(smem + b.tap_off);
  if (tid < 4) *reinterpret_cast<v4i*>(smem + b.zero_off + 16 * tid) = (v4i){0, 0, 0, 0};
  if (tid < 64) {
    int dl = 0;
    if (tid < p.taps && !b.list) {
      const int tr = tid / d.kw, tc = tid - tr * d.kw;
      dl = tr * d.wp + (b.s2 ? (tc & 1) * b.we + (tc >> 1) : tc);
    }
    s_tap[tid] = dl;
  }
  if constexpr (MASKED) {
    for (int i = tid; i < d.kpad / 16; i += NT)
      *reinterpret_cast<v4i*>(smem + b.mask_off + 16 * i) = *reinterpret_cast<const v4i*>(d.kmask + 16 * i);
  }
  __syncthreads();  // before any LDS-DMA is in flight (a barrier then would drain it)

  // ---- this lane's pixels (column tile j: m0 + wn*16*TN + 16j + lane&15): decoded with
  // one division, then stepped by 16; pixels past M stand in for the last one (not stored)
  auto lane_pixels = [&](Pix (&pix)[TN]) {
    Pix last;
    decode(p.M - 1, last);
    Pix cur;
    const int mb = m0 + wn * 16 * TN + px;
    decode(mb < p.M ? mb : p.M - 1, cur);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int m = mb + 16 * j;
      Pix P = cur;
      P.m = m;
      P.ok = m < p.M;
      if (!P.ok) P = last, P.ok = false;
      pix[j] = P;
      cur.wo += 16;
      while (cur.wo >= d.wo) {
        cur.wo -= d.wo;
        if (++cur.ho == d.ho) cur.ho = 0, ++cur.n;
      }
    }
  };
  int bq16[TN];  // byte offset within a band plane of each column tile's pixel (tap 0)
  {
    Pix pix[TN];
    lane_pixels(pix);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const Pix& P = pix[j];
      const int q = b.list ? (P.ok ? P.m : p.M - 1) - m0
                           : (P.n * d.hp + P.ho * d.sh - R0) * d.wp + P.wo;  // column wo*sw: wo (stride 2: even half)
      bq16[j] = 16 * q;
    }
  }
  static_assert(NPL == 1 || NPL == 2 || NPL == 4, "16-byte planes per band pixel");
  static_assert(!MASKED || NPL == 1, "masked (space-to-depth) stems have 16-channel band pixels");
  const int tsub = NPL == 4 ? 0 : (NPL == 2 ? g >> 1 : g);  // which tap of a stage this lane's bytes hold
  const int lpo = (g & (NPL - 1)) * b.plane;                // this lane's plane

  // ---- weights: 16 rows x 64 B per DMA, slots XOR-swizzled by row bit 2 (source side)
  const int8_t* wblk = w + (int64_t)c0 * d.kpad;
  uint32_t aoff[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int row = 16 * ((wave + W * j) % C::AP) + (lane >> 2);
    const int crow = (c0 + row < d.cout_pad ? row : d.cout_pad - 1 - c0);
    aoff[j] = (uint32_t)(crow * d.kpad + 16 * ((lane & 3) ^ (((row >> 2) & 1) << 1)));
  }
  const int offa = (wm * 16 * TM + px) * 64 + 16 * (g ^ (((px >> 2) & 1) << 1));

  if (p.epi_early) stage_epi<C, EK>(p, x, smem + p.epi_off, c0, wave, lane);  // oldest DMAs: land under the loop

  // ---- DMA.  Band piece j of this wave = 1 KiB of the band buffer at piece (wave + W*j):
  // plane pl, band pixels [64*(.), +64); its global source is recomputed on the fly.
  auto band_src = [&](int j, int c) -> uint32_t {
    const int id = wave + W * j;               // uniform
    int pl = id / b.ppp;
    const int qb = (id - pl * b.ppp) * 64;
    pl = pl < NPL ? pl : NPL - 1;              // slack pieces past the last plane re-read valid bytes
    int q = qb + lane;
    q = q < NBP ? q : NBP - 1;
    const int r = (int)__umulhi((uint32_t)q, b.wp_magic);
    const int ci = q - r * d.wp;
    const int col = b.s2 ? (ci < b.we ? 2 * ci : 2 * (ci - b.we) + 1) : ci;
    return (uint32_t)(((R0 + r) * d.wp + col) * d.cp + 16 * pl + c * 16 * NPL);
  };
  auto glds = [&](const int8_t* src, int8_t* dst) {
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)dst, 16, 0, 0);
  };
  auto koff = [&](int c, int s) -> uint32_t { return (uint32_t)(NPL == 4 ? s * d.cp + 64 * c : 64 * s); };
  const int KT = b.kt;
  // DMA group of stage (c, s), issued D-1 stages ahead: its weights (NA pieces) and NBS band
  // pieces -- slice s-(D-1) of chunk c+1 when c+1 < nc and s >= D-1, otherwise dummies (the
  // input's zero page into this wave's scratch KiB, one L2 line).  Every group is exactly
  // NA + NBS DMA per wave, so every wait below is a compile-time vmcnt.
  auto issue_group = [&](int c, int s, int slot) {
    if (QNN_ABLATE == 1) return;
    const uint32_t ko = koff(c, s);
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      uint32_t off = aoff[j] + ko;
      asm volatile("" : "+v"(off));
      glds(wblk + off, smem + slot * STAGE_A + ((wave + W * j) % C::AP) * 1024);
    }
    const int cn = c + 1, bj0 = NBS * (s - (D - 1));
    const bool slice = cn < b.nc && s >= D - 1;
    int8_t* bdst = smem + b.band_off + (cn & 1) * b.bufsz;
#pragma unroll
    for (int u = 0; u < NBS; ++u) {
      const int j = bj0 + u;
      const bool real = slice && j < b.nbw;
      uint32_t off = band_src(real ? j : 0, cn);
      asm volatile("" : "+v"(off));
      const int8_t* src = real ? x + off : x + d.zero_off;
      int8_t* dst = real ? bdst + (wave + W * j) * 1024 : smem + b.dummy_off + wave * 1024;
      glds(src, dst);
    }
  };

  v4i acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4i){0, 0, 0, 0};
  int sumq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] = 0;
  int sacc[PPTMAX];
#pragma unroll
  for (int u = 0; u < PPTMAX; ++u) sacc[u] = 0;

  // band offset (pixels) of stage s's tap for this lane's K bytes (uniform when npl == 4)
  auto tap_of = [&](int s) -> int {
    if (b.list) return 0;
    int tt = NPL == 4 ? s : s * (4 / NPL) + tsub;
    if (tt >= p.taps) tt = 0;  // padded taps: any valid band bytes (their weights are 0, masked in sums)
    const int tr = (tt * p.kw_magic) >> 16, tc = tt - tr * d.kw;
    return tr * d.wp + (b.s2 ? (tc & 1) * b.we + (tc >> 1) : tc);
  };
  // Fragment reads are inline asm: the compiler's waitcnt pass cannot see that the next
  // stage's reads are younger than the registers the current MFMAs use (it waits
  // lgkmcnt(0) there); the counts are kept by hand (lds_wait) instead.
  auto read_frags = [&](auto slotc, int bi, int s, v4i (&fa)[TM], v4i (&fb)[TN]) {
    constexpr int AO = decltype(slotc)::value * STAGE_A;
#pragma unroll
    for (int i = 0; i < TM; ++i)
    {
      v4i r;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(offa), "n"(AO + i * 1024));
      fa[i] = r;
    }
    const int base = b.band_off + bi * b.bufsz + lpo + 16 * tap_of(s);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int addr = base + bq16[j];
      v4i r;
      asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
      fb[j] = r;
    }
  };
  auto mma = [&](const v4i (&fa)[TM], const v4i (&fb)[TN], int s) {
    if constexpr (MASKED) {
      const v4i mk = *reinterpret_cast<const v4i*>(smem + b.mask_off + 64 * s + 16 * g);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int sm = __builtin_amdgcn_sdot4(fb[j].x, mk.x, sumq[j], false);
        sm = __builtin_amdgcn_sdot4(fb[j].y, mk.y, sm, false);
        sm = __builtin_amdgcn_sdot4(fb[j].z, mk.z, sm, false);
        sumq[j] = __builtin_amdgcn_sdot4(fb[j].w, mk.w, sm, false);
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (QNN_ABLATE == 2) {
          asm volatile("" ::"v"(fa[i]), "v"(fb[j]));
          acc[i][j][0] += fa[i].x;
        } else {
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
      }
    __builtin_amdgcn_s_setprio(0);
  };
  // channel sums of the band chunk in buffer bi (every band pixel, all planes)
  auto band_sums = [&](int bi) {
    const int8_t* bb = smem + b.band_off + bi * b.bufsz;
    const int ones = 0x01010101;
#pragma unroll
    for (int u = 0; u < PPTMAX; ++u) {
      const int q = tid + NT * u;
      if (q < NBP) {
        int sm = sacc[u];
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          const v4i v = *reinterpret_cast<const v4i*>(bb + pl * b.plane + 16 * q);
          sm = __builtin_amdgcn_sdot4(v.x, ones, sm, false);
          sm = __builtin_amdgcn_sdot4(v.y, ones, sm, false);
          sm = __builtin_amdgcn_sdot4(v.z, ones, sm, false);
          sm = __builtin_amdgcn_sdot4(v.w, ones, sm, false);
        }
        sacc[u] = sm;
      }
    }
  };
  // ---- main loop.  Stage k = (c, s) lives in weight slot k % D and band buffer c & 1.
  // Before the barrier of stage k each wave waits for its own DMA group of stage k (issued
  // D-1 stages earlier; the band chunk it reads was completed by older groups); the D-2
  // younger groups stay in flight.  After the barrier the slot of stage k-1 is refilled
  // with stage k+D-1's group.  Two waves per SIMD: one wave's LDS reads and DMA issue hide
  // under its partner's MFMAs.  Branch-free apart from the chunk-start channel sums.
  constexpr int YOUNG = (D - 2) * (NA + NBS);
  {  // chunk 0's band, then the groups of stages 0 .. D-2 (clamped to the last stage)
#pragma unroll
    for (int j = 0; j < NBWMAX; ++j) {
      if (j < b.nbw) {
        uint32_t off = band_src(j, 0);
        asm volatile("" : "+v"(off));
        glds(x + off, smem + b.band_off + (wave + W * j) * 1024);
      }
    }
  }
  int ca = 0, sa = 0;  // the newest issued group's stage
#pragma unroll
  for (int k = 0; k < D - 1; ++k) {
    issue_group(ca, sa, k);
    if (k + 1 < D - 1 && ca * b.ns + sa + 1 < KT)
      if (++sa == b.ns) sa = 0, ++ca;
  }
  v4i fa[TM], fb[TN];
  int s = 0, bi = 0;
  auto step = [&](auto slotc) {
    constexpr int SL = decltype(slotc)::value;
    wait_vmcnt<YOUNG>();
    __builtin_amdgcn_s_barrier();
    if (ca * b.ns + sa + 1 < KT)
      if (++sa == b.ns) sa = 0, ++ca;
    issue_group(ca, sa, (SL + D - 1) % D);
    if constexpr (!MASKED)
      if (s == 0) band_sums(bi);
    read_frags(slotc, bi, s, fa, fb);
    lds_wait<0>();
    mma(fa, fb, s);
    if (++s == b.ns) s = 0, bi ^= 1;
  };
  for (int k = 0; k < KT; k += D) {
    step(std::integral_constant<int, 0>{});
    if (k + 1 < KT) step(std::integral_constant<int, 1>{});
    if (k + 2 < KT) step(std::integral_constant<int, 2>{});
    if constexpr (D == 4)
      if (k + 3 < KT) step(std::integral_constant<int, 3>{});
  }
  wait_vmcnt<0>();  // the clamped tail DMAs still write LDS

  // ---- sum_valid(q'_x) per output pixel
  if constexpr (MASKED) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      sumq[j] += __shfl_xor(sumq[j], 16, 64);
      sumq[j] += __shfl_xor(sumq[j], 32, 64);
    }
  } else {
    int* s_S = reinterpret_cast<int*>(smem + b.s_off);
#pragma unroll
    for (int u = 0; u < PPTMAX; ++u) {
      const int q = tid + NT * u;
      if (q < NBP) s_S[q] = sacc[u];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int sm = 0;
      const int q = bq16[j] >> 4;
      for (int tt = 0; tt < p.taps; ++tt) sm += s_S[q + s_tap[tt]];
      sumq[j] = sm;
    }
  }
  __syncthreads();  // main-loop LDS is reused by the epilogue
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
    stage_epi<C, EK>(p, x, smem + p.epi_off, c0, wave, lane);
    wait_vmcnt<0>();
    __syncthreads();
  }
  {
    Pix pix[TN];
    lane_pixels(pix);
    int pcls[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) pcls[j] = p.e.hcls[pix[j].ho] * p.e.nwc + p.e.wcls[pix[j].wo];
    epilogue16<C, EK>(p, acc, sumq, pcls, pix, smem, c0, wm, lane);
  }
}

// ------------------------------------------------------------------ host side
// Fills the band plan; returns the main-loop LDS bytes, or -1 if the layer / tile does not fit.
static int band16(const Params& p, int BM, int BN, int nt, int D, int bpc, Band16& b) {
  const qnn_conv_desc& d = p.d;
  if (d.sh != d.sw || (d.sh != 1 && d.sh != 2)) return -1;
  const int npl = d.cp >= 64 ? 4 : d.cp / 16;
  if (d.kmask && npl != 1) return -1;
  b.npl = npl;
  b.tps = 4 / npl;
  const int taps_pad = (p.taps + b.tps - 1) / b.tps * b.tps;
  if (taps_pad > 64) return -1;
  b.nc = npl == 4 ? d.cp / 64 : 1;
  b.ns = taps_pad / b.tps;
  b.kt = b.nc * b.ns;
  if ((npl < 4 ? b.ns * 64 : p.taps * d.cp) > d.kpad) return -1;
  b.list = p.taps == 1;
  if (b.list) return -1;  // 1x1: qconv.hip's ring kernels (no im2col re-reads to save)
  b.s2 = !b.list && d.sh == 2;
  b.we = (d.wp + 1) / 2;
  b.wp_magic = (uint32_t)((0x100000000ULL + (uint64_t)d.wp - 1) / (uint64_t)d.wp);
  int64_t nbp;
  if (b.list) {
    nbp = BN;
  } else {  // BN consecutive output pixels span at most RO + 1 output rows and `cross` image boundaries
    const int RO = (BN + d.wo - 2) / d.wo;
    const int cross = (d.ho - 1 + RO) / d.ho;
    nbp = (int64_t)(RO * d.sh + cross * (d.hp - d.ho * d.sh) + d.kh) * d.wp;
  }
  if (nbp > PPTMAX * nt) return -1;
  b.plane = (int)cdiv(nbp * 16, 1024) * 1024;
  b.ppp = b.plane / 1024;
  const int W = nt / 64;
  b.nbw = (int)cdiv(npl * b.ppp, W);
  if (b.nbw > NBWMAX) return -1;
  b.bufsz = b.nbw * W * 1024;
  // chunk c+1's band is issued in NBS-piece slices with the DMA groups of stages (c, D-1 .. ns-1)
  if (b.nc > 1 && b.nbw > NBS * (b.ns - D + 1)) return -1;
  b.nbuf = b.nc > 1 ? 2 : 1;
  b.band_off = D * BM * 64;
  b.dummy_off = b.band_off + b.nbuf * b.bufsz;
  b.zero_off = b.dummy_off + W * 1024;
  b.tap_off = b.zero_off + 64;
  b.s_off = b.tap_off + 256;
  b.mask_off = b.s_off + (int)nbp * 4;
  const int lds = b.mask_off + (d.kmask ? d.kpad : 0);
  if (lds > LDS_MAX / bpc) return -1;
  return lds;
}

template <class C>
static int plan_lds(int lds_main, Params& q) {
  lds_main = (lds_main + 15) & ~15;
  const int k = epi_kind(q.e);
  const int epi = 4 * (7 + q.e.nclass) * C::BM + (k == EK_LUT ? 256 * C::BM : 0);
  int lds;
  if (lds_main + epi <= LDS_MAX / C::BPC) {
    q.epi_early = 1, q.epi_off = lds_main;
    lds = lds_main + epi;
  } else {
    q.epi_early = 0, q.epi_off = 0;
    lds = epi > lds_main ? epi : lds_main;
  }
  q.scr_off = 0;
  return lds > LDS_MAX ? -1 : lds;
}

template <class C, int EK, int NPL, bool MASKED>
static int launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  auto kern = qconv16_kernel<C, EK, NPL, MASKED>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  Band16 b;
  const int main = band16(p, C::BM, C::BN, C::NT, C::D, C::BPC, b);
  if (main < 0) return arg_error("tile configuration not built for this layer / epilogue kind");
  Params q = p;
  const int lds = plan_lds<C>(main, q);
  if (lds < 0) return arg_error("conv tile needs more than 160 KiB of LDS (too many border classes)");
  const int nblk = (int)(cdiv(p.M, C::BN) * cdiv(p.d.cout, C::BM));
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(C::NT), lds, s, x, w, q, b);
  return QNN_OK;
}

template <class C, int EK>
static int launch_m(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  const int npl = p.d.cp >= 64 ? 4 : p.d.cp / 16;
  if (npl == 4 && !p.d.kmask) return launch<C, EK, 4, false>(x, w, p, s);
  if constexpr (C::BM == 64) {  // few-channel inputs (stems, CIFAR): narrow output tiles only
    if (p.d.kmask) return launch<C, EK, 1, true>(x, w, p, s);
    if (npl == 2) return launch<C, EK, 2, false>(x, w, p, s);
    if (npl == 1) return launch<C, EK, 1, false>(x, w, p, s);
  }
  return arg_error("tile configuration not built for this layer / epilogue kind");
}

template <class C>
static int launch_ek(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  switch (epi_kind(p.e)) {
    case EK_NCHW: return launch_m<C, EK_NCHW>(x, w, p, s);
    case EK_LUT: return launch_m<C, EK_LUT>(x, w, p, s);
    case EK_BNCODE: return launch_m<C, EK_BNCODE>(x, w, p, s);
    default:
      if constexpr (C::TM * C::TN > 16) return arg_error("tile configuration not built for this layer / epilogue kind");
      else return launch_m<C, EK_GEN>(x, w, p, s);
  }
}

//   id   block (cout x px)   waves (each)          blocks/CU  (all: two waves per SIMD)
//   0    256 x 256           8 (64 x 128)          1
//   1    256 x 208           8 (32 x 208)          1   (a 14x14 image + 12 px: 242 tiles for R50 l3)
//   2    128 x 256           8 (64 x 64)           1
//   3    256 x 128           8 (64 x 64)           1
//   4     64 x 256           4 (64 x 64)           2
//   5    128 x 128           4 (64 x 64)           2
//   6     64 x 128           4 (64 x 32)           2-4
//   7     64 x 512           8 (64 x 64)           1   (64-channel layers: one weight stream per CU)
using Q0 = Cfg<4, 2, 4, 8, 4, 1>;
using Q1 = Cfg<8, 1, 2, 13, 4, 1>;
using Q2 = Cfg<2, 4, 4, 4, 4, 1>;
using Q3 = Cfg<4, 2, 4, 4, 4, 1>;
using Q4 = Cfg<1, 4, 4, 4, 4, 2>;
using Q5 = Cfg<2, 2, 4, 4, 4, 2>;
using Q6 = Cfg<1, 4, 4, 2, 4, 2>;
using Q7 = Cfg<1, 8, 4, 4, 4, 1>;
constexpr int NQ = 8;
struct Info {
  int bm, bn, nt, bpc, acc_tiles;
  float rate;
};
static const Info INFO[NQ] = {
    {256, 256, 512, 1, 32, 0.74f}, {256, 208, 512, 1, 26, 0.70f}, {128, 256, 512, 1, 16, 0.55f},
    {256, 128, 512, 1, 16, 0.55f}, {64, 256, 256, 2, 16, 0.55f},  {128, 128, 256, 2, 16, 0.55f},
    {64, 128, 256, 2, 8, 0.45f},   {64, 512, 512, 1, 16, 0.50f},
};

}  // namespace q16

int q16_count() { return q16::NQ; }

void q16_tile(int k, int* bm, int* bn) {
  *bm = q16::INFO[k].bm;
  *bn = q16::INFO[k].bn;
}

bool q16_ok(int k, const Params& p) {
  using namespace q16;
  if (k < 0 || k >= NQ) return false;
  const Info& f = INFO[k];
  if (epi_kind(p.e) == EK_GEN && f.acc_tiles > 16) return false;  // the general chain spills beside 128 acc regs
  if (p.e.nres > 0 || (p.e.out_bncode && p.e.bncode_tiled)) return false;  // residual code chains: qconv.hip only
  if ((p.d.kmask || p.d.cp < 64) && f.bm != 64) return false;
  Band16 b;
  return band16(p, f.bm, f.bn, f.nt, 4, f.bpc, b) >= 0;
}

double q16_cost(int k, const Params& p) {
  const q16::Info& c = q16::INFO[k];
  const int64_t tiles = cdiv(p.M, c.bn) * cdiv(p.d.cout, c.bm);
  const int64_t slots = (int64_t)NUM_CU * c.bpc;
  const int64_t rounds = cdiv(tiles, slots);
  const double share = tiles < slots ? (double)cdiv(tiles, NUM_CU) : (double)c.bpc;
  return (double)rounds * share * c.bm * c.bn * p.d.kpad / c.rate;
}

int q16_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  using namespace q16;
  switch (k) {
    case 0: return launch_ek<Q0>(x, w, p, s);
    case 1: return launch_ek<Q1>(x, w, p, s);
    case 2: return launch_ek<Q2>(x, w, p, s);
    case 3: return launch_ek<Q3>(x, w, p, s);
    case 4: return launch_ek<Q4>(x, w, p, s);
    case 5: return launch_ek<Q5>(x, w, p, s);
    case 6: return launch_ek<Q6>(x, w, p, s);
    default: return launch_ek<Q7>(x, w, p, s);
  }
}

}  // namespace qnn
