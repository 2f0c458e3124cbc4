// Resident-band int8 convolution with two priority teams (v_mfma_i32_16x16x64_i8): the eval
// forward of QConv2d (models/modules/quantize.py:314-349) for the deep 3x3 layers whose whole
// input band fits one CU's LDS beside the epilogue data -- ResNet-50 layer 3's 256@14x14 (the
// north star's headline, one 14x14 image per block) and its 512@7x7 pairs.  Same exact
// decomposition and epilogue arithmetic as qconv_rb.hip, so the outputs are
// bitwise those of every other tile configuration.
//
// qconv_rb.hip's resident-band kernel runs its phases in series -- the whole band lands, the
// K loop runs, the channel sums of the band are reduced, the epilogue runs -- and at one image
// per CU (ResNet-50 b256 on 256 CUs) nothing else hides them: about half of a block's life is
// outside the K loop.  Here one 512-thread block (two waves per SIMD) owns BM = 256 output
// channels x the block's pixels, split into two TEAMS of four waves (one wave per SIMD each):
//
// * team 0 (waves 0-3, channels [0, 128)) runs at s_setprio 2, team 1 (waves 4-7, channels
//   [128, 256)) at 0.  Their K loops share each SIMD's matrix pipe; team 0 wins every
//   arbitration, so it finishes its K loop first and runs its epilogue (VALU, LDS, stores)
//   while team 1's MFMAs still fill the pipe.  Only team 1's epilogue is exposed.
// * the band lands in K-group chunks (planes 2g, 2g+1 = input channels [64g, 64g + 64) of every
//   band pixel).  EVERY wave of both teams loads it: each wave issues ppp / 4 of a chunk's
//   2 ppp 1 KiB pieces (issue_own; chunk 0 in the prologue, chunk g + 1 during taps 0-3 of
//   chunk g), waits for its own pieces with a counted vmcnt that leaves its younger weight
//   loads in flight (so a wave's in-order vmcnt waits do cover its own band DMA), and adds 1
//   to the chunk's LDS counter; every wave polls for all 8 arrivals before its first step of a
//   chunk.  No workgroup barrier after the start.  The stagger is team 0's priority only.
// * sum_valid(q'_x): as its pieces of a chunk land, every wave sums the bytes each of its lanes
//   moved (v_dot4 against 1s) into a per-band-pixel channel sum in LDS (sum_chunk); after the
//   K loop one team-0 lane per output pixel sums its taps.  Each team stages its own epilogue
//   data (per-channel vectors, border table, code LUT) by LDS-DMA during its last chunk.
#include <stdlib.h>

#include <type_traits>
#include <utility>

#include "qconv_common.h"
#include "epi16.h"

#ifndef QNN_RBP_PRIO
#define QNN_RBP_PRIO 1  // 0: both teams at priority 0 (diagnostic A/B)
#endif
#ifndef QNN_STAMP
#define QNN_STAMP 0  // diagnostic builds only (make stamp_rbp): per-wave s_memtime phase stamps
#endif
#if QNN_STAMP
// [block][wave][8]: realtime start/end (100 MHz); cycles: to chunk 0, K loop, pixel sums ready,
// epilogue data ready, epilogue code, store drain
__device__ unsigned long long qnn_rbp_stamps[1 << 18];
#define RBP_TS(v)                                                                         \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#else
#define RBP_TS(v) ((void)0)
#endif

namespace qnn {
namespace rbp {

template <class F, int... J>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, J...>) {
  (f(std::integral_constant<int, J>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int N>
__device__ __forceinline__ void lds_wait() {
  static_assert(N >= 0 && N < 16, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// LDS accesses that may run while LDS-DMA is in flight are inline asm: the compiler's waitcnt
// pass cannot tell them apart from the DMA'd band and would put a vmcnt(0) -- the whole band --
// in front of every compiler-visible LDS access that follows the DMA issue
__device__ __forceinline__ void lds_add(int* p, int v) {
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_add_u32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ int lds_load(const int* p) {
  int v;
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}

// LDS counters: one lane adds; waiters poll (the counters live in the block's own LDS, so a
// plain workgroup-scope atomic is the whole protocol; LDS-DMA data a counter announces was
// waited for by its issuing wave's vmcnt before the add)
__device__ __forceinline__ void arrive(int* c, int lane) {
  __builtin_amdgcn_sched_barrier(0);
  if (lane == 0) lds_add(c, 1);
  __builtin_amdgcn_sched_barrier(0);
}
// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [0, 63] (prologue only)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  static_for<64>([&](auto c) {
    if (n == decltype(c)::value) wait_vmcnt<decltype(c)::value>();
  });
}
__device__ __forceinline__ void poll(int* c, int target) {
  __builtin_amdgcn_sched_barrier(0);
  while (lds_load(c) < target) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_sched_barrier(0);
}

// 8 waves, TM = 2 (32 channels per wave, BM = 256), TN 16-pixel tiles per wave (every pixel of
// the block), DA = 3 weight register slots (2 K steps of weights in flight)
template <int TN_>
struct Cfg {
  static constexpr int WGM = 8, WGN = 1, TM = 2, TN = TN_, DA = 3, BPC = 1;
  static constexpr int W = 8, NT = 512, BM = 256, BN = 16 * TN;
};

constexpr int SYNC_INTS = 32;  // [0, 16) chunk counters, [16] pixel sums, [17 + team] epilogue data, [20] band sums

struct Geo {
  int rows;        // flattened output rows (n*ho) per block
  int nbands;      // blocks along the pixels
  int nbrows;      // padded input rows of a band
  int wb, we, s2;  // band row width (= wp); stride 2: even columns first, we = (wp + 1) / 2
  int nbp;         // band pixels
  int pl;          // bytes per 32-byte plane (1 KiB multiple)
  int ppp;         // 1 KiB DMA pieces per plane
  int sync_off;    // LDS: SYNC_INTS counters, then the per-pixel channel sums [BN]
  int ps_off;      // LDS: the channel sum of every band pixel [nbp]
  int cls_off;     // LDS: hcls[ho] * nwc, wcls[wo]
  int lut;         // EK_LUT: the 256-byte code table is staged (else evaluated)
  int lds;         // dynamic LDS bytes
};

// ---------------------------------------------------------------- kernel
template <class C, int EK>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void qconv_rbp_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ w, const Params p, const Geo g) {
  constexpr int BM = C::BM, TM = C::TM, TN = C::TN, DA = C::DA, NT = C::NT;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];

  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int team = wave >> 2, tw = wave & 3;
  const int wm = wave;  // 32-channel group of the block
#if QNN_STAMP
  unsigned long long ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0, ts4 = 0, ts5 = 0, ts6 = 0;
  unsigned long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // team 1's prologue: issued, chunks 0-3, sums, staged
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  RBP_TS(ts0);
#endif
#if QNN_RBP_PRIO
  if (team == 0) __builtin_amdgcn_s_setprio(2);
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
  const int r0 = band * g.rows;
  const int nrows_all = d.n * d.ho;
  const int R0 = (r0 / d.ho) * d.hp + (r0 % d.ho) * d.sh;  // first padded input row (batch-flat)
  const int rows_in = d.n * d.hp;

  int* s_sync = reinterpret_cast<int*>(smem + g.sync_off);
  int* s_sum = s_sync + SYNC_INTS;
  int* s_hc = reinterpret_cast<int*>(smem + g.cls_off);
  int* s_ps = reinterpret_cast<int*>(smem + g.ps_off);

  auto tap_off = [&](int tap) {  // band pixel offset of tap (tr, tc); t / kw by p.kw_magic (t < 64)
    const int tr = (tap * p.kw_magic) >> 16, tc = tap - tr * d.kw;
    return tr * g.wb + (g.s2 ? (tc & 1) * g.we + (tc >> 1) : tc);
  };

  // ---- band DMA (team 1): piece r of plane v = band pixels [32r, 32r + 32), lane i pixel
  // + (i >> 1), 16-byte half i & 1; past the band: the last pixel again (identical bytes)
  auto issue_piece = [&](int r, int v) {
    int b = r * 32 + (lane >> 1);
    b = b < g.nbp ? b : g.nbp - 1;
    const int br = b / g.wb, cc = b - br * g.wb;
    const int col = g.s2 ? (cc < g.we ? 2 * cc : 2 * (cc - g.we) + 1) : cc;
    int row = R0 + br;
    row = row < rows_in ? row : rows_in - 1;  // past the batch: feeds only pixels never stored
    const uint32_t off =
        cc >= d.wp ? (uint32_t)d.zero_off : (uint32_t)((row * d.wp + col) * d.cp + 32 * v + 16 * (lane & 1));
    const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(smem + v * g.pl + r * 1024));
    // inline asm: the compiler neither counts these in its vmcnt waits (a wave's VMEM ops finish
    // in order, so unseen older ops only lengthen its waits) nor fences LDS accesses behind them;
    // team 1 waits for them itself, counted (wait_vmcnt_rt), before anything reads the band
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(dst), "v"(off), "s"(x) : "memory", "m0");
  };
  // Chunk gch = planes 2gch, 2gch + 1 = 2 ppp pieces, NPW = ppp / 4 per wave (geometry: ppp % 4
  // == 0); this wave's piece i of it is piece k = wave + 8 i.
  auto issue_own = [&](int gch, int i) {
    const int k = wave + 8 * i, hi = k >= g.ppp;
    issue_piece(k - (hi ? g.ppp : 0), 2 * gch + hi);
  };
  // sum_valid(q'_x), part 1: once a wave's pieces of chunk gch have landed, each lane sums the
  // 16 bytes it moved itself (v_dot4 against 1s), the two halves of a pixel combine, and the
  // pixel's channel sum accumulates in LDS (exact integer adds in any order)
  auto sum_chunk = [&](int gch) {
    for (int k = wave; k < 2 * g.ppp; k += 8) {
      const int hi = k >= g.ppp, r = k - (hi ? g.ppp : 0);
      v4i a;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(a)
                   : "v"((uint32_t)(uintptr_t)(smem + (2 * gch + hi) * g.pl + r * 1024 + 16 * lane))
                   : "memory");
      int s = __builtin_amdgcn_sdot4(a.x, 0x01010101, 0, false);
      s = __builtin_amdgcn_sdot4(a.y, 0x01010101, s, false);
      s = __builtin_amdgcn_sdot4(a.z, 0x01010101, s, false);
      s = __builtin_amdgcn_sdot4(a.w, 0x01010101, s, false);
      s += __builtin_amdgcn_update_dpp(0, s, 0xB1, 0xF, 0xF, false);  // + lane ^ 1 (quad_perm 1,0,3,2)
      const int b = r * 32 + (lane >> 1);
      if ((lane & 1) == 0 && b < g.nbp) lds_add(&s_ps[b], s);
    }
  };

  // LDS-DMA in inline asm (a lane's bytes land at the wave-uniform LDS address + lane * size):
  // invisible to the compiler's vmcnt bookkeeping, waited for explicitly (wait_vmcnt<0> before
  // the epilogue), so the K loop's weight waits stay counted
  auto dma4 = [&](const void* src, int8_t* ldst) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(m), "v"(src) : "memory", "m0");
  };
  auto dma16 = [&](const void* src, int8_t* ldst) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m), "v"(src) : "memory", "m0");
  };
  // ---- the team's epilogue data by LDS-DMA (qconv_common.h stage_epi's layout; this team's
  // 64-channel chunks k = 2 team, 2 team + 1)
  const bool lut_on = EK == EK_LUT && g.lut;
  auto stage_team = [&] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int cmax = d.cout - 1;
    const int nvec = (EK != EK_NCHW && e.bn_mean) ? 7 : 3;
    const int nf = (nvec + e.nclass) * 2;
    int8_t* dst = smem + p.epi_off;
    for (int jb = tw; jb < nf; jb += 4) {
      const int v = jb >> 1, k = 2 * team + (jb & 1);
      const int arr = v < nvec ? v : 7 + (v - nvec);
      int c = c0 + 64 * k + lane;
      c = c < cmax ? c : cmax;
      const float* src;
      switch (arr) {
        case 0: src = e.sxsw; break;
        case 1: src = e.sxbw; break;
        case 2:
          if (!e.bias) {  // no bias: zeros from the input's 128-byte zero page
            src = reinterpret_cast<const float*>(x + d.zero_off);
            c = lane & 31;
          } else {
            src = e.bias;
          }
          break;
        case 3: src = e.bn_mean; break;
        case 4: src = e.bn_sq; break;
        case 5: src = e.bn_wq; break;
        case 6: src = e.bn_bq; break;
        default: src = e.table + (int64_t)(arr - 7) * d.cout; break;
      }
      dma4(src + c, dst + 4 * (arr * BM + 64 * k));
    }
    if (lut_on) {
      int8_t* lut = dst + 4 * (7 + e.nclass) * BM;
      for (int jl = 32 * team + tw; jl < 32 * team + 32; jl += 4) {
        int c = c0 + 4 * jl + (lane >> 4);
        c = c < cmax ? c : cmax;
        dma16(e.lut + (int64_t)c * 256 + 16 * (lane & 15), lut + 1024 * jl);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };

  // ---- this lane's pixels: block pixel q = j*16 + (lane & 15); past the block (or the
  // batch) they stand in for the block's last pixel and are never stored
  const int npx_blk = __builtin_amdgcn_readfirstlane((r0 + g.rows <= nrows_all ? g.rows : nrows_all - r0) * d.wo);
  int pb[TN];  // band byte offset of tap (0, 0) in the fragment's plane
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int q = j * 16 + (lane & 15);
    q = q < npx_blk ? q : npx_blk - 1;
    const int rr = q / d.wo, col = q - rr * d.wo;
    const int r = r0 + rr, n = r / d.ho, ho = r - n * d.ho;
    pb[j] = ((n * d.hp + ho * d.sh - R0) * g.wb + col) * 32 + (lane >> 5) * g.pl + 16 * ((lane >> 4) & 1);
  }

  // ---- weights: rows c0 + 32 wm + 16 i + (lane & 15), K bytes 16 (lane >> 4) of each step;
  // K steps group-major: step (gk, tap) = weight bytes tap * cp + 64 gk, band planes 2gk, 2gk+1
  const int8_t* wblk = w + (int64_t)c0 * d.kpad;
  uint32_t aoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int row = 32 * wm + 16 * i + (lane & 15);
    row = c0 + row < d.cout_pad ? row : d.cout_pad - 1 - c0;
    aoff[i] = (uint32_t)(row * d.kpad + 16 * (lane >> 4));
  }
  const int G = d.cp / 64, taps = p.taps;
  v4i fa[DA][TM];
  int lg = 0, lt = 0;  // the next step to load
  auto load_a = [&](v4i (&dst)[TM]) __attribute__((always_inline)) {
    const int8_t* base = wblk + lt * d.cp + 64 * lg;
#pragma unroll
    for (int i = 0; i < TM; ++i) dst[i] = *reinterpret_cast<const v4i*>(base + aoff[i]);
    if (++lt == taps) {
      if (lg + 1 < G) lt = 0, ++lg;
      else lt = taps - 1;  // clamp at the last step
    }
  };

  // ---- prologue: every wave issues its pieces of chunk 0 and the first DA - 1 steps' weights,
  // publishes the chunk once its pieces landed (the vmcnt leaves the weight loads in flight)
  // and sums the bytes it moved
  const int NPW = g.ppp / 4;
  for (int i = tid; i < SYNC_INTS + C::BN; i += NT) s_sync[i] = 0;
  for (int i = tid; i < g.nbp; i += NT) s_ps[i] = 0;
  // the only workgroup barrier (the counters are zero).  A raw s_barrier: __syncthreads()'s
  // release fence would also wait for every VMEM op in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#if QNN_STAMP
  RBP_TS(tp[0]);
#endif
  for (int i = 0; i < NPW; ++i) issue_own(0, i);
#pragma unroll
  for (int s = 0; s < DA - 1; ++s) load_a(fa[s]);
#if QNN_STAMP
  RBP_TS(tp[1]);
#endif
  wait_vmcnt<(DA - 1) * TM>();
#if QNN_STAMP
  RBP_TS(tp[2]);
#endif
  arrive(&s_sync[0], lane);
  sum_chunk(0);
#if QNN_STAMP
  RBP_TS(tp[3]);
#endif

  v4i acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4i){0, 0, 0, 0};
  auto step = [&](auto slotc, int gk, int tap) __attribute__((always_inline)) {
    constexpr int SL = decltype(slotc)::value;
    const int boff = 2 * gk * g.pl + 32 * tap_off(tap);
    v4i fb[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      v4i r;
      asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(pb[j] + boff));
      fb[j] = r;
    }
    static_for<TN>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      lds_wait<(TN - 1 - j < 15 ? TN - 1 - j : 15)>();
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[SL][i], fb[j], acc[i][j], 0, 0, 0);
    });
    __builtin_amdgcn_sched_barrier(0);
    // refill slot (SL + DA - 1) % DA, last read one step earlier (never the slot just read:
    // DESIGN.md §4, tools/asm_mfma_war_check.py)
    load_a(fa[(SL + DA - 1) % DA]);
  };
  // The next chunk's pieces, one per wave every second step (after that step's weight loads:
  // taps 1 and 3), published at the start of tap 6: every VMEM op issued after the last piece
  // by then is one of the 2 TM weight loads of taps 4 and 5, so a counted vmcnt(2 TM) covers
  // it, and the compiler's own weight waits before tap 6 are for loads issued before it -- the
  // DMA never stalls the K loop unless a piece takes two steps to land.  (Geometry: NPW <= 2,
  // taps == 9.)  Straight-line per group: no VMEM op the compiler sees but the weight loads.
  if (G == 1) arrive(&s_sync[20], lane);
#pragma nounroll
  for (int gk = 0; gk < G; ++gk) {
    poll(&s_sync[gk], 8);  // chunk gk landed (every wave's pieces)
#if QNN_STAMP
    if (gk == 0) RBP_TS(ts1);
#endif
    const bool more = gk + 1 < G;
#pragma nounroll
    for (int t0 = 0; t0 < taps; t0 += 3) {
      if (more && t0 == 6) {
        wait_vmcnt<2 * TM>();
        arrive(&s_sync[gk + 1], lane);
        sum_chunk(gk + 1);
        if (gk + 2 == G) arrive(&s_sync[20], lane);  // this wave's band-pixel sums are all in
      }
      step(std::integral_constant<int, 0>{}, gk, t0);
      if (more && t0 == 3 && NPW > 1) issue_own(gk + 1, 1);
      step(std::integral_constant<int, 1>{}, gk, t0 + 1);
      if (t0 == 0) {
        if (more) issue_own(gk + 1, 0);
        else stage_team();  // the team's epilogue data, behind every chunk
      }
      step(std::integral_constant<int, 2>{}, gk, t0 + 2);
    }
  }
#if QNN_STAMP
  RBP_TS(ts2);
#endif
  // ---- sum_valid(q'_x), part 2, by the first team out of its K loop (team 0, priority): one
  // lane per output pixel sums its taps of the band-pixel sums (padding codes are 0, so this is
  // the receptive field's exact sum)
  if (team == 0) {
    if (tw == 0)  // the border-class tables (ho + wo entries: more than one wave's lanes at 56x56)
      for (int i = lane; i < d.ho + d.wo; i += 64) s_hc[i] = i < d.ho ? e.hcls[i] * e.nwc : e.wcls[i - d.ho];
    poll(&s_sync[20], 8);
    for (int q = 64 * tw + lane; q < C::BN; q += 256) {
      int qq = q < npx_blk ? q : npx_blk - 1;
      const int rr = qq / d.wo, col = qq - rr * d.wo;
      const int r = r0 + rr, n = r / d.ho, ho = r - n * d.ho;
      const int b0 = (n * d.hp + ho * d.sh - R0) * g.wb + col;
      int sm = 0;
      for (int tt = 0; tt < taps; ++tt) sm += s_ps[b0 + tap_off(tt)];
      s_sum[q] = sm;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    arrive(&s_sync[16], lane);
  }
  poll(&s_sync[16], 4);  // the pixel sums
  int sumq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] = s_sum[16 * j + (lane & 15)];
#if QNN_STAMP
  RBP_TS(ts3);
#endif
  // the team's epilogue data (staged by its four waves) and this wave's tail weight loads
  wait_vmcnt<0>();
  arrive(&s_sync[17 + team], lane);
  poll(&s_sync[17 + team], 4);
#if QNN_STAMP
  RBP_TS(ts4);
#endif

  // ---- epilogue (qconv_rb.hip's, this wave's 32 channels x TN tiles)
  {
    const int HoWo = d.ho * d.wo;
    int cq = lane & 15;
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
    if (lut_on && c0 + BM <= d.cout && c0 + BM <= e.code0_cp) {
      // fast path of the common case (a full channel tile, the code table staged)
      const float* s_f = reinterpret_cast<const float*>(smem + p.epi_off);
      const int8_t* s_lut = smem + p.epi_off + 4 * (7 + e.nclass) * BM;
      const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
      const int gq = lane >> 4;
      float4 sw[TM], bw[TM], bi[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int cl = 32 * wm + 16 * i + 4 * gq;
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
                                       e.code0_cp + c0 + 32 * wm + 4 * gq;
        const float* tp = s_f + (7 + pc) * BM + 32 * wm + 4 * gq;
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
          const int8_t* lp = s_lut + (32 * wm + 16 * i + 4 * gq) * 256;
          const int b0 = (uint8_t)lp[__float_as_uint(q0.x) & 255u];
          const int b1 = (uint8_t)lp[256 + (__float_as_uint(q0.y) & 255u)];
          const int b2 = (uint8_t)lp[512 + (__float_as_uint(q1.x) & 255u)];
          const int b3 = (uint8_t)lp[768 + (__float_as_uint(q1.y) & 255u)];
          *reinterpret_cast<int*>(op + 16 * i) = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
        }
      }
    } else {
      q16::epilogue_rb<C, EK>(p, acc, sumq, pixel, smem, c0, wm, lane, lut_on ? 1 : 0);
    }
  }
#if QNN_STAMP
  RBP_TS(ts5);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  RBP_TS(ts6);
  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && blockIdx.x < (1 << 18) / 128) {
    unsigned long long* o = qnn_rbp_stamps + ((size_t)blockIdx.x * 8 + wave) * 16;
    o[0] = rt0; o[1] = rt1; o[2] = ts1 - ts0; o[3] = ts2 - ts1; o[4] = ts3 - ts2; o[5] = ts4 - ts3;
    o[6] = ts5 - ts4; o[7] = ts6 - ts5;
    for (int i = 0; i < 7; ++i) o[8 + i] = tp[i] ? tp[i] - ts0 : 0;
  }
#endif
}

// ---------------------------------------------------------------- host side
// Rows per block: k whole images when they fit the pixel columns, else the largest divisor of
// ho that does; the first candidate whose band + epilogue data fit LDS and that gives at least
// one block per CU, else the first that fits.  Returns the LDS bytes or -1.
static int geometry(const Params& p, int BM, int BN, int ek, Geo& g) {
  const qnn_conv_desc& d = p.d;
  if (p.taps != 9 || d.kmask || d.cp % 64 != 0 || d.cp > 1024) return -1;
  const int G = d.cp / 64;
  if (d.sh != d.sw || (d.sh != 1 && d.sh != 2)) return -1;
  if (d.kpad < p.taps * d.cp) return -1;
  if (ek == EK_GEN) return -1;  // residual chains: qconv_rb.hip
  g.s2 = d.sh == 2;
  g.wb = d.wp;
  g.we = (d.wp + 1) / 2;
  const int npl = d.cp / 32, img = d.ho * d.wo;
  const int epi_vec = 4 * (7 + p.e.nclass) * BM;
  auto fit = [&](int rows, int nbrows, int lut) {
    g.rows = rows;
    g.nbrows = nbrows;
    g.nbp = nbrows * g.wb;
    g.pl = (int)cdiv((int64_t)g.nbp * 32, 1024) * 1024;
    g.ppp = g.pl / 1024;
    if (g.ppp % 4 != 0) g.ppp += 4 - g.ppp % 4, g.pl = 1024 * g.ppp;  // every wave moves ppp / 4 pieces a chunk
    g.sync_off = npl * g.pl;
    g.ps_off = g.sync_off + 4 * (SYNC_INTS + BN);
    g.cls_off = g.ps_off + 4 * g.nbp;
    const int epi_off = (g.cls_off + 4 * (d.ho + d.wo) + 15) & ~15;
    g.lut = lut;
    g.lds = epi_off + epi_vec + (lut ? 256 * BM : 0);
    if (g.ppp / 4 > 2) return -1;  // the next chunk is issued and published within a group
    return g.lds <= LDS_MAX ? epi_off : -1;
  };
  const int nby = (int)cdiv(d.cout, BM);
  int best_rows = 0, best_nbrows = 0, first_rows = 0, first_nbrows = 0;
  auto consider = [&](int rows, int nbrows) {
    if (best_rows || fit(rows, nbrows, 0) < 0) return;
    if (!first_rows) first_rows = rows, first_nbrows = nbrows;
    if (cdiv((int64_t)d.n * d.ho, rows) * nby >= NUM_CU) best_rows = rows, best_nbrows = nbrows;
  };
  if (img <= BN)
    for (int k = BN / img < d.n ? BN / img : d.n; k >= 1; --k) consider(k * d.ho, (k - 1) * d.hp + (d.ho - 1) * d.sh + d.kh);
  for (int rows = d.ho - 1; rows >= 1; --rows)
    if (d.ho % rows == 0 && rows * d.wo <= BN) consider(rows, (rows - 1) * d.sh + d.kh);
  if (!best_rows) best_rows = first_rows, best_nbrows = first_nbrows;
  if (!best_rows) return -1;
  // the code LUT beside the band when it fits (else the same ops evaluated)
  int off = fit(best_rows, best_nbrows, ek == EK_LUT ? 1 : 0);
  if (off < 0) off = fit(best_rows, best_nbrows, 0);
  if (off < 0) return -1;
  g.nbands = (int)cdiv((int64_t)d.n * d.ho, g.rows);
  return off;
}

template <class C, int EK>
static int launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  auto kern = qconv_rbp_kernel<C, EK>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  Geo g;
  const int off = geometry(p, C::BM, C::BN, EK, g);
  if (off < 0) return arg_error("tile configuration not built for this layer / epilogue kind");
  Params q = p;
  q.epi_off = off;
  q.epi_early = 1;
  q.scr_off = 0;
  const int nblk = g.nbands * (int)cdiv(p.d.cout, C::BM);
  if (occ) {
    int n = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, C::NT, g.lds);
    if (e != hipSuccess) return hip_check(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    occ->blocks_per_cu = n, occ->lds = g.lds, occ->grid = nblk;
    return QNN_OK;
  }
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(C::NT), g.lds, s, x, w, q, g);
  return QNN_OK;
}

template <class C>
static int launch_ek(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  switch (epi_kind(p.e)) {
    case EK_NCHW: return launch<C, EK_NCHW>(x, w, p, s, occ);
    case EK_LUT: return launch<C, EK_LUT>(x, w, p, s, occ);
    case EK_BNCODE: return launch<C, EK_BNCODE>(x, w, p, s, occ);
    default: return arg_error("tile configuration not built for this layer / epilogue kind");
  }
}

//   id  block (cout x px cols)  fits
//   0   256 x 208               one 14x14 image (ResNet-50 layer 3 at b256; 196 of 208 columns)
//   1   256 x 112               half a 14x14 image (7 rows) or two 7x7 images (layer 4)
using P0 = Cfg<13>;
using P1 = Cfg<7>;
constexpr int NP = 2;
struct Info {
  int bm, bn;
  float rate;
};
static const Info INFO[NP] = {{256, 208, 1.60f}, {256, 112, 1.30f}};

}  // namespace rbp

int rbp_count() { return rbp::NP; }

#if QNN_STAMP
extern "C" int qnn_debug_stamps_rbp(void* dst, size_t bytes) {
  if (bytes > sizeof(::qnn_rbp_stamps)) bytes = sizeof(::qnn_rbp_stamps);
  return hip_check(hipMemcpyFromSymbol(dst, HIP_SYMBOL(::qnn_rbp_stamps), bytes), "stamps");
}
#endif

void rbp_tile(int k, int* bm, int* bn) {
  *bm = rbp::INFO[k].bm;
  *bn = rbp::INFO[k].bn;
}

bool rbp_ok(int k, const Params& p) {
  if (k < 0 || k >= rbp::NP) return false;
  rbp::Geo g;
  return rbp::geometry(p, rbp::INFO[k].bm, rbp::INFO[k].bn, epi_kind(p.e), g) >= 0;
}

int64_t rbp_blocks(int k, const Params& p) {
  rbp::Geo g;
  if (rbp::geometry(p, rbp::INFO[k].bm, rbp::INFO[k].bn, epi_kind(p.e), g) < 0) return 0;
  return (int64_t)g.nbands * cdiv(p.d.cout, rbp::INFO[k].bm);
}

double rbp_cost(int k, const Params& p) {
  const rbp::Info& f = rbp::INFO[k];
  rbp::Geo g;
  if (rbp::geometry(p, f.bm, f.bn, epi_kind(p.e), g) < 0) return 1e30;
  const int64_t tiles = (int64_t)g.nbands * cdiv(p.d.cout, f.bm);
  const int64_t rounds = cdiv(tiles, NUM_CU);
  const double share = tiles < NUM_CU ? 1.0 : 1.0;
  return (double)rounds * share * f.bm * f.bn * (p.taps * p.d.cp) / f.rate;
}

int rbp_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  switch (k) {
    case 0: return rbp::launch_ek<rbp::P0>(x, w, p, s, occ);
    default: return rbp::launch_ek<rbp::P1>(x, w, p, s, occ);
  }
}

}  // namespace qnn
