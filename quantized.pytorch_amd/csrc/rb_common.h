// Shared by the resident-band kernels (qconv_rb.hip: whole band before the K loop;
// qconv_rs.hip: the band streamed in chunks): tile configurations, band geometry.
#pragma once
#include <type_traits>
#include <utility>

#include "qconv_common.h"
#include "epi16.h"

#ifndef QNN_STAMP
#define QNN_STAMP 0  // diagnostic builds only: per-wave s_memtime phase stamps
#endif
#if QNN_STAMP
#define RB_TS(v)                                                                          \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#else
#define RB_TS(v) ((void)0)
#endif

namespace qnn {
namespace rb {

template <class F, int... J>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, J...>) {
  (f(std::integral_constant<int, J>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// s_waitcnt lgkmcnt(N) for the hand-counted inline-asm LDS reads; the scheduling barrier keeps
// the compiler from hoisting register-only MFMAs above it
template <int N>
__device__ __forceinline__ void lds_wait() {
  static_assert(N >= 0 && N < 16, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// WGM x WGN waves; a wave owns TM 16-channel tiles x TN 16-pixel tiles; DA weight register
// slots per wave (DA - 1 K steps in flight); BPC blocks per CU the registers and LDS must allow.
// s_waitcnt vmcnt(n) for a wave-uniform run-time n (clamped to the counter's 63: a longer wait)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  n = n < 63 ? n : 63;
  static_for<64>([&](auto c) {
    if (n == decltype(c)::value) wait_vmcnt<decltype(c)::value>();
  });
}

template <int WGM_, int WGN_, int TM_, int TN_, int DA_, int BPC_>
struct Cfg {
  static constexpr int WGM = WGM_, WGN = WGN_, TM = TM_, TN = TN_, DA = DA_, BPC = BPC_;
  static constexpr int W = WGM * WGN, NT = 64 * W;
  static constexpr int BM = WGM * TM * 16;  // output channels per block
  static constexpr int BN = WGN * TN * 16;  // pixel columns per block (>= the block's pixels)
};

constexpr int NBW_MAX = 16;  // band DMA pieces per wave

struct Geo {
  int rows;       // flattened output rows (n*ho) per block
  int npx;        // output pixels per block (rows * wo)
  int nbands;     // blocks along the pixels
  int nbrows;     // padded input rows of a band
  int wb, we, s2; // band row width (= wp); stride 2: even columns first, we = (wp + 1) / 2
  int nbp;        // band pixels (nbrows * wb)
  int pl;         // bytes per 32-byte plane (1 KiB multiple)
  int npl;        // planes (cp / 32)
  int ppp;        // 1 KiB DMA pieces per plane
  int nbw;        // band DMA pieces per wave
  int lut;        // EK_LUT: the 256-byte-per-channel code table is staged (else evaluated)
  int psum_off;   // LDS: int channel sum of each band pixel
  int tap_off;    // LDS: int band offset (pixels) of each tap
  int cls_off;    // LDS: int hcls[ho] * nwc, then wcls[wo]
  int main_bytes; // LDS of the main loop (band + psum + taps)
};


struct Info {
  int bm, bn, w, bpc, acc_tiles;
  float rate;
};

// Rows per block: whole images when an image fits the pixel columns, else the largest
// divisor of ho that does (so no block straddles an image and every band has the same
// height) and whose band fits LDS.  Returns the main-loop LDS bytes or -1.
static int geometry(const Params& p, int BM, int BN, int W, int bpc, int epi_min, Geo& g) {
  const qnn_conv_desc& d = p.d;
  if (p.taps <= 1 || d.kmask || d.cp % 64 != 0) return -1;
  if (d.sh != d.sw || (d.sh != 1 && d.sh != 2)) return -1;
  if (d.kpad < p.taps * d.cp) return -1;
  if ((d.cp / 64) * p.taps % 3 != 0) return -1;  // K steps in whole rounds of the DA = 3 weight ring
  g.s2 = d.sh == 2;
  g.we = (d.wp + 1) / 2;
  g.npl = d.cp / 32;
  const int img = d.ho * d.wo;
  auto fit = [&](int rows, int nbrows) {
    g.rows = rows;
    g.npx = rows * d.wo;
    g.nbrows = nbrows;
    g.nbp = nbrows * g.wb;
    g.pl = (int)cdiv((int64_t)g.nbp * 32, 1024) * 1024;
    g.ppp = g.pl / 1024;
    g.nbw = (int)cdiv(g.ppp, W) * g.npl;
    g.psum_off = g.npl * g.pl;
    g.tap_off = g.psum_off + ((g.nbp * 4 + 15) & ~15);
    g.cls_off = g.tap_off + 4 * MAX_TAPS;
    g.main_bytes = (g.cls_off + 4 * (d.ho + d.wo) + 15) & ~15;  // the epilogue data after it: 16-B aligned
    return g.nbw <= 4 * NBW_MAX && g.main_bytes + epi_min <= LDS_MAX / bpc;
  };
  bool ok = false;
  // candidates, largest first: k whole images, then divisors of ho; the first that fits LDS
  // and gives at least one block per CU, else the first that fits
  const int nby = (int)cdiv(d.cout, BM);
  int best_rows = 0, best_nbrows = 0;
  g.wb = d.wp;
  {
    int first_rows = 0, first_nbrows = 0;
    auto consider = [&](int rows, int nbrows) {
      if (ok || !fit(rows, nbrows)) return;
      if (!first_rows) first_rows = rows, first_nbrows = nbrows;
      if (cdiv((int64_t)d.n * d.ho, rows) * nby >= NUM_CU) ok = true, best_rows = rows, best_nbrows = nbrows;
    };
    if (img <= BN)
      for (int k = BN / img < d.n ? BN / img : d.n; k >= 1; --k) consider(k * d.ho, (k - 1) * d.hp + (d.ho - 1) * d.sh + d.kh);
    for (int rows = d.ho - 1; rows >= 1; --rows)
      if (d.ho % rows == 0 && rows * d.wo <= BN) consider(rows, (rows - 1) * d.sh + d.kh);
    if (!ok && first_rows) ok = true, best_rows = first_rows, best_nbrows = first_nbrows;
  }
  if (ok) fit(best_rows, best_nbrows);
  if (!ok) return -1;
  g.nbands = (int)cdiv((int64_t)d.n * d.ho, g.rows);
  return g.main_bytes;
}

static int epi_bytes(const Params& p, int BM) {
  const int k = epi_kind(p.e);
  return 4 * (7 + p.e.nclass) * BM + (k == EK_GEN ? 16 * p.e.nres * BM : 0);  // no LUT: EK_LUT is evaluated
}

// LDS bytes of one block and the Params/Geo it runs with, or a negative status
}  // namespace rb
}  // namespace qnn
