// Streamed resident-band int8 convolution on v_mfma_i32_16x16x64_i8 (configurations 56-61): the
// eval forward of QConv2d (models/modules/quantize.py:314-349) for 3x3 layers whose whole-image
// band fits LDS, bitwise the other configurations (SURVEY.md §0.5 decomposition, shared epilogue).
#include "rb_common.h"

namespace qnn {
namespace rb {

// ---------------------------------------------------------------- streamed resident band (rs)
// qconv_rb_kernel's tile and main loop (one block per CU owns whole images x BM channels, the
// band resident in LDS as 32-byte planes, each wave's weights straight into VGPRs), with the
// block's serial phases taken off the critical path:
// * the band arrives in CHUNKS of 2H planes (64H channels) in the order the K loop consumes
//   them; the loop starts when chunk 0 has landed.  A wave's VMEM operations complete in order
//   (one vmcnt), so every LDS-DMA a wave issues is implicitly waited for by its next weight wait
//   after it: an in-loop DMA gets DA - 1 K steps to land, no more.  Hence the issue order at
//   kernel start is chunk 0, the first DA - 1 weight steps, then (left in flight) chunk 1 and the
//   epilogue data, and each later chunk c + 1 is issued at chunk c's boundary; a raw s_barrier at
//   each boundary publishes the chunk to the other waves;
// * sum_valid(q'_x): each thread sums its band pixels' channels chunk by chunk at the chunk
//   boundaries (v_dot4 against 1s); after the last, the block's output pixels' 9-tap box sums are
//   computed once (one LDS word per pixel) behind one more barrier, so the epilogue reads one
//   word per pixel tile;
// * each wave DMAs the epilogue data of ITS OWN channels (per-channel vectors, border table, the
//   EK_LUT code-table rows) and waits only for its own DMA: no workgroup barrier after the K loop.
// The DMAs are inline asm (global_load_lds with m0), invisible to the compiler's waitcnt pass:
// it neither drains them before the band reads nor miscounts its weight waits (invisible older
// VMEM ops only make a counted wait stricter).  Outputs are bitwise those of every other
// configuration (the same contraction and epilogue arithmetic).
#if QNN_STAMP
__device__ unsigned long long qnn_rs_stamps[1 << 18];
#endif

// LATE: chunk 1 and the epilogue data issued after chunk 0's barrier instead of at kernel start
// (their issue then stays out of chunk 0's wait; the first in-loop weight wait covers them)
template <class C, int EK, int H, int LATE>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(C::BPC * C::W / 4))) void qconv_rs_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ w, const Params p, const Geo g) {
  constexpr int BM = C::BM, W = C::W, TM = C::TM, TN = C::TN, DA = C::DA, NT = C::NT;
  constexpr int CPL = 2 * H;  // planes per chunk
  static_assert(C::DA >= 1 && C::DA <= 4, "the K loop unrolls at most four weight slots per pass");
  constexpr int NPT = 1;      // band pixels / output pixels per thread (geometry: nbp, npx <= NT)
  constexpr int CW = 16 * TM;  // this wave's channels
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];

  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
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
  const int r0 = band * g.rows;
  const int nrows_all = d.n * d.ho;
  const int R0 = (r0 / d.ho) * d.hp + (r0 % d.ho) * d.sh;
  const int rows_in = d.n * d.hp;

  // ---- band DMA (inline asm): piece (r, v) = 1 KiB of plane v, band pixels [32r, 32r + 32),
  // lane i pixel + (i >> 1), half i & 1; past the band the last pixel again (identical bytes)
  auto issue_piece = [&](int r, int v) {
    r = r < g.ppp ? r : g.ppp - 1;
    int b = r * 32 + (lane >> 1);
    b = b < g.nbp ? b : g.nbp - 1;
    const int br = b / g.wb, cc = b - br * g.wb;
    const int col = g.s2 ? (cc < g.we ? 2 * cc : 2 * (cc - g.we) + 1) : cc;
    int row = R0 + br;
    row = row < rows_in ? row : rows_in - 1;  // past the batch: feeds only pixels never stored
    const uint32_t off =
        cc >= d.wp ? (uint32_t)d.zero_off : (uint32_t)((row * d.wp + col) * d.cp + 32 * v + 16 * (lane & 1));
    const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(smem + v * g.pl + r * 1024));
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(dst), "v"(off), "s"(x) : "memory", "m0");
  };
  const int nchunk = g.npl / CPL;
  const int npr = (g.ppp + W - 1) / W;  // this wave's ranges r = wave + W*k of each plane
  const int ppc = npr * CPL;             // its pieces of one chunk
  auto issue_chunk = [&](int c) {
    for (int i = 0; i < ppc; ++i) issue_piece(wave + W * (i / CPL), c * CPL + i % CPL);
  };

  // ---- the epilogue data of this wave's channels cw0 .. cw0 + CW (qconv_common.h stage_epi's
  // layout): per vector / table array one 4-byte-per-lane DMA per 64 channels, then the EK_LUT
  // code-table rows (1 KiB = 4 rows per 16-byte-per-lane DMA)
  const bool lut_on = EK == EK_LUT && g.lut;
  const bool lutfast = lut_on && c0 + BM <= d.cout && c0 + BM <= e.code0_cp;  // block-uniform
  int8_t* const epi = smem + p.epi_off;
  const int cw0 = wm * CW;
  const int cmax = d.cout - 1;
  constexpr int VJ = (CW + 63) / 64;  // DMAs per array
  const int nvec = (EK != EK_NCHW && e.bn_mean) ? 7 : 3;
  const int narr = nvec + e.nclass + (EK == EK_GEN ? 4 * e.nres : 0);
  const int njobs = narr * VJ + (lut_on ? CW / 4 : 0);  // this wave's epilogue DMAs
  auto issue_epi = [&] {
    for (int v = 0; v < narr; ++v) {
      const int arr = v < nvec ? v : 7 + (v - nvec);
      const float* src;
      bool zero = false;
      switch (arr) {
        case 0: src = e.sxsw; break;
        case 1: src = e.sxbw; break;
        case 2: src = e.bias; zero = !e.bias; break;  // no bias: zeros from the input's zero page
        case 3: src = e.bn_mean; break;
        case 4: src = e.bn_sq; break;
        case 5: src = e.bn_wq; break;
        case 6: src = e.bn_bq; break;
        default:
          if (arr - 7 < e.nclass) {
            src = e.table + (int64_t)(arr - 7) * d.cout;
          } else {
            const int lk = arr - 7 - e.nclass, l = lk >> 2, k4 = lk & 3;
            const qnn_res_link& rl = e.res[l];
            src = k4 == 0 ? rl.mean : k4 == 1 ? rl.sq : k4 == 2 ? rl.wq : rl.bq;
          }
          break;
      }
#pragma unroll
      for (int kk = 0; kk < VJ; ++kk) {
        int c = c0 + cw0 + 64 * kk + lane;
        c = c < cmax ? c : cmax;
        const float* sp = zero ? reinterpret_cast<const float*>(x + d.zero_off) + (lane & 31) : src + c;
        const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(epi + 4 * (arr * BM + cw0 + 64 * kk)));
        if (CW % 64 == 0 || 64 * kk + lane < CW)  // lanes past this wave's channels write nothing
          asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(m), "v"(sp) : "memory", "m0");
      }
    }
    if (lut_on) {
      for (int jl = 0; jl < CW / 4; ++jl) {  // rows cw0 + 4 jl .. + 3
        int c = c0 + cw0 + 4 * jl + (lane >> 4);
        c = c < cmax ? c : cmax;
        const int8_t* src = e.lut + (int64_t)c * 256 + 16 * (lane & 15);
        const uint32_t m =
            __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(epi + 4 * (7 + e.nclass) * BM + 256 * (cw0 + 4 * jl)));
        asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m), "v"(src) : "memory", "m0");
      }
    }
  };

  // ---- the lane's band offset of output tile j (block pixel (wn*TN + j)*16 + (lane & 15); past
  // the block it stands in for the block's last pixel and is never stored)
  const int npx_blk = __builtin_amdgcn_readfirstlane((r0 + g.rows <= nrows_all ? g.rows : nrows_all - r0) * d.wo);
  auto band_px = [&](int q) {  // band pixel of tap (0, 0) of block pixel q
    q = q < npx_blk ? q : npx_blk - 1;
    const int rr = q / d.wo, col = q - rr * d.wo;
    const int r = r0 + rr, n = r / d.ho, ho = r - n * d.ho;
    return (n * d.hp + ho * d.sh - R0) * g.wb + col;
  };
  const int lsel = (lane >> 5) * g.pl + 16 * ((lane >> 4) & 1);
  int pb[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) pb[j] = band_px((wn * TN + j) * 16 + (lane & 15)) * 32 + lsel;

  int* s_hc = reinterpret_cast<int*>(smem + g.cls_off);  // hcls[ho], then wcls[wo] (raw class ids)
  int* s_ps = reinterpret_cast<int*>(smem + g.psum_off);  // band pixel channel sums
  // the block's output pixels: {box sum of q', border class, flattened pixel m, n << 16 | ho << 8 | wo}
  int4* s_px = reinterpret_cast<int4*>(smem + p.scr_off);

  // ---- weights: rows c0 + cw0 + 16*i + (lane & 15), K bytes 16*(lane >> 4) of each step
  const int8_t* wblk = w + (int64_t)c0 * d.kpad;
  uint32_t aoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int row = cw0 + 16 * i + (lane & 15);
    row = c0 + row < d.cout_pad ? row : d.cout_pad - 1 - c0;
    aoff[i] = (uint32_t)(row * d.kpad + 16 * (lane >> 4));
  }
  const int KS = (d.cp / 64) * p.taps;
  const int SPC = H * p.taps;  // K steps per chunk
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
  v4i fa[DA][TM];
  Cur cl = {0, 0, 0, 0, 0};
  auto load_a = [&](v4i (&dst)[TM]) {
    const int8_t* base = wblk + kbytes(cl);
#pragma unroll
    for (int i = 0; i < TM; ++i) dst[i] = *reinterpret_cast<const v4i*>(base + aoff[i]);
    if (H * cl.gp + cl.h < d.cp / 64 - 1 || cl.t < p.taps - 1 || cl.h < H - 1) advance(cl);  // clamp at the last step
  };

  // issue order at start: the border classes and chunk 0, the first weights, chunk 1 (or the
  // epilogue data); the class tables by 4-byte-per-lane DMA (wave 0), 64 entries per job
  if (wave == 0) {
    for (int i0 = 0; i0 < d.ho + d.wo; i0 += 64) {
      const int i = i0 + lane;
      const int* src = i < d.ho ? p.e.hcls + i : p.e.wcls + (i < d.ho + d.wo ? i - d.ho : d.wo - 1);
      const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(s_hc + i0));
      if (i < d.ho + d.wo)
        asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(m), "v"(src) : "memory", "m0");
    }
  }
  issue_chunk(0);
#pragma unroll
  for (int s = 0; s < DA - 1; ++s) load_a(fa[s]);
  // chunk 1 and the epilogue data (L2-resident); issued before the loop, whose registers would
  // otherwise carry every epilogue pointer through the K steps
  if (!LATE) {
    if (nchunk > 1) issue_chunk(1);
    issue_epi();
  }
#if QNN_STAMP
  unsigned long long ta = 0, tb = 0, tc = 0;
  RB_TS(ta);
#endif


  // channel sums of this thread's band pixels, accumulated chunk by chunk; after the last chunk
  // the output pixels' box sums (two barriers: all band sums written, all box sums read them)
  int psum[NPT];
#pragma unroll
  for (int u = 0; u < NPT; ++u) psum[u] = 0;
  auto sum_chunk = [&](int c) {
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int b = tid + NT * u;
      if (b < g.nbp) {
        int sm[4] = {0, 0, 0, 0};
#pragma unroll
        for (int vv = 0; vv < CPL; ++vv) {
          const int8_t* pp = smem + (c * CPL + vv) * g.pl + 32 * b;
          const v4i a = *reinterpret_cast<const v4i*>(pp);
          const v4i cc = *reinterpret_cast<const v4i*>(pp + 16);
          sm[0] = __builtin_amdgcn_sdot4(a.x, 0x01010101, sm[0], false);
          sm[1] = __builtin_amdgcn_sdot4(a.y, 0x01010101, sm[1], false);
          sm[2] = __builtin_amdgcn_sdot4(a.z, 0x01010101, sm[2], false);
          sm[3] = __builtin_amdgcn_sdot4(a.w, 0x01010101, sm[3], false);
          sm[0] = __builtin_amdgcn_sdot4(cc.x, 0x01010101, sm[0], false);
          sm[1] = __builtin_amdgcn_sdot4(cc.y, 0x01010101, sm[1], false);
          sm[2] = __builtin_amdgcn_sdot4(cc.z, 0x01010101, sm[2], false);
          sm[3] = __builtin_amdgcn_sdot4(cc.w, 0x01010101, sm[3], false);
        }
        psum[u] += (sm[0] + sm[1]) + (sm[2] + sm[3]);
      }
    }
    if (c == nchunk - 1) {
#pragma unroll
      for (int u = 0; u < NPT; ++u)
        if (tid + NT * u < g.nbp) s_ps[tid + NT * u] = psum[u];
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      // each output pixel of the block, once: its receptive-field sum, border class and coordinates
      // (the epilogue then reads one 16-byte word per pixel tile: no divisions, no loops)
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const int q = tid + NT * u;
        if (q < npx_blk) {
          const int b0 = band_px(q);
          int bx = 0, tr = 0, tc = 0;
          for (int tt = 0; tt < p.taps; ++tt) {
            bx += s_ps[b0 + tr * g.wb + (g.s2 ? (tc & 1) * g.we + (tc >> 1) : tc)];
            if (++tc == d.kw) tc = 0, ++tr;
          }
          const int m = r0 * d.wo + q, HoWo = d.ho * d.wo;
          const int n = m / HoWo, ho = (m - n * HoWo) / d.wo, wo = m - n * HoWo - ho * d.wo;
          const int pc = s_hc[ho] * e.nwc + s_hc[d.ho + wo];
          // the code-table path: the class row's byte offset and the code0 pixel's (32-bit: rs_plan)
          s_px[q] = lutfast ? make_int4(bx, 4 * (7 + pc) * BM,
                                        ((n * e.code0_hp + ho + e.code0_pad) * e.code0_wp + wo + e.code0_pad) *
                                                e.code0_cp + c0,
                                        bx)
                            : make_int4(bx, pc, m, (n << 16) | (ho << 8) | wo);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };

  // chunk 0 and the border classes (this wave's DMA: counted, chunk 1's pieces and the first
  // weights behind them), then every wave's
  // (chunk 1's pieces and the epilogue data stay in flight: the first in-loop weight wait
  // covers them)
  if (LATE) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DA - 1) * TM) : "memory");
  else wait_vmcnt_rt((DA - 1) * TM + (nchunk > 1 ? ppc : 0) + njobs);
#if QNN_STAMP
  RB_TS(tb);
#endif
  asm volatile("s_barrier" ::: "memory");
#if QNN_STAMP
  RB_TS(tc);
#endif
  if (LATE) {
    if (nchunk > 1) issue_chunk(1);
    issue_epi();
  }
  sum_chunk(0);
#if QNN_STAMP
  RB_TS(ts1);
#endif

  v4i acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4i){0, 0, 0, 0};
  Cur cc = {0, 0, 0, 0, 0};
  int chunk = 0;
  auto step = [&](auto slotc) {
    constexpr int SL = decltype(slotc)::value;
    const int dt = cc.tr * g.wb + (g.s2 ? (cc.tc & 1) * g.we + (cc.tc >> 1) : cc.tc);
    const int boff = (2 * (H * cc.gp + cc.h)) * g.pl + 32 * dt;
    v4i fb[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      v4i r;
      asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(pb[j] + boff));
      fb[j] = r;
    }
    static_for<TN>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      lds_wait<TN - 1 - j>();
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[SL][i], fb[j], acc[i][j], 0, 0, 0);
    });
    __builtin_amdgcn_sched_barrier(0);
    load_a(fa[(SL + DA - 1) % DA]);
    advance(cc);
  };
#pragma nounroll
  for (int k0 = 0; k0 < KS; k0 += DA) {
    if (k0 > 0 && k0 % SPC == 0) {  // chunk boundary: this wave's pieces landed (counted), then every wave's
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DA - 1) * TM) : "memory");
      asm volatile("s_barrier" ::: "memory");
      ++chunk;
      if (chunk + 1 < nchunk) issue_chunk(chunk + 1);
      sum_chunk(chunk);
    }
    step(std::integral_constant<int, 0>{});
    if constexpr (DA > 1) step(std::integral_constant<int, 1>{});
    if constexpr (DA > 2) step(std::integral_constant<int, 2>{});
    if constexpr (DA > 3) step(std::integral_constant<int, 3>{});
  }
#if QNN_STAMP
  RB_TS(ts2);
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's epilogue data, the clamped tail weights
#if QNN_STAMP
  RB_TS(ts3);
#endif
#if QNN_STAMP
  RB_TS(ts5);
#endif
  if (lutfast) {
    // conv -> RangeBN -> ReLU -> next quantizer by the code table, software-pipelined over the
    // pixel tiles: tile j+1's pixel word and class rows are read while tile j's table bytes are
    const float* s_f = reinterpret_cast<const float*>(epi);
    const int8_t* s_lut = epi + 4 * (7 + e.nclass) * BM;
    const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
    const int gq = lane >> 4;
    const int cwl = cw0 + 4 * gq;  // this lane's first local channel of channel tile 0
    float4 sw[TM], bw[TM], bi[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      sw[i] = *reinterpret_cast<const float4*>(s_f + cwl + 16 * i);
      bw[i] = *reinterpret_cast<const float4*>(s_f + BM + cwl + 16 * i);
      bi[i] = *reinterpret_cast<const float4*>(s_f + 2 * BM + cwl + 16 * i);
    }
    auto pxq = [&](int j) {
      const int q = (wn * TN + j) * 16 + (lane & 15);
      return q < npx_blk ? q : npx_blk - 1;  // past the block: the last pixel again (same bytes)
    };
    auto rows = [&](int off, float4 (&tb)[TM]) {
      const float* tp = reinterpret_cast<const float*>(epi + off) + cwl;
#pragma unroll
      for (int i = 0; i < TM; ++i) tb[i] = *reinterpret_cast<const float4*>(tp + 16 * i);
    };
    // LDS returns in order: tile j+1's class rows are requested before tile j's table bytes, and
    // the pixel word two tiles ahead, so no wait for one tile's rows also waits for its bytes
    int4 pxc = s_px[pxq(0)];
    float4 tbc[TM];
    rows(pxc.y, tbc);
    int4 pxn = TN > 1 ? s_px[pxq(1)] : pxc;
    // tile j-1's table bytes are combined and stored after tile j's are requested
    int bp[TM][4];
    int8_t* opp = nullptr;
    auto put = [&](int8_t* op, const int (&b)[TM][4]) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        *reinterpret_cast<int*>(op + 16 * i) = b[i][0] | (b[i][1] << 8) | (b[i][2] << 16) | (b[i][3] << 24);
    };
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float4 tbn[TM];
      if (j + 1 < TN) rows(pxn.y, tbn);
      int4 pxnn = pxn;
      if (j + 2 < TN) pxnn = s_px[pxq(j + 2)];
      __builtin_amdgcn_sched_barrier(0);  // (the scheduler would sink these reads to their uses)
      // (.w repeats the sum: a field of the 16-byte read left unused would be reallocated while
      // the read is in flight, which costs a full lgkmcnt(0) wait)
      const f2 p2 = {(float)pxc.x, (float)pxc.w};
      int bq[TM][4];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const v4i& a = acc[i][j];
        const f2 a01 = {(float)a[0], (float)a[1]}, a23 = {(float)a[2], (float)a[3]};
        const f2 v0 = pfma((f2){sw[i].x, sw[i].y}, a01, pfma((f2){bw[i].x, bw[i].y}, p2, (f2){tbc[i].x, tbc[i].y})) +
                      (f2){bi[i].x, bi[i].y};
        const f2 v1 = pfma((f2){sw[i].z, sw[i].w}, a23, pfma((f2){bw[i].z, bw[i].w}, p2, (f2){tbc[i].z, tbc[i].w})) +
                      (f2){bi[i].z, bi[i].w};
        const f2 q0 = qclamp2(v0, bnp) + MAGIC_U8, q1 = qclamp2(v1, bnp) + MAGIC_U8;
        const uint8_t* lp = reinterpret_cast<const uint8_t*>(s_lut) + (cwl + 16 * i) * 256;
        bq[i][0] = lp[__float_as_uint(q0.x) & 255u];
        bq[i][1] = lp[256 + (__float_as_uint(q0.y) & 255u)];
        bq[i][2] = lp[512 + (__float_as_uint(q1.x) & 255u)];
        bq[i][3] = lp[768 + (__float_as_uint(q1.y) & 255u)];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (j > 0) put(opp, bp);
      opp = e.out_code0 + (uint32_t)pxc.z + cwl;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) bp[i][k] = bq[i][k];
      if (j + 1 < TN) {
        pxc = pxn;
        pxn = pxnn;
#pragma unroll
        for (int i = 0; i < TM; ++i) tbc[i] = tbn[i];
      }
    }
    put(opp, bp);
  } else {
    int sumq[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int q = (wn * TN + j) * 16 + (lane & 15);
      q = q < npx_blk ? q : npx_blk - 1;
      sumq[j] = s_px[q].x;
    }
    // this lane's pixel of tile j from the block's pixel table (a slot past the block stands in
    // for the block's last pixel and is never stored)
    auto pixel = [&](int j, q16::Pix& P, int& pc) {
      const int q = (wn * TN + j) * 16 + (lane & 15);
      P.ok = q < npx_blk;
      const int4 px = s_px[P.ok ? q : npx_blk - 1];
      pc = px.y;
      P.m = px.z;
      P.n = (int)((unsigned)px.w >> 16);
      P.ho = (px.w >> 8) & 255;
      P.wo = px.w & 255;
    };
    q16::epilogue_rb<C, EK>(p, acc, sumq, pixel, smem, c0, wm, lane, g.lut);
  }
#if QNN_STAMP
  RB_TS(ts6);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  RB_TS(ts4);
  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && blockIdx.x < (1 << 18) / (8 * W)) {
    unsigned long long* o = qnn_rs_stamps + ((size_t)blockIdx.x * W + wave) * 8;
    // issue (DMA + first weights), chunk-0 wait, its barrier, K loop (chunk-0 sums included),
    // epilogue (epilogue-data wait and box sums included), store drain
    o[0] = rt0; o[1] = rt1; o[2] = ta - ts0; o[3] = tb - ta; o[4] = tc - tb; o[5] = ts2 - tc;
    o[6] = ts6 - ts2; o[7] = ts4 - ts6;
  }
#endif
}

// ---------------------------------------------------------------- rs host side
// LDS of an rs block (band + sums + taps + classes, then the epilogue data, the EK_LUT code table
// when it fits) and the geometry checks the streamed chunks need; -1 if the layer does not fit.
template <class C, int EK, int H>
static int rs_plan(const Params& p, Params& q, Geo& g) {
  const int main = geometry(p, C::BM, C::BN, C::W, 1, 0, g);
  if (main < 0) return -1;
  const int cpl = 2 * H, spc = H * p.taps;
  // one DMA range per wave and plane (the chunk-0 wait counts pieces at compile time); chunk
  // boundaries on whole DA-step groups; one band pixel and one output pixel per thread
  if (g.npl % cpl || spc % C::DA || g.nbp > C::NT || g.npx > C::NT) return -1;
  if (p.d.ho > 255 || p.d.wo > 255 || p.d.n > 65535) return -1;  // (the pixel table's packed coordinates)
  q = p;
  const int box = 16 * g.npx;  // the pixel table (int4 per output pixel)
  int epi = epi_bytes(p, C::BM);
  g.lut = 0;
  // (the code-table path addresses code0 with 32-bit pixel offsets)
  const bool off32 = p.e.out_code0 == nullptr ||
                     (int64_t)p.d.n * p.e.code0_hp * p.e.code0_wp * p.e.code0_cp < ((int64_t)1 << 31);
  // BPC > 1: co-resident blocks (one's start-up and epilogue under the other's K loop), so the
  // block fits LDS_MAX / BPC and leaves the code table out (the epilogue evaluates the chain)
  const int lds_max = LDS_MAX / C::BPC;
  if (EK == EK_LUT && C::BPC == 1 && off32 && main + box + epi + 256 * C::BM <= lds_max) g.lut = 1, epi += 256 * C::BM;
  if (main + box + epi > lds_max) return -1;
  // the chunk-0 wait counts this wave's DMAs still allowed in flight: chunk 1's pieces, the
  // epilogue jobs and the first weights, within vmcnt's 6 bits
  const int npr = (g.ppp + C::W - 1) / C::W, cw = 16 * C::TM, vj = (cw + 63) / 64;
  const int narr = ((EK != EK_NCHW && p.e.bn_mean) ? 7 : 3) + p.e.nclass + (EK == EK_GEN ? 4 * p.e.nres : 0);
  if (npr * cpl + (C::DA - 1) * C::TM + narr * vj + (g.lut ? cw / 4 : 0) > 63) return -1;
  q.epi_early = 1, q.scr_off = main, q.epi_off = main + box;
  return main + box + epi;
}

template <class C, int EK, int H, int LATE>
static int rs_launch_k(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  auto kern = qconv_rs_kernel<C, EK, H, LATE>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  Geo g;
  Params q;
  const int lds = rs_plan<C, EK, H>(p, q, g);
  if (lds < 0) return arg_error("tile configuration not built for this layer / epilogue kind");
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

template <class C, int H, int LATE>
static int rs_launch_ek(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  switch (epi_kind(p.e)) {
    case EK_NCHW: return rs_launch_k<C, EK_NCHW, H, LATE>(x, w, p, s, occ);
    case EK_LUT: return rs_launch_k<C, EK_LUT, H, LATE>(x, w, p, s, occ);
    case EK_BNCODE: return rs_launch_k<C, EK_BNCODE, H, LATE>(x, w, p, s, occ);
    default:  // the general chain spills beside more than 16 accumulator tiles: not built
      if constexpr (C::TM * C::TN > 16) return arg_error("tile configuration not built for this layer / epilogue kind");
      else return rs_launch_k<C, EK_GEN, H, LATE>(x, w, p, s, occ);
  }
}

template <class C, int H>
static bool rs_ok_h(const Params& p) {
  if (p.d.cp < 128 * H) return false;  // (a 64-channel layer has one chunk of H = 1)
  Params q;
  Geo g;
  switch (epi_kind(p.e)) {
    case EK_NCHW: return rs_plan<C, EK_NCHW, H>(p, q, g) >= 0;
    case EK_LUT: return rs_plan<C, EK_LUT, H>(p, q, g) >= 0;
    case EK_BNCODE: return rs_plan<C, EK_BNCODE, H>(p, q, g) >= 0;
    default: return C::TM * C::TN <= 16 && rs_plan<C, EK_GEN, H>(p, q, g) >= 0;
  }
}

//   id  block (cout x px cols)  waves (each)    K chunks   chunk 1 + epilogue data
//   0   256 x 208               8 (32 x 208)    128 ch     at start        14x14 images (ResNet-50 layer 3, b256)
//   1   256 x 208               8 (32 x 208)    64 ch      at start
//   2   256 x 208               8 (32 x 208)    128 ch     after chunk 0
//   3   256 x 208               8 (32 x 208)    64 ch      after chunk 0
//   4   256 x 224               8 (64 x 112)    128 ch     at start        each band fragment feeds 4 MFMAs
//   5   256 x 112               8 (32 x 112)    128 ch     at start        half 14x14 images (ResNet-18 layer 3, b128)
//   6   256 x 112               8 (32 x 112)    64 ch      after chunk 0
//   7   128 x 112               8 (16 x 112)    128 ch     at start        2 images of 7x7 on 512 channels (layer 4, b128)
using S0 = Cfg<8, 1, 2, 13, 3, 1>;
using S2 = Cfg<4, 2, 4, 7, 3, 1>;
using S3 = Cfg<8, 1, 2, 7, 3, 1>;
using S5 = Cfg<8, 1, 1, 7, 4, 1>;
constexpr int NS = 8;
static const Info SINFO[NS] = {
    {256, 208, 8, 1, 26, 1.55f}, {256, 208, 8, 1, 26, 1.55f}, {256, 208, 8, 1, 26, 1.55f},
    {256, 208, 8, 1, 26, 1.55f}, {256, 224, 8, 1, 28, 1.55f}, {256, 112, 8, 1, 14, 1.10f},
    {256, 112, 8, 1, 14, 1.10f}, {128, 112, 8, 1, 7, 0.80f},
};

template <int K, class F>
static auto rs_cfg(F&& f) {
  using I2 = std::integral_constant<int, 2>;
  using I1 = std::integral_constant<int, 1>;
  using I0 = std::integral_constant<int, 0>;
  if constexpr (K == 0) return f(S0{}, I2{}, I0{});
  else if constexpr (K == 1) return f(S0{}, I1{}, I0{});
  else if constexpr (K == 2) return f(S0{}, I2{}, I1{});
  else if constexpr (K == 3) return f(S0{}, I1{}, I1{});
  else if constexpr (K == 4) return f(S2{}, I2{}, I0{});
  else if constexpr (K == 5) return f(S3{}, I2{}, I0{});
  else if constexpr (K == 6) return f(S3{}, I1{}, I1{});
  else return f(S5{}, I2{}, I0{});
}

template <int K>
static bool rs_ok_k(const Params& p) {
  return rs_cfg<K>([&](auto c, auto h, auto) { return rs_ok_h<decltype(c), decltype(h)::value>(p); });
}
template <int K>
static int rs_launch_kk(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  return rs_cfg<K>([&](auto c, auto h, auto late) {
    if (!rs_ok_h<decltype(c), decltype(h)::value>(p))
      return arg_error("tile configuration not built for this layer / epilogue kind");
    return rs_launch_ek<decltype(c), decltype(h)::value, decltype(late)::value>(x, w, p, s, occ);
  });
}

}  // namespace rb

int rs_count() { return rb::NS; }

void rs_tile(int k, int* bm, int* bn) {
  *bm = rb::SINFO[k].bm;
  *bn = rb::SINFO[k].bn;
}

bool rs_ok(int k, const Params& p) {
  using namespace rb;
  switch (k) {
    case 0: return rs_ok_k<0>(p);
    case 1: return rs_ok_k<1>(p);
    case 2: return rs_ok_k<2>(p);
    case 3: return rs_ok_k<3>(p);
    case 4: return rs_ok_k<4>(p);
    case 5: return rs_ok_k<5>(p);
    case 6: return rs_ok_k<6>(p);
    case 7: return rs_ok_k<7>(p);
    default: return false;
  }
}

int64_t rs_blocks(int k, const Params& p) {
  const rb::Info& f = rb::SINFO[k];
  rb::Geo g;
  if (rb::geometry(p, f.bm, f.bn, f.w, 1, 0, g) < 0) return 0;
  return (int64_t)g.nbands * cdiv(p.d.cout, f.bm);
}

double rs_cost(int k, const Params& p) {
  const rb::Info& f = rb::SINFO[k];
  rb::Geo g;
  if (rb::geometry(p, f.bm, f.bn, f.w, 1, 0, g) < 0) return 1e30;
  const int64_t tiles = (int64_t)g.nbands * cdiv(p.d.cout, f.bm);
  return (double)cdiv(tiles, NUM_CU) * f.bm * f.bn * (p.taps * p.d.cp) / f.rate;
}

int rs_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ) {
  using namespace rb;
  switch (k) {
    case 0: return rs_launch_kk<0>(x, w, p, s, occ);
    case 1: return rs_launch_kk<1>(x, w, p, s, occ);
    case 2: return rs_launch_kk<2>(x, w, p, s, occ);
    case 3: return rs_launch_kk<3>(x, w, p, s, occ);
    case 4: return rs_launch_kk<4>(x, w, p, s, occ);
    case 5: return rs_launch_kk<5>(x, w, p, s, occ);
    case 6: return rs_launch_kk<6>(x, w, p, s, occ);
    default: return rs_launch_kk<7>(x, w, p, s, occ);
  }
}

#if QNN_STAMP
extern "C" int qnn_debug_stamps_rs(void* dst, size_t bytes) {
  if (bytes > sizeof(::qnn::rb::qnn_rs_stamps)) bytes = sizeof(::qnn::rb::qnn_rs_stamps);
  return hip_check(hipMemcpyFromSymbol(dst, HIP_SYMBOL(::qnn::rb::qnn_rs_stamps), bytes), "stamps");
}
#endif
}  // namespace qnn
