// ResNet stem fused with its max-pool: the space-to-depth stem conv (7x7/2 as 4x4 taps x 16
// channels, resnet_quantized.py:171-174), RangeBN's input quantization of its output
// (quantize.py:461-462) and nn.MaxPool2d(3, 2, 1) of relu(RangeBN(.)) (resnet_quantized.py:140-143)
// in one kernel.  The unfused path writes the stem's full-resolution RangeBN codes to HBM and
// reads them back in qnn_maxpool_bn (103 MB each way at ResNet-18 b128); here they live in LDS.
//
// The kernel is persistent: one block per CU walks the items (PR pooled rows of one image each;
// all pooled columns, all 64 channels), staging the epilogue data and code tables once and
// double-buffering the band: item i + 1's band lands by LDS-DMA under item i's tiles and pooling.
// Per item:
//  0. the padded space-to-depth input rows those stem rows read -- one contiguous stretch of
//     the NHWC16 codes -- land in LDS by LDS-DMA (the BAND), with the epilogue data and tables;
//  1. the stem rows its windows read (2*PR + 1, fewer at the image edge) are computed with
//     16x16x64 MFMAs whose B fragment lanes are one 16-byte chunk of one tap of one band pixel
//     (ds_read_b128; every input byte crosses L2 once per block, no global-load latency in the
//     tile loop), sum_valid(q') by an all-ones MFMA against the K mask, with the exact
//     decomposition and EK_BNCODE arithmetic of every other conv kernel (epi16.h), so the
//     codes are bitwise the unfused kernel's; they go to LDS as [row][col][64] bytes;
//  2. every pooled (pixel, 16 channels) reduces its window in LDS with qnn_maxpool_bn's
//     algorithm (graph.hip): relu o RangeBN is monotone per channel, so the direction is folded
//     into the codes with an XOR and the window reduction is a bytewise max; outputs as
//     qnn_maxpool_bn: the pooled codes (byte C-tile, a residual chain start) and the consumer
//     codes through the per-channel tables (qnn_bn_code_lut).
// One stem row per block boundary is computed twice (the window overlap), 1/(2*PR) extra.
#include "qconv_common.h"
#include "epi16.h"

#ifndef QNN_STAMP
#define QNN_STAMP 0  // diagnostic builds only (make spstamp): per-wave s_memtime phase sums
#endif
#if QNN_STAMP
// [block][wave][8]: realtime start/end (100 MHz); cycles: prologue, item tops (band wait +
// barrier), tiles, mid barrier, pooling; items
__device__ unsigned long long qnn_sp_stamps[1 << 16];
#define SP_TS(v)                                                                          \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#else
#define SP_TS(v) ((void)0)
#endif

#ifndef QNN_SP_ABLATE
#define QNN_SP_ABLATE 0  // diagnostic builds only: 1 no MFMA, 2 no tile epilogue, 3 no pooling, 4 no band DMA
#endif

namespace qnn {
namespace sp {

constexpr int C = 64;    // stem channels (one 64-channel block, 4 MFMA row tiles)
constexpr int TM = 4;
#ifndef QNN_SP_W
#define QNN_SP_W 12  // three waves per SIMD (measured: 8 waves 97.5 / 184.8 us, 12 waves 90.0 / 165-168 at
                     // ResNet-18 b128 / ResNet-50 b256, profiles/r5_stem_ablation.txt)
#endif
#ifndef QNN_SP_DB
#define QNN_SP_DB 1
#endif
constexpr int W = QNN_SP_W;  // waves: each takes every W-th 16-pixel stem tile, all 64 channels
// 1: two band buffers, the next item's band lands under this item's tiles; 0: one, refilled
// under this item's pooling (less LDS: more blocks per CU)
constexpr bool DB = QNN_SP_DB;
constexpr int NT = 64 * W;
// more than two waves per SIMD (QNN_SP_W 12: three): the VGPR budget drops to 168, so the
// channel vectors are read from LDS where used and the tiles are not software-pipelined
constexpr bool LEAN = W > 8;
#ifndef QNN_SP_PR
#define QNN_SP_PR 4
#endif
constexpr int PR = QNN_SP_PR;  // pooled rows per block (4: 9 stem rows, 1/8 of them computed twice)

struct Cfg {  // what stage_epi expects
  static constexpr int BM = 64, W = sp::W;
};

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// q = m / D, r = m % D for 0 <= m < 2^24: the float quotient is off by at most one, fixed up
// exactly (qconv_direct.hip's fdivmod) -- a few VALU ops where an integer division costs ~40
__device__ __forceinline__ void fdivmod(int m, int D, float invD, int& q, int& r) {
  q = (int)((float)m * invD);
  r = m - (int)__umul24((unsigned)q, (unsigned)D);
  if (r < 0) --q, r += D;
  if (r >= D) ++q, r -= D;
}
// s_waitcnt vmcnt(n) for a wave-uniform run-time n (clamped to 63: vector memory operations
// complete in issue order, so at most n younger ones in flight still means every older one is done)
template <int N = 0>
__device__ __forceinline__ void wait_vmcnt_upto(int n) {
  if constexpr (N < 63) {
    if (n <= N) {
      wait_vmcnt<N>();
      return;
    }
    wait_vmcnt_upto<N + 1>(n);
  } else {
    wait_vmcnt<63>();
  }
}

struct Pool {
  int ho, wo;            // pooled output
  int nrg;               // row groups per image (ceil(ho / PR))
  uint8_t* out_code;     // nullable: pooled RangeBN input codes, byte C-tile
  const int8_t* lut0;    // nullable with code0
  qnn_code_out c0;
  const int8_t* lut1;
  qnn_code_out c1;
  int nitems;            // n * nrg
  int lds_codes, lds_lut0, lds_lut1, lds_dir, lds_hc, lds_band, lds_band_bytes, lds_zero, lds_mask;  // LDS offsets
};

template <int KS, bool MASKED, bool BIAS>
__global__ __launch_bounds__(NT) void stem_pool_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ w,
                                                       const Params p, const Pool pl) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const qnn_conv_desc& d = p.d;
  const qnn_epilogue& e = p.e;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // item -> (image, first pooled row, stem rows [sr_lo, sr_hi], padded input rows of its band)
  struct Item {
    int img, pr0, npr, sr_lo, sr_hi, npx, ntile, R0, band_bytes;
  };
  auto item = [&](int it) {
    Item q;
    q.img = it / pl.nrg;
    q.pr0 = (it - q.img * pl.nrg) * PR;
    q.npr = min(PR, pl.ho - q.pr0);
    // stem rows the windows of pooled rows [pr0, pr0 + npr) read (MaxPool2d(3, 2, 1))
    q.sr_lo = max(2 * q.pr0 - 1, 0);
    q.sr_hi = min(2 * (q.pr0 + q.npr - 1) + 1, d.ho - 1);
    q.npx = (q.sr_hi - q.sr_lo + 1) * d.wo;
    q.ntile = (q.npx + 15) >> 4;
    q.R0 = q.img * d.hp + q.sr_lo * d.sh;
    q.band_bytes = ((q.sr_hi - q.sr_lo) * d.sh + d.kh) * d.wp * d.cp;
    return q;
  };
  // ---- the band of an item: padded input rows [R0, R0 + nbr) of its image, one contiguous
  // stretch of nbr * wp * cp bytes, by 1 KiB LDS-DMA pieces (past its end: the zero page), in
  // inline asm -- invisible to the compiler's waitcnt bookkeeping, which would otherwise fence
  // every LDS read of the tile loop behind it; waited for explicitly (vmcnt(0) per item)
  auto issue_band = [&](const Item& q, int buf) {
    const int64_t src0 = (int64_t)q.R0 * d.wp * d.cp;
    const uint32_t dst0 = (uint32_t)(uintptr_t)(smem + pl.lds_band + buf * pl.lds_band_bytes);
    for (int pc = wave; pc * 1024 < q.band_bytes && QNN_SP_ABLATE != 4; pc += W) {
      const int o = pc * 1024 + 16 * lane;
      const int64_t src = o < q.band_bytes ? src0 + o : (int64_t)d.zero_off;
      const uint32_t m = __builtin_amdgcn_readfirstlane(dst0 + pc * 1024);
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m), "v"(x + src) : "memory", "m0");
    }
  };
  int it = blockIdx.x;
  if (it >= pl.nitems) return;
#if QNN_STAMP
  unsigned long long t0 = 0, ta = 0, tb = 0, c_pro = 0, c_top = 0, c_tile = 0, c_mid = 0, c_pool = 0, nit = 0;
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  SP_TS(t0);
#endif
  issue_band(item(it), 0);
  // ---- staged once: epilogue vectors + border table (stage_epi), code tables, border classes
  stage_epi<Cfg, EK_BNCODE>(p, x, smem, 0, wave, lane);
  auto stage_lut = [&](const int8_t* lut, int off) {
    for (int jl = wave; jl < C / 4; jl += W)
      __builtin_amdgcn_global_load_lds((const void*)(lut + jl * 1024 + 16 * lane), (lds_ptr_t)(smem + off + 1024 * jl),
                                       16, 0, 0);
  };
  if (pl.lut0) stage_lut(pl.lut0, pl.lds_lut0);
  if (pl.lut1) stage_lut(pl.lut1, pl.lds_lut1);
  int* s_hc = reinterpret_cast<int*>(smem + pl.lds_hc);
  for (int i = tid; i < d.ho + d.wo; i += NT) s_hc[i] = i < d.ho ? e.hcls[i] * e.nwc : e.wcls[i - d.ho];
  if (tid < 4) reinterpret_cast<int*>(smem + pl.lds_zero)[tid] = 0;
  if constexpr (MASKED && LEAN)  // the K mask, read per tile (no registers to hold it)
    for (int i = tid; i < d.kpad / 16; i += NT)
      *reinterpret_cast<v4i*>(smem + pl.lds_mask + 16 * i) = *reinterpret_cast<const v4i*>(d.kmask + 16 * i);

  // ---- the K chunks of this lane: tap u / cpg, 16 channels each, as band byte offsets from
  // the tile pixel's tap (0, 0); chunks past the taps read a 16-byte zero slot
  const int cpg = d.cp >> 4, kreal = p.taps * cpg;
  int doff[KS];
  v4i fa[KS][TM], ones[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int u = 4 * s + g;
    const int tap = u / cpg, tr = tap / d.kw, tc = tap - tr * d.kw;
    doff[s] = u < kreal ? (tr * d.wp + tc) * d.cp + 16 * (u - tap * cpg) : -1;
#pragma unroll
    for (int i = 0; i < TM; ++i)
      fa[s][i] = *reinterpret_cast<const v4i*>(w + (int64_t)(16 * i + (lane & 15)) * d.kpad + 64 * s + 16 * g);
    if constexpr (MASKED && !LEAN) ones[s] = *reinterpret_cast<const v4i*>(d.kmask + 64 * s + 16 * g);
    else ones[s] = (v4i){0x01010101, 0x01010101, 0x01010101, 0x01010101};
  }
  wait_vmcnt<0>();  // staged data, tables, weights (and the first band)
  __syncthreads();
  const float* s_f = reinterpret_cast<const float*>(smem);
  const QParams bnp = make_qparams(e.bn_neg_min, e.bn_scale, e.bn_qmax);
  float4 sw[TM], bw[TM], bi[TM];
  auto chan_vecs = [&](int i) {  // the channel vectors of row tile i (LEAN: read at use)
    const int cl = 16 * i + 4 * g;
    sw[i] = *reinterpret_cast<const float4*>(s_f + cl);
    bw[i] = *reinterpret_cast<const float4*>(s_f + C + cl);
    if constexpr (BIAS) bi[i] = *reinterpret_cast<const float4*>(s_f + 2 * C + cl);
  };
  if constexpr (!LEAN) {
#pragma unroll
    for (int i = 0; i < TM; ++i) chan_vecs(i);
  }
  // the stem codes, [stem pixel][64 bytes] with the channels of each pixel in LANE order: byte
  // 16 g + 4 i + u is channel 16 i + 4 g + u, so a tile lane (4 g) stores its 16 codes as one
  // conflict-free 16-byte write (channel order: 4-byte writes at a 64-byte pixel stride, 8-way
  // bank conflicts); a pooling chunk cg then holds channels 16 k + 4 cg + u (k, u < 4)
  uint8_t* s_codes = reinterpret_cast<uint8_t*>(smem + pl.lds_codes);
  // pool direction per channel (the same lane order): 0xff where relu o RangeBN is non-increasing
  // (sq * wq < 0).  The tiles store their codes XOR the direction (the pooling's folded form), so
  // the window reduction is a plain bytewise max and only its result is unfolded.
  uint8_t* s_dir = reinterpret_cast<uint8_t*>(smem + pl.lds_dir);
  if (tid < C) {
    const int ch = 16 * ((tid >> 2) & 3) + 4 * (tid >> 4) + (tid & 3);
    s_dir[tid] = (s_f[4 * C + ch] * s_f[5 * C + ch]) < 0.f ? 0xff : 0;
  }
  uint32_t dirw[TM];  // this lane's four channels of each row tile
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    dirw[i] = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ch = 16 * i + 4 * g + u;
      dirw[i] |= ((s_f[4 * C + ch] * s_f[5 * C + ch]) < 0.f ? 0xffu : 0u) << (8 * u);
    }
  }
  const float inv_wo = 1.0f / (float)d.wo, inv_pwo = 1.0f / (float)pl.wo;
  const int ct = (C + 31) >> 5;

  // global stores the wave issued since the current item's band DMA (the previous item's pooled
  // codes): the band is waited for with those left in flight
  int nst = 0;
  const int st_per = (pl.out_code ? 4 : 0) + (pl.c0.ptr ? 4 : 0) + (pl.c1.ptr ? 4 : 0);
#if QNN_STAMP
  SP_TS(ta);
  c_pro = ta - t0;
#endif
  for (int buf = 0; it < pl.nitems; it += gridDim.x, buf ^= (DB ? 1 : 0)) {
    const Item q = item(it);
#if QNN_STAMP
    SP_TS(ta);
    ++nit;
#endif
    // this item's band landed (every wave's pieces) and the previous item's pooling is done
    // with the codes: then the next item's band DMA goes into the other buffer, whose last
    // reader (the previous item's tiles) finished before the previous barrier.  A raw barrier
    // (__syncthreads would also wait for the pooled-code stores)
    wait_vmcnt_upto(__builtin_amdgcn_readfirstlane(nst));
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    nst = 0;
#if QNN_STAMP
    SP_TS(tb);
    c_top += tb - ta;
    ta = tb;
#endif
    if (DB && it + (int)gridDim.x < pl.nitems) issue_band(item(it + gridDim.x), buf ^ 1);
    const int band = pl.lds_band + buf * pl.lds_band_bytes;
    auto load_b = [&](int t, v4i (&fb)[KS], int& lr, int& col) {
      int qq = t * 16 + (lane & 15);
      qq = qq < q.npx ? qq : q.npx - 1;  // past the rows: the last pixel again (its store is skipped)
      fdivmod(qq, d.wo, inv_wo, lr, col);
      const int base = band + (lr * d.sh * d.wp + col * d.sw) * d.cp;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        fb[s] = *reinterpret_cast<const v4i*>(smem + (doff[s] >= 0 ? base + doff[s] : pl.lds_zero));
    };

    // ---- 1. stem tiles: wave w takes tiles w, w + W, ...  Software-pipelined: tile t + W's
    //         MFMAs are issued before tile t's epilogue (two accumulator sets), so the matrix pipe
    //         runs under the epilogue's VALU work instead of between epilogues; each tile's
    //         fragments are read from the band a tile earlier still.
    struct Acc {
      v4i a[TM], s;
    };
    auto mfmas = [&](const v4i (&fb)[KS], Acc& A) {
      A.s = (v4i){0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < TM; ++i) A.a[i] = (v4i){0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (QNN_SP_ABLATE == 1) {
          asm volatile("" ::"v"(fb[s]));
          A.s[0] += fb[s][0];
          continue;
        }
        v4i o = ones[s];
        if constexpr (MASKED && LEAN) o = *reinterpret_cast<const v4i*>(smem + pl.lds_mask + 64 * s + 16 * g);
        A.s = __builtin_amdgcn_mfma_i32_16x16x64_i8(o, fb[s], A.s, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < TM; ++i) A.a[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[s][i], fb[s], A.a[i], 0, 0, 0);
      }
    };
    auto epilogue = [&](int t, int lr, int col, const Acc& A) {
      const bool ok = t * 16 + (lane & 15) < q.npx;
      uint8_t* dst = s_codes + (lr * d.wo + col) * C + 16 * g;
      if (QNN_SP_ABLATE == 2) {
        int z = A.s[0];
#pragma unroll
        for (int i = 0; i < TM; ++i) z ^= A.a[i][0] ^ A.a[i][1] ^ A.a[i][2] ^ A.a[i][3];
        if (ok) *reinterpret_cast<int*>(dst) = z;
        return;
      }
      const int pc = s_hc[q.sr_lo + lr] + s_hc[d.ho + col];
      const f2 p2 = {(float)A.s[0], (float)A.s[0]};
      int kk[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int cl = 16 * i + 4 * g;
        const float4 tb = *reinterpret_cast<const float4*>(s_f + (7 + pc) * C + cl);
        if constexpr (LEAN) chan_vecs(i);
        const v4i& a = A.a[i];
        const f2 a01 = {(float)a[0], (float)a[1]}, a23 = {(float)a[2], (float)a[3]};
        // the exact decomposition with the op order of every conv epilogue (epi16.h conv_out4)
        f2 v0 = pfma((f2){sw[i].x, sw[i].y}, a01, pfma((f2){bw[i].x, bw[i].y}, p2, (f2){tb.x, tb.y}));
        f2 v1 = pfma((f2){sw[i].z, sw[i].w}, a23, pfma((f2){bw[i].z, bw[i].w}, p2, (f2){tb.z, tb.w}));
        if constexpr (BIAS) {  // (without one the other kernels add staged zeros: v + 0 differs from v
                               // only for v = -0, and -0 and +0 quantize to the same code)
          v0 = v0 + (f2){bi[i].x, bi[i].y};
          v1 = v1 + (f2){bi[i].z, bi[i].w};
        }
        const int kb = pack4(qclamp2(v0, bnp) + MAGIC_U8, qclamp2(v1, bnp) + MAGIC_U8);  // EK_BNCODE
        kk[i] = kb ^ (int)dirw[i];
      }
      if (ok) *reinterpret_cast<int4*>(dst) = make_int4(kk[0], kk[1], kk[2], kk[3]);
    };
    // one tile's MFMAs interleaved with the previous tile's epilogue: 1 MFMA per 8 VALU
    auto interleave = [] {
#pragma unroll
      for (int k = 0; k < 5 * KS; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);  // VALU
      }
    };
    if constexpr (LEAN) {
      Acc A;
      for (int t = wave; t < q.ntile; t += W) {
        v4i fb[KS];
        int lr, col;
        load_b(t, fb, lr, col);
        mfmas(fb, A);
        epilogue(t, lr, col, A);
      }
    } else {
    Acc A0, A1;
    v4i fnx[KS];
    int t = wave, nlr = 0, ncol = 0, lrA = 0, colA = 0, lrB = 0, colB = 0;
    if (t < q.ntile) {
      load_b(t, fnx, lrA, colA);
      mfmas(fnx, A0);
      load_b(t + W, fnx, nlr, ncol);  // (past the last tile: clamped reads, results discarded)
    }
    // unrolled by two: each accumulator set keeps its registers.  Branch-free steps (the next
    // tile's MFMAs and fragment reads run even past the last tile, on clamped pixels, and are
    // discarded), so the scheduler can interleave them with the epilogue.
    while (t < q.ntile) {
      mfmas(fnx, A1);
      lrB = nlr, colB = ncol;
      load_b(t + 2 * W, fnx, nlr, ncol);
      epilogue(t, lrA, colA, A0);
      interleave();
      t += W;
      if (t >= q.ntile) break;
      mfmas(fnx, A0);
      lrA = nlr, colA = ncol;
      load_b(t + 2 * W, fnx, nlr, ncol);
      epilogue(t, lrB, colB, A1);
      interleave();
      t += W;
    }
    }
#if QNN_STAMP
    SP_TS(tb);
    c_tile += tb - ta;
    ta = tb;
#endif
    // the codes are in LDS (raw barrier: the next item's band DMA stays in flight)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#if QNN_STAMP
    SP_TS(tb);
    c_mid += tb - ta;
    ta = tb;
#endif
    // one band buffer: the tiles are done with it, the next item's band lands under the pooling
    if (!DB && it + (int)gridDim.x < pl.nitems) issue_band(item(it + gridDim.x), 0);

    // ---- 2. pooled (pixel, 16 channels) items, channel groups fastest.  MaxPool2d pads with
    //         -inf: an out-of-image tap is clamped to the nearest in-image row / column, which
    //         lies inside the same window (2*oy and 2*pc are always in the image), and the max is
    //         idempotent.  The folded bytes are reduced as even / odd halves in u16 lanes
    //         (v_perm_b32 splits, v_pk_max_u16), rejoined once.
    for (int pi = tid; pi < q.npr * pl.wo * 4 && QNN_SP_ABLATE != 3; pi += NT) {
      const int cg = pi & 3, pxi = pi >> 2;
      int prl, pc;
      fdivmod(pxi, pl.wo, inv_pwo, prl, pc);
      const int oy = q.pr0 + prl, cb = 16 * cg;
      const uint4 dm = *reinterpret_cast<const uint4*>(s_dir + cb);
      int roff[3], coff[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int sy = min(max(2 * oy - 1 + r, 0), d.ho - 1);
        roff[r] = (min(max(sy, q.sr_lo), q.sr_hi) - q.sr_lo) * d.wo * C + cb;
        coff[r] = min(max(2 * pc - 1 + r, 0), d.wo - 1) * C;
      }
      u16x2 lo[4], hi[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) lo[k] = hi[k] = (u16x2){0, 0};
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) {
          const uint4 v = *reinterpret_cast<const uint4*>(s_codes + roff[r] + coff[s2]);
          const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            lo[k] = __builtin_elementwise_max(lo[k], __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(0u, vv[k], 0x0c020c00u)));
            hi[k] = __builtin_elementwise_max(hi[k], __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(0u, vv[k], 0x0c030c01u)));
          }
        }
      uint4 best;
      best.x = __builtin_bit_cast(uint32_t, lo[0]) | (__builtin_bit_cast(uint32_t, hi[0]) << 8);
      best.y = __builtin_bit_cast(uint32_t, lo[1]) | (__builtin_bit_cast(uint32_t, hi[1]) << 8);
      best.z = __builtin_bit_cast(uint32_t, lo[2]) | (__builtin_bit_cast(uint32_t, hi[2]) << 8);
      best.w = __builtin_bit_cast(uint32_t, lo[3]) | (__builtin_bit_cast(uint32_t, hi[3]) << 8);
      const uint32_t qd[4] = {best.x ^ dm.x, best.y ^ dm.y, best.z ^ dm.z, best.w ^ dm.w};
      const int64_t m = ((int64_t)q.img * pl.ho + oy) * pl.wo + pc;
      nst += st_per;
      if (pl.out_code) {
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int ch = 16 * s4 + 4 * cg;  // the chunk's dword s4: channels ch .. ch + 3
          *reinterpret_cast<uint32_t*>(pl.out_code + btile_off((int)(m >> 5), ch >> 5, ct, (int)(m & 31) + 32 * ((ch >> 2) & 1)) +
                                       4 * ((ch & 31) >> 3)) = qd[s4];
        }
      }
#pragma unroll
      for (int o = 0; o < 2; ++o) {
        const qnn_code_out& co = o ? pl.c1 : pl.c0;
        if (!co.ptr) continue;
        const int8_t* sl = smem + (o ? pl.lds_lut1 : pl.lds_lut0);
        int8_t* op = co.ptr + (((int64_t)q.img * co.hp + oy + co.pad) * co.wp + pc + co.pad) * co.cp + 4 * cg;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          int r4 = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int ch = 16 * s4 + 4 * cg + u;
            r4 |= ((int)(uint8_t)sl[ch * 256 + ((qd[s4] >> (8 * u)) & 255)]) << (8 * u);
          }
          *reinterpret_cast<int*>(op + 16 * s4) = r4;
        }
      }
    }
#if QNN_STAMP
    SP_TS(tb);
    c_pool += tb - ta;
#endif
  }
#if QNN_STAMP
  const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && blockIdx.x < (1 << 16) / (8 * W)) {
    unsigned long long* o = qnn_sp_stamps + ((size_t)blockIdx.x * W + wave) * 8;
    o[0] = rt0, o[1] = rt1, o[2] = c_pro, o[3] = c_top, o[4] = c_tile, o[5] = c_mid, o[6] = c_pool, o[7] = nit;
  }
#endif
}

template <int KS, bool MASKED, bool BIAS>
static int launch(const int8_t* x, const int8_t* w, const Params& p, const Pool& pl0, hipStream_t s) {
  auto kern = stem_pool_kernel<KS, MASKED, BIAS>;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  if (attr != hipSuccess) return hip_check(attr, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  Pool pl = pl0;
  int off = (4 * (7 + p.e.nclass) * C + 15) & ~15;  // stage_epi's EK_BNCODE data
  pl.lds_hc = off;
  off += (4 * (p.d.ho + p.d.wo) + 15) & ~15;
  pl.lds_dir = off;
  off += C;
  pl.lds_lut0 = off;
  off += pl.lut0 ? 256 * C : 0;
  pl.lds_lut1 = off;
  off += pl.lut1 ? 256 * C : 0;
  pl.lds_zero = off;
  off += 16;
  pl.lds_mask = off;  // (LEAN + masked: the K mask, kpad <= 256 bytes)
  off += LEAN && p.d.kmask ? 256 : 0;
  pl.lds_band = off;  // two bands: (2 PR + 1) stem rows read (2 PR) * sh + kh padded input rows, 1 KiB pieces
  pl.lds_band_bytes = (int)cdiv((int64_t)(2 * PR * p.d.sh + p.d.kh) * p.d.wp * p.d.cp, 1024) * 1024;
  off += (DB ? 2 : 1) * pl.lds_band_bytes;
  pl.lds_codes = off;
  off += (2 * PR + 1) * p.d.wo * C;
  if (off > LDS_MAX) return arg_error("stem max-pool tile needs more than 160 KiB of LDS");
  pl.nitems = p.d.n * pl.nrg;
  int per_cu = 0;  // persistent: as many blocks as fit at once, each walking the items
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, NT, off) != hipSuccess || per_cu < 1) per_cu = 1;
  const int nblk = (int)std::min<int64_t>(pl.nitems, (int64_t)device_cu_count() * per_cu);
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(NT), off, s, x, w, p, pl);
  return QNN_OK;
}

}  // namespace sp

#if QNN_STAMP
extern "C" int qnn_debug_stamps_sp(void* dst, size_t bytes) {
  if (bytes > sizeof(::qnn_sp_stamps)) bytes = sizeof(::qnn_sp_stamps);
  return hip_check(hipMemcpyFromSymbol(dst, HIP_SYMBOL(::qnn_sp_stamps), bytes), "stamps");
}
#endif

int stem_pool_launch(const int8_t* x, const int8_t* w, const Params& p, int pool_ho, int pool_wo, uint8_t* out_code,
                     const int8_t* lut0, const qnn_code_out& c0, const int8_t* lut1, const qnn_code_out& c1,
                     hipStream_t s) {
  using namespace sp;
  const qnn_conv_desc& d = p.d;
  if (d.cout != C || d.cout_pad < C || d.kpad > 256 || d.kpad % 64 || d.cp % 16 || p.taps * d.cp > d.kpad)
    return arg_error("stem max-pool: 64 output channels and a short reduction (kpad <= 256) only");
  if (pool_ho != (d.ho + 2 - 3) / 2 + 1 || pool_wo != (d.wo + 2 - 3) / 2 + 1)
    return arg_error("stem max-pool: MaxPool2d(3, 2, 1) output size expected");
  Pool pl{};
  pl.ho = pool_ho, pl.wo = pool_wo, pl.nrg = (pool_ho + PR - 1) / PR;
  pl.out_code = out_code, pl.lut0 = lut0, pl.c0 = c0, pl.lut1 = lut1, pl.c1 = c1;
  const bool m = d.kmask != nullptr;
  // the bias as a template parameter: a run-time test inside the tile loop is if-converted into
  // an add and a select per output
  auto go = [&](auto ks) {
    constexpr int K = decltype(ks)::value;
    if (p.e.bias) return m ? launch<K, true, true>(x, w, p, pl, s) : launch<K, false, true>(x, w, p, pl, s);
    return m ? launch<K, true, false>(x, w, p, pl, s) : launch<K, false, false>(x, w, p, pl, s);
  };
  switch ((p.taps * (d.cp >> 4) + 3) >> 2) {
    case 1: return go(std::integral_constant<int, 1>{});
    case 2: return go(std::integral_constant<int, 2>{});
    case 3: return go(std::integral_constant<int, 3>{});
    default: return go(std::integral_constant<int, 4>{});
  }
}

}  // namespace qnn
