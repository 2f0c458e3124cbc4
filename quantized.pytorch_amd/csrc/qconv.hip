// int8 MFMA implicit-GEMM convolution: the eval forward of QConv2d / QLinear
// (models/modules/quantize.py:314-349, :398-428; biprecision's out1+out2-out1
// is one contraction).  CDNA4 / gfx950: v_mfma_i32_32x32x32_i8.
//
// GEMM view  D[c][m] = sum_k Wq'[c][k] * Xq'[k][m]
//   c: output channel  -> MFMA rows    (operand A: packed weights [cout_pad][kpad])
//   m: output pixel    -> MFMA columns (operand B: implicit im2col of the NHWC8 codes)
//   k: (kh, kw, ci) tap-major, ci padded to Cp = 16 * 2^j
// The input is SPATIALLY PRE-PADDED ([n][hp][wp][cp], border code' = 0): zero
// padding of x_hat contributes nothing to any term of the exact decomposition
// (SURVEY.md §0.5), so the gather has no bounds checks at all and goes straight
// HBM -> LDS with global_load_lds_dwordx4.  Chunks past K read a zero page.
//
// Epilogue: y = s_x*s_w[c]*acc + s_x*b_w[c]*sum_valid(q'_x) + b_x*sum_valid(w_hat[c]) (+ bias)
//   sum_valid(q'_x): v_dot4 of the B fragments against 1s (exact, in-loop);
//   border term: per (row class, col class, c) table staged in LDS.
// Then either the drop-in output (fp32 NCHW, the reference module boundary), or
// the fused chain of the model graph: RangeBN eval (quantize.py:461-499, exact
// fp32 op order) -> + residual -> ReLU -> fp32 NHWC and/or requantized NHWC8
// codes for up to two consumer convs (their QuantMeasure ranges).
//
// Block: 256 threads = 4 waves, each wave a 64x64 tile (2x2 MFMA 32x32x32).
// K stage = 128 bytes; two LDS stages filled by LDS-DMA, counted vmcnt, raw
// s_barrier; rows XOR-swizzled so ds_read_b128 fragment reads are conflict-free.
#include <stdlib.h>

#include "qnn_internal.h"

namespace qnn {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int MAX_TAPS = 64;
constexpr int MAX_CLASSES = 32;
constexpr int MAX_MASK = 1024;
constexpr int KPAD_ALIGN = 128;  // packed weight rows are multiples of 128 bytes (any BK divides)

struct Params {
  qnn_conv_desc d;
  qnn_epilogue e;
  int M;        // n*ho*wo
  int taps;     // kh*kw
  int lgcpt;    // log2(cp/16)
  int nstage;   // kpad / BK
};

// Byte offset of 16-byte chunk `chunk` of LDS row `row` (rows of BK bytes): XOR swizzle so
// that the 16-lane groups of a ds_read_b128 fragment read (16 rows, one chunk) hit 16
// distinct 16-B bank slots: BK=128 (2 rows per 256-B bank row) xor (row>>1)&7,
// BK=64 (4 rows per bank row) xor (row>>2)&3.
template <int BK>
__device__ __forceinline__ int swz(int row, int chunk) {
  if constexpr (BK == 128) return row * BK + ((chunk ^ ((row >> 1) & 7)) << 4);
  else return row * BK + ((chunk ^ ((row >> 2) & 3)) << 4);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void store_code4(int8_t* p, float4 v, float nm, float s, float inv, float qmax) {
  int b0 = (int)quant_code_fast(v.x, nm, s, inv, qmax) - 128;
  int b1 = (int)quant_code_fast(v.y, nm, s, inv, qmax) - 128;
  int b2 = (int)quant_code_fast(v.z, nm, s, inv, qmax) - 128;
  int b3 = (int)quant_code_fast(v.w, nm, s, inv, qmax) - 128;
  *reinterpret_cast<int*>(p) = (b0 & 255) | ((b1 & 255) << 8) | ((b2 & 255) << 16) | ((b3 & 255) << 24);
}

// Epilogue shared by the implicit-GEMM and halo kernels.  sumq[j]: full receptive-field
// sum of q'_x for this lane's pixel of column tile j.  smem: >= epilogue LDS bytes.
template <int BM, bool FUSED>
__device__ __forceinline__ void epilogue(const Params& p, v16i (&acc)[2][2], const int (&sumq)[2], int8_t* smem,
                                         int m0, int c0, int wm, int wn, int lane) {
  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, frow = lane & 31, fh = lane >> 5;
  const int HoWo = d.ho * d.wo;
  const qnn_epilogue& e = p.e;
  float* s_f = reinterpret_cast<float*>(smem);  // main-loop LDS is free now
  // [0,BM) sxsw  [BM,2BM) sxbw  [2BM,3BM) bias  [3BM..7BM) bn mean/sq/wq/bq  [7BM..) table[cls][BM]
  const int nparam = 7 * BM;
  for (int i = tid; i < BM; i += 256) {
    const int c = c0 + i;
    const bool ok = c < d.cout;
    s_f[i] = ok ? e.sxsw[c] : 0.f;
    s_f[BM + i] = ok ? e.sxbw[c] : 0.f;
    s_f[2 * BM + i] = (ok && e.bias) ? e.bias[c] : 0.f;
    if (FUSED && e.bn_mean) {
      s_f[3 * BM + i] = ok ? e.bn_mean[c] : 0.f;
      s_f[4 * BM + i] = ok ? e.bn_sq[c] : 0.f;
      s_f[5 * BM + i] = ok ? e.bn_wq[c] : 0.f;
      s_f[6 * BM + i] = ok ? e.bn_bq[c] : 0.f;
    }
  }
  for (int i = tid; i < e.nclass * BM; i += 256) {
    const int cls = i / BM, c = c0 + (i - cls * BM);
    s_f[nparam + i] = c < d.cout ? e.table[cls * d.cout + c] : 0.f;
  }
  int8_t* s_lut = smem + 4 * (7 + MAX_CLASSES) * BM;  // [BM][256] next-layer codes (FUSED && e.lut)
  if (FUSED && e.lut) {
    for (int i = tid; i < BM * 16; i += 256) {
      const int c = c0 + (i >> 4);
      if (c < d.cout)
        *reinterpret_cast<v4i*>(s_lut + 16 * i) = *reinterpret_cast<const v4i*>(e.lut + (int64_t)c * 256 + 16 * (i & 15));
    }
  }
  __syncthreads();
  const float bn_inv = 1.0f / e.bn_scale, c0_inv = 1.0f / e.code0_scale, c1_inv = 1.0f / e.code1_scale;

  // per-pixel (lane) state for the two 32-pixel column tiles of this wave
  int pm[2], pn[2], phw[2], pho[2], pwo[2], ptab[2];
  float psq[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = m0 + wn * 64 + j * 32 + frow;
    pm[j] = m;
    const int mm = m < p.M ? m : p.M - 1;
    pn[j] = mm / HoWo;
    phw[j] = mm - pn[j] * HoWo;
    pho[j] = phw[j] / d.wo;
    pwo[j] = phw[j] - pho[j] * d.wo;
    ptab[j] = nparam + (e.hcls[pho[j]] * e.nwc + e.wcls[pwo[j]]) * BM;
    psq[j] = (float)sumq[j];
  }
  // channel groups outer (params loaded once), pixel tiles inner
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int cl = wm * 64 + i * 32 + 8 * g + 4 * fh;  // local channel of reg 4g (+u)
      const int c = c0 + cl;
      if (FUSED && c >= d.cout) continue;  // cout % 4 == 0 in fused mode
      float a_sxsw[4], a_sxbw[4], a_bias[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a_sxsw[u] = s_f[cl + u];
        a_sxbw[u] = s_f[BM + cl + u];
        a_bias[u] = s_f[2 * BM + cl + u];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (pm[j] >= p.M) continue;
        const int m = pm[j], n = pn[j], hw = phw[j], ho = pho[j], wo = pwo[j];
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float y = fmaf(a_sxsw[u], (float)acc[i][j][4 * g + u], fmaf(a_sxbw[u], psq[j], s_f[ptab[j] + cl + u]));
          v[u] = y + a_bias[u];
        }
        if (!FUSED) {
          float* yp = e.out_f32 + ((int64_t)n * d.cout + c) * HoWo + hw;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (c + u < d.cout) yp[(int64_t)u * HoWo] = v[u];
          continue;
        }
        if (e.lut) {  // conv -> RangeBN -> ReLU -> next quantizer, tabulated per channel (exact)
          int r = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int q = (int)quant_code_fast(v[u], e.bn_neg_min, e.bn_scale, bn_inv, e.bn_qmax);
            r |= ((int)(uint8_t)s_lut[(cl + u) * 256 + q]) << (8 * u);
          }
          const int64_t a = (((int64_t)n * e.code0_hp + ho + e.code0_pad) * e.code0_wp + wo + e.code0_pad) * e.code0_cp + c;
          *reinterpret_cast<int*>(e.out_code0 + a) = r;
          continue;
        }
        if (e.bn_mean) {
          int qb[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            qb[u] = (int)quant_code_fast(v[u], e.bn_neg_min, e.bn_scale, bn_inv, e.bn_qmax);  // RangeBN.quantize_input
          if (e.out_bncode) {
            *reinterpret_cast<int*>(e.out_bncode + (int64_t)m * d.cout + c) =
                qb[0] | (qb[1] << 8) | (qb[2] << 16) | (qb[3] << 24);
            if (!e.out_f32 && !e.out_code0) continue;  // stem before the code-domain max-pool
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int l = cl + u;
            float o = dequant((float)qb[u], e.bn_scale, e.bn_min) - s_f[3 * BM + l];  // x - mean
            o = o * s_f[4 * BM + l];                                                   // * q(scale)
            o = o * s_f[5 * BM + l];                                                   // * q(weight)
            v[u] = o + s_f[6 * BM + l];                                                // + q(bias)
          }
        }
        float4 o4 = make_float4(v[0], v[1], v[2], v[3]);
        if (e.residual) {
          const float4 r4 = *reinterpret_cast<const float4*>(e.residual + (int64_t)m * d.cout + c);
          o4.x = o4.x + r4.x; o4.y = o4.y + r4.y; o4.z = o4.z + r4.z; o4.w = o4.w + r4.w;
        }
        if (e.relu) {
          o4.x = fmaxf(o4.x, 0.f); o4.y = fmaxf(o4.y, 0.f); o4.z = fmaxf(o4.z, 0.f); o4.w = fmaxf(o4.w, 0.f);
        }
        if (e.out_f32) *reinterpret_cast<float4*>(e.out_f32 + (int64_t)m * d.cout + c) = o4;
        if (e.out_code0) {
          const int64_t a = (((int64_t)n * e.code0_hp + ho + e.code0_pad) * e.code0_wp + wo + e.code0_pad) * e.code0_cp + c;
          store_code4(e.out_code0 + a, o4, e.code0_neg_min, e.code0_scale, c0_inv, e.code0_qmax);
        }
        if (e.out_code1) {
          const int64_t a = (((int64_t)n * e.code1_hp + ho + e.code1_pad) * e.code1_wp + wo + e.code1_pad) * e.code1_cp + c;
          store_code4(e.out_code1 + a, o4, e.code1_neg_min, e.code1_scale, c1_inv, e.code1_qmax);
        }
      }
    }
  }
}

template <int BM, int BN, int BK, bool FUSED, bool MASKED>
__global__ __launch_bounds__(256) void qconv_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ w,
                                                    const Params p) {
  constexpr int WM = BM / 64, WN = BN / 64;
  static_assert(WM * WN == 4, "4 waves of 64x64");
  static_assert(BK == 64 || BK == 128, "BK");
  constexpr int CPR = BK / 16;    // 16-B chunks per LDS row
  constexpr int RPI = 1024 / BK;  // rows per 1 KiB LDS-DMA wave-instruction
  constexpr int NA = BM / (4 * RPI);  // glds per wave per stage for A
  constexpr int NB = BN / (4 * RPI);
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int MAIN = 2 * STAGE + 4 * MAX_TAPS + (MASKED ? MAX_MASK : 0);
  constexpr int EPI = 4 * (7 + MAX_CLASSES) * BM + (FUSED ? 256 * BM : 0);  // params, border table, LUT
  // one LDS object (a second __shared__ array can make hipcc drain vmcnt before ds_reads)
  __shared__ __attribute__((aligned(16))) int8_t smem[MAIN > EPI ? MAIN : EPI];
  int* s_tap = reinterpret_cast<int*>(smem + 2 * STAGE);
  int8_t* s_mask = smem + 2 * STAGE + 4 * MAX_TAPS;

  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // ---- XCD-aware, bijective block -> tile map: each XCD gets a contiguous run of
  // tiles, output-channel tiles fastest so blocks sharing an activation tile share L2
  const int nby = (d.cout + BM - 1) / BM;
  const int nbx = (p.M + BN - 1) / BN;
  const int nblk = nbx * nby;
  int t;
  {
    const int b = blockIdx.x, xcd = b & 7, q = nblk >> 3, r = nblk & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int m0 = (t / nby) * BN;
  const int c0 = (t % nby) * BM;
  const int HoWo = d.ho * d.wo;

  if (tid < p.taps) s_tap[tid] = ((tid / d.kw) * d.wp + (tid % d.kw)) * d.cp;
  if constexpr (MASKED) {
    for (int i = tid; i < d.kpad / 16; i += 256)
      *reinterpret_cast<v4i*>(s_mask + 16 * i) = *reinterpret_cast<const v4i*>(d.kmask + 16 * i);
  }

  // ---- per-lane load state
  uint32_t boff[NB];
  int bchunk[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int row = RPI * (wave + 4 * j) + lane / CPR;
    int m = m0 + row;
    if (m > p.M - 1) m = p.M - 1;
    const int n = m / HoWo, rem = m - n * HoWo, ho = rem / d.wo, wo = rem - ho * d.wo;
    boff[j] = (uint32_t)(((n * d.hp + ho * d.sh) * d.wp + wo * d.sw) * d.cp);
    bchunk[j] = (swz<BK>(row, lane % CPR) - row * BK) >> 4;  // the chunk that lands in this lane's slot
  }
  const int8_t* aptr[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int row = RPI * (wave + 4 * j) + lane / CPR;
    aptr[j] = w + (int64_t)(c0 + row) * d.kpad + (swz<BK>(row, lane % CPR) - row * BK);
  }
  const int cpt_mask = (1 << p.lgcpt) - 1;
  __syncthreads();  // s_tap

  auto issue = [&](int st, int buf) {
    int8_t* sa = smem + buf * STAGE;
    int8_t* sb = sa + BM * BK;
#pragma unroll
    for (int j = 0; j < NA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(aptr[j] + st * BK),
                                       (lds_ptr_t)(sa + (wave + 4 * j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int kc = st * CPR + bchunk[j];
      const int tap = kc >> p.lgcpt;
      uint32_t off = tap < p.taps ? boff[j] + (uint32_t)s_tap[tap] + (uint32_t)((kc & cpt_mask) << 4)
                                  : (uint32_t)d.zero_off;
      asm volatile("" : "+v"(off));  // keep ONE per-lane-address load (no saddr/vaddr branch split)
      __builtin_amdgcn_global_load_lds((const void*)(x + off), (lds_ptr_t)(sb + (wave + 4 * j) * 1024), 16, 0, 0);
    }
  };

  v16i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (v16i){0};
  int sumq[2] = {0, 0};

  const int frow = lane & 31, fh = lane >> 5;
  issue(0, 0);
  const int nstage = p.d.kpad / BK;
  for (int st = 0; st < nstage; ++st) {
    const int buf = st & 1;
    if (st + 1 < nstage) {
      issue(st + 1, buf ^ 1);
      wait_vmcnt<NA + NB>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    const int8_t* sa = smem + buf * STAGE;
    const int8_t* sb = sa + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int chunk = 2 * ks + fh;
      v4i fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const v4i*>(sa + swz<BK>(wm * 64 + i * 32 + frow, chunk));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        fb[j] = *reinterpret_cast<const v4i*>(sb + swz<BK>(wn * 64 + j * 32 + frow, chunk));
        v4i ones = {0x01010101, 0x01010101, 0x01010101, 0x01010101};
        if constexpr (MASKED) ones = *reinterpret_cast<const v4i*>(s_mask + st * BK + 16 * chunk);
        int s = __builtin_amdgcn_sdot4(fb[j].x, ones.x, sumq[j], false);
        s = __builtin_amdgcn_sdot4(fb[j].y, ones.y, s, false);
        s = __builtin_amdgcn_sdot4(fb[j].z, ones.z, s, false);
        sumq[j] = __builtin_amdgcn_sdot4(fb[j].w, ones.w, s, false);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_barrier();
  }

  // ================================================================ epilogue
#pragma unroll
  for (int j = 0; j < 2; ++j) sumq[j] += __shfl_xor(sumq[j], 32, 64);
  __syncthreads();  // main-loop LDS is reused by the epilogue
  epilogue<BM, FUSED>(p, acc, sumq, smem, m0, c0, wm, wn, lane);
}

// ============================================================================ halo kernel
// For kh x kw convs with Cp >= 32 (the ResNet 3x3s).  The implicit-GEMM kernel above
// re-gathers every activation byte once per tap (9x for 3x3) through L1, which caps
// it at the per-CU load bandwidth.  Here a block loads, per channel chunk of CK bytes,
// the BAND of padded input rows covering its pixel tile's receptive field into LDS
// ONCE (rows [n0*hp + ho0*sh, n1*hp + ho1*sh + kh - 1] of the flattened padded
// buffer, every column, CK channels), then serves all kh*kw taps' B fragments from
// it; only the per-tap weight slice [BM][CK] streams (LDS-DMA, double-buffered).
// sum_valid(q'_x) comes from per-band-pixel channel sums S[q] (one v_dot4 pass per
// band pixel instead of one per fragment), summed over the taps of each pixel.
constexpr int MAX_BAND = 40960;

template <int CPR>
__device__ __forceinline__ int swz_c(int idx, int chunk) {
  // chunk slot of 16-B chunk `chunk` in LDS row `idx` (rows of 16*CPR bytes): conflict-free
  // ds_read_b128 over 16 consecutive rows
  return chunk ^ ((idx / (16 / CPR)) & (CPR - 1));
}

template <int BM, int BN, int CK, bool FUSED>
__global__ __launch_bounds__(256) void qconv_halo_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ w,
                                                         const Params p) {
  constexpr int WM = BM / 64, WN = BN / 64;
  static_assert(WM * WN == 4, "4 waves of 64x64");
  constexpr int CPR = CK / 16;
  constexpr int A_BYTES = BM * CK;
  constexpr int NPA = A_BYTES / 1024;  // 1-KiB LDS-DMA pieces per weight slice
  static_assert(NPA % 4 == 0, "every wave issues the same number of weight pieces");
  constexpr int BAND_PIX = MAX_BAND / CK;
  constexpr int OFF_S = MAX_BAND + 1024;            // band + slack for a partial last piece
  constexpr int OFF_A = OFF_S + 4 * BAND_PIX;
  constexpr int MAIN = OFF_A + 2 * A_BYTES;
  constexpr int EPI = 4 * (7 + MAX_CLASSES) * BM + (FUSED ? 256 * BM : 0);
  __shared__ __attribute__((aligned(16))) int8_t smem[MAIN > EPI ? MAIN : EPI];
  int8_t* s_band = smem;
  int* s_sum = reinterpret_cast<int*>(smem + OFF_S);
  int8_t* s_a = smem + OFF_A;

  const qnn_conv_desc& d = p.d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int frow = lane & 31, fh = lane >> 5;

  const int nby = (d.cout + BM - 1) / BM;
  const int nblk = ((p.M + BN - 1) / BN) * nby;
  int t;
  {
    const int b = blockIdx.x, xcd = b & 7, q = nblk >> 3, r = nblk & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int m0 = (t / nby) * BN;
  const int c0 = (t % nby) * BM;
  const int HoWo = d.ho * d.wo;

  // band rows of this pixel tile (flattened padded rows n*hp + row)
  int rlo, rhi;
  {
    const int mA = m0, mB = min(m0 + BN, p.M) - 1;
    const int nA = mA / HoWo, hoA = (mA - nA * HoWo) / d.wo;
    const int nB = mB / HoWo, hoB = (mB - nB * HoWo) / d.wo;
    rlo = nA * d.hp + hoA * d.sh;
    rhi = nB * d.hp + hoB * d.sh + d.kh - 1;
  }
  const int band_pix = (rhi - rlo + 1) * d.wp;
  const int band_pieces = (band_pix * CK + 1023) >> 10;
  const int8_t* xband = x + (int64_t)rlo * d.wp * d.cp;

  // per-lane band pixel of tap (0,0) for the two 32-pixel column tiles
  int P[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int m = m0 + wn * 64 + j * 32 + frow;
    if (m > p.M - 1) m = p.M - 1;
    const int n = m / HoWo, rem = m - n * HoWo, ho = rem / d.wo, wo = rem - ho * d.wo;
    P[j] = (n * d.hp + ho * d.sh - rlo) * d.wp + wo * d.sw;
  }
  // per-lane A fragment row offsets (fixed)
  int arow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) arow[i] = wm * 64 + i * 32 + frow;

  const int taps = p.taps;
  const int nch = d.cp / CK;
  const int nsteps = nch * taps;

  auto issue_a = [&](int step, int buf) {
    const int ch = step / taps, tp = step - ch * taps;
    const int8_t* src = w + (int64_t)c0 * d.kpad + tp * d.cp + ch * CK;
#pragma unroll
    for (int k = 0; k < NPA / 4; ++k) {
      const int pc = wave + 4 * k;
      const int L = pc * 64 + lane, row = L / CPR, slot = L % CPR;
      __builtin_amdgcn_global_load_lds((const void*)(src + (int64_t)row * d.kpad + 16 * swz_c<CPR>(row, slot)),
                                       (lds_ptr_t)(s_a + buf * A_BYTES + pc * 1024), 16, 0, 0);
    }
  };
  auto issue_band = [&](int ch) {
    const int8_t* src = xband + ch * CK;
    for (int pc = wave; pc < band_pieces; pc += 4) {
      const int L = pc * 64 + lane, q = L / CPR, slot = L % CPR;
      uint32_t off = q < band_pix ? (uint32_t)(q * d.cp + 16 * swz_c<CPR>(q, slot))
                                  : (uint32_t)(d.zero_off - (int64_t)rlo * d.wp * d.cp - ch * CK);
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_global_load_lds((const void*)(src + off), (lds_ptr_t)(s_band + pc * 1024), 16, 0, 0);
    }
  };

  v16i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (v16i){0};
  int sumq[2] = {0, 0};

  issue_a(0, 0);
  for (int ch = 0; ch < nch; ++ch) {
    issue_band(ch);
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    // per-band-pixel channel sums of the codes (exact)
    for (int q = tid; q < band_pix; q += 256) {
      int ssum = 0;
#pragma unroll
      for (int c = 0; c < CPR; ++c) {
        const v4i v = *reinterpret_cast<const v4i*>(s_band + q * CK + 16 * c);
        ssum = __builtin_amdgcn_sdot4(v.x, 0x01010101, ssum, false);
        ssum = __builtin_amdgcn_sdot4(v.y, 0x01010101, ssum, false);
        ssum = __builtin_amdgcn_sdot4(v.z, 0x01010101, ssum, false);
        ssum = __builtin_amdgcn_sdot4(v.w, 0x01010101, ssum, false);
      }
      s_sum[q] = ssum;
    }
    __syncthreads();
    for (int tp = 0; tp < taps; ++tp) {
      const int step = ch * taps + tp;
      const int buf = step & 1;
      if (step + 1 < nsteps) {
        issue_a(step + 1, buf ^ 1);
        wait_vmcnt<NPA / 4>();
      } else {
        wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
      const int r = tp / d.kw, sx = tp - r * d.kw;
      const int toff = r * d.wp + sx;
      const int8_t* sa = s_a + buf * A_BYTES;
      int bidx[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bidx[j] = P[j] + toff;
        sumq[j] += s_sum[bidx[j]];
      }
#pragma unroll
      for (int ks = 0; ks < CK / 32; ++ks) {
        const int chunk = 2 * ks + fh;
        v4i fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          fa[i] = *reinterpret_cast<const v4i*>(sa + arow[i] * CK + 16 * swz_c<CPR>(arow[i], chunk));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[j] = *reinterpret_cast<const v4i*>(s_band + bidx[j] * CK + 16 * swz_c<CPR>(bidx[j], chunk));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_barrier();
    }
  }
  __syncthreads();
  epilogue<BM, FUSED>(p, acc, sumq, smem, m0, c0, wm, wn, lane);
}

// Largest band (bytes per channel byte) over the pixel tiles of one launch.
static int64_t max_band_rows(const Params& p, int BN) {
  const qnn_conv_desc& d = p.d;
  const int HoWo = d.ho * d.wo;
  int64_t worst = 0;
  for (int m0 = 0; m0 < p.M; m0 += BN) {
    const int mB = (m0 + BN < p.M ? m0 + BN : p.M) - 1;
    const int nA = m0 / HoWo, hoA = (m0 - nA * HoWo) / d.wo;
    const int nB = mB / HoWo, hoB = (mB - nB * HoWo) / d.wo;
    const int64_t rows = (int64_t)(nB * d.hp + hoB * d.sh + d.kh - 1) - (nA * d.hp + hoA * d.sh) + 1;
    if (rows > worst) worst = rows;
  }
  return worst;
}

template <int BM, int BN, int CK, bool FUSED>
static void launch_halo(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  const int nblk = (int)(cdiv(p.M, BN) * cdiv(p.d.cout, BM));
  hipLaunchKernelGGL((qconv_halo_kernel<BM, BN, CK, FUSED>), dim3(nblk), dim3(256), 0, s, x, w, p);
}

// Picks the halo kernel's channel chunk (0 = not applicable).  QNN_HALO=0 disables it.
static int pick_halo_ck(const Params& p, int BM, int BN) {
  static int enabled = [] {
    const char* v = getenv("QNN_HALO");
    return v ? atoi(v) : 1;
  }();
  const qnn_conv_desc& d = p.d;
  if (!enabled || d.kmask || d.kh * d.kw < 2 || d.cp < 32) return 0;
  const int64_t rows = max_band_rows(p, BN);
  for (int ck : {128, 64, 32}) {
    if (d.cp % ck) continue;
    if ((BM * ck / 1024) % 4) continue;
    if (rows * d.wp * ck <= MAX_BAND) return ck;
  }
  return 0;
}

template <int BM, int BN, bool FUSED>
static bool try_halo(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  switch (pick_halo_ck(p, BM, BN)) {
    case 128: launch_halo<BM, BN, 128, FUSED>(x, w, p, s); return true;
    case 64: launch_halo<BM, BN, 64, FUSED>(x, w, p, s); return true;
    case 32:
      if constexpr (BM == 128) {
        launch_halo<BM, BN, 32, FUSED>(x, w, p, s);
        return true;
      }
      return false;
    default: return false;
  }
}

template <int BM, int BN, int BK, bool FUSED>
static void launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  const int nblk = (int)(cdiv(p.M, BN) * cdiv(p.d.cout, BM));
  if (p.d.kmask)
    hipLaunchKernelGGL((qconv_kernel<BM, BN, BK, FUSED, true>), dim3(nblk), dim3(256), 0, s, x, w, p);
  else
    hipLaunchKernelGGL((qconv_kernel<BM, BN, BK, FUSED, false>), dim3(nblk), dim3(256), 0, s, x, w, p);
}

// K-stage depth: 64-byte stages halve the LDS of a block (more blocks per CU to hide
// DMA latency and overlap one block's epilogue with another's MFMAs).  QNN_CONV_BK
// overrides (64 / 128) for A/B measurements.
static int pick_bk(const Params& p) {
  static int forced = [] {
    const char* v = getenv("QNN_CONV_BK");
    return v ? atoi(v) : 0;
  }();
  if (forced == 64 || forced == 128) return forced;
  return p.d.cout <= 64 ? 64 : 128;  // measured: BK=64 wins on 64-channel layers, 128 on wider
}

template <int BM, int BN, bool FUSED>
static void launch_bk(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s) {
  if (try_halo<BM, BN, FUSED>(x, w, p, s)) return;
  if (pick_bk(p) == 128) launch<BM, BN, 128, FUSED>(x, w, p, s);
  else launch<BM, BN, 64, FUSED>(x, w, p, s);
}

}  // namespace qnn

using namespace qnn;

extern "C" int qnn_qconv2d_fwd(const int8_t* x, const int8_t* wq, const qnn_conv_desc* desc, const qnn_epilogue* epi,
                               qnn_stream_t stream) {
  QNN_REQUIRE(desc && epi, "null descriptor");
  const qnn_conv_desc& d = *desc;
  const qnn_epilogue& e = *epi;
  QNN_REQUIRE(d.n >= 0 && d.hp > 0 && d.wp > 0 && d.cout > 0 && d.kh > 0 && d.kw > 0 && d.sh > 0 && d.sw > 0,
              "bad shape");
  QNN_REQUIRE(d.cp >= 16 && (d.cp & (d.cp - 1)) == 0, "cp must be 16 * 2^j");
  QNN_REQUIRE(d.kh * d.kw <= MAX_TAPS, "at most 64 taps");
  QNN_REQUIRE(d.ho > 0 && d.wo > 0 && (d.ho - 1) * d.sh + d.kh <= d.hp && (d.wo - 1) * d.sw + d.kw <= d.wp,
              "ho/wo exceed the padded input");
  QNN_REQUIRE(d.kpad % KPAD_ALIGN == 0 && d.kpad >= d.kh * d.kw * d.cp, "kpad must be a multiple of 128 covering K");
  QNN_REQUIRE((int64_t)d.n * d.hp * d.wp * d.cp < (1LL << 31) && d.zero_off >= 0 && d.zero_off % 16 == 0,
              "input too large or bad zero_off");
  QNN_REQUIRE(!d.kmask || (d.kpad <= MAX_MASK && (((uintptr_t)d.kmask) & 15) == 0), "kmask: kpad <= 1024, 16-B aligned");
  QNN_REQUIRE(e.nclass > 0 && e.nclass <= MAX_CLASSES && e.nwc > 0, "border classes out of range");
  QNN_REQUIRE(e.mode == 0 || e.mode == 1, "mode must be 0 (drop-in NCHW) or 1 (fused NHWC)");
  if (d.n == 0) return QNN_OK;
  QNN_REQUIRE(x && wq && e.sxsw && e.sxbw && e.table && e.hcls && e.wcls, "null pointer");
  QNN_REQUIRE((((uintptr_t)x) & 15) == 0 && (((uintptr_t)wq) & 15) == 0, "x/wq must be 16-byte aligned");
  if (e.mode == 0) {
    QNN_REQUIRE(e.out_f32 != nullptr, "mode 0 needs out_f32");
  } else {
    QNN_REQUIRE(d.cout % 4 == 0, "fused mode needs cout % 4 == 0");
    QNN_REQUIRE(!e.bn_mean || (e.bn_sq && e.bn_wq && e.bn_bq && e.bn_scale > 0.f), "incomplete RangeBN");
    QNN_REQUIRE(!e.out_code0 || (e.code0_cp % 4 == 0 && e.code0_scale > 0.f), "bad code0");
    QNN_REQUIRE(!e.out_code1 || (e.code1_cp % 4 == 0 && e.code1_scale > 0.f), "bad code1");
    QNN_REQUIRE(e.out_f32 || e.out_code0 || e.out_code1 || e.out_bncode, "fused mode without an output");
    QNN_REQUIRE(!e.lut || (e.bn_mean && e.out_code0 && !e.residual && !e.out_f32 && !e.out_code1 && !e.out_bncode &&
                           (((uintptr_t)e.lut) & 15) == 0),
                "lut needs RangeBN, exactly one code output, no residual/fp32/bncode, 16-B aligned");
  }
  Params p;
  p.d = d;
  p.e = e;
  const int64_t M = (int64_t)d.n * d.ho * d.wo;
  QNN_REQUIRE(M < (1LL << 31), "too many output pixels");
  p.M = (int)M;
  p.taps = d.kh * d.kw;
  p.lgcpt = __builtin_ctz(d.cp / 16);
  p.nstage = 0;
  hipStream_t s = (hipStream_t)stream;
  const bool narrow = d.cout <= 64;
  QNN_REQUIRE(d.cout_pad >= (narrow ? 64 : 128) * (int)cdiv(d.cout, narrow ? 64 : 128), "cout_pad too small");
  if (e.mode == 0) {
    if (narrow) launch_bk<64, 256, false>(x, wq, p, s);
    else launch_bk<128, 128, false>(x, wq, p, s);
  } else {
    if (narrow) launch_bk<64, 256, true>(x, wq, p, s);
    else launch_bk<128, 128, true>(x, wq, p, s);
  }
  QNN_LAUNCH_CHECK("qnn_qconv2d_fwd");
  return QNN_OK;
}
