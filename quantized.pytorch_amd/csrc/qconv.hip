// int8 MFMA implicit-GEMM convolution for the eval forward of QConv2d / QLinear
// (models/modules/quantize.py:314-349 and :398-428; biprecision is one contraction,
// SURVEY.md §0.3).  CDNA4 / gfx950 only: v_mfma_i32_32x32x32_i8.
//
// GEMM view:  D[c][m] = sum_k Wq'[c][k] * Xq'[k][m]
//   c = output channel (MFMA rows, operand A = packed weights [cout_pad][kpad])
//   m = output pixel n*Ho*Wo + ho*Wo + wo (MFMA columns, operand B gathered from
//       the NHWC8 activation codes: implicit im2col, zero outside the image)
//   k = (kh, kw, ci) tap-major, ci padded to Cp (16-byte chunks, one tap each)
// Exact decomposition of the reference fp32 conv of dequantized operands
// (SURVEY.md §0.5), evaluated in the epilogue:
//   y = s_x*s_w[c]*acc + s_x*b_w[c]*sum_valid(q'_x) + b_x*sum_valid(w_hat[c]) (+ bias[c])
// sum_valid(q'_x) is accumulated in-loop from the B fragments (v_dot4 against 1s);
// the border-aware third term comes from a per-(row class, col class, c) table.
//
// Block: 256 threads = 4 waves laid out WM x WN; each wave owns TM x TN tiles of
// 32x32; BK = 64 bytes of K per LDS stage, double-buffered, register-staged
// loads (issue early, write after compute), XOR-swizzled 16-B chunks so the
// ds_read_b128 fragment reads are bank-conflict free.
#include "qnn_internal.h"

namespace qnn {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

struct ConvParams {
  const int8_t* x;   // [N][H][W][Cp]
  const int8_t* w;   // [cout_pad][kpad]
  float* y;
  const float* sxsw;
  const float* sxbw;
  const float* table;
  const int* hcls;
  const int* wcls;
  const float* bias;
  int N, H, W, Cp, Cout, KH, KW, SH, SW, PH, PW, Ho, Wo;
  int K;     // KH*KW*Cp (real)
  int kpad;  // packed row stride, multiple of 64
  int M;     // N*Ho*Wo
  int nwc;
  int out_layout;
};

constexpr int BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 2) & 3)) << 4); }

template <int WM, int WN, int TM, int TN>
__global__ __launch_bounds__(256) void qconv_mfma_kernel(const ConvParams p) {
  constexpr int BM = WM * TM * 32;  // output channels per block
  constexpr int BN = WN * TN * 32;  // output pixels per block
  constexpr int A_LD = BM * 4 / 256;  // 16-B chunks per thread per stage
  constexpr int B_LD = BN * 4 / 256;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(A_LD >= 1 && B_LD >= 1, "tile too small");

  __shared__ __attribute__((aligned(16))) int8_t smem[2 * (BM + BN) * BK];
  auto sA = [&](int b) { return smem + b * (BM * BK); };
  auto sB = [&](int b) { return smem + 2 * BM * BK + b * (BN * BK); };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int m0 = blockIdx.x * BN;
  const int c0 = blockIdx.y * BM;
  const int HoWo = p.Ho * p.Wo;

  // ---- per-thread gather state for B (activation) chunks
  const int8_t* bptr[B_LD];
  int bh[B_LD], bw[B_LD];
  int bci[B_LD], br[B_LD], bs[B_LD];
  int bk[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    int q = tid + 256 * i;
    int prow = q >> 2, cj = q & 3;
    int m = m0 + prow;
    if (m < p.M) {
      int n = m / HoWo;
      int hw = m - n * HoWo;
      int ho = hw / p.Wo;
      int wo = hw - ho * p.Wo;
      bh[i] = ho * p.SH - p.PH;
      bw[i] = wo * p.SW - p.PW;
      bptr[i] = p.x + (int64_t)n * p.H * p.W * p.Cp;
    } else {
      bh[i] = -100000;  // never in bounds
      bw[i] = 0;
      bptr[i] = p.x;
    }
    // k = 16*cj within the first stage
    int k = 16 * cj;
    int tap = k / p.Cp;
    bci[i] = k - tap * p.Cp;
    br[i] = tap / p.KW;
    bs[i] = tap - br[i] * p.KW;
    bk[i] = k;
  }
  const int8_t* aptr[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    int q = tid + 256 * i;
    aptr[i] = p.w + (int64_t)(c0 + (q >> 2)) * p.kpad + 16 * (q & 3);
  }

  v4i ra[A_LD], rb[B_LD];
  auto load_stage = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) ra[i] = *reinterpret_cast<const v4i*>(aptr[i] + k0);
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      v4i v = {0, 0, 0, 0};
      int hi = bh[i] + br[i], wi = bw[i] + bs[i];
      if (bk[i] < p.K && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
        v = *reinterpret_cast<const v4i*>(bptr[i] + ((int64_t)(hi * p.W + wi) * p.Cp + bci[i]));
      rb[i] = v;
      // advance this chunk's k by BK
      bk[i] += BK;
      bci[i] += BK;
      while (bci[i] >= p.Cp) {
        bci[i] -= p.Cp;
        if (++bs[i] == p.KW) {
          bs[i] = 0;
          ++br[i];
        }
      }
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      int q = tid + 256 * i;
      *reinterpret_cast<v4i*>(sA(buf) + swz(q >> 2, q & 3)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      int q = tid + 256 * i;
      *reinterpret_cast<v4i*>(sB(buf) + swz(q >> 2, q & 3)) = rb[i];
    }
  };

  v16i acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v16i){0};
  int sumq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] = 0;

  const int nstage = p.kpad / BK;
  load_stage(0);
  store_stage(0);
  __syncthreads();

  const int frow = lane & 31, fh = lane >> 5;
  for (int st = 0; st < nstage; ++st) {
    const int buf = st & 1;
    if (st + 1 < nstage) load_stage((st + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = 2 * ks + fh;
      v4i fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const v4i*>(sA(buf) + swz(wm * TM * 32 + i * 32 + frow, chunk));
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        fb[j] = *reinterpret_cast<const v4i*>(sB(buf) + swz(wn * TN * 32 + j * 32 + frow, chunk));
        int s = __builtin_amdgcn_sdot4(fb[j].x, 0x01010101, 0, false);
        s = __builtin_amdgcn_sdot4(fb[j].y, 0x01010101, s, false);
        s = __builtin_amdgcn_sdot4(fb[j].z, 0x01010101, s, false);
        s = __builtin_amdgcn_sdot4(fb[j].w, 0x01010101, s, false);
        sumq[j] += s;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nstage) store_stage(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue
#pragma unroll
  for (int j = 0; j < TN; ++j) sumq[j] += __shfl_xor(sumq[j], 32, 64);

#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int m = m0 + wn * TN * 32 + j * 32 + frow;
    if (m >= p.M) continue;
    const int n = m / HoWo;
    const int hw = m - n * HoWo;
    const int ho = hw / p.Wo;
    const int wo = hw - ho * p.Wo;
    const float* trow = p.table + (int64_t)(p.hcls[ho] * p.nwc + p.wcls[wo]) * p.Cout;
    const float sq = (float)sumq[j];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = c0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        if (c >= p.Cout) continue;
        float v = fmaf(p.sxsw[c], (float)acc[i][j][r], fmaf(p.sxbw[c], sq, trow[c]));
        if (p.bias) v = v + p.bias[c];
        if (p.out_layout == 0)
          p.y[((int64_t)n * p.Cout + c) * HoWo + hw] = v;
        else
          p.y[(int64_t)m * p.Cout + c] = v;
      }
    }
  }
}

template <int WM, int WN, int TM, int TN>
static int launch(const ConvParams& p, hipStream_t stream) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  dim3 grid((unsigned)cdiv(p.M, BN), (unsigned)cdiv(p.Cout, BM));
  hipLaunchKernelGGL((qconv_mfma_kernel<WM, WN, TM, TN>), grid, dim3(256), 0, stream, p);
  QNN_LAUNCH_CHECK("qnn_qconv2d_fwd");
  return QNN_OK;
}

}  // namespace qnn

using namespace qnn;

extern "C" int qnn_qconv2d_fwd(const int8_t* x, int n, int h, int w, int cp, const int8_t* wq, int cout, int cout_pad,
                               int kh, int kw, int sh, int sw, int ph, int pw, int ho, int wo, const float* sxsw,
                               const float* sxbw, const float* table, const int* hcls, const int* wcls, int nwc,
                               const float* bias, float* y, int out_layout, qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && h > 0 && w > 0 && cout > 0 && kh > 0 && kw > 0 && sh > 0 && sw > 0 && ph >= 0 && pw >= 0,
              "bad shape");
  QNN_REQUIRE(cp > 0 && cp % 16 == 0, "cp must be a positive multiple of 16");
  QNN_REQUIRE(ho == (h + 2 * ph - kh) / sh + 1 && wo == (w + 2 * pw - kw) / sw + 1, "ho/wo inconsistent");
  QNN_REQUIRE(out_layout == 0 || out_layout == 1, "out_layout must be 0 or 1");
  QNN_REQUIRE(nwc > 0, "nwc must be > 0");
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(x && wq && sxsw && sxbw && table && hcls && wcls && y, "null pointer");
  QNN_REQUIRE((((uintptr_t)x) & 15) == 0 && (((uintptr_t)wq) & 15) == 0, "x/wq must be 16-byte aligned");
  ConvParams p;
  p.x = x; p.w = wq; p.y = y; p.sxsw = sxsw; p.sxbw = sxbw; p.table = table; p.hcls = hcls; p.wcls = wcls;
  p.bias = bias;
  p.N = n; p.H = h; p.W = w; p.Cp = cp; p.Cout = cout; p.KH = kh; p.KW = kw; p.SH = sh; p.SW = sw; p.PH = ph; p.PW = pw;
  p.Ho = ho; p.Wo = wo;
  p.K = kh * kw * cp;
  p.kpad = (int)(cdiv((int64_t)p.K, BK) * BK);
  int64_t M = (int64_t)n * ho * wo;
  QNN_REQUIRE(M < (1LL << 31), "too many output pixels");
  p.M = (int)M;
  p.nwc = nwc;
  p.out_layout = out_layout;
  hipStream_t s = (hipStream_t)stream;
  // tile choice: 64-channel tiles for narrow layers, 128x128 otherwise
  if (cout <= 64) {
    QNN_REQUIRE(cout_pad >= 64 && cout_pad % 64 == 0, "cout_pad must be a multiple of 64 (>= 64)");
    return launch<1, 4, 2, 2>(p, s);  // 64 x 256
  }
  QNN_REQUIRE(cout_pad % 128 == 0, "cout_pad must be a multiple of 128 when cout > 64");
  return launch<2, 2, 2, 2>(p, s);    // 128 x 128
}
