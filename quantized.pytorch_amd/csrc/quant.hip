// Quantizer, weight pre-pack, RangeBN and depthwise kernels of the qnn C ABI.
// Reference semantics: models/modules/quantize.py (see include/qnn.h per entry).
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "qnn_internal.h"

namespace qnn {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return QNN_OK;
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  return QNN_ERR_HIP;
}

int arg_error(const char* what) {
  set_error(std::string("invalid argument: ") + what);
  return QNN_ERR_ARG;
}

// ------------------------------------------------------------------ fake quant
__global__ void fake_quant_kernel(const float* __restrict__ x, float* y, int64_t n, float neg_min,
                                  float min, float scale, float qmax) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (; i < n; i += stride) {
    if (i + 4 <= n && ((((uintptr_t)(x + i)) | ((uintptr_t)(y + i))) & 15) == 0) {
      float4 v = *reinterpret_cast<const float4*>(x + i);
      v.x = fake_quant(v.x, neg_min, min, scale, qmax);
      v.y = fake_quant(v.y, neg_min, min, scale, qmax);
      v.z = fake_quant(v.z, neg_min, min, scale, qmax);
      v.w = fake_quant(v.w, neg_min, min, scale, qmax);
      *reinterpret_cast<float4*>(y + i) = v;
    } else {
      for (int64_t j = i; j < n && j < i + 4; ++j) y[j] = fake_quant(x[j], neg_min, min, scale, qmax);
    }
  }
}

__global__ void fake_quant_rows_kernel(const float* __restrict__ x, float* y, int rows, int64_t cols,
                                       const float* __restrict__ mins, const float* __restrict__ maxs, float qmax) {
  const int r = blockIdx.y;
  const float mn = mins[r], mx = maxs[r];
  float s = (mx - mn) / qmax;  // quantize.py:71 (tensor scale, fp32)
  s = fmaxf(s, 1e-8f);         // :73
  const float* xr = x + (int64_t)r * cols;
  float* yr = y + (int64_t)r * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cols; i += (int64_t)gridDim.x * blockDim.x)
    yr[i] = fake_quant(xr[i], -mn, mn, s, qmax);
}

// One 1024-thread block: range of the vector, then quantize it.
__global__ __launch_bounds__(1024) void fake_quant_vec_kernel(const float* __restrict__ x, float* y, int n,
                                                              float qmax, int scale_mode, float* range_out) {
  __shared__ float smin[16], smax[16];
  __shared__ float s_params[3];
  float lo = INFINITY, hi = -INFINITY;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float v = x[i];
    lo = fminf(lo, v);
    hi = fmaxf(hi, v);
  }
  lo = wave_min(lo);
  hi = wave_max(hi);
  int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    smin[wid] = lo;
    smax[wid] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int nw = (blockDim.x + 63) >> 6;
    float mn = smin[0], mx = smax[0];
    for (int k = 1; k < nw; ++k) {
      mn = fminf(mn, smin[k]);
      mx = fmaxf(mx, smax[k]);
    }
    float s;
    if (scale_mode == 0) {
      s = (mx - mn) / qmax;           // tensor scale (quantize.py:71), fp32
      s = fmaxf(s, 1e-8f);            // scale.clamp_(1e-8)      (:73)
    } else {
      double sd = ((double)mx - (double)mn) / (double)qmax;  // Python float scale (:71)
      sd = sd > 1e-8 ? sd : 1e-8;                             // max(scale, 1e-8) (:75)
      s = (float)sd;                                          // cast at div_/mul_
    }
    s_params[0] = mn;
    s_params[1] = mx;
    s_params[2] = s;
    if (range_out) {
      range_out[0] = mn;
      range_out[1] = mx;
    }
  }
  __syncthreads();
  float mn = s_params[0], s = s_params[2];
  for (int i = threadIdx.x; i < n; i += blockDim.x) y[i] = fake_quant(x[i], -mn, mn, s, qmax);
}

// ------------------------------------------------------------------ NCHW -> padded NHWC8
// One thread per (padded pixel, 16-channel group): interior pixels quantize 16
// channels (reads coalesced along w), border pixels / pad channels write code' 0.
__global__ void quantize_nchw_nhwc8_kernel(const float* __restrict__ x, int8_t* __restrict__ q, int n, int c, int h,
                                           int w, int pad, int cp, float neg_min, float scale, float qmax) {
  const int hp = h + 2 * pad, wp = w + 2 * pad, groups = cp >> 4;
  const int64_t npix = (int64_t)n * hp * wp;
  const int64_t total = npix * groups;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = idx % npix;
    const int g = (int)(idx / npix);
    const int wq = (int)(pix % wp);
    const int64_t t = pix / wp;
    const int hq = (int)(t % hp);
    const int64_t img = t / hp;
    const int iy = hq - pad, ix = wq - pad;
    union {
      int8_t b[16];
      int4 v;
    } out;
    out.v = make_int4(0, 0, 0, 0);
    if (iy >= 0 && iy < h && ix >= 0 && ix < w) {
      const float* src = x + (img * c) * (int64_t)h * w + (int64_t)iy * w + ix;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int ch = g * 16 + j;
        if (ch < c) out.b[j] = (int8_t)((int)quant_code(src[(int64_t)ch * h * w], neg_min, scale, qmax) - 128);
      }
    }
    *reinterpret_cast<int4*>(q + pix * cp + g * 16) = out.v;
  }
  if (blockIdx.x == 0 && threadIdx.x < 8)  // 128-byte zero page after the tensor
    *reinterpret_cast<int4*>(q + npix * cp + 16 * threadIdx.x) = make_int4(0, 0, 0, 0);
}

// Space-to-depth codes (factor 2): z[n][h2][w2][(2u+v)*c + ci], 16 channels.  One thread per
// s2d pixel: its 4*c input values (2 rows x 2 columns x c channels, code' 0 outside the image)
// are loaded together -- for a wave, each of the 4*c loads reads 64 values two floats apart,
// so every input byte is fetched from HBM once and L1 serves the interleaved half --
// quantized (quant_code_fast == IEEE division, bit for bit) and stored as one 16-byte pixel.
// No LDS, no barrier: all 12 loads of every lane are in flight at once.
__global__ __launch_bounds__(256) void quantize_s2d_kernel(const float* __restrict__ x, int8_t* __restrict__ z, int n,
                                                           int c, int h, int w, int pad, int hz, int wz, float neg_min,
                                                           float scale, float qmax) {
  const float inv = 1.0f / scale;
  const int64_t total = (int64_t)n * hz * wz;
  const int64_t hw = (int64_t)h * w;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int w2 = (int)(i % wz);
    const int64_t r = i / wz;
    const int h2 = (int)(r % hz), img = (int)(r / hz);
    float v[16];
    bool ok[4];
#pragma unroll
    for (int uv = 0; uv < 4; ++uv) {
      const int iy = 2 * h2 + (uv >> 1) - pad, ix = 2 * w2 + (uv & 1) - pad;
      ok[uv] = iy >= 0 && iy < h && ix >= 0 && ix < w;
      const float* src = x + (int64_t)img * c * hw + (ok[uv] ? (int64_t)iy * w + ix : 0);
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) v[uv * 4 + ci] = ci < c ? src[ci * hw] : 0.f;
    }
    union {
      int8_t b[16];
      int4 q;
    } out;
    out.q = make_int4(0, 0, 0, 0);
#pragma unroll
    for (int uv = 0; uv < 4; ++uv)
#pragma unroll
      for (int ci = 0; ci < 4; ++ci)
        if (ci < c && ok[uv])
          out.b[uv * c + ci] = (int8_t)((int)quant_code_fast(v[uv * 4 + ci], neg_min, scale, inv, qmax) - 128);
    *reinterpret_cast<int4*>(z + i * 16) = out.q;
  }
  if (blockIdx.x == 0 && threadIdx.x < 8)
    *reinterpret_cast<int4*>(z + (int64_t)n * hz * wz * 16 + 16 * threadIdx.x) = make_int4(0, 0, 0, 0);
}

// The same space-to-depth codes, two s2d pixels (four input columns) per thread, for w % 4 == 0
// and a 16-byte aligned x: every input row segment is read as the two aligned float4s around
// it (a whole wave instruction = 1 KiB contiguous; the neighbour's shared float4 hits L1), so
// the reads are 16 bytes per lane instead of 4 at a 2-float stride; each code byte is
// quant_code_fast of the same float, so the codes are bitwise quantize_s2d_kernel's.
// OFF = (4 - pad % 4) % 4: where column 4k - pad sits in its float4; CH = c (compile-time, so
// every code byte's position is too and nothing goes through scratch)
template <int OFF, int CH>
__global__ __launch_bounds__(256) void quantize_s2d_x2_kernel(const float* __restrict__ x, int8_t* __restrict__ z,
                                                              int n, int h, int w, int pad, int hz, int wz,
                                                              float neg_min, float scale, float qmax) {
  constexpr int c = CH;
  const float inv = 1.0f / scale;
  const int wz2 = (wz + 1) >> 1;
  const int64_t total = (int64_t)n * hz * wz2;
  const int64_t hw = (int64_t)h * w;
  constexpr int off = OFF;  // column 4k - pad = 4a + off, a = floor((4k - pad) / 4)
  const int w4 = w >> 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % wz2);
    const int64_t r = i / wz2;
    const int h2 = (int)(r % hz), img = (int)(r / hz);
    const int a = (4 * k - pad - off) >> 2;  // exact: 4k - pad - off is a multiple of 4
    float v[2][4][4];                        // [row][channel][column 0..3 = 4k - pad ..]
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int iy = 2 * h2 + rr - pad;
      const bool rok = iy >= 0 && iy < h;
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) {
        float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
        if (ci < c && rok) {
          const float4* row = reinterpret_cast<const float4*>(x + ((int64_t)img * c + ci) * hw + (int64_t)iy * w);
          if (a >= 0 && a < w4) A = row[a];
          if (a + 1 >= 0 && a + 1 < w4) B = row[a + 1];
        }
        const float e[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) v[rr][ci][j] = e[off + j];
      }
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int w2 = 2 * k + p;
      if (w2 >= wz) break;
      union {
        int8_t b[16];
        int4 q;
      } out;
      out.q = make_int4(0, 0, 0, 0);
#pragma unroll
      for (int uv = 0; uv < 4; ++uv) {
        const int rr = uv >> 1, u = uv & 1;
        const int iy = 2 * h2 + rr - pad, ix = 2 * w2 + u - pad;
        const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
#pragma unroll
        for (int ci = 0; ci < 4; ++ci)
          if (ci < c && ok)
            out.b[uv * c + ci] = (int8_t)((int)quant_code_fast(v[rr][ci][2 * p + u], neg_min, scale, inv, qmax) - 128);
      }
      *reinterpret_cast<int4*>(z + (r * wz + w2) * 16) = out.q;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 8)
    *reinterpret_cast<int4*>(z + (int64_t)n * hz * wz * 16 + 16 * threadIdx.x) = make_int4(0, 0, 0, 0);
}

// quantize_s2d_x2_kernel's codes with one wave per s2d row (lane k = pair k of the row, wz2 <= 64):
// the row's image and height come from the wave-uniform row index on the scalar unit, so no lane
// divides (the grid-stride form spent ~3 64-bit divisions per pair), and the tail zero page is
// written by the first block.  Bitwise quantize_s2d_x2_kernel's (same loads, same quotients).
template <int OFF, int CH>
__global__ __launch_bounds__(256) void quantize_s2d_rows_kernel(const float* __restrict__ x, int8_t* __restrict__ z,
                                                                int n, int h, int w, int pad, int hz, int wz,
                                                                float neg_min, float scale, float qmax) {
  constexpr int c = CH;
  constexpr int off = OFF;
  const float inv = 1.0f / scale;
  const int wz2 = (wz + 1) >> 1;
  const int r = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));  // s2d row (img, h2)
  const int k = threadIdx.x & 63;
  if (r < n * hz && k < wz2) {
    const int img = r / hz, h2 = r - img * hz;
    const int64_t hw = (int64_t)h * w;
    const int w4 = w >> 2;
    const int a = (4 * k - pad - off) >> 2;
    float v[2][4][4];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int iy = 2 * h2 + rr - pad;
      const bool rok = iy >= 0 && iy < h;
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) {
        float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
        if (ci < c && rok) {
          const float4* row = reinterpret_cast<const float4*>(x + ((int64_t)img * c + ci) * hw + (int64_t)iy * w);
          if (a >= 0 && a < w4) A = row[a];
          if (a + 1 >= 0 && a + 1 < w4) B = row[a + 1];
        }
        const float e[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) v[rr][ci][j] = e[off + j];
      }
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int w2 = 2 * k + p;
      if (w2 >= wz) break;
      union {
        int8_t b[16];
        int4 q;
      } out;
      out.q = make_int4(0, 0, 0, 0);
#pragma unroll
      for (int uv = 0; uv < 4; ++uv) {
        const int rr = uv >> 1, u = uv & 1;
        const int iy = 2 * h2 + rr - pad, ix = 2 * w2 + u - pad;
        const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
#pragma unroll
        for (int ci = 0; ci < 4; ++ci)
          if (ci < c && ok)
            out.b[uv * c + ci] = (int8_t)((int)quant_code_fast(v[rr][ci][2 * p + u], neg_min, scale, inv, qmax) - 128);
      }
      *reinterpret_cast<int4*>(z + ((int64_t)r * wz + w2) * 16) = out.q;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 8)
    *reinterpret_cast<int4*>(z + (int64_t)n * hz * wz * 16 + 16 * threadIdx.x) = make_int4(0, 0, 0, 0);
}

// ------------------------------------------------------------------ generic drop-in conv
// F.conv2d(input_, qweight, qbias, stride, padding, dilation, groups) of QConv2d.forward
// (quantize.py:342-344) for the shapes the int8 MFMA path does not take: dilation != 1, grouped
// convs other than depthwise, unequal / string ('same', 'valid') padding.  A correctness path, not
// a tuned one: one thread per output, the input fake-quantized on the fly with the quantizer's own
// op order (quant_code -> dequant, quantize.py:89-100), the products of the fake-quantized operands
// summed in fp64 and rounded once, then + the quantized bias (as the reference's conv adds it).
__global__ __launch_bounds__(256) void qconv_generic_kernel(const float* __restrict__ x, int n, int c, int h, int w,
                                                            float neg_min, float xmin, float scale, float qmax,
                                                            const float* __restrict__ w_hat, int cout, int groups,
                                                            int kh, int kw, int sh, int sw, int pt, int pl, int dh,
                                                            int dw, int ho, int wo, const float* __restrict__ bias,
                                                            float* __restrict__ y) {
  const int cin_g = c / groups, cout_g = cout / groups;
  const int64_t total = (int64_t)n * cout * ho * wo;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(i % wo);
    int64_t r = i / wo;
    const int oy = (int)(r % ho);
    r /= ho;
    const int co = (int)(r % cout), img = (int)(r / cout);
    const int g = co / cout_g;
    const float* wp = w_hat + (int64_t)co * cin_g * kh * kw;
    double acc = 0.0;
    for (int ci = 0; ci < cin_g; ++ci) {
      const float* xp = x + ((int64_t)img * c + g * cin_g + ci) * h * w;
      for (int ky = 0; ky < kh; ++ky) {
        const int iy = oy * sh - pt + ky * dh;
        if (iy < 0 || iy >= h) continue;
        for (int kx = 0; kx < kw; ++kx) {
          const int ix = ox * sw - pl + kx * dw;
          if (ix < 0 || ix >= w) continue;
          const float xq = fake_quant(xp[(int64_t)iy * w + ix], neg_min, xmin, scale, qmax);
          acc += (double)xq * (double)wp[(ci * kh + ky) * kw + kx];
        }
      }
    }
    float v = (float)acc;
    if (bias) v = v + bias[co];
    y[i] = v;
  }
}

// ------------------------------------------------------------------ gradient quantizer
// quantize.py:76-97 with enforce_true_zero (the binding of UniformQuantizeGrad.backward):
// the reference's in-place op order, one element per lane, four per thread
__global__ __launch_bounds__(256) void grad_quant_kernel(const float* __restrict__ g, const float* __restrict__ noise,
                                                         float* __restrict__ out, int64_t n, float scale, float zp,
                                                         float qmax) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float t = g[i] / scale;  // output.div_(scale)
    t = t + zp;              // .add_(zero_point)
    if (noise) t = t + noise[i];
    t = rintf(fminf(fmaxf(t, 0.0f), qmax));  // clamp_(qmin, qmax).round_()
    t = t + (-zp);                           // add_(-zero_point)
    out[i] = t * scale;                      // .mul_(scale)
  }
}

// ------------------------------------------------------------------ weight pack
// One block per (padded) output channel.  Deterministic fp64 tap sums.
__global__ __launch_bounds__(256) void pack_weight_kernel(const float* __restrict__ w, int cout, int cin_g, int kh,
                                                          int kw, int cin_pad, int kpad, int s2d, float qmax,
                                                          const float* w_min_in, const float* w_max_in,
                                                          int8_t* __restrict__ wq, float* s_w, float* b_w,
                                                          float* tap_sum, float* w_hat, float* w_min_out,
                                                          float* w_max_out) {
  const int c = blockIdx.x;
  const int taps = kh * kw;
  const int E = cin_g * taps;
  int8_t* row = wq + (int64_t)c * kpad;
  if (c >= cout) {
    for (int i = threadIdx.x; i < kpad; i += blockDim.x) row[i] = 0;
    return;
  }
  __shared__ float s_mm[2][4];
  __shared__ double s_red[4];
  const float* wc = w + (int64_t)c * E;
  float mn, mx;
  if (w_min_in && w_max_in) {
    mn = w_min_in[c];
    mx = w_max_in[c];
  } else {
    float lo = INFINITY, hi = -INFINITY;
    for (int i = threadIdx.x; i < E; i += blockDim.x) {
      lo = fminf(lo, wc[i]);
      hi = fmaxf(hi, wc[i]);
    }
    lo = wave_min(lo);
    hi = wave_max(hi);
    if ((threadIdx.x & 63) == 0) {
      s_mm[0][threadIdx.x >> 6] = lo;
      s_mm[1][threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    mn = fminf(fminf(s_mm[0][0], s_mm[0][1]), fminf(s_mm[0][2], s_mm[0][3]));
    mx = fmaxf(fmaxf(s_mm[1][0], s_mm[1][1]), fmaxf(s_mm[1][2], s_mm[1][3]));
  }
  float s = (mx - mn) / qmax;  // quantize.py:71 (tensor, fp32)
  s = fmaxf(s, 1e-8f);         // :73
  const float neg_min = -mn;
  if (threadIdx.x == 0) {
    s_w[c] = s;
    b_w[c] = (float)(128.0 * (double)s + (double)mn);
    if (w_min_out) w_min_out[c] = mn;
    if (w_max_out) w_max_out[c] = mx;
  }
  const int pkw = s2d ? (kw + 1) / 2 : kw;
  const int ptaps = s2d ? ((kh + 1) / 2) * pkw : taps;
  for (int i = threadIdx.x; i < kpad; i += blockDim.x) {
    int8_t code = 0;
    const int tap = i / cin_pad;
    const int cc = i - tap * cin_pad;
    int r = -1, sx = -1, ci = -1;
    if (tap < ptaps) {
      if (!s2d) {
        if (cc < cin_g) { r = tap / kw; sx = tap - r * kw; ci = cc; }
      } else if (cc < 4 * cin_g) {
        const int uv = cc / cin_g, a = tap / pkw, b = tap - a * pkw;
        ci = cc - uv * cin_g;
        r = 2 * a + (uv >> 1);
        sx = 2 * b + (uv & 1);
        if (r >= kh || sx >= kw) r = -1;
      }
    }
    if (r >= 0) code = (int8_t)((int)quant_code(wc[ci * taps + r * kw + sx], neg_min, s, qmax) - 128);
    row[i] = code;
  }
  if (w_hat) {
    for (int e = threadIdx.x; e < E; e += blockDim.x)
      w_hat[(int64_t)c * E + e] = fake_quant(wc[e], neg_min, mn, s, qmax);
  }
  if (tap_sum) {
    for (int tap = 0; tap < taps; ++tap) {
      double acc = 0.0;
      for (int ci = threadIdx.x; ci < cin_g; ci += blockDim.x)
        acc += (double)fake_quant(wc[ci * taps + tap], neg_min, mn, s, qmax);
      acc = wave_sum(acc);
      __syncthreads();
      if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = acc;
      __syncthreads();
      if (threadIdx.x == 0) tap_sum[(int64_t)c * taps + tap] = (float)(s_red[0] + s_red[1] + s_red[2] + s_red[3]);
    }
  }
}

__global__ void border_table_kernel(const float* __restrict__ tap_sum, int cout, int kh, int kw,
                                    const int* __restrict__ hrange, int nhc, const int* __restrict__ wrange,
                                    int nwc, float b_x, float* __restrict__ table) {
  int64_t total = (int64_t)nhc * nwc * cout;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % cout);
    int cls = (int)(i / cout);
    int wc = cls % nwc, hc = cls / nwc;
    double acc = 0.0;
    for (int r = hrange[2 * hc]; r < hrange[2 * hc + 1]; ++r)
      for (int s = wrange[2 * wc]; s < wrange[2 * wc + 1]; ++s) acc += (double)tap_sum[(int64_t)c * kh * kw + r * kw + s];
    table[i] = (float)((double)b_x * acc);
  }
}

// ------------------------------------------------------------------ RangeBN eval
__device__ __forceinline__ float rangebn_one(float x, float neg_min, float min, float scale, float qmax, float mu,
                                             float sq, float wq, float bq) {
  float xh = fake_quant(x, neg_min, min, scale, qmax);  // quantize_input  :462
  float o = xh - mu;                                     // x - mean        :488
  o = o * sq;                                            // * q(scale)      :488-489
  o = o * wq;                                            // * q(weight)     :495
  return o + bq;                                         // + q(bias)       :499
}

__global__ void rangebn_kernel(const float* __restrict__ x, float* y, int64_t total, int c, int hw, float neg_min,
                               float min, float scale, float qmax, const float* __restrict__ mean,
                               const float* __restrict__ sq, const float* __restrict__ wq,
                               const float* __restrict__ bq, const float* residual, int relu) {
  const bool vec = (hw & 3) == 0;
  int64_t step = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < total; i += step) {
    if (vec) {
      int ch = (int)((i / hw) % c);
      float mu = mean[ch], a = sq[ch], b = wq[ch], d = bq[ch];
      float4 v = *reinterpret_cast<const float4*>(x + i);
      float4 o;
      o.x = rangebn_one(v.x, neg_min, min, scale, qmax, mu, a, b, d);
      o.y = rangebn_one(v.y, neg_min, min, scale, qmax, mu, a, b, d);
      o.z = rangebn_one(v.z, neg_min, min, scale, qmax, mu, a, b, d);
      o.w = rangebn_one(v.w, neg_min, min, scale, qmax, mu, a, b, d);
      if (residual) {
        float4 r = *reinterpret_cast<const float4*>(residual + i);
        o.x = o.x + r.x; o.y = o.y + r.y; o.z = o.z + r.z; o.w = o.w + r.w;
      }
      if (relu) {
        o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
      }
      *reinterpret_cast<float4*>(y + i) = o;
    } else {
      for (int64_t j = i; j < total && j < i + 4; ++j) {
        int ch = (int)((j / hw) % c);
        float o = rangebn_one(x[j], neg_min, min, scale, qmax, mean[ch], sq[ch], wq[ch], bq[ch]);
        if (residual) o = o + residual[j];
        if (relu) o = fmaxf(o, 0.f);
        y[j] = o;
      }
    }
  }
}

// ------------------------------------------------------------------ depthwise
__global__ void dwconv_kernel(const float* __restrict__ x, int n, int c, int h, int w,
                              const float* __restrict__ w_hat, int kh, int kw, int sh, int sw, int ph, int pw,
                              int ho, int wo, float neg_min, float min, float scale, float qmax,
                              const float* __restrict__ bias, float* __restrict__ y) {
  int64_t total = (int64_t)n * c * ho * wo;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int ox = (int)(i % wo);
    int64_t t = i / wo;
    int oy = (int)(t % ho);
    int64_t nc = t / ho;
    int ch = (int)(nc % c);
    const float* xp = x + nc * h * w;
    const float* wp = w_hat + (int64_t)ch * kh * kw;
    float acc = 0.f;
    for (int r = 0; r < kh; ++r) {
      int iy = oy * sh - ph + r;
      if (iy < 0 || iy >= h) continue;
      for (int s = 0; s < kw; ++s) {
        int ix = ox * sw - pw + s;
        if (ix < 0 || ix >= w) continue;
        float xh = fake_quant(xp[iy * w + ix], neg_min, min, scale, qmax);
        acc = fmaf(xh, wp[r * kw + s], acc);
      }
    }
    if (bias) acc = acc + bias[ch];
    y[i] = acc;
  }
}

static int grid_for(int64_t work, int block) {
  int64_t g = cdiv(work, block);
  if (g > 256 * 32) g = 256 * 32;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace qnn

using namespace qnn;

extern "C" {

int qnn_abi_version(void) { return QNN_ABI_VERSION; }

const char* qnn_last_error(void) { return qnn::g_last_error.c_str(); }

int qnn_fake_quant_f32(const float* x, float* y, int64_t n, float neg_min, float min, float scale, float qmax,
                       qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0, "n < 0");
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(x && y, "null pointer");
  QNN_REQUIRE(scale > 0.f, "scale must be > 0");
  hipLaunchKernelGGL(fake_quant_kernel, dim3(grid_for(cdiv(n, 4), 256)), dim3(256), 0, (hipStream_t)stream, x, y,
                     n, neg_min, min, scale, qmax);
  QNN_LAUNCH_CHECK("qnn_fake_quant_f32");
  return QNN_OK;
}

int qnn_fake_quant_rows_f32(const float* x, float* y, int rows, int64_t cols, const float* mins, const float* maxs,
                            float qmax, qnn_stream_t stream) {
  QNN_REQUIRE(rows >= 0 && cols >= 0 && rows <= 65535, "bad shape (rows must be <= 65535)");
  if (rows == 0 || cols == 0) return QNN_OK;
  QNN_REQUIRE(x && y && mins && maxs, "null pointer");
  int gx = (int)cdiv(cols, 256);
  if (gx > 64) gx = 64;
  hipLaunchKernelGGL(fake_quant_rows_kernel, dim3(gx, rows), dim3(256), 0, (hipStream_t)stream, x, y, rows, cols, mins,
                     maxs, qmax);
  QNN_LAUNCH_CHECK("qnn_fake_quant_rows_f32");
  return QNN_OK;
}

int qnn_fake_quant_vec_f32(const float* x, float* y, int n, float qmax, int scale_mode, float* range_out,
                           qnn_stream_t stream) {
  QNN_REQUIRE(n > 0 && n <= 65536, "n must be in [1, 65536]");
  QNN_REQUIRE(x && y, "null pointer");
  QNN_REQUIRE(scale_mode == 0 || scale_mode == 1, "scale_mode must be 0 or 1");
  hipLaunchKernelGGL(fake_quant_vec_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, x, y, n, qmax, scale_mode,
                     range_out);
  QNN_LAUNCH_CHECK("qnn_fake_quant_vec_f32");
  return QNN_OK;
}

int qnn_grad_quant_f32(const float* g, const float* noise, float* out, int64_t n, float scale, float zero_point,
                       float qmax, qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0, "n must be >= 0");
  QNN_REQUIRE(scale > 0.f, "scale must be > 0");
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(g && out, "null pointer");
  hipLaunchKernelGGL(grad_quant_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, g, noise, out, n,
                     scale, zero_point, qmax);
  QNN_LAUNCH_CHECK("qnn_grad_quant_f32");
  return QNN_OK;
}

// The same codes, 4 pixels per thread (w % 4 == 0, x 16-byte aligned): one float4 load per
// channel (16 of them in flight: 64 values), 16 codes per pixel as one 16-byte store.  Lanes take
// the cp / 16 channel groups fastest, so a store instruction's lanes write whole 64-128-byte
// pixels, then the pixel quads along the row (a load instruction: cp / 16 planes x 256 B).  The
// padding ring is written by the threads past the interior.  32-bit indices (checked by the host).
__global__ __launch_bounds__(256) void quantize_nchw_nhwc8_q4_kernel(const float* __restrict__ x, int8_t* __restrict__ q,
                                                                     int n, int c, int h, int w, int pad, int cp,
                                                                     float neg_min, float scale, float qmax) {
  const int hp = h + 2 * pad, wp = w + 2 * pad, G = cp >> 4, wq = w >> 2;
  const int interior = n * h * wq * G;
  const int ring = n * (hp * wp - h * w) * G;  // border pixels x groups
  const float inv = 1.0f / scale;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < interior + ring; idx += gridDim.x * blockDim.x) {
    if (idx < interior) {
      const int g = idx % G, r = idx / G;
      const int qd = r % wq, r2 = r / wq;
      const int y = r2 % h, img = r2 / h;
      const float* src = x + ((size_t)img * c * h + y) * w + 4 * qd;
      const size_t hw = (size_t)h * w;
      float4 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {  // channels past c re-read channel c - 1 (masked below): no
        const int ch = min(16 * g + j, c - 1);  // per-load branch
        v[j] = *reinterpret_cast<const float4*>(src + ch * hw);
      }
      int8_t* dst = q + (((size_t)img * hp + y + pad) * wp + pad + 4 * qd) * cp + 16 * g;
#pragma unroll
      for (int px = 0; px < 4; ++px) {
        unsigned wd[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          unsigned b = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = 4 * k + u;
            const float f = px == 0 ? v[j].x : px == 1 ? v[j].y : px == 2 ? v[j].z : v[j].w;
            const unsigned code = (unsigned)(int)quant_code_fast(f, neg_min, scale, inv, qmax) - 128u;
            b |= ((16 * g + j < c ? code : 0u) & 255u) << (8 * u);
          }
          wd[k] = b;
        }
        *reinterpret_cast<int4*>(dst + px * cp) = make_int4((int)wd[0], (int)wd[1], (int)wd[2], (int)wd[3]);
      }
    } else {
      // border pixel k of an image: the top pad rows, the bottom pad rows, then each interior row's
      // left and right pad columns
      const int k = idx - interior, g = k % G, r = k / G;
      const int per_img = hp * wp - h * w, img = r / per_img, b = r % per_img;
      const int top = pad * wp;
      int y, col;
      if (b < 2 * top) {
        y = b < top ? b / wp : h + pad + (b - top) / wp;
        col = (b < top ? b : b - top) % wp;
      } else {
        const int e = b - 2 * top, side = 2 * pad;
        y = pad + e / side;
        const int s = e % side;
        col = s < pad ? s : w + s;
      }
      *reinterpret_cast<int4*>(q + (((size_t)img * hp + y) * wp + col) * cp + 16 * g) = make_int4(0, 0, 0, 0);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 8)  // 128-byte zero page after the tensor
    *reinterpret_cast<int4*>(q + (size_t)n * hp * wp * cp + 16 * threadIdx.x) = make_int4(0, 0, 0, 0);
}

int qnn_quantize_nchw_to_nhwc8(const float* x, int8_t* q, int n, int c, int h, int w, int pad, int cp,
                               float neg_min, float scale, float qmax, qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && c > 0 && h > 0 && w > 0 && pad >= 0, "bad shape");
  QNN_REQUIRE(cp >= c && cp % 16 == 0, "cp must be a multiple of 16 and >= c");
  QNN_REQUIRE(scale > 0.f, "scale must be > 0");
  QNN_REQUIRE(q && (n == 0 || x), "null pointer");
  QNN_REQUIRE((((uintptr_t)q) & 15) == 0, "q must be 16-byte aligned");
  int64_t work = (int64_t)n * (h + 2 * pad) * (w + 2 * pad) * (cp / 16);
  if (w % 4 == 0 && (((uintptr_t)x) & 15) == 0 && work < (1LL << 31) && (int64_t)n * c * h * w < (1LL << 31)) {
    const int64_t t4 = (int64_t)n * h * (w / 4) * (cp / 16) + (int64_t)n * ((h + 2 * pad) * (w + 2 * pad) - h * w) * (cp / 16);
    hipLaunchKernelGGL(quantize_nchw_nhwc8_q4_kernel, dim3(grid_for(t4 > 0 ? t4 : 1, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, q, n, c, h, w, pad, cp, neg_min, scale, qmax);
    QNN_LAUNCH_CHECK("qnn_quantize_nchw_to_nhwc8");
    return QNN_OK;
  }
  hipLaunchKernelGGL(quantize_nchw_nhwc8_kernel, dim3(grid_for(work > 0 ? work : 1, 256)), dim3(256), 0,
                     (hipStream_t)stream, x, q, n, c, h, w, pad, cp, neg_min, scale, qmax);
  QNN_LAUNCH_CHECK("qnn_quantize_nchw_to_nhwc8");
  return QNN_OK;
}

int qnn_qconv2d_generic_fwd(const float* x, int n, int c, int h, int w, float neg_min, float xmin, float scale,
                            float qmax, const float* w_hat, int cout, int groups, int kh, int kw, int sh, int sw,
                            int pad_top, int pad_left, int dil_h, int dil_w, int ho, int wo, const float* bias,
                            float* y, qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && c > 0 && h > 0 && w > 0 && cout > 0 && groups > 0 && c % groups == 0 && cout % groups == 0 &&
                  kh > 0 && kw > 0 && sh > 0 && sw > 0 && pad_top >= 0 && pad_left >= 0 && dil_h > 0 && dil_w > 0 &&
                  ho > 0 && wo > 0,
              "bad shape");
  QNN_REQUIRE(scale > 0.f, "scale must be > 0");
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(x && w_hat && y, "null pointer");
  const int64_t total = (int64_t)n * cout * ho * wo;
  hipLaunchKernelGGL(qconv_generic_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, x, n, c, h,
                     w, neg_min, xmin, scale, qmax, w_hat, cout, groups, kh, kw, sh, sw, pad_top, pad_left, dil_h,
                     dil_w, ho, wo, bias, y);
  QNN_LAUNCH_CHECK("qnn_qconv2d_generic_fwd");
  return QNN_OK;
}

int qnn_quantize_nchw_to_s2d8(const float* x, int8_t* z, int n, int c, int h, int w, int pad, int hz, int wz,
                              float neg_min, float scale, float qmax, qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && c > 0 && 4 * c <= 16 && h > 0 && w > 0 && pad >= 0 && hz > 0 && wz > 0, "bad shape");
  QNN_REQUIRE(scale > 0.f, "scale must be > 0");
  QNN_REQUIRE(z && (n == 0 || x), "null pointer");
  QNN_REQUIRE((((uintptr_t)z) & 15) == 0, "z must be 16-byte aligned");
  const int64_t total = (int64_t)n * hz * wz;
  if (w % 4 == 0 && (((uintptr_t)x) & 15) == 0) {
    const int64_t pairs = (int64_t)n * hz * ((wz + 1) / 2);
    const dim3 grid(grid_for(pairs > 0 ? pairs : 1, 256));
    const int64_t rows = (int64_t)n * hz;
    const bool by_rows = (wz + 1) / 2 <= 64 && rows < ((int64_t)1 << 30);
    const dim3 grid_rows((unsigned)(rows > 0 ? (rows + 3) / 4 : 1));
    auto go = [&](auto offc) {
      constexpr int O = decltype(offc)::value;
      if (by_rows) {
        switch (c) {
          case 1: hipLaunchKernelGGL((quantize_s2d_rows_kernel<O, 1>), grid_rows, dim3(256), 0, (hipStream_t)stream, x, z, n, h, w, pad, hz, wz, neg_min, scale, qmax); break;
          case 2: hipLaunchKernelGGL((quantize_s2d_rows_kernel<O, 2>), grid_rows, dim3(256), 0, (hipStream_t)stream, x, z, n, h, w, pad, hz, wz, neg_min, scale, qmax); break;
          case 3: hipLaunchKernelGGL((quantize_s2d_rows_kernel<O, 3>), grid_rows, dim3(256), 0, (hipStream_t)stream, x, z, n, h, w, pad, hz, wz, neg_min, scale, qmax); break;
          default: hipLaunchKernelGGL((quantize_s2d_rows_kernel<O, 4>), grid_rows, dim3(256), 0, (hipStream_t)stream, x, z, n, h, w, pad, hz, wz, neg_min, scale, qmax); break;
        }
        return;
      }
      switch (c) {
        case 1: hipLaunchKernelGGL((quantize_s2d_x2_kernel<O, 1>), grid, dim3(256), 0, (hipStream_t)stream, x, z, n, h, w, pad, hz, wz, neg_min, scale, qmax); break;
        case 2: hipLaunchKernelGGL((quantize_s2d_x2_kernel<O, 2>), grid, dim3(256), 0, (hipStream_t)stream, x, z, n, h, w, pad, hz, wz, neg_min, scale, qmax); break;
        case 3: hipLaunchKernelGGL((quantize_s2d_x2_kernel<O, 3>), grid, dim3(256), 0, (hipStream_t)stream, x, z, n, h, w, pad, hz, wz, neg_min, scale, qmax); break;
        default: hipLaunchKernelGGL((quantize_s2d_x2_kernel<O, 4>), grid, dim3(256), 0, (hipStream_t)stream, x, z, n, h, w, pad, hz, wz, neg_min, scale, qmax); break;
      }
    };
    switch ((4 - (pad & 3)) & 3) {
      case 0: go(std::integral_constant<int, 0>{}); break;
      case 1: go(std::integral_constant<int, 1>{}); break;
      case 2: go(std::integral_constant<int, 2>{}); break;
      default: go(std::integral_constant<int, 3>{}); break;
    }
  } else {
    hipLaunchKernelGGL(quantize_s2d_kernel, dim3(grid_for(total > 0 ? total : 1, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, z, n, c, h, w, pad, hz, wz, neg_min, scale, qmax);
  }
  QNN_LAUNCH_CHECK("qnn_quantize_nchw_to_s2d8");
  return QNN_OK;
}

int qnn_pack_weight_i8(const float* w, int cout, int cin_g, int kh, int kw, int cin_pad, int cout_pad, int s2d,
                       float qmax, const float* w_min_in, const float* w_max_in, int8_t* wq, float* s_w, float* b_w,
                       float* tap_sum, float* w_hat, float* w_min_out, float* w_max_out, qnn_stream_t stream) {
  QNN_REQUIRE(cout > 0 && cin_g > 0 && kh > 0 && kw > 0, "bad shape");
  QNN_REQUIRE(s2d == 0 || s2d == 2, "s2d must be 0 or 2");
  QNN_REQUIRE(cin_pad >= (s2d ? 4 * cin_g : cin_g) && cout_pad >= cout, "padding smaller than shape");
  QNN_REQUIRE(w && wq && s_w && b_w, "null pointer");
  QNN_REQUIRE((w_min_in == nullptr) == (w_max_in == nullptr), "w_min_in/w_max_in must both be set or both null");
  const int64_t ptaps = s2d ? (int64_t)((kh + 1) / 2) * ((kw + 1) / 2) : (int64_t)kh * kw;
  const int kpad = (int)(cdiv(ptaps * cin_pad, 128) * 128);
  hipLaunchKernelGGL(pack_weight_kernel, dim3(cout_pad), dim3(256), 0, (hipStream_t)stream, w, cout, cin_g, kh, kw,
                     cin_pad, kpad, s2d, qmax, w_min_in, w_max_in, wq, s_w, b_w, tap_sum, w_hat, w_min_out, w_max_out);
  QNN_LAUNCH_CHECK("qnn_pack_weight_i8");
  return QNN_OK;
}

int qnn_conv_border_table(const float* tap_sum, int cout, int kh, int kw, const int* hrange, int nhc,
                          const int* wrange, int nwc, float b_x, float* table, qnn_stream_t stream) {
  QNN_REQUIRE(cout > 0 && kh > 0 && kw > 0 && nhc > 0 && nwc > 0, "bad shape");
  QNN_REQUIRE(tap_sum && hrange && wrange && table, "null pointer");
  int64_t work = (int64_t)nhc * nwc * cout;
  hipLaunchKernelGGL(border_table_kernel, dim3(grid_for(work, 256)), dim3(256), 0, (hipStream_t)stream, tap_sum, cout,
                     kh, kw, hrange, nhc, wrange, nwc, b_x, table);
  QNN_LAUNCH_CHECK("qnn_conv_border_table");
  return QNN_OK;
}

int qnn_rangebn_f32(const float* x, float* y, int n, int c, int hw, float neg_min, float min, float scale, float qmax,
                    const float* mean, const float* sq, const float* wq, const float* bq, const float* residual,
                    int relu, qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && c > 0 && hw > 0, "bad shape");
  QNN_REQUIRE(scale > 0.f, "scale must be > 0");
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(x && y && mean && sq && wq && bq, "null pointer");
  int64_t total = (int64_t)n * c * hw;
  if ((hw & 3) == 0) {
    QNN_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && (!residual || ((uintptr_t)residual & 15) == 0),
                "x/y/residual must be 16-byte aligned");
  }
  hipLaunchKernelGGL(rangebn_kernel, dim3(grid_for(cdiv(total, 4), 256)), dim3(256), 0, (hipStream_t)stream, x, y,
                     total, c, hw, neg_min, min, scale, qmax, mean, sq, wq, bq, residual, relu);
  QNN_LAUNCH_CHECK("qnn_rangebn_f32");
  return QNN_OK;
}

int qnn_dwconv2d_fwd(const float* x, int n, int c, int h, int w, const float* w_hat, int kh, int kw, int sh, int sw,
                     int ph, int pw, int ho, int wo, float neg_min, float min, float scale, float qmax,
                     const float* bias, float* y, qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && c > 0 && h > 0 && w > 0 && kh > 0 && kw > 0 && sh > 0 && sw > 0, "bad shape");
  QNN_REQUIRE(ho == (h + 2 * ph - kh) / sh + 1 && wo == (w + 2 * pw - kw) / sw + 1, "ho/wo inconsistent");
  QNN_REQUIRE(scale > 0.f, "scale must be > 0");
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(x && w_hat && y, "null pointer");
  int64_t total = (int64_t)n * c * ho * wo;
  hipLaunchKernelGGL(dwconv_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, x, n, c, h, w,
                     w_hat, kh, kw, sh, sw, ph, pw, ho, wo, neg_min, min, scale, qmax, bias, y);
  QNN_LAUNCH_CHECK("qnn_dwconv2d_fwd");
  return QNN_OK;
}

}  // extern "C"
