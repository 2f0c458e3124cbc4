// Fused model-graph kernels around the int8 contraction (HBM-bound, NHWC, coalesced
// along channels, 4 channels per thread): code-domain max-pool, fused depthwise conv,
// avg-pool head.  Reference semantics cited per entry in include/qnn.h.
#include <string.h>

#include "qnn_internal.h"

namespace qnn {

__device__ __forceinline__ float bn_apply(float q, const qnn_bn_params& b, int c) {
  float o = dequant(q, b.scale, b.min) - b.mean[c];  // (x - mean)      quantize.py:488
  o = o * b.sq[c];                                    // * q(scale)      :488-489
  o = o * b.wq[c];                                    // * q(weight)     :495
  return o + b.bq[c];                                 // + q(bias)       :499
}

__device__ __forceinline__ void put_code4(const qnn_code_out& o, int n, int h, int w, int c, const float v[4]) {
  int8_t* p = o.ptr + (((int64_t)n * o.hp + h + o.pad) * o.wp + w + o.pad) * o.cp + c;
  int r = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) r |= (((int)quant_code(v[u], o.neg_min, o.scale, o.qmax) - 128) & 255) << (8 * u);
  *reinterpret_cast<int*>(p) = r;
}

__device__ __forceinline__ void decode_pix(int64_t i, int cg, int wo, int ho, int& g, int& ox, int& oy, int& img) {
  g = (int)(i % cg);
  int64_t t = i / cg;
  ox = (int)(t % wo);
  t /= wo;
  oy = (int)(t % ho);
  img = (int)(t / ho);
}

// ------------------------------------------------------------------ max-pool on RangeBN codes
__device__ __forceinline__ void put_lut4(const qnn_code_out& o, const int8_t* __restrict__ lut, int n, int h, int w,
                                         int c, const int q[4]) {
  int8_t* p = o.ptr + (((int64_t)n * o.hp + h + o.pad) * o.wp + w + o.pad) * o.cp + c;
  int r = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) r |= ((int)(uint8_t)lut[(c + u) * 256 + q[u]]) << (8 * u);
  *reinterpret_cast<int*>(p) = r;
}

__global__ void maxpool_lut_kernel(const uint8_t* __restrict__ q, int n, int h, int w, int c, int k, int stride,
                                   int pad, int ho, int wo, const uint8_t* __restrict__ dir,
                                   const float* __restrict__ vlut, float* out_f32, const int8_t* __restrict__ lut0,
                                   qnn_code_out c0, const int8_t* __restrict__ lut1, qnn_code_out c1) {
  const int cg = c >> 2;
  const int64_t total = (int64_t)n * ho * wo * cg;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int g, ox, oy, img;
    decode_pix(i, cg, wo, ho, g, ox, oy, img);
    const int cbase = 4 * g;
    const uint32_t dmask = *reinterpret_cast<const uint32_t*>(dir + cbase);  // 1 byte per channel
    int hi4[4] = {-1, -1, -1, -1}, lo4[4] = {256, 256, 256, 256};
    for (int r = 0; r < k; ++r) {
      const int iy = oy * stride - pad + r;
      if (iy < 0 || iy >= h) continue;  // MaxPool2d pads with -inf
      for (int s = 0; s < k; ++s) {
        const int ix = ox * stride - pad + s;
        if (ix < 0 || ix >= w) continue;
        const uint32_t v = *reinterpret_cast<const uint32_t*>(q + (((int64_t)img * h + iy) * w + ix) * c + cbase);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int b = (v >> (8 * u)) & 255;
          hi4[u] = max(hi4[u], b);
          lo4[u] = min(lo4[u], b);
        }
      }
    }
    int qs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) qs[u] = ((dmask >> (8 * u)) & 255) ? lo4[u] : hi4[u];
    if (out_f32) {
      const float4 o = make_float4(vlut[(cbase + 0) * 256 + qs[0]], vlut[(cbase + 1) * 256 + qs[1]],
                                   vlut[(cbase + 2) * 256 + qs[2]], vlut[(cbase + 3) * 256 + qs[3]]);
      *reinterpret_cast<float4*>(out_f32 + (((int64_t)img * ho + oy) * wo + ox) * c + cbase) = o;
    }
    if (c0.ptr) put_lut4(c0, lut0, img, oy, ox, cbase, qs);
    if (c1.ptr) put_lut4(c1, lut1, img, oy, ox, cbase, qs);
  }
}

__global__ void bn_value_lut_kernel(qnn_bn_params bn, int c, int relu, float* vlut, uint8_t* dir) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c * 256) return;
  const int ch = i >> 8, qv = i & 255;
  float v = bn_apply((float)qv, bn, ch);
  vlut[i] = relu ? fmaxf(v, 0.f) : v;
  if (qv == 0) dir[ch] = (bn.sq[ch] * bn.wq[ch]) < 0.f ? 1 : 0;
}

// ------------------------------------------------------------------ depthwise, fused
// x: padded NHWC8 [n][hp][wp][cp], image interior at [pad, pad+h) x [pad, pad+w).
// Taps outside the image are skipped: zero padding applies to x_hat (quantize.py:343),
// and code' 0 there is NOT x_hat = 0 for a direct fp32 sum.
__global__ void dwconv_fused_kernel(const int8_t* __restrict__ x, int n, int h, int w, int pad, int hp, int wp,
                                    int cp, int c, const float* __restrict__ wt, int kh, int kw, int sh, int sw,
                                    int ho, int wo, float x_min, float x_scale, const float* bias, qnn_bn_params bn,
                                    int has_bn, int relu, float* out_f32, qnn_code_out c0) {
  const int cg = c >> 2;
  const int64_t total = (int64_t)n * ho * wo * cg;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int g, ox, oy, img;
    decode_pix(i, cg, wo, ho, g, ox, oy, img);
    const int cbase = 4 * g;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < kh; ++r) {
      const int py = oy * sh + r;  // padded-buffer row; image row py - pad
      if (py < pad || py >= pad + h) continue;
      for (int s = 0; s < kw; ++s) {
        const int px = ox * sw + s;
        if (px < pad || px >= pad + w) continue;
        const uint32_t v = *reinterpret_cast<const uint32_t*>(x + (((int64_t)img * hp + py) * wp + px) * cp + cbase);
        const float4 w4 = *reinterpret_cast<const float4*>(wt + (int64_t)(r * kw + s) * c + cbase);
        const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int code = (int)(int8_t)((v >> (8 * u)) & 255) + 128;
          acc[u] = fmaf(dequant((float)code, x_scale, x_min), wv[u], acc[u]);
        }
      }
    }
    float val[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ch = cbase + u;
      float y = bias ? acc[u] + bias[ch] : acc[u];
      if (has_bn) y = bn_apply(quant_code(y, bn.neg_min, bn.scale, bn.qmax), bn, ch);
      val[u] = relu ? fmaxf(y, 0.f) : y;
    }
    if (out_f32)
      *reinterpret_cast<float4*>(out_f32 + (((int64_t)img * ho + oy) * wo + ox) * c + cbase) =
          make_float4(val[0], val[1], val[2], val[3]);
    if (c0.ptr) put_code4(c0, img, oy, ox, cbase, val);
  }
}

// ------------------------------------------------------------------ RangeBN -> code LUT
__global__ void bn_code_lut_kernel(qnn_bn_params bn, int c, int relu, qnn_code_out nx, int8_t* lut) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c * 256) return;
  const int ch = i >> 8, q = i & 255;
  float v = bn_apply((float)q, bn, ch);
  if (relu) v = fmaxf(v, 0.f);
  lut[i] = (int8_t)((int)quant_code(v, nx.neg_min, nx.scale, nx.qmax) - 128);
}

// ------------------------------------------------------------------ avg-pool head
__global__ void avgpool_quant_kernel(const float* __restrict__ x, int n, int hw, int c, float* out_f32,
                                     qnn_code_out c0) {
  const int cg = c >> 2;
  const int64_t total = (int64_t)n * cg;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(i % cg);
    const int img = (int)(i / cg);
    const float* p = x + (int64_t)img * hw * c + 4 * g;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int t = 0; t < hw; ++t) {
      const float4 v = *reinterpret_cast<const float4*>(p + (int64_t)t * c);
      s.x = s.x + v.x; s.y = s.y + v.y; s.z = s.z + v.z; s.w = s.w + v.w;
    }
    const float d = (float)hw;
    const float val[4] = {s.x / d, s.y / d, s.z / d, s.w / d};
    if (out_f32)
      *reinterpret_cast<float4*>(out_f32 + (int64_t)img * c + 4 * g) = make_float4(val[0], val[1], val[2], val[3]);
    if (c0.ptr) put_code4(c0, img, 0, 0, 4 * g, val);
  }
}

static int grid_for(int64_t work) {
  int64_t g = cdiv(work, 256);
  if (g > 256 * 32) g = 256 * 32;
  return (int)(g < 1 ? 1 : g);
}

static qnn_code_out none_code() {
  qnn_code_out o;
  memset(&o, 0, sizeof(o));
  return o;
}

static int check_code(const qnn_code_out* o, int c, const char* what) {
  if (!o || !o->ptr) return QNN_OK;
  if (o->cp < c || o->cp % 4 || o->scale <= 0.f || o->pad < 0 || (((uintptr_t)o->ptr) & 3))
    return arg_error(what);
  return QNN_OK;
}

}  // namespace qnn

using namespace qnn;

extern "C" {

int qnn_bn_value_lut(const qnn_bn_params* bn, int c, int relu, float* vlut, uint8_t* dir, qnn_stream_t stream) {
  QNN_REQUIRE(c > 0 && bn && bn->mean && bn->sq && bn->wq && bn->bq && bn->scale > 0.f, "bad RangeBN params");
  QNN_REQUIRE(vlut && dir, "null output");
  hipLaunchKernelGGL(bn_value_lut_kernel, dim3((unsigned)cdiv((int64_t)c * 256, 256)), dim3(256), 0,
                     (hipStream_t)stream, *bn, c, relu, vlut, dir);
  QNN_LAUNCH_CHECK("qnn_bn_value_lut");
  return QNN_OK;
}

int qnn_maxpool_lut(const uint8_t* q, int n, int h, int w, int c, int k, int stride, int pad, int ho, int wo,
                    const uint8_t* dir, const float* vlut, float* out_f32, const int8_t* lut0,
                    const qnn_code_out* code0, const int8_t* lut1, const qnn_code_out* code1,
                    qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0 && k > 0 && stride > 0 && pad >= 0, "bad shape");
  QNN_REQUIRE(ho == (h + 2 * pad - k) / stride + 1 && wo == (w + 2 * pad - k) / stride + 1, "ho/wo inconsistent");
  QNN_REQUIRE(dir && (((uintptr_t)dir) & 3) == 0, "dir must be non-null and 4-byte aligned");
  QNN_REQUIRE(!out_f32 || vlut, "out_f32 needs vlut");
  QNN_REQUIRE(!(code0 && code0->ptr) || lut0, "code0 needs lut0");
  QNN_REQUIRE(!(code1 && code1->ptr) || lut1, "code1 needs lut1");
  if (int rc = check_code(code0, c, "bad code0")) return rc;
  if (int rc = check_code(code1, c, "bad code1")) return rc;
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(q, "null input");
  const qnn_code_out c0 = code0 ? *code0 : none_code(), c1 = code1 ? *code1 : none_code();
  hipLaunchKernelGGL(maxpool_lut_kernel, dim3(grid_for((int64_t)n * ho * wo * (c / 4))), dim3(256), 0,
                     (hipStream_t)stream, q, n, h, w, c, k, stride, pad, ho, wo, dir, vlut, out_f32, lut0, c0, lut1, c1);
  QNN_LAUNCH_CHECK("qnn_maxpool_lut");
  return QNN_OK;
}

int qnn_dwconv_fused(const int8_t* x, int n, int h, int w, int pad, int hp, int wp, int cp, int c,
                     const float* w_hat_t, int kh, int kw, int sh, int sw, int ho, int wo, float x_min, float x_scale,
                     const float* bias, const qnn_bn_params* bn, int relu, float* out_f32, const qnn_code_out* code0,
                     qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0 && cp >= c && cp % 4 == 0 && kh > 0 && kw > 0 &&
                  sh > 0 && sw > 0 && pad >= 0,
              "bad shape");
  QNN_REQUIRE(hp >= h + 2 * pad && wp >= w + 2 * pad, "padded buffer smaller than image");
  QNN_REQUIRE(ho == (h + 2 * pad - kh) / sh + 1 && wo == (w + 2 * pad - kw) / sw + 1, "ho/wo inconsistent");
  QNN_REQUIRE(x_scale > 0.f, "x_scale must be > 0");
  QNN_REQUIRE(!bn || (bn->mean && bn->sq && bn->wq && bn->bq && bn->scale > 0.f), "bad RangeBN params");
  QNN_REQUIRE(out_f32 || (code0 && code0->ptr), "no output");
  if (int rc = check_code(code0, c, "bad code0")) return rc;
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(x && w_hat_t, "null pointer");
  qnn_bn_params b;
  memset(&b, 0, sizeof(b));
  if (bn) b = *bn;
  const qnn_code_out c0 = code0 ? *code0 : none_code();
  hipLaunchKernelGGL(dwconv_fused_kernel, dim3(grid_for((int64_t)n * ho * wo * (c / 4))), dim3(256), 0,
                     (hipStream_t)stream, x, n, h, w, pad, hp, wp, cp, c, w_hat_t, kh, kw, sh, sw, ho, wo, x_min,
                     x_scale, bias, b, bn ? 1 : 0, relu, out_f32, c0);
  QNN_LAUNCH_CHECK("qnn_dwconv_fused");
  return QNN_OK;
}

int qnn_bn_code_lut(const qnn_bn_params* bn, int c, int relu, const qnn_code_out* next, int8_t* lut,
                    qnn_stream_t stream) {
  QNN_REQUIRE(c > 0 && bn && bn->mean && bn->sq && bn->wq && bn->bq && bn->scale > 0.f, "bad RangeBN params");
  QNN_REQUIRE(next && next->scale > 0.f && lut, "bad next range / null lut");
  hipLaunchKernelGGL(bn_code_lut_kernel, dim3((unsigned)cdiv((int64_t)c * 256, 256)), dim3(256), 0,
                     (hipStream_t)stream, *bn, c, relu, *next, lut);
  QNN_LAUNCH_CHECK("qnn_bn_code_lut");
  return QNN_OK;
}

int qnn_avgpool_quant(const float* x, int n, int hw, int c, float* out_f32, const qnn_code_out* code0,
                      qnn_stream_t stream) {
  QNN_REQUIRE(n >= 0 && hw > 0 && c > 0 && c % 4 == 0, "bad shape");
  QNN_REQUIRE(out_f32 || (code0 && code0->ptr), "no output");
  if (int rc = check_code(code0, c, "bad code0")) return rc;
  if (n == 0) return QNN_OK;
  QNN_REQUIRE(x, "null input");
  const qnn_code_out c0 = code0 ? *code0 : none_code();
  hipLaunchKernelGGL(avgpool_quant_kernel, dim3(grid_for((int64_t)n * (c / 4))), dim3(256), 0, (hipStream_t)stream, x,
                     n, hw, c, out_f32, c0);
  QNN_LAUNCH_CHECK("qnn_avgpool_quant");
  return QNN_OK;
}

}  // extern "C"
