/* qnn.h — C ABI of the MI355X (gfx950) int8 QConv2d / QLinear inference path.
 *
 * Drop-in boundary for the eval forward of `QConv2d` / `QLinear` of
 * amishacorns/quantized.pytorch (models/modules/quantize.py).  The reference is
 * pure Python with no FFI; each entry point below names the
 * reference code whose behaviour it replaces.  Conventions:
 *   - plain device pointers; the caller owns all memory (PyTorch tensors);
 *   - an explicit stream (`qnn_stream_t` is `hipStream_t`); every call is
 *     asynchronous on that stream, re-entrant per stream, and never allocates,
 *     synchronises or copies host<->device (hipGraph-capturable);
 *   - the return value is a status code; on failure `qnn_last_error()` returns a
 *     thread-local message;
 *   - activation codes are stored shifted to int8: q' = q - 128, q in [0, 255];
 *   - no global mutable state.
 * Layouts: "NCHW" fp32 is the reference's module-boundary layout; "NHWC8" is
 * int8 codes [N][H][W][Cp] with Cp = round_up(C, 16) (padding channels hold 0).
 */
#ifndef QNN_H_
#define QNN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* qnn_stream_t; /* == hipStream_t */

enum {
  QNN_OK = 0,
  QNN_ERR_ARG = 1,         /* invalid argument (shape, pointer, unsupported combination) */
  QNN_ERR_HIP = 2,         /* HIP runtime error (launch failure, ...) */
  QNN_ERR_UNSUPPORTED = 3  /* valid in the reference but not implemented here */
};

#define QNN_ABI_VERSION 1

int qnn_abi_version(void);
const char* qnn_last_error(void);

/* ---------------------------------------------------------------- quantizer */

/* UniformQuantize.forward with a host-side range (quantize.py:159-160 -> :42-103,
 * effective asymmetric branch :89-100).  Replaces `quantize(x, b, float(min), float(max))`
 * as called by QuantMeasure.forward eval (quantize.py:249).
 * y[i] = fl(fl(q*scale) + min), q = rint(clamp(fl(fl(x[i] + neg_min) / scale), 0, qmax)).
 * `scale` is the fp32 rounding of the reference's double-precision scale
 * max((max-min)/qmax, 1e-8) (quantize.py:71-75).  x and y may alias. */
int qnn_fake_quant_f32(const float* x, float* y, int64_t n, float neg_min, float min, float scale,
                       float qmax, qnn_stream_t stream);

/* UniformQuantize.forward on a small vector whose range is taken from the vector
 * itself, computed on device (no host sync):
 *   scale_mode 0: tensor range, fp32 scale  — `quantize(b, min_value=b.min(), max_value=b.max())`
 *                 (QConv2d/QLinear bias, quantize.py:328-340) and `quantize(b)` with
 *                 min/max None (RangeBN bias, :498 -> :45-55; identical for 1-D input);
 *   scale_mode 1: Python-float range, double scale — `quantize(v, b, float(v.min()), float(v.max()))`
 *                 (RangeBN scale/weight, :486-494).
 * n <= 65536.  Optionally writes the range used to range_out[0..1] (nullable). */
int qnn_fake_quant_vec_f32(const float* x, float* y, int n, float qmax, int scale_mode,
                           float* range_out, qnn_stream_t stream);

/* UniformQuantize.forward with a tensor range per row (fp32 scale), as the
 * per-output-channel weight quantization of QConv2d/QLinear (quantize.py:332-334,
 * weight_min/max of shape (Cout,1,..)) and the generic `quantize(x, b, t_min, t_max)`:
 * row r of x ([rows][cols], contiguous) uses mins[r], maxs[r]; rows == 1 with
 * scalar (0-dim) tensors.  s = clamp(fl(fl(max-min)/qmax), 1e-8) (:71-73). */
int qnn_fake_quant_rows_f32(const float* x, float* y, int rows, int64_t cols, const float* mins,
                            const float* maxs, float qmax, qnn_stream_t stream);

/* Activation codes for the int8 path: NCHW fp32 -> NHWC8 (q - 128), channel pad 0.
 * The per-tensor QuantMeasure range (quantize.py:241-249) is (min, scale). */
int qnn_quantize_nchw_to_nhwc8(const float* x, int8_t* q, int n, int c, int h, int w, int cp,
                               float neg_min, float scale, float qmax, qnn_stream_t stream);

/* Per-output-channel weight quantization + pre-pack for the int8 contraction.
 * Replaces QConv2d.forward :317-334 / QLinear.forward :401-415 (per_channel=True):
 *   weight_min/max = w.flatten(1).min/max(-1)   (or the given ones when frozen: w_min_in/w_max_in non-null)
 *   s_w = clamp(fl(fl(max-min)/qmax), 1e-8);  q_w = rint(clamp(fl(fl(w + (-min)) / s_w), 0, qmax))
 * Outputs (all device buffers):
 *   wq      [cout_pad][kh][kw][cin_pad] int8 codes q_w - 128 (zero in padding rows/channels)
 *   s_w     [cout]  fp32 scale;  b_w [cout] fp32 = 128*s_w + min (double-rounded once)
 *   tap_sum [cout][kh*kw] fp32 = sum_ci of the dequantized weights w_hat (fp64 accumulation)
 *   w_hat   [cout][cin_g*kh*kw] fp32 dequantized weights (nullable)
 *   w_min_out / w_max_out [cout] (nullable): the ranges used (the reference stores them in
 *   the weight_min/weight_max buffers). */
int qnn_pack_weight_i8(const float* w, int cout, int cin_g, int kh, int kw, int cin_pad, int cout_pad,
                       float qmax, const float* w_min_in, const float* w_max_in, int8_t* wq, float* s_w,
                       float* b_w, float* tap_sum, float* w_hat, float* w_min_out, float* w_max_out,
                       qnn_stream_t stream);

/* Border-aware zero-point table of the exact int8 decomposition:
 *   table[hc][wc][c] = b_x * sum_{kh in hrange[hc], kw in wrange[wc]} tap_sum[c][kh][kw]
 * hrange/wrange are [lo, hi) tap ranges, 2 ints per class (host-computed from geometry). */
int qnn_conv_border_table(const float* tap_sum, int cout, int kh, int kw, const int* hrange, int nhc,
                          const int* wrange, int nwc, float b_x, float* table, qnn_stream_t stream);

/* ---------------------------------------------------------------- contraction */

/* Eval forward of QConv2d (quantize.py:314-349; biprecision's out1+out2-out1 is
 * bitwise one conv) on pre-quantized operands, int8 MFMA
 * implicit GEMM (v_mfma_i32_32x32x32_i8), exact int32 accumulation, fp32 epilogue:
 *   y[n][c][p] = sxsw[c]*acc + sxbw[c]*sum_valid(q'_x) + table[hcls[ho]][wcls[wo]][c] + bias[c]
 * with sxsw = s_x*s_w, sxbw = s_x*b_w.  groups must be 1 (depthwise: qnn_dwconv2d_fwd).
 * x: NHWC8 [n][h][w][cp]; wq: from qnn_pack_weight_i8 (cin_pad == cp).
 * out_layout 0: y is NCHW fp32 [n][cout][ho][wo]; 1: y is NHWC fp32 [n][ho][wo][cout].
 * bias nullable (already fake-quantized, quantize.py:336-340). */
int qnn_qconv2d_fwd(const int8_t* x, int n, int h, int w, int cp, const int8_t* wq, int cout,
                    int cout_pad, int kh, int kw, int sh, int sw, int ph, int pw, int ho, int wo,
                    const float* sxsw, const float* sxbw, const float* table, const int* hcls,
                    const int* wcls, int nwc, const float* bias, float* y, int out_layout,
                    qnn_stream_t stream);

/* Depthwise (groups == cin == cout) eval forward: fake-quantize-on-load of x
 * (QuantMeasure range) times the dequantized weights w_hat [c][kh*kw] plus the
 * fake-quantized bias, fp32.  NCHW in, NCHW out. */
int qnn_dwconv2d_fwd(const float* x, int n, int c, int h, int w, const float* w_hat, int kh, int kw,
                     int sh, int sw, int ph, int pw, int ho, int wo, float neg_min, float min, float scale,
                     float qmax, const float* bias, float* y, qnn_stream_t stream);

/* ---------------------------------------------------------------- RangeBN */

/* RangeBN.forward eval for NCHW fp32 (quantize.py:461-505):
 *   x_hat = fake_quant(x; QuantMeasure range)            (:462)
 *   out   = fl(fl(fl(x_hat - mean[c]) * sq[c]) * wq[c]) + bq[c]   (:488-499)
 * sq/wq/bq are the fake-quantized running_var / weight / bias (qnn_fake_quant_vec_f32).
 * Optional fusions of the model graph that follows (resnet_quantized.py:52-68):
 *   residual (nullable): out = fl(out + residual);  relu != 0: out = max(out, 0). */
int qnn_rangebn_f32(const float* x, float* y, int n, int c, int hw, float neg_min, float min, float scale,
                    float qmax, const float* mean, const float* sq, const float* wq, const float* bq,
                    const float* residual, int relu, qnn_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* QNN_H_ */
