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

#define QNN_ABI_VERSION 9

int qnn_abi_version(void);
const char* qnn_last_error(void);

/* Device-side error word of the current device: bit QNN_DEVERR_PB_SPIN is raised by a
 * persistent-band convolution wave (configurations 45-49, qnn_qconv2d_fwd_nchw_f32) that gave up
 * one of its bounded hand-off waits -- that launch's outputs are then unreliable.  Reads the word
 * into *flags (nullable) and clears it when clear != 0.  Synchronizes the device. */
enum { QNN_DEVERR_PB_SPIN = 1 };
int qnn_device_errors(uint32_t* flags, int clear);
/* Test hook: the iteration bound of those waits (limit >= 0; 0 gives every wait up at once, so a
 * test can force the error path); limit < 0 restores the default. */
int qnn_debug_set_spin_limit(int limit);

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

/* The gradient quantizer of training (quantize.py:123-139, UniformQuantizeGrad.backward):
 * UniformQuantize().apply(grad, num_bits, min, max, stochastic, inplace) binds
 * enforce_true_zero = True, so per element, in the reference's op order (:76-97):
 *   t = g / scale; t = t + zero_point; [t = t + noise]; t = rint(clamp(t, 0, qmax));
 *   out = (t - zero_point) * scale
 * with scale = max((max - min) / qmax, 1e-8) and zero_point = int(clamp(-min / scale, 0, qmax))
 * computed by the caller in double from the Python-float range, as the reference does.
 * noise (nullable = not stochastic): the uniform(-0.5, 0.5) draw, one per element. */
int qnn_grad_quant_f32(const float* g, const float* noise, float* out, int64_t n, float scale, float zero_point,
                       float qmax, qnn_stream_t stream);

/* UniformQuantize.forward with a tensor range per row (fp32 scale), as the
 * per-output-channel weight quantization of QConv2d/QLinear (quantize.py:332-334,
 * weight_min/max of shape (Cout,1,..)) and the generic `quantize(x, b, t_min, t_max)`:
 * row r of x ([rows][cols], contiguous) uses mins[r], maxs[r]; rows == 1 with
 * scalar (0-dim) tensors.  s = clamp(fl(fl(max-min)/qmax), 1e-8) (:71-73). */
int qnn_fake_quant_rows_f32(const float* x, float* y, int rows, int64_t cols, const float* mins,
                            const float* maxs, float qmax, qnn_stream_t stream);

/* Activation codes for the int8 path: NCHW fp32 -> spatially padded NHWC8
 * [n][h+2*pad][w+2*pad][cp] holding q - 128 (quantize.py:89-95 codes), with the
 * border and channel padding written as code' 0 — zero padding of x_hat adds
 * nothing to the exact decomposition — followed by a 128-byte
 * zero tail (the conv's zero page, at byte offset n*(h+2p)*(w+2p)*cp).  The buffer
 * must hold that many bytes + 128.  Range: QuantMeasure's (min, scale). */
int qnn_quantize_nchw_to_nhwc8(const float* x, int8_t* q, int n, int c, int h, int w, int pad, int cp,
                               float neg_min, float scale, float qmax, qnn_stream_t stream);

/* Same codes in space-to-depth form for stride-2 convs on few channels (the
 * 7x7/2 and 3x3/2 stems): z[n][h2][w2][(2u+v)*c + ci] = code(x[n][ci][2*h2+u-pad][2*w2+v-pad])
 * (code' 0 outside the image), 4*c <= 16 = cpz, z is [n][hz][wz][16] + 128-byte zero tail.
 * A kh x kw stride-2 conv becomes a ceil(kh/2) x ceil(kw/2) stride-1 conv on z. */
int qnn_quantize_nchw_to_s2d8(const float* x, int8_t* z, int n, int c, int h, int w, int pad, int hz, int wz,
                              float neg_min, float scale, float qmax, qnn_stream_t stream);

/* Per-output-channel weight quantization + pre-pack for the int8 contraction.
 * Replaces QConv2d.forward :317-334 / QLinear.forward :401-415 (per_channel=True):
 *   weight_min/max = w.flatten(1).min/max(-1)   (or the given ones when frozen: w_min_in/w_max_in non-null)
 *   s_w = clamp(fl(fl(max-min)/qmax), 1e-8);  q_w = rint(clamp(fl(fl(w + (-min)) / s_w), 0, qmax))
 * Packed rows (stride kpad = round_up(taps * cin_pad, 128) bytes, codes q_w - 128, zeros
 * in every padding position and in rows >= cout):
 *   s2d == 0: [cout_pad][kh][kw][cin_pad]
 *   s2d == 2: [cout_pad][ceil(kh/2)][ceil(kw/2)][cin_pad] with channel (2u+v)*cin_g + ci
 *             holding tap (2a+u, 2b+v) — the space-to-depth weights (cin_pad >= 4*cin_g).
 * Other outputs (device buffers):
 *   s_w [cout] fp32 scale;  b_w [cout] fp32 = 128*s_w + min (double-rounded once)
 *   tap_sum [cout][kh*kw] fp32 = sum_ci of the dequantized weights w_hat, ORIGINAL taps
 *   w_hat   [cout][cin_g*kh*kw] fp32 dequantized weights (nullable)
 *   w_min_out / w_max_out [cout] (nullable): the ranges used (the reference stores them in
 *   the weight_min/weight_max buffers). */
int qnn_pack_weight_i8(const float* w, int cout, int cin_g, int kh, int kw, int cin_pad, int cout_pad, int s2d,
                       float qmax, const float* w_min_in, const float* w_max_in, int8_t* wq, float* s_w,
                       float* b_w, float* tap_sum, float* w_hat, float* w_min_out, float* w_max_out,
                       qnn_stream_t stream);

/* Border-aware zero-point table of the exact int8 decomposition:
 *   table[hc][wc][c] = b_x * sum_{kh in hrange[hc], kw in wrange[wc]} tap_sum[c][kh][kw]
 * hrange/wrange are [lo, hi) tap ranges, 2 ints per class (host-computed from geometry). */
int qnn_conv_border_table(const float* tap_sum, int cout, int kh, int kw, const int* hrange, int nhc,
                          const int* wrange, int nwc, float b_x, float* table, qnn_stream_t stream);

/* ---------------------------------------------------------------- contraction */

/* Geometry of one int8 contraction over a spatially pre-padded NHWC8 input. */
typedef struct qnn_conv_desc {
  int n, hp, wp, cp;   /* input codes [n][hp][wp][cp], cp = 16 * 2^j, border = code' 0   */
  int zero_off;        /* byte offset from x of >= 16 zero bytes (reads past K land here)  */
  int cout, cout_pad;  /* output channels; packed weight rows (>= round_up(cout, 64|128))  */
  int kh, kw, sh, sw;  /* taps and strides in the padded input's coordinates               */
  int ho, wo;          /* output pixel (ho, wo) reads input rows ho*sh + r, cols wo*sw + s */
  int kpad;            /* packed weight row stride in bytes (multiple of 128)              */
  const int8_t* kmask; /* nullable: [kpad] 0/1 per K byte, 1 where the packed weights hold a
                          real (tap, channel); sum_valid(q'_x) then counts only those bytes.
                          Needed by space-to-depth stems (their 2x2-tap grid over-covers the
                          kernel); NULL = every byte counts (codes past K are 0).  kpad <= 1024 */
  int tile;            /* tile configuration: 0 = chosen by the library's cost model, k + 1 =
                          configuration k of qnn_conv_plan (callers that autotune pass their
                          measured best; the result is identical for every configuration) */
} qnn_conv_desc;

/* Epilogue of the contraction.  Always:
 *   y = sxsw[c]*acc + sxbw[c]*sum_valid(q'_x) + table[hcls[ho]*nwc + wcls[wo]][c] (+ bias[c])
 * (exact decomposition; table = b_x * border-aware sum of w_hat, from
 * qnn_conv_border_table over the ORIGINAL unpadded geometry).
 * mode 0 (drop-in): out_f32 = y as NCHW fp32 [n][cout][ho][wo] — QConv2d.forward's output.
 * mode 1 (fused model graph, resnet_quantized.py:52-68/:93-113, mobilenet_quantized.py:38-48):
 *   v = bn_mean ? RangeBN_eval(y) : y     (quantize.py:461-499, exact fp32 op order;
 *                                          out_bncode receives RangeBN's input code)
 *   v = residual ? fl(v + residual) : v   (fp32 [m][cout], NHWC or C-tile, see f32_tiled)
 *   v = relu ? max(v, 0) : v
 *   out_f32 = v (fp32 [m][cout], NHWC or C-tile);  out_code{0,1} = codes of v for a consumer
 *   conv with QuantMeasure range (neg_min, scale, qmax), written into that consumer's padded
 *   NHWC8 buffer [n][hp][wp][cp] at (ho + pad, wo + pad); channels [cout, cp) of every
 *   16-byte group the block covers are written as code' 0.  cout % 16 == 0, cp % 16 == 0.
 *
 * C-tile layout (f32_tiled != 0): the fp32 image of the MFMA 32x32 accumulators, so the
 * epilogue reads/writes it with one coalesced 1-KiB access per wave-instruction:
 *   index(m, c) = (((m/32)*CT + c/32)*4 + (c%32)/8)*256 + (m%32 + 32*((c/4)%2))*4 + c%4
 * with CT = ceil(cout/32); a map holds ceil(M/32)*32 * CT*32 floats.  Producer and
 * consumer of a residual agree on it (qnn_maxpool_bn, qnn_avgpool_quant take it too). */
/* One link of a residual code chain (qnn_epilogue.res): the RangeBN input codes a producer
 * wrote (its out_bncode, byte C-tile layout) and that RangeBN's eval parameters, so a
 * consumer recomputes the producer's fp32 value op for op:
 *   g(q) = fl(fl(fl(fl(q*scale) + min) - mean[c]) * sq[c]) * wq[c]) + bq[c]   (quantize.py:488-499)
 * Byte C-tile layout of a [m][cout] code map (the MFMA accumulator image, 1 byte per value):
 *   index(m, c) = (((m/32)*CT + c/32)*64 + m%32 + 32*((c/4)%2))*16 + 4*((c%32)/8) + c%4
 * so a wave reads / writes a 32x32 sub-tile as one coalesced 16-byte access per lane. */
typedef struct qnn_res_link {
  const uint8_t* code;
  const float* mean;
  const float* sq;
  const float* wq;
  const float* bq;
  float min, scale;
} qnn_res_link;
#define QNN_MAX_RES 4

typedef struct qnn_epilogue {
  int mode;
  const float* sxsw;
  const float* sxbw;
  const float* table;
  const int* hcls;
  const int* wcls;
  int nwc, nclass;
  const float* bias;
  const float* bn_mean;
  const float* bn_sq;
  const float* bn_wq;
  const float* bn_bq;
  float bn_neg_min, bn_min, bn_scale, bn_qmax;
  const float* residual;
  int relu;
  float* out_f32;
  uint8_t* out_bncode;
  int8_t* out_code0;
  int code0_cp, code0_pad, code0_hp, code0_wp;
  float code0_neg_min, code0_scale, code0_qmax;
  int8_t* out_code1;
  int code1_cp, code1_pad, code1_hp, code1_wp;
  float code1_neg_min, code1_scale, code1_qmax;
  const int8_t* lut;  /* nullable [cout][256]: out_code0 = lut[c][RangeBN input code] — the
                         whole RangeBN -> ReLU -> consumer-quantizer chain tabulated per
                         channel (qnn_bn_code_lut); needs bn, out_code0 only, no residual */
  int f32_tiled;      /* mode 1: residual and out_f32 in the C-tile layout (else NHWC)     */
  /* Residual as a code chain (mode 1, resnet_quantized.py:60-68 / :105-113): instead of
   * reading an fp32 block input, recompute it from 1-byte codes (res[], qnn_res_link):
   *   r = residual ? residual (fp32)                                   (links 0 .. nres-1)
   *                : (res_relu0 ? max(g_0(q_0), 0) : g_0(q_0))         (links 1 .. nres-1)
   *   r = max(g_l(q_l) + r, 0)   for each remaining link l            (a block's output)
   * the first form continues a chain from an fp32 checkpoint, the second starts it from a
   * downsample branch's RangeBN codes (res_relu0 = 0) or the stem max-pool's (= 1).  The
   * result is bitwise the fp32 map the producers would have stored.  0 <= nres <= 4. */
  int nres;
  int res_relu0;
  qnn_res_link res[QNN_MAX_RES];
  int bncode_tiled;   /* out_bncode in the byte C-tile layout (a chain link), else NHWC uint8 */
} qnn_epilogue;

/* Eval forward of QConv2d / QLinear (quantize.py:314-349, :398-428; biprecision's
 * out1 + out2 - out1 is bitwise one conv) on pre-quantized operands:
 * int8 MFMA implicit GEMM (v_mfma_i32_32x32x32_i8), exact int32 accumulation, fp32
 * epilogue as described by `epi`.  groups == 1 (depthwise: qnn_dwconv2d_fwd). */
int qnn_qconv2d_fwd(const int8_t* x, const int8_t* wq, const qnn_conv_desc* desc, const qnn_epilogue* epi,
                    qnn_stream_t stream);

/* The drop-in QConv2d forward from the module's own fp32 NCHW input (quantize.py:314-354: the
 * input quantizer, then the conv), one launch: the persistent-band kernel quantizes each input
 * band into LDS (x + neg_min over scale, round, clamp to [0, qmax]: bitwise the codes
 * qnn_quantize_nchw_to_nhwc8 writes) instead of reading a code tensor.  desc is the layer's
 * descriptor for that code tensor (hp = h + 2 pad, wp = w + 2 pad, cp >= c); epi mode 0 (fp32
 * NCHW out).  tile: 0 = the cheapest persistent-band configuration that fits, k + 1 =
 * configuration k.  Returns QNN_ERR_UNSUPPORTED when none fits (3x3 on 64 or 128 padded input
 * channels, stride 1 or 2): the caller quantizes and calls qnn_qconv2d_fwd instead. */
int qnn_qconv2d_fwd_nchw_f32(const float* x, int c, int h, int w, int pad, float neg_min, float scale, float qmax,
                             const int8_t* wq, const qnn_conv_desc* desc, const qnn_epilogue* epi, int tile,
                             qnn_stream_t stream);

/* Tile plan qnn_qconv2d_fwd would use for this layer (introspection for benchmarks and
 * profiles; no GPU work): configuration id, block tile (cout x pixels), and the number of
 * block tiles (the persistent direct-fragment grid loops over them: qnn_conv_occupancy.grid
 * is the launched grid).  Any out pointer may be NULL. */
int qnn_conv_plan(const qnn_conv_desc* desc, const qnn_epilogue* epi, int* cfg, int* bm, int* bn, int* nblk);

/* Launch resources of the configuration qnn_qconv2d_fwd would use (resident-band and
 * direct-fragment configurations, ids >= 26): co-resident blocks per CU at its dynamic LDS
 * (registers and LDS, hipOccupancyMaxActiveBlocksPerMultiprocessor), LDS bytes per block,
 * and the launched grid.  No GPU work.  Any out pointer may be NULL. */
int qnn_conv_occupancy(const qnn_conv_desc* desc, const qnn_epilogue* epi, int* cfg, int* blocks_per_cu,
                       int* lds_bytes, int* grid);

/* Number of tile configurations (valid qnn_conv_desc.tile values are 1 .. count).  Those with
 * ids 12-25 are the halo-band kernels for kh x kw > 1: the block's input rows are read into
 * LDS once per K chunk and every tap reads them at a shifted LDS address (no im2col
 * re-reads from L2); ids 26-30 the resident-band kernels (whole output rows per block, the
 * band of ALL input channels loaded once, weights streamed straight into registers, no
 * barrier in the K loop; kh x kw > 1, cp % 64 == 0; id 30 runs two blocks per CU); ids 31-33
 * the direct-fragment kernels for
 * short reductions (kpad <= 256: the space-to-depth stems, narrow 1x1s; every B fragment one
 * 16-byte load of one tap of one input pixel, persistent blocks).  An explicit tile that is
 * not built for the layer / epilogue kind is an argument error. */
int qnn_conv_tile_count(void);

/* The kernel family of tile configuration `cfg` (0-based, as qnn_conv_plan reports it): the
 * device function's name -- "qconv_kernel" (LDS-DMA ring), "qconv_pp_kernel" (ping-pong),
 * "qconv_band_kernel", "qconv16_kernel", "qconv_rb_kernel" (resident band) or
 * "qconv_direct_kernel" -- as rocprof's kernel trace names its dispatches; NULL when out of
 * range.  No GPU work. */
const char* qnn_conv_tile_kernel(int cfg);

/* Depthwise (groups == cin == cout) eval forward: fake-quantize-on-load of x
 * (QuantMeasure range) times the dequantized weights w_hat [c][kh*kw] plus the
 * fake-quantized bias, fp32.  NCHW in, NCHW out. */
int qnn_dwconv2d_fwd(const float* x, int n, int c, int h, int w, const float* w_hat, int kh, int kw,
                     int sh, int sw, int ph, int pw, int ho, int wo, float neg_min, float min, float scale,
                     float qmax, const float* bias, float* y, qnn_stream_t stream);

/* ---------------------------------------------------------------- RCCL gather (§8(e)) */

/* The one collective of the data-parallel eval forward: every rank's [B/W, classes] fp32
 * logits gathered to the root over RCCL (xGMI), replacing nn.DataParallel's gather
 * (reference main.py:345 scatters the batch and gathers the outputs every forward).  One
 * process per GPU; the communicator is the library's only global mutable state.
 *   qnn_comm_unique_id: on one rank, an opaque id (QNN_COMM_ID_BYTES) to share with the others
 *                       (any out-of-band channel: torch.distributed broadcast, a file, MPI);
 *   qnn_comm_init:      on every rank, with the same id (ncclCommInitRank; blocks until all join);
 *   qnn_gather_f32:     recv[r * count .. ] = rank r's send[0 .. count) on the root (recv is
 *                       ignored elsewhere), enqueued on `stream`;
 *   qnn_comm_destroy:   collective teardown. */
#define QNN_COMM_ID_BYTES 128
int qnn_comm_unique_id(void* id, size_t bytes);
int qnn_comm_init(int rank, int world, const void* unique_id);
int qnn_gather_f32(const float* send, float* recv, size_t count, int root, qnn_stream_t stream);
int qnn_comm_destroy(void);

/* ---------------------------------------------------------------- calibration (§8(f2)) */

/* QuantMeasure's train-branch statistics (models/modules/quantize.py:225-236) of x viewed
 * as [rows][row_len] (rows = batch, input_.view(input_.size(0), -1)):
 *   out[0] = mean over rows of min(row)      (:226-227)
 *   out[1] = mean over rows of max(row)      (:229-230)
 *   out[2] = mean(x), out[3] = std(x, unbiased)   (:232-233)
 * Deterministic fixed-order reductions accumulated in fp64 (the reference reduces in fp32
 * torch order; agreement ~1e-6 relative).  The caller applies the momentum updates
 * (:216-219) and the aciq range (:238-239).  work: qnn_measure_stats_work(rows) doubles of
 * device scratch.  Replaces the torch reductions of QuantMeasure.forward in training mode. */
int64_t qnn_measure_stats_work(int64_t rows);
int qnn_measure_stats_f32(const float* x, int64_t rows, int64_t row_len, double* work, float* out,
                          qnn_stream_t stream);

/* RangeBN's train-branch statistics (quantize.py:466-472) of x [b][c][hw] (NCHW): per
 * channel c, over the sequence q = bi*hw + p (x.transpose(0, 1) flattened) split into
 * num_chunks equal chunks:
 *   mean_max[c] = mean_k max(chunk k)   mean_min[c] = mean_k min(chunk k)   mean[c] = mean(q)
 * b*hw % num_chunks == 0 (the reference's view).  The caller forms scale (:473-476) and the
 * momentum updates (:478-482).  work: 3 * c * num_chunks doubles. */
int qnn_rangebn_stats_f32(const float* x, int b, int c, int hw, int num_chunks, double* work, float* mean_max,
                          float* mean_min, float* mean, qnn_stream_t stream);

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

/* ---------------------------------------------------------------- fused model graph */

/* RangeBN eval parameters (quantize.py:461-499) for the fused kernels below. */
typedef struct qnn_bn_params {
  const float* mean;  /* running_mean [c]                        */
  const float* sq;    /* fake-quantized running_var [c]          */
  const float* wq;    /* fake-quantized weight [c]               */
  const float* bq;    /* fake-quantized bias [c]                 */
  float neg_min, min, scale, qmax;  /* RangeBN.quantize_input range */
} qnn_bn_params;

/* Where and how to write requantized codes for a consumer conv: its QuantMeasure range
 * and its padded NHWC8 input buffer [n][hp][wp][cp] (value at (h + pad, w + pad)). */
typedef struct qnn_code_out {
  int8_t* ptr;
  int cp, pad, hp, wp;
  float neg_min, scale, qmax;
} qnn_code_out;

/* Per-channel code -> code table of the chain RangeBN eval -> [ReLU] -> consumer quantizer
 * (quantize.py:461-499 then :89-95), evaluated with the same device arithmetic as the
 * fused epilogue: lut[c][q] = code'(relu(f_c(q)); next range) for q in 0..255.
 * It makes the chain exact AND division-free in the conv epilogue. */
int qnn_bn_code_lut(const qnn_bn_params* bn, int c, int relu, const qnn_code_out* next, int8_t* lut,
                    qnn_stream_t stream);

/* ResNet stem max-pool (nn.MaxPool2d(k, stride, pad), resnet_quantized.py:174) fused with
 * the ReLU and RangeBN before it (:140-143), on RangeBN's input codes q [n][h][w][c]
 * (uint8, the stem conv's out_bncode).  g_c = [relu o] RangeBN_eval is monotone in the
 * code (non-increasing where sq*wq < 0), so max over the window of g_c(q_i) = g_c(max q_i)
 * (min where decreasing); padding positions are skipped (-inf).  Outputs: out_f32 =
 * g_c(q*) (fp32 [m][c], NHWC or C-tile by f32_tiled; nullable), out_code = q* itself (the
 * byte C-tile layout of qnn_res_link: a residual chain start with res_relu0 = relu;
 * nullable) and codes lut{0,1}[c][q*] (qnn_bn_code_lut) into consumer buffers code{0,1}
 * (nullable).  c % 16 == 0. */
int qnn_maxpool_bn(const uint8_t* q, int n, int h, int w, int c, int k, int stride, int pad, int ho, int wo,
                   const qnn_bn_params* bn, int relu, float* out_f32, int f32_tiled, uint8_t* out_code,
                   const int8_t* lut0, const qnn_code_out* code0, const int8_t* lut1, const qnn_code_out* code1,
                   qnn_stream_t stream);

/* The ResNet stem (resnet_quantized.py:171-174, :140-143) in one launch: the contraction of
 * qnn_qconv2d_fwd (a short reduction, kpad <= 256, 64 output channels: the space-to-depth 7x7/2
 * stem) with its RangeBN's input codes (mode 1, bn_* of epi, as out_bncode would receive them),
 * then nn.MaxPool2d(3, 2, 1) of ReLU o RangeBN on those codes and the outputs of
 * qnn_maxpool_bn: out_code (pooled codes, byte C-tile; nullable) and codes lut{0,1}[c][q*] into
 * consumer buffers code{0,1} (nullable).  Bitwise qnn_qconv2d_fwd (out_bncode) followed by
 * qnn_maxpool_bn, without the full-resolution codes ever reaching memory.  pool_ho/pool_wo:
 * the pooled size ((ho - 1) / 2 + 1). */
int qnn_qconv2d_maxpool_fwd(const int8_t* x, const int8_t* wq, const qnn_conv_desc* desc, const qnn_epilogue* epi,
                            int pool_ho, int pool_wo, uint8_t* out_code, const int8_t* lut0,
                            const qnn_code_out* code0, const int8_t* lut1, const qnn_code_out* code1,
                            qnn_stream_t stream);

/* Depthwise QConv2d (groups == c, mobilenet_quantized.py:38-40) fused with its RangeBN and
 * ReLU (:41-42) on padded NHWC8 codes x [n][hp][wp][cp] whose image interior is
 * [pad, pad+h) x [pad, pad+w); taps outside it are skipped (zero padding of x_hat):
 *   y = sum_taps x_hat * w_hat + bias, x_hat = fl(fl((q'+128) * x_scale) + x_min)  (the
 *   reference's fake-quantized input values exactly), w_hat_t [kh*kw][c], bias = q(bias);
 *   v = bn ? RangeBN_eval(y) : y;  v = relu ? max(v, 0) : v
 * Outputs: out_f32 NHWC [n][ho][wo][c] (nullable), codes for one consumer (nullable). */
int qnn_dwconv_fused(const int8_t* x, int n, int h, int w, int pad, int hp, int wp, int cp, int c,
                     const float* w_hat_t, int kh, int kw, int sh, int sw, int ho, int wo, float x_min, float x_scale,
                     const float* bias, const qnn_bn_params* bn, int relu, float* out_f32,
                     const qnn_code_out* code0, qnn_stream_t stream);

/* The same operation always on the generic depthwise kernel (any kh x kw, stride, channel
 * count): the bitwise reference the tests hold qnn_dwconv_fused's 3x3 fast kernel to. */
int qnn_dwconv_fused_generic(const int8_t* x, int n, int h, int w, int pad, int hp, int wp, int cp, int c,
                             const float* w_hat_t, int kh, int kw, int sh, int sw, int ho, int wo, float x_min,
                             float x_scale, const float* bias, const qnn_bn_params* bn, int relu, float* out_f32,
                             const qnn_code_out* code0, qnn_stream_t stream);

/* qnn_dwconv_fused with RangeBN -> ReLU -> the consumer's quantizer looked up instead of
 * evaluated: lut = qnn_bn_code_lut(bn, c, relu, code0) ([c][256] over the RangeBN input code,
 * bitwise the evaluated chain), codes out only, 3x3 stride 1 or 2, c % 4 == 0 (and c % 128 == 0
 * above 128 channels), lut 16-byte aligned; anything else is an argument error (round 4: the
 * MobileNet engine's depthwise launches). */
int qnn_dwconv_fused_lut(const int8_t* x, int n, int h, int w, int pad, int hp, int wp, int cp, int c,
                         const float* w_hat_t, int kh, int kw, int sh, int sw, int ho, int wo, float x_min,
                         float x_scale, const float* bias, const qnn_bn_params* bn, const int8_t* lut,
                         const qnn_code_out* code0, qnn_stream_t stream);

/* nn.AvgPool2d(k) over the whole k x k map (resnet_quantized.py:153, mobilenet_quantized.py:157)
 * on fp32 x [n*hw][c] (NHWC, or the C-tile layout when x_tiled): mean = (sum in row-major
 * tap order) / hw; writes out_f32 [n][c]
 * (nullable) and the codes of the classifier's QuantMeasure into code0 (hp = wp = 1). */
int qnn_avgpool_quant(const float* x, int n, int hw, int c, int x_tiled, float* out_f32,
                      const qnn_code_out* code0, qnn_stream_t stream);

/* The drop-in QConv2d forward (quantize.py:314-349) for the shapes the int8 MFMA path does not
 * take -- dilation != 1, grouped convs other than depthwise, unequal or 'same' padding -- from the
 * module's fp32 NCHW input: F.conv2d(input_, qweight, qbias, stride, padding, dilation, groups) on
 * the fake-quantized input (quantized on the fly with the QuantMeasure range neg_min / xmin /
 * scale / qmax) and w_hat, the fake-quantized weight [cout][c / groups][kh][kw] (qnn_pack_weight_i8's
 * w_hat); products summed in fp64, rounded once, + bias (the quantized bias, nullable).  Zero
 * padding pad_top / pad_left before the first row / column (the bottom / right padding follows from
 * ho / wo).  A correctness path (one thread per output), not a tuned kernel. */
int qnn_qconv2d_generic_fwd(const float* x, int n, int c, int h, int w, float neg_min, float xmin, float scale,
                            float qmax, const float* w_hat, int cout, int groups, int kh, int kw, int sh, int sw,
                            int pad_top, int pad_left, int dil_h, int dil_w, int ho, int wo, const float* bias,
                            float* y, qnn_stream_t stream);

/* The residual-chain tail of a ResNet block's last conv as a launch of its own (the "split"
 * general epilogue; resnet_quantized.py:60-68 / :105-113 after the conv): bncode holds that
 * conv's RangeBN input codes [n*ho*wo][c] in the byte C-tile layout (qnn_qconv2d_fwd with
 * epi->out_bncode, bncode_tiled = 1 and no other output), and this evaluates what the fused
 * general epilogue computes from them -- RangeBN (epi->bn_*), + the block input (epi->residual
 * or the chain epi->res[0 .. nres-1], res_relu0), ReLU (epi->relu) -- into epi->out_f32 (C-tile
 * when f32_tiled, else NHWC) and the codes epi->out_code0 / out_code1 (code*_ fields), bitwise
 * the fused epilogue's outputs.  The conv-only fields of epi are ignored.  c % 16 == 0. */
int qnn_chain_epilogue(const uint8_t* bncode, int n, int ho, int wo, int c, const qnn_epilogue* epi,
                       qnn_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* QNN_H_ */
