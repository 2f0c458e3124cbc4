// Calibration statistics: the measure-mode reductions main.py:154-205
// runs over calibration batches, on the device.
//   qnn_measure_stats_f32  QuantMeasure train branch (models/modules/quantize.py:225-236)
//   qnn_rangebn_stats_f32  RangeBN train branch (quantize.py:466-472)
// HBM-bound single passes (fp32 in, a few doubles out).  Every reduction has a fixed
// shape and order (grid and block sizes depend only on the tensor shape), accumulated in
// fp64, so results are deterministic run to run and within ~1e-6 relative of the
// reference's fp32 torch reductions (whose own order is unspecified).  The momentum
// updates of the running buffers stay in the caller (torch, op for op as :216-219, :478-482).
#include <float.h>

#include "qnn_internal.h"

namespace qnn {

constexpr int STAT_BLOCKS = 1024;  // moment partials of qnn_measure_stats_f32
constexpr int ST = 256;            // threads per block

template <class T, class Op>
__device__ __forceinline__ T block_reduce(T v, T* sh, Op op) {
  // fixed tree: wave shuffles then the 4 wave results in order
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  T r = sh[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = op(r, sh[w]);
  return r;
}

struct Min { __device__ float operator()(float a, float b) const { return fminf(a, b); } };
struct Max { __device__ float operator()(float a, float b) const { return fmaxf(a, b); } };
struct Add { __device__ double operator()(double a, double b) const { return a + b; } };

// one block per row: min and max of x[row, :]
__global__ __launch_bounds__(ST) void row_minmax_kernel(const float* __restrict__ x, int64_t row_len,
                                                        double* __restrict__ rmm) {
  __shared__ float sh[ST / 64];
  const float* r = x + (int64_t)blockIdx.x * row_len;
  float mn = FLT_MAX, mx = -FLT_MAX;
  for (int64_t i = threadIdx.x; i < row_len; i += ST) {
    const float v = r[i];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  mn = block_reduce(mn, sh, Min());
  mx = block_reduce(mx, sh, Max());
  if (threadIdx.x == 0) rmm[2 * blockIdx.x] = mn, rmm[2 * blockIdx.x + 1] = mx;
}

// block g: sum and sum of squares (fp64) of elements g*ST + t + k*STAT_BLOCKS*ST
__global__ __launch_bounds__(ST) void moments_kernel(const float* __restrict__ x, int64_t n, double* __restrict__ part) {
  __shared__ double sh[ST / 64];
  double s = 0.0, q = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * ST + threadIdx.x; i < n; i += (int64_t)STAT_BLOCKS * ST) {
    const double v = (double)x[i];
    s += v;
    q += v * v;
  }
  s = block_reduce(s, sh, Add());
  q = block_reduce(q, sh, Add());
  if (threadIdx.x == 0) part[2 * blockIdx.x] = s, part[2 * blockIdx.x + 1] = q;
}

__global__ void measure_final_kernel(const double* __restrict__ rmm, int64_t rows, const double* __restrict__ part,
                                     int64_t n, float* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double smin = 0.0, smax = 0.0;
  for (int64_t b = 0; b < rows; ++b) smin += rmm[2 * b], smax += rmm[2 * b + 1];
  double s = 0.0, q = 0.0;
  for (int g = 0; g < STAT_BLOCKS; ++g) s += part[2 * g], q += part[2 * g + 1];
  const double mean = s / (double)n;
  double var = n > 1 ? (q - s * mean) / (double)(n - 1) : NAN;  // torch: std of one element is nan
  if (var < 0.0) var = 0.0;
  out[0] = (float)(smin / (double)rows);
  out[1] = (float)(smax / (double)rows);
  out[2] = (float)mean;
  out[3] = (float)sqrt(var);
}

// block (k, c): max, min, sum of chunk k of channel c, the sequence s = b*hw + p
__global__ __launch_bounds__(ST) void rangebn_chunk_kernel(const float* __restrict__ x, int c, int hw, int64_t lc,
                                                           double* __restrict__ part) {
  __shared__ float shf[ST / 64];
  __shared__ double shd[ST / 64];
  const int k = blockIdx.x, ch = blockIdx.y;
  float mn = FLT_MAX, mx = -FLT_MAX;
  double s = 0.0;
  for (int64_t t = threadIdx.x; t < lc; t += ST) {
    const int64_t q = (int64_t)k * lc + t, b = q / hw, p = q - b * hw;
    const float v = x[(b * c + ch) * hw + p];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
    s += (double)v;
  }
  mn = block_reduce(mn, shf, Min());
  mx = block_reduce(mx, shf, Max());
  s = block_reduce(s, shd, Add());
  if (threadIdx.x == 0) {
    double* o = part + ((int64_t)ch * gridDim.x + k) * 3;
    o[0] = mx, o[1] = mn, o[2] = s;
  }
}

__global__ void rangebn_final_kernel(const double* __restrict__ part, int c, int nchunks, int64_t total,
                                     float* mean_max, float* mean_min, float* mean) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  double smx = 0.0, smn = 0.0, s = 0.0;
  for (int k = 0; k < nchunks; ++k) {
    const double* o = part + ((int64_t)ch * nchunks + k) * 3;
    smx += o[0], smn += o[1], s += o[2];
  }
  mean_max[ch] = (float)(smx / nchunks);
  mean_min[ch] = (float)(smn / nchunks);
  mean[ch] = (float)(s / (double)total);
}

}  // namespace qnn

using namespace qnn;

extern "C" {

int64_t qnn_measure_stats_work(int64_t rows) { return 2 * (int64_t)STAT_BLOCKS + 2 * (rows > 0 ? rows : 0); }

int qnn_measure_stats_f32(const float* x, int64_t rows, int64_t row_len, double* work, float* out,
                          qnn_stream_t stream) {
  QNN_REQUIRE(rows > 0 && row_len > 0 && rows < (1LL << 31), "need rows > 0, row_len > 0");
  QNN_REQUIRE(x && work && out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  double* part = work;
  double* rmm = work + 2 * STAT_BLOCKS;
  hipLaunchKernelGGL(row_minmax_kernel, dim3((unsigned)rows), dim3(ST), 0, s, x, row_len, rmm);
  QNN_LAUNCH_CHECK("qnn_measure_stats_f32");
  hipLaunchKernelGGL(moments_kernel, dim3(STAT_BLOCKS), dim3(ST), 0, s, x, rows * row_len, part);
  QNN_LAUNCH_CHECK("qnn_measure_stats_f32");
  hipLaunchKernelGGL(measure_final_kernel, dim3(1), dim3(64), 0, s, rmm, rows, part, rows * row_len, out);
  QNN_LAUNCH_CHECK("qnn_measure_stats_f32");
  return QNN_OK;
}

int qnn_rangebn_stats_f32(const float* x, int b, int c, int hw, int num_chunks, double* work, float* mean_max,
                          float* mean_min, float* mean, qnn_stream_t stream) {
  QNN_REQUIRE(b > 0 && c > 0 && hw > 0 && num_chunks > 0 && c < 65536, "bad shape");
  const int64_t total = (int64_t)b * hw;
  QNN_REQUIRE(total % num_chunks == 0, "b*h*w must be a multiple of num_chunks (quantize.py:469 view)");
  QNN_REQUIRE(x && work && mean_max && mean_min && mean, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(rangebn_chunk_kernel, dim3((unsigned)num_chunks, (unsigned)c), dim3(ST), 0, s, x, c, hw,
                     total / num_chunks, work);
  QNN_LAUNCH_CHECK("qnn_rangebn_stats_f32");
  hipLaunchKernelGGL(rangebn_final_kernel, dim3((unsigned)cdiv(c, 256)), dim3(256), 0, s, work, c, num_chunks, total,
                     mean_max, mean_min, mean);
  QNN_LAUNCH_CHECK("qnn_rangebn_stats_f32");
  return QNN_OK;
}

}  // extern "C"
