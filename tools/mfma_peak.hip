// Microbenchmark: sustained int8 / bf16 MFMA rate on this MI355X (the roofline's "peak").
// Every wave runs a long chain of independent MFMAs on register operands (4 or 8
// accumulators, no memory traffic); 1 or 2 waves per SIMD; every CU busy.  Random
// operands (DVFS depends on data).  Prints achieved T(FL)OP/s and the in-kernel clock
// (s_memtime / s_memrealtime ratio, MI355X_MICROARCH.md 'DVFS give-back' item 6).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o tools/mfma_peak && ./tools/mfma_peak
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef short v8s __attribute__((ext_vector_type(8)));

template <int KIND>  // 0: i8 32x32x32, 1: i8 16x16x64, 2: bf16 32x32x16, 3: bf16 16x16x32
__global__ void mfma_loop(const int* __restrict__ seed, int iters, int* out, unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  v4i a = {seed[lane], seed[lane + 64], seed[lane + 128], seed[lane + 192]};
  v4i b = {seed[lane + 256], seed[lane + 320], seed[lane + 384], seed[lane + 448]};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  int res = 0;
  if constexpr (KIND == 0) {
    v16i c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) res ^= c0[r] ^ c1[r] ^ c2[r] ^ c3[r];
  } else if constexpr (KIND == 1) {
    v4i c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0}, c4 = {0}, c5 = {0}, c6 = {0}, c7 = {0};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, c3, 0, 0, 0);
      c4 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c4, 0, 0, 0);
      c5 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, c5, 0, 0, 0);
      c6 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, c6, 0, 0, 0);
      c7 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, c7, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) res ^= c0[r] ^ c1[r] ^ c2[r] ^ c3[r] ^ c4[r] ^ c5[r] ^ c6[r] ^ c7[r];
  } else if constexpr (KIND == 2) {
    v8s x = __builtin_bit_cast(v8s, a), y = __builtin_bit_cast(v8s, b);
    v16f c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(y, x, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(y, y, c3, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) res ^= __float_as_int(c0[r] + c1[r] + c2[r] + c3[r]);
  } else {
    v8s x = __builtin_bit_cast(v8s, a), y = __builtin_bit_cast(v8s, b);
    v4f c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0}, c4 = {0}, c5 = {0}, c6 = {0}, c7 = {0};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y, x, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y, y, c3, 0, 0, 0);
      c4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, c4, 0, 0, 0);
      c5 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y, x, c5, 0, 0, 0);
      c6 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c6, 0, 0, 0);
      c7 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y, y, c7, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) res ^= __float_as_int(c0[r] + c1[r] + c2[r] + c3[r] + c4[r] + c5[r] + c6[r] + c7[r]);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = res;  // keeps every MFMA live
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int KIND>
static void run(const char* name, double ops_per_mfma, int mfma_per_iter, int waves_per_simd, const int* seed, int* out,
                unsigned long long* clk) {
  const int cus = 256, threads = 256 * waves_per_simd, iters = 20000;
  const int blocks = cus;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {  // warm (clock settles) then measure
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop<KIND>, dim3(blocks), dim3(threads), 0, 0, seed, iters, out, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
  }
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[512];
  hipMemcpy(h, clk, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
  double ratio = 0;
  for (int i = 0; i < blocks; ++i) ratio += (double)h[2 * i] / (double)h[2 * i + 1];
  ratio /= blocks;  // shader cycles per 100 MHz tick
  const double mfma = (double)blocks * (threads / 64) * iters * mfma_per_iter;
  const double tops = mfma * ops_per_mfma / (ms * 1e-3) / 1e12;
  printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"tops\": %.1f, \"clock_ghz\": %.3f, "
         "\"cycles_per_mfma\": %.2f}\n",
         name, waves_per_simd, ms, tops, ratio * 0.1,
         (ms * 1e-3) * ratio * 1e8 / (mfma / blocks / 4));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  int* seed;
  int* out;
  unsigned long long* clk;
  hipMalloc(&seed, 512 * sizeof(int));
  hipMalloc(&out, 256 * 512 * sizeof(int));
  hipMalloc(&clk, 2 * 256 * sizeof(unsigned long long));
  int h[512];
  srand(7);
  for (int i = 0; i < 512; ++i) h[i] = rand() ^ (rand() << 16);
  hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
  for (int w = 1; w <= 2; ++w) {
    run<0>("i8_32x32x32", 2.0 * 32 * 32 * 32, 4, w, seed, out, clk);
    run<1>("i8_16x16x64", 2.0 * 16 * 16 * 64, 8, w, seed, out, clk);
    run<2>("bf16_32x32x16", 2.0 * 32 * 32 * 16, 4, w, seed, out, clk);
    run<3>("bf16_16x16x32", 2.0 * 16 * 16 * 32, 8, w, seed, out, clk);
  }
  return 0;
}
