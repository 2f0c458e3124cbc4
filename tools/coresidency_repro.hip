// Standalone reproducer for the round-3 co-residency corruption: does a packed-FP32
// VALU op (v_pk_fma_f32) in one workgroup return a wrong element while ANOTHER workgroup's MFMA
// loop runs on the same SIMD -- with nothing else of the conv kernels involved?
//
// Two kinds of 256-thread workgroups share every CU (64 KiB of LDS each caps a CU at two):
//   MFMA blocks  -- a long v_mfma_i32_16x16x64_i8 loop on register accumulators (12 independent
//                   chains, the resident-band kernel's issue pattern), result to a sink;
//   packed blocks -- v_pk_fma_f32 with the operand forms the failing epilogue used (src1 broadcast,
//                   op_sel_hi:[1,0,1]; and the plain form), each checked against the same fma done
//                   as two v_fma_f32 on the same inputs, mismatches counted per lane group.
// Even block ids are MFMA, odd packed; the grid is 2 x 256 x ROUNDS blocks.
//
//   hipcc --offload-arch=gfx950 -O3 tools/coresidency_repro.hip -o tools/coresidency_repro
//   ./tools/coresidency_repro [launches]
// prints the mismatch count per lane group (0-15, 16-31, 32-47, 48-63) and exits 1 if any.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int ITERS = 4096;  // loop trips per block (a few tens of us per launch)
constexpr int ROUNDS = 4;

__global__ __launch_bounds__(256) void mixed(unsigned long long* err, int* sink, const float* in, int seed) {
  extern __shared__ int lds[];  // 64 KiB: two blocks per CU
  const int lane = threadIdx.x & 63;
  if (blockIdx.x % 2 == 0) {
    // ---- MFMA block
    v4i a = {seed + lane, 3 * lane + 1, 5, 7 - lane};
    v4i b = {lane, 11, seed ^ lane, 13};
    v4i acc[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) acc[i] = (v4i){i, 0, 0, 0};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int i = 0; i < 12; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
      a.x += 1;
    }
    int s = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) s ^= acc[i][0] ^ acc[i][1] ^ acc[i][2] ^ acc[i][3];
    lds[threadIdx.x] = s;
    __syncthreads();
    sink[blockIdx.x * 256 + threadIdx.x] = lds[255 - threadIdx.x];
    return;
  }
  // ---- packed-FP32 block
  const int t = (blockIdx.x * 256 + threadIdx.x) & 4095;
  f2 x = {in[t], in[(t + 1) & 4095]};
  f2 y = {in[(t + 7) & 4095], in[(t + 9) & 4095]};
  float z = in[(t + 13) & 4095];
  unsigned long long bad = 0;
  for (int it = 0; it < ITERS; ++it) {
    f2 p, q;
    // the failing epilogue's form: src1 a single register broadcast to both halves
    const f2 zz = {z, -z};  // src1 a pair whose HIGH register is never read (op_sel_hi 0 for src1)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(p) : "v"(x), "v"(zz), "v"(y));
    // the plain form
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(q) : "v"(x), "v"(y), "v"(x));
    float p0, p1, q0, q1;
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(p0) : "v"(x.x), "v"(z), "v"(y.x));
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(p1) : "v"(x.y), "v"(z), "v"(y.y));
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(q0) : "v"(x.x), "v"(y.x), "v"(x.x));
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(q1) : "v"(x.y), "v"(y.y), "v"(x.y));
    const bool ok = __float_as_uint(p.x) == __float_as_uint(p0) && __float_as_uint(p.y) == __float_as_uint(p1) &&
                    __float_as_uint(q.x) == __float_as_uint(q0) && __float_as_uint(q.y) == __float_as_uint(q1);
    bad += ok ? 0 : 1;
    // next inputs (keeps the values bounded and changing)
    x.x = p0 * 0.5f + 0.25f;
    x.y = q1 * 0.5f - 0.25f;
    y.x = q0 * 0.125f;
    z = p1 * 0.0625f + 1.0f;
  }
  if (bad) atomicAdd(&err[lane >> 4], bad);
  lds[threadIdx.x] = (int)bad;
}

int main(int argc, char** argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 200;
  const int grid = 2 * 256 * ROUNDS;
  unsigned long long* err;
  int* sink;
  float* in;
  if (hipMalloc(&err, 4 * sizeof(unsigned long long)) || hipMalloc(&sink, (size_t)grid * 256 * sizeof(int)) ||
      hipMalloc(&in, 4096 * sizeof(float)))
    return 2;
  std::vector<float> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = 0.5f + (float)((i * 2654435761u) % 1000) / 997.0f;
  hipMemcpy(in, h.data(), 4096 * sizeof(float), hipMemcpyHostToDevice);
  hipMemset(err, 0, 4 * sizeof(unsigned long long));
  hipFuncSetAttribute((const void*)mixed, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int l = 0; l < launches; ++l) hipLaunchKernelGGL(mixed, dim3(grid), dim3(256), 64 * 1024, 0, err, sink, in, l);
  hipEventRecord(e1);
  if (hipEventSynchronize(e1) != hipSuccess) return 3;
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long he[4];
  hipMemcpy(he, err, sizeof(he), hipMemcpyDeviceToHost);
  const double checks = (double)launches * (grid / 2) * 256 * ITERS;
  printf("{\"launches\": %d, \"packed_checks\": %.3e, \"ms_per_launch\": %.3f, "
         "\"mismatches_by_lane_group\": [%llu, %llu, %llu, %llu]}\n",
         launches, checks, ms / launches, he[0], he[1], he[2], he[3]);
  return (he[0] | he[1] | he[2] | he[3]) ? 1 : 0;
}
