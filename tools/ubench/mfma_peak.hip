// Dense-MFMA calibration for the MFMA-utilisation figure (tools/mfma_util.py): every SIMD of the chip runs
// independent chains of v_mfma_f32_16x16x32_f16 back to back (8 accumulators per wave, no memory traffic in the
// loop), so SQ_VALU_MFMA_BUSY_CYCLES normalised by (kernel cycles x SIMDs) must read close to 1.0 here, and the
// event-timed rate is the chip's dense f16 MFMA rate at the clock it holds under this load.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/mfma_peak.hip -o build_ab/mfma_peak
// Run:   build_ab/mfma_peak [iters] [waves_per_simd]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mfma(int iters, float* out) {
  const int lane = threadIdx.x & 63;
  half8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (_Float16)(0.001f * (lane + i));
    b[i] = (_Float16)(0.002f * (lane - i));
  }
  float4v c[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = float4v{0.f, 0.f, 0.f, 0.f};
  // eight accumulate chains in one asm statement per iteration (the compiler's allocation of the builtin's chains
  // shuffled them through AGPR copies every iteration); the closing pad covers MFMA D -> compiler reader
  for (int it = 0; it < iters; ++it) {
    asm volatile(
        "v_mfma_f32_16x16x32_f16 %0, %8, %9, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %1, %8, %9, %1\n\t"
        "v_mfma_f32_16x16x32_f16 %2, %8, %9, %2\n\t"
        "v_mfma_f32_16x16x32_f16 %3, %8, %9, %3\n\t"
        "v_mfma_f32_16x16x32_f16 %4, %8, %9, %4\n\t"
        "v_mfma_f32_16x16x32_f16 %5, %8, %9, %5\n\t"
        "v_mfma_f32_16x16x32_f16 %6, %8, %9, %6\n\t"
        "v_mfma_f32_16x16x32_f16 %7, %8, %9, %7"
        : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7])
        : "v"(a), "v"(b));
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += c[k][0] + c[k][1] + c[k][2] + c[k][3];
  if (s == 1234.5f) out[0] = s;   // keeps the chains alive
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const int wps = argc > 2 ? atoi(argv[2]) : 1;   // waves per SIMD
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int wgs = cus * wps;                       // 4 waves (256 threads) per WG: one per SIMD
  float* out;
  (void)hipMalloc(&out, 64);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_mfma<<<wgs, 256>>>(iters / 10, out);
  (void)hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) k_mfma<<<wgs, 256>>>(iters, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2.0 * 16 * 16 * 32 * 8.0 * iters * (double)wgs * 4 * reps;
  printf("{\"cus\": %d, \"wgs\": %d, \"iters\": %d, \"ms_per_launch\": %.4f, \"tflops\": %.1f, \"mfma_per_simd\": %lld}\n",
         cus, wgs, iters, ms / reps, flop / (ms * 1e-3) / 1e12, (long long)8 * iters * wps);
  return 0;
}
