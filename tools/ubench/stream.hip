// Per-CU streaming rate vs. bytes in flight: each WG reads `per_wg` bytes of a 43 MB-class
// working set that is re-read (L2/MALL resident) -- the node-step access shape.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int THREADS, int LOADS>
__global__ __launch_bounds__(THREADS) void k_stream(const float4* src, int64_t per_wg4, int64_t wrap4, float* out) {
  const float4* p = src + ((int64_t)blockIdx.x * per_wg4) % wrap4;
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < per_wg4; i += (int64_t)THREADS * LOADS) {
    float4 v[LOADS];
#pragma unroll
    for (int k = 0; k < LOADS; ++k) v[k] = p[min(i + (int64_t)THREADS * k, per_wg4 - 1)];
#pragma unroll
    for (int k = 0; k < LOADS; ++k) s += v[k].x + v[k].w;
  }
  if (s == 12345.f) out[0] = s;
}

template <int THREADS, int LOADS>
void run(const float4* src, int wgs, int64_t per_wg_bytes, int64_t wrap_bytes, float* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int i = 0; i < 10; ++i) k_stream<THREADS, LOADS><<<wgs, THREADS>>>(src, per_wg_bytes / 16, wrap_bytes / 16, out);
  (void)hipEventRecord(e0);
  const int reps = 100;
  for (int i = 0; i < reps; ++i) k_stream<THREADS, LOADS><<<wgs, THREADS>>>(src, per_wg_bytes / 16, wrap_bytes / 16, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const float us = ms * 1e3f / reps;
  printf("threads %4d loads %2d wgs %4d per_wg %6lld KB wrap %5lld MB: %7.2f us  %7.1f GB/s total\n", THREADS, LOADS, wgs,
         (long long)per_wg_bytes / 1024, (long long)wrap_bytes >> 20, us, (double)wgs * per_wg_bytes / us / 1e3);
}

int main() {
  float4* src;
  float* out;
  (void)hipMalloc(&src, 1ll << 30);
  (void)hipMemset(src, 0, 1ll << 30);
  (void)hipMalloc(&out, 64);
  const int64_t KB = 1024, MB = 1 << 20;
  // node-update shape: 308 WGs x 140 KB over a 5.6 MB set
  run<256, 8>(src, 308, 140 * KB, 6 * MB, out);
  run<256, 16>(src, 308, 140 * KB, 6 * MB, out);
  run<1024, 8>(src, 308, 140 * KB, 6 * MB, out);
  run<1024, 4>(src, 308, 140 * KB, 6 * MB, out);
  run<512, 8>(src, 616, 70 * KB, 6 * MB, out);
  run<256, 8>(src, 1232, 35 * KB, 6 * MB, out);
  run<1024, 8>(src, 1232, 35 * KB, 6 * MB, out);
  // streaming from HBM (1 GB set)
  run<256, 8>(src, 2048, 512 * KB, 1024 * MB, out);
  run<1024, 8>(src, 1024, 1024 * KB, 1024 * MB, out);
  // empty-ish
  run<256, 8>(src, 308, 1 * KB, 6 * MB, out);
  return 0;
}
