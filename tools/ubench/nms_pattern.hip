// Read rate of the NMS unit access patterns over a C3-sized heatmap batch (8 x 17 x 640 x 640 fp32, 222.8 MB),
// loads only (a max-reduction keeps them live), persistent waves walking units like nms_strips_kernel:
//   A: 16-row units of 64 lanes x 1 column (dword loads, 20 rows per unit: 16 + 2 halo rows each side), the
//      current kernel's pattern (60 output columns per unit);
//   B: 16-row units of 64 lanes x 4 columns (dwordx4 loads, 1 KB per row), 248 output columns per unit.
// usage (GPU box): hipcc -O3 --offload-arch=gfx950 tools/ubench/nms_pattern.hip -o /tmp/nmsp && /tmp/nmsp
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int B = 8, J = 17, H = 640, W = 640, SR = 16, P = 2;

template <int COLS, int PREFETCH>
__global__ __launch_bounds__(256) void k_units(const float* s, float* out) {
  const int lane = threadIdx.x & 63;
  constexpr int SC = 64 * COLS - (COLS == 1 ? 2 * P : 8);     // output columns per unit
  const int nsx = (W + SC - 1) / SC, nb = H / SR, units = nb * nsx, total = B * J * units;
  const int stride = gridDim.x * 4;
  float acc = 0.f;
  for (int u = blockIdx.x * 4 + (threadIdx.x >> 6); u < total; u += stride) {
    const int plane = u / units, rem = u - plane * units, band = rem / nsx, strip = rem - band * nsx;
    const float* pl = s + (size_t)plane * H * W;
    const int y0 = band * SR;
    if (COLS == 1) {
      const int x = min(max(strip * SC - P + lane, 0), W - 1);
      float r[SR + 2 * P];
#pragma unroll
      for (int i = 0; i < SR + 2 * P; ++i) r[i] = pl[(size_t)min(max(y0 - P + i, 0), H - 1) * W + x];
#pragma unroll
      for (int i = 0; i < SR + 2 * P; ++i) acc = fmaxf(acc, r[i]);
    } else {
      const int x = min(max(strip * SC - 4 + 4 * lane, 0), W - 4);
      float4 r[SR + 2 * P];
#pragma unroll
      for (int i = 0; i < SR + 2 * P; ++i)
        r[i] = *reinterpret_cast<const float4*>(pl + (size_t)min(max(y0 - P + i, 0), H - 1) * W + x);
#pragma unroll
      for (int i = 0; i < SR + 2 * P; ++i) acc = fmaxf(acc, fmaxf(fmaxf(r[i].x, r[i].y), fmaxf(r[i].z, r[i].w)));
    }
  }
  if (acc == 12345.f) out[0] = acc;
}

template <int COLS>
void run(const float* s, float* out, int wg_per_cu, int cus) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = wg_per_cu * cus;
  for (int i = 0; i < 5; ++i) k_units<COLS, 0><<<grid, 256>>>(s, out);
  (void)hipEventRecord(e0);
  const int reps = 50;
  for (int i = 0; i < reps; ++i) k_units<COLS, 0><<<grid, 256>>>(s, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / reps, bytes = (double)B * J * H * W * 4;
  printf("cols/lane %d, %d WG/CU: %7.2f us  %7.1f GB/s (of the 222.8 MB batch)\n", COLS, wg_per_cu, us, bytes / us / 1e3);
}

int main() {
  float *s, *out;
  const size_t n = (size_t)B * J * H * W;
  (void)hipMalloc(&s, n * 4);
  (void)hipMemset(s, 0, n * 4);
  (void)hipMalloc(&out, 64);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int wpc : {2, 4, 5, 8}) run<1>(s, out, wpc, cus);
  for (int wpc : {2, 3, 4, 5, 8}) run<4>(s, out, wpc, cus);
  return 0;
}
