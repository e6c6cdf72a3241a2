// Shared device/host helpers for the gfx950 kernels of libpemp.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/pemp.h"

namespace pemp {

// Correctly rounded fp32 division (HIP's `/` is IEEE-correct by default and never contracted; ocml
// has no __fdiv_rn under OCML_BASIC_ROUNDED_OPERATIONS, see the Makefile)
__device__ __forceinline__ float div_rn(float a, float b) { return a / b; }


// ---- error reporting (thread-local last error, returned through pemp_last_error) ----
void set_error(const char* fmt, ...);

#define PEMP_CHECK_ARG(cond, ...)                \
  do {                                           \
    if (!(cond)) {                               \
      ::pemp::set_error(__VA_ARGS__);            \
      return PEMP_ERR_INVALID_ARG;               \
    }                                            \
  } while (0)

#define PEMP_HIP(call)                                                             \
  do {                                                                             \
    hipError_t e_ = (call);                                                        \
    if (e_ != hipSuccess) {                                                        \
      ::pemp::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),     \
                        __FILE__, __LINE__);                                        \
      return PEMP_ERR_HIP;                                                         \
    }                                                                              \
  } while (0)

// PEMP_DEBUG_SYNC=1 in the environment: synchronise after every launch and report the failing
// kernel by source line (fault localisation in one run; never on in measured runs).
bool debug_sync();

// true while the opt-in event profiler records (its hipEvent calls must not be graph-captured)
bool prof_active();
// launches a site should issue per event pair: R for a "label@R" profiler filter matching `label`
// (launch sites that are idempotent may repeat to amortise the event overhead), else 1
int prof_repeat(const char* label);

// host-side launch timing (diagnostics builds with -DPEMP_HOST_TRACE, run with PEMP_HOST_TRACE=1): a timestamp
// per launch check, printed by pemp_host_trace_dump(); compiled out of the product library
#ifdef PEMP_HOST_TRACE
void host_mark(int line);
extern bool g_host_trace;
#define PEMP_HOST_MARK() \
  do {                   \
    if (::pemp::g_host_trace) ::pemp::host_mark(__LINE__); \
  } while (0)
#else
#define PEMP_HOST_MARK() \
  do {                   \
  } while (0)
#endif

#define PEMP_LAUNCH_CHECK()                                                        \
  do {                                                                             \
    PEMP_HOST_MARK();                                                              \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ == hipSuccess && ::pemp::debug_sync()) e_ = hipDeviceSynchronize();     \
    if (e_ != hipSuccess) {                                                        \
      ::pemp::set_error("kernel failed: %s (%s:%d)", hipGetErrorString(e_),        \
                        __FILE__, __LINE__);                                        \
      fprintf(stderr, "[pemp] %s\n", ::pemp_last_error());                        \
      return PEMP_ERR_HIP;                                                         \
    }                                                                              \
  } while (0)

// RAII: records a hipEvent pair around a launch when the profiler is enabled for `label`.
class ProfScope {
 public:
  ProfScope(const char* label, hipStream_t st);
  ~ProfScope();

 private:
  hipStream_t st_;
  int slot_;
};

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// compute units of the current device (cached per process; 256 on MI355X)
static inline int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) return 256;
    return v;
  }();
  return n;
}

// Workspace carving: bump allocator over a caller-owned buffer (256-B aligned slices).
struct Carver {
  char* base;
  size_t used;
  explicit Carver(void* b) : base(static_cast<char*>(b)), used(0) {}
  template <typename T>
  T* take(size_t count) {
    used = align_up(used, 256);
    T* p = reinterpret_cast<T*>(base ? base + used : nullptr);
    used += count * sizeof(T);
    return p;
  }
};

// ---- device helpers ----
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  // v_mfma_f32_16x16x4_f32: exact f32 fma chain (k ordered), 16x16 tile, K = 4.
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Cross-lane sums without the LDS pipe (gfx950 v_permlane16_swap / v_permlane32_swap, DPP in-row moves). A
// __shfl_xor lowers to a ds_bpermute (an LDS round trip in the dependency chain); these stay in the VALU.
// permlane16_swap(x, x) leaves rows (0, 0, 2, 2) in one result and (1, 1, 3, 3) in the other, so their sum is
// x[lane] + x[lane ^ 16] in every lane; permlane32_swap likewise for lane ^ 32. Each sum is the same two operands as
// x + __shfl_xor(x, 16 / 32), so the results are bit-identical to the shuffle forms.
#ifndef PEMP_PERMLANE
#define PEMP_PERMLANE 1   // 0: the __shfl_xor forms (A/B builds)
#endif
__device__ __forceinline__ float xsum16(float v) {
  if (!PEMP_PERMLANE) return v + __shfl_xor(v, 16);
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}
__device__ __forceinline__ float xsum32(float v) {
  if (!PEMP_PERMLANE) return v + __shfl_xor(v, 32);
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}
// v summed over the lanes c, c + 16, c + 32, c + 48 (the four 16-lane rows), in every lane
__device__ __forceinline__ float xsum_rows(float v) { return xsum32(xsum16(v)); }
__device__ __forceinline__ float xmax_rows(float v) {
  if (!PEMP_PERMLANE) {
    v = fmaxf(v, __shfl_xor(v, 16));
    return fmaxf(v, __shfl_xor(v, 32));
  }
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// integer sum over all 64 lanes, in every lane: xor 1, xor 2 (quad_perm), half-row and row mirrors, then the row swaps
__device__ __forceinline__ int wave_sum_i32(int v) {
  if (!PEMP_PERMLANE) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
  }
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);   // row_half_mirror
  v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);   // row_mirror
  const auto a = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  v = (int)(a[0] + a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
  return (int)(b[0] + b[1]);
}

}  // namespace pemp
