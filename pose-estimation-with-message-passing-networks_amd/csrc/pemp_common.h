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

}  // namespace pemp
