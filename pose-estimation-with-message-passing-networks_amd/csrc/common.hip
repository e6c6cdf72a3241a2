// Library-level entry points: ABI version, thread-local error string, device check.
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "pemp_common.h"

namespace pemp {
static thread_local char g_err[512] = "";

bool debug_sync() {
  static const bool on = [] {
    const char* v = getenv("PEMP_DEBUG_SYNC");
    return v && v[0] && v[0] != '0';
  }();
  return on;
}

#ifdef PEMP_HOST_TRACE   // diagnostics build only (-DPEMP_HOST_TRACE, tools/host_trace.py)
bool g_host_trace = [] {
  const char* v = getenv("PEMP_HOST_TRACE");
  return v && v[0] && v[0] != '0';
}();
namespace {
std::mutex g_ht_mu;
std::vector<std::pair<int, long long>> g_ht;   // (source line of the launch check, steady-clock ns)
}
void host_mark(int line) {
  const long long t = std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
  std::lock_guard<std::mutex> lk(g_ht_mu);
  if (g_ht.size() < (1u << 20)) g_ht.emplace_back(line, t);
}
#endif

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ---- opt-in event profiler: hipEvents recorded on the launch stream around selected kernels ----
namespace {
struct Pending {
  std::string label;
  hipEvent_t a, b;
  int reps;
};
std::mutex g_prof_mu;
std::string g_prof_filter;
int g_prof_repeat = 1;     // "label@R": matching launch sites issue their launch R times per event pair
std::vector<Pending> g_pending;
std::vector<hipEvent_t> g_pool;
struct Agg {
  long count = 0;
  double ms = 0.0;
};
std::map<std::string, Agg> g_agg;

hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

ProfScope::ProfScope(const char* label, hipStream_t st) : st_(st), slot_(-1) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (g_prof_filter.empty()) return;
  if (g_prof_filter != "*" && std::string(label).find(g_prof_filter) == std::string::npos) return;
  Pending p{label, take_event(), take_event(), g_prof_repeat};
  if (!p.a || !p.b) return;
  (void)hipEventRecord(p.a, st);
  g_pending.push_back(p);
  slot_ = (int)g_pending.size() - 1;
}

ProfScope::~ProfScope() {
  if (slot_ < 0) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  (void)hipEventRecord(g_pending[slot_].b, st_);
}

int prof_repeat(const char* label) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (g_prof_filter.empty() || g_prof_repeat <= 1) return 1;
  if (g_prof_filter != "*" && std::string(label).find(g_prof_filter) == std::string::npos) return 1;
  return g_prof_repeat;
}

bool prof_active() {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  return !g_prof_filter.empty();
}

}  // namespace pemp

extern "C" int pemp_prof_enable(const char* filter) {
  std::lock_guard<std::mutex> lk(pemp::g_prof_mu);
  std::string f = filter ? filter : "";
  int reps = 1;
  const size_t at = f.find('@');
  if (at != std::string::npos) {
    reps = atoi(f.c_str() + at + 1);
    f = f.substr(0, at);
  }
  pemp::g_prof_filter = f;
  pemp::g_prof_repeat = reps > 1 ? reps : 1;
  return PEMP_OK;
}

extern "C" int pemp_prof_report(char* buf, size_t len) {
  std::lock_guard<std::mutex> lk(pemp::g_prof_mu);
  for (auto& p : pemp::g_pending) {
    float ms = 0.f;
    PEMP_HIP(hipEventSynchronize(p.b));
    PEMP_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    auto& a = pemp::g_agg[p.label];
    a.count += p.reps;
    a.ms += ms;
    pemp::g_pool.push_back(p.a);
    pemp::g_pool.push_back(p.b);
  }
  pemp::g_pending.clear();
  std::string out;
  char line[160];
  for (auto& kv : pemp::g_agg) {
    snprintf(line, sizeof(line), "%s %ld %.6f\n", kv.first.c_str(), kv.second.count, kv.second.ms);
    out += line;
  }
  pemp::g_agg.clear();
  if (buf && len) {
    strncpy(buf, out.c_str(), len - 1);
    buf[len - 1] = 0;
  }
  return (int)out.size();
}

extern "C" int pemp_abi_version(void) { return PEMP_ABI_VERSION; }

extern "C" const char* pemp_last_error(void) { return pemp::g_err; }

extern "C" int pemp_device_check(void) {
  int dev = 0;
  PEMP_HIP(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  PEMP_HIP(hipGetDeviceProperties(&prop, dev));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    pemp::set_error("device %d is %s, libpemp is built for gfx950 (MI355X)", dev, prop.gcnArchName);
    return PEMP_ERR_UNSUPPORTED;
  }
  return PEMP_OK;
}

#ifdef PEMP_HOST_TRACE
// diagnostics build (-DPEMP_HOST_TRACE, run with PEMP_HOST_TRACE=1; not part of the C-ABI of include/pemp.h):
// prints the host time between consecutive launch checks (source lines) since the last dump to stderr, then
// clears; returns the number of marks
extern "C" int pemp_host_trace_dump(void) {
  std::lock_guard<std::mutex> lk(pemp::g_ht_mu);
  const int n = (int)pemp::g_ht.size();
  for (int i = 0; i < n; ++i) fprintf(stderr, "[ht] %lld line %d\n", pemp::g_ht[i].second, pemp::g_ht[i].first);
  pemp::g_ht.clear();
  return n;
}
#endif
