// Pose grouping — restates:
//   Utils.py:1445-1455          pred_to_ann prefix: node threshold joint_scores > th, PyG subgraph
//                               (an edge survives iff both ends survive; no relabelling)
//   correlation_clustering_utils.py:99-151
//                               extract_edge_matrix(update=True) + update_graph_with_edge_matrix: dense
//                               adjacency of the surviving edges, averaged with its transpose in fp32
//                               ((a + b) / 2), or a + transpose when its lower triangle sums to zero
//   correlation_clustering_utils.py:187-245
//                               cluster_andres_graph(complete=False): upper-triangle edges, weight
//                               w - 0.5, andres GAEC, 1 = joined
//   Utils.py:499-514            pred_to_person (GAEC / threshold branches)
//   Utils.py:672-743            graph_cluster_to_persons: connected components (scipy labels: in order of
//                               each component's lowest node), class re-typing, best-scoring joint per type
//
// The edge pass is a GPU kernel over the batched graph (one thread per edge; the reverse edge is found by a
// binary search inside its CSR row of the (src, dst)-sorted edge list). Greedy additive edge contraction is inherently sequential: it
// runs on the host, one image per thread, restating andres::graph::multicut::greedyAdditiveEdgeContraction
// (andres graph, the library behind the reference's missing andres_graph_wrapper; not vendored): a max-heap of
// (a, b, w, edition) entries ordered by w only (std::priority_queue, so ties resolve exactly as libstdc++'s
// heap does), per-vertex std::map adjacency, contraction of the endpoint with fewer neighbours into the
// other, stale entries skipped by edition, stop at the first entry with w < 0.
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <queue>
#include <thread>
#include <vector>

#include "pemp_common.h"

using namespace pemp;

namespace {

// row_start[v] = first edge with src >= v (v = 0..N): the CSR rows of the (src, dst)-sorted edge list
__global__ __launch_bounds__(256) void pose_row_start_kernel(const int64_t* __restrict__ ei, int64_t E, int64_t N,
                                                             int64_t* __restrict__ row_start) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v > N) return;
  int64_t lo = 0, hi = E;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (ei[mid] < v) lo = mid + 1; else hi = mid;
  }
  row_start[v] = lo;
}

// w[e] = fl32(pred[e] + pred[rev(e)]) for a surviving upper edge (src < dst) in mode 0 (GAEC), pred[e] for
// every surviving edge in mode 1 (threshold), NaN otherwise. flags[B] bit 0: edge_index is not strictly
// (src, dst)-sorted; bit 2: a node index outside [0, N), never dereferenced (the per-image bits come
// from pose_image_flags_kernel).
__global__ __launch_bounds__(256) void pose_edge_weights_kernel(const int64_t* __restrict__ ei, int64_t E,
                                                                const float* __restrict__ pred,
                                                                const float* __restrict__ score, float th,
                                                                int use_th, const int64_t* __restrict__ node_off,
                                                                int B, int mode,
                                                                const int64_t* __restrict__ row_start, int64_t N,
                                                                float* __restrict__ w, int* __restrict__ flags) {
  for (int64_t e0 = (int64_t)blockIdx.x * blockDim.x; e0 < E; e0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = e0 + threadIdx.x;
    const bool live = e < E;
    const int64_t s = live ? ei[e] : ei[E - 1], d = live ? ei[E + e] : ei[2 * E - 1];
    if (live && e + 1 < E) {
      const int64_t s1 = ei[e + 1], d1 = ei[E + e + 1];
      if (s1 < s || (s1 == s && d1 <= d)) atomicOr(&flags[B], 1);
    }
    // node indices outside [0, N): flagged (bit 2, raised as an error by the caller), never dereferenced
    const bool inr = s >= 0 && s < N && d >= 0 && d < N;
    if (live && !inr) atomicOr(&flags[B], 4);
    const bool keep = live && inr && (!use_th || (score[s] > th && score[d] > th));
    const float p = live ? pred[e] : 0.f;
    float out = __int_as_float(0x7fc00000);
    if (keep) {
      if (mode == 1) {
        out = p;
      } else if (s < d) {
        // reverse edge (d, s): binary search for dst == s inside row d only (a few cached steps)
        int64_t lo = 0, hi = 0;
        if (d >= 0 && d < N) {
          lo = row_start[d];
          hi = row_start[d + 1];
        }
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (ei[E + mid] < s) lo = mid + 1; else hi = mid;
        }
        const float q = (lo < E && d >= 0 && d < N && lo < row_start[d + 1] && ei[E + lo] == s) ? pred[lo] : 0.f;
        out = p + q;
      }
    }
    if (live) w[e] = out;
  }
}

// flags[b] (bit 0: a surviving src > dst edge with pred != 0; bit 1: a surviving edge) over image b's edge
// range [row_start[node_off[b]], row_start[node_off[b + 1]]): grid (chunks, B), a block-wide OR per chunk and
// one atomic per block (a handful per image instead of one per wave on a few hot addresses).
__global__ __launch_bounds__(256) void pose_image_flags_kernel(const int64_t* __restrict__ ei, int64_t E,
                                                               const float* __restrict__ pred,
                                                               const float* __restrict__ score, float th, int use_th,
                                                               const int64_t* __restrict__ node_off,
                                                               const int64_t* __restrict__ row_start, int64_t N,
                                                               int* __restrict__ flags) {
  const int b = blockIdx.y;
  const int64_t lo = row_start[node_off[b]], hi = row_start[node_off[b + 1]];
  const int64_t chunk = (hi - lo + gridDim.x - 1) / gridDim.x;
  const int64_t c0 = lo + chunk * blockIdx.x, c1 = min(hi, c0 + chunk);
  int bits = 0;
  for (int64_t e = c0 + threadIdx.x; e < c1; e += blockDim.x) {
    const int64_t s = ei[e], d = ei[E + e];
    if (!(s >= 0 && s < N && d >= 0 && d < N)) continue;   // flagged by pose_edge_weights_kernel
    if (use_th && !(score[s] > th && score[d] > th)) continue;
    bits |= 2 | ((s > d && pred[e] != 0.f) ? 1 : 0);
  }
  const int b1 = __syncthreads_or(bits & 1), b2 = __syncthreads_or(bits & 2);
  if (threadIdx.x == 0 && (b1 | b2)) atomicOr(&flags[b], (b1 ? 1 : 0) | (b2 ? 2 : 0));
}

struct GaecEdge {
  size_t a, b, edition;
  double w;
  GaecEdge(size_t a_, size_t b_, double w_) : a(a_ < b_ ? a_ : b_), b(a_ < b_ ? b_ : a_), edition(0), w(w_) {}
  bool operator<(const GaecEdge& o) const { return w < o.w; }
};

// One image's edges (image-local endpoints, weights) as pemp_pose_cluster buckets them.
struct EdgeList {
  const uint32_t* a;
  const uint32_t* b;
  const double* w;
  size_t m;
};

// Greedy additive edge contraction over n vertices; root[v] = the cluster representative of v.
void gaec(size_t n, const EdgeList& el, std::vector<size_t>& root) {
  std::vector<std::map<size_t, double>> adj(n);
  std::vector<std::map<size_t, size_t>> editions(n);
  std::priority_queue<GaecEdge> q;
  for (size_t i = 0; i < el.m; ++i) {
    adj[el.a[i]][el.b[i]] += el.w[i];
    adj[el.b[i]][el.a[i]] += el.w[i];
    GaecEdge e(el.a[i], el.b[i], el.w[i]);
    e.edition = ++editions[e.a][e.b];
    q.push(e);
  }
  std::vector<size_t> parent(n), rank(n, 0);
  for (size_t v = 0; v < n; ++v) parent[v] = v;
  auto find = [&](size_t v) {
    while (parent[v] != v) {
      parent[v] = parent[parent[v]];
      v = parent[v];
    }
    return v;
  };
  while (!q.empty()) {
    // andres pops, skips stale entries and stops at the first live one with w < 0; every entry below a negative
    // top is negative too, so no contraction can follow once the top is negative: stop there instead of popping
    // the (mostly stale) negative entries one by one (the same partition; ~3x less time, gaec_dense alike)
    if (q.top().w < 0.0) break;
    const GaecEdge e = q.top();
    q.pop();
    const auto& aa = adj[e.a];
    if (aa.empty() || aa.find(e.b) == aa.end() || e.edition < editions[e.a][e.b]) continue;
    size_t keep = e.a, merge = e.b;
    if (adj[keep].size() < adj[merge].size()) std::swap(keep, merge);
    {
      size_t rk = find(keep), rm = find(merge);
      if (rk != rm) {
        if (rank[rk] < rank[rm]) std::swap(rk, rm);
        parent[rm] = rk;
        if (rank[rk] == rank[rm]) ++rank[rk];
      }
    }
    for (const auto& p : adj[merge]) {
      if (p.first == keep) continue;
      adj[keep][p.first] += p.second;
      adj[p.first][keep] += p.second;
      GaecEdge ne(keep, p.first, adj[keep][p.first]);
      ne.edition = ++editions[ne.a][ne.b];
      q.push(ne);
    }
    for (const auto& p : adj[merge]) adj[p.first].erase(merge);
    adj[merge].clear();
  }
  root.resize(n);
  for (size_t v = 0; v < n; ++v) root[v] = find(v);
}

// The same algorithm on dense n x n adjacency (weights, existence, edition counters, degrees): the
// neighbours of a vertex are visited by a row scan in ascending vertex order, i.e. in std::map order, the
// heap sees the identical push sequence, and every weight is the same sequence of double additions — so
// the result is identical to gaec() above, ties included (tests compare both against the oracle).
// 16-byte heap entry for the dense path (n <= 65535): the heap compares w only, so the entry layout does
// not change the pop order.
struct GaecEdge16 {
  double w;
  uint32_t edition;
  uint16_t a, b;
  GaecEdge16(size_t a_, size_t b_, double w_)
      : w(w_), edition(0), a((uint16_t)(a_ < b_ ? a_ : b_)), b((uint16_t)(a_ < b_ ? b_ : a_)) {}
  bool operator<(const GaecEdge16& o) const { return w < o.w; }
};

// The n x n per-pair arrays of both GAEC forms: one per-thread arena (gaec_fast and its gaec_dense fallback run one
// after the other on one thread, never together), reused across images and calls (fresh multi-100 KB blocks are
// mmap'ed, and their page faults serialise threads that cluster in parallel). An image above GAEC_KEEP_N vertices
// releases the arena afterwards, so one large image does not pin n^2 x 13 bytes per pool thread for the life of
// the process (2048 vertices: 54 MB per thread).
constexpr size_t GAEC_KEEP_N = 1024;
struct GaecScratch {
  std::vector<double> w;
  std::vector<uint32_t> ed;
  std::vector<uint8_t> ex;
};
GaecScratch& gaec_scratch() {
  static thread_local GaecScratch s;
  return s;
}
void gaec_release_if_large(size_t n) {
  if (n <= GAEC_KEEP_N) return;
  GaecScratch& s = gaec_scratch();
  std::vector<double>().swap(s.w);
  std::vector<uint32_t>().swap(s.ed);
  std::vector<uint8_t>().swap(s.ex);
}

void gaec_dense(size_t n, const EdgeList& el, std::vector<size_t>& root) {
  std::vector<double>& wt = gaec_scratch().w;
  std::vector<uint32_t>& ed = gaec_scratch().ed;
  std::vector<uint8_t>& ex = gaec_scratch().ex;
  static thread_local std::vector<uint32_t> deg;
  static thread_local std::vector<GaecEdge16> qstore;
  wt.assign(n * n, 0.0);
  ed.assign(n * n, 0);
  ex.assign(n * n, 0);
  deg.assign(n, 0);
  auto link = [&](size_t a, size_t b) {
    if (!ex[a * n + b]) {
      ex[a * n + b] = ex[b * n + a] = 1;
      ++deg[a];
      ++deg[b];
    }
  };
  // the queue's vector reserved up front (initial edges + one push per neighbour per contraction bound)
  qstore.clear();
  qstore.reserve(el.m + n * 8 + 64);
  std::priority_queue<GaecEdge16> q(std::less<GaecEdge16>(), std::move(qstore));
  for (size_t i = 0; i < el.m; ++i) {
    link(el.a[i], el.b[i]);
    wt[el.a[i] * n + el.b[i]] += el.w[i];
    wt[el.b[i] * n + el.a[i]] += el.w[i];
    GaecEdge16 e(el.a[i], el.b[i], el.w[i]);
    e.edition = ++ed[e.a * n + e.b];
    q.push(e);
  }
  std::vector<size_t> parent(n), rank(n, 0);
  for (size_t v = 0; v < n; ++v) parent[v] = v;
  auto find = [&](size_t v) {
    while (parent[v] != v) {
      parent[v] = parent[parent[v]];
      v = parent[v];
    }
    return v;
  };
  while (!q.empty()) {
    if (q.top().w < 0.0) break;   // (see gaec)
    const GaecEdge16 e = q.top();
    q.pop();
    if (!ex[e.a * n + e.b] || e.edition < ed[e.a * n + e.b]) continue;
    size_t keep = e.a, merge = e.b;
    if (deg[keep] < deg[merge]) std::swap(keep, merge);
    {
      size_t rk = find(keep), rm = find(merge);
      if (rk != rm) {
        if (rank[rk] < rank[rm]) std::swap(rk, rm);
        parent[rm] = rk;
        if (rank[rk] == rank[rm]) ++rank[rk];
      }
    }
    const uint8_t* row = &ex[merge * n];
    for (size_t p = 0; p < n; ++p) {
      if (!row[p] || p == keep) continue;
      const double pw = wt[merge * n + p];
      link(keep, p);
      wt[keep * n + p] += pw;
      wt[p * n + keep] += pw;
      GaecEdge16 ne(keep, p, wt[keep * n + p]);
      ne.edition = ++ed[ne.a * n + ne.b];
      q.push(ne);
    }
    for (size_t p = 0; p < n; ++p) {
      if (!ex[merge * n + p]) continue;
      ex[merge * n + p] = ex[p * n + merge] = 0;
      wt[merge * n + p] = wt[p * n + merge] = 0.0;
      --deg[p];
    }
    deg[merge] = 0;
  }
  root.resize(n);
  for (size_t v = 0; v < n; ++v) root[v] = find(v);
  // keep the heap's capacity for the next image (priority_queue exposes its container only to derived classes)
  struct Drain : std::priority_queue<GaecEdge16> {
    static std::vector<GaecEdge16>& c_of(std::priority_queue<GaecEdge16>& pq) { return pq.*(&Drain::c); }
  };
  qstore = std::move(Drain::c_of(q));
}

// gaec_dense with a heap of the non-negative entries only. andres' loop stops at the first negative heap top and
// never contracts a negative entry, so the negative entries matter only through the heap layout, i.e. through the
// order in which EQUAL weights pop. When every live entry popped for a contraction is strictly larger than every
// other entry in the heap at that moment, both heaps contract the same edges in the same order (a max-heap pops
// the unique maximum whatever its layout; stale entries are skipped by both) and the partitions are identical.
// So: the same adjacency, degrees, weights and edition counters as gaec_dense (every update counted, pushed or
// not), a heap of the entries with w >= 0, and at each contraction a check that the next top does not equal the
// popped weight. On such a tie it returns false and the caller runs gaec_dense (the exact libstdc++ heap order).
// C3 / C5 shapes: 20-40x fewer heap entries (the fully graph's edges between persons are negative).
bool gaec_fast(size_t n, const EdgeList& el, std::vector<size_t>& root) {
  // Per unordered pair (a, b), a < b, at a * n + b of two n x n arrays whose upper triangle alone is used (and
  // cleared): the weight (double) and the edition counter (uint32; 0 = no edge: every edge's first update counts
  // one). Split arrays, so the triangle's working set (12 bytes per pair, 1.5 MB at n = 502) stays in a core's
  // L2 through the row and column walks of the contractions. The initial edges (sorted by (src, dst), src < dst)
  // fill the rows in order. A merged vertex is only marked dead (its pairs are never read again: the walks visit
  // the alive vertices, a popped entry with a dead end is stale). Within one contraction every pair is updated
  // once, so the order of the walk does not change any weight (the same double additions).
  std::vector<double>& W = gaec_scratch().w;
  std::vector<uint32_t>& ED = gaec_scratch().ed;
  static thread_local std::vector<uint32_t> deg;
  static thread_local std::vector<uint8_t> alive;
  static thread_local std::vector<uint32_t> live;   // the alive vertices, ascending
  static thread_local std::vector<GaecEdge16> qstore;
  if (W.size() < n * n || ED.size() < n * n) {
    W.resize(n * n);
    ED.resize(n * n);
  }
  for (size_t a = 0; a + 1 < n; ++a) {
    std::fill(W.begin() + a * n + a + 1, W.begin() + (a + 1) * n, 0.0);
    std::fill(ED.begin() + a * n + a + 1, ED.begin() + (a + 1) * n, 0u);
  }
  deg.assign(n, 0);
  alive.assign(n, 1);
  live.resize(n);
  for (size_t v = 0; v < n; ++v) live[v] = (uint32_t)v;
  auto ix = [n](size_t a, size_t b) { return a < b ? a * n + b : b * n + a; };
  qstore.clear();
  std::priority_queue<GaecEdge16> q(std::less<GaecEdge16>(), std::move(qstore));
  struct Drain : std::priority_queue<GaecEdge16> {
    static std::vector<GaecEdge16>& c_of(std::priority_queue<GaecEdge16>& pq) { return pq.*(&Drain::c); }
  };
  for (size_t i = 0; i < el.m; ++i) {
    const size_t a = el.a[i], b = el.b[i], k = ix(a, b);
    if (!ED[k]) {
      ++deg[a];
      ++deg[b];
    }
    W[k] += el.w[i];
    GaecEdge16 e(a, b, el.w[i]);
    e.edition = ++ED[k];
    if (!(e.w < 0.0)) q.push(e);
  }
  std::vector<size_t> parent(n), rank(n, 0);
  for (size_t v = 0; v < n; ++v) parent[v] = v;
  auto find = [&](size_t v) {
    while (parent[v] != v) {
      parent[v] = parent[parent[v]];
      v = parent[v];
    }
    return v;
  };
  bool exact = true;
  while (!q.empty()) {
    const GaecEdge16 e = q.top();
    q.pop();
    if (!alive[e.a] || !alive[e.b]) continue;
    const size_t ke = (size_t)e.a * n + e.b;
    if (!ED[ke] || e.edition < ED[ke]) continue;
    if (!q.empty() && q.top().w == e.w) {   // an equal weight: its pop order is the full heap's to decide
      exact = false;
      break;
    }
    size_t keep = e.a, merge = e.b;
    if (deg[keep] < deg[merge]) std::swap(keep, merge);
    {
      size_t rk = find(keep), rm = find(merge);
      if (rk != rm) {
        if (rank[rk] < rank[rm]) std::swap(rk, rm);
        parent[rm] = rk;
        if (rank[rk] == rank[rm]) ++rank[rk];
      }
    }
    for (const uint32_t pv : live) {
      const size_t p = pv;
      if (p == merge) continue;
      const size_t km = ix(merge, p);
      if (!ED[km]) continue;
      --deg[p];                      // the edge (p, merge) goes with merge (p == keep included)
      if (p == keep) continue;
      const size_t kk = ix(keep, p);
      if (!ED[kk]) {
        ++deg[keep];
        ++deg[p];
      }
      const double nw = W[kk] + W[km];
      W[kk] = nw;
      GaecEdge16 ne(keep, p, nw);
      ne.edition = ++ED[kk];
      if (!(nw < 0.0)) q.push(ne);
    }
    alive[merge] = 0;
    deg[merge] = 0;
    live.erase(std::lower_bound(live.begin(), live.end(), (uint32_t)merge));
  }
  qstore = std::move(Drain::c_of(q));
  if (!exact) return false;
  root.resize(n);
  for (size_t v = 0; v < n; ++v) root[v] = find(v);
  return true;
}

// Persistent host workers for the per-image loops (one image per task): a call hands out tasks through an atomic
// counter and the calling thread works too, so no thread is created per call (std::thread creation and the first
// touch of each new thread's stack cost more than a 153-node GAEC). Calls are serialised by the pool's mutex.
class HostPool {
 public:
  void run(int tasks, int threads, const std::function<void(int)>& fn) {
    threads = std::max(1, std::min(threads, tasks));
    if (threads == 1) {
      for (int i = 0; i < tasks; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> call(call_mu_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      while ((int)workers_.size() < threads - 1) workers_.emplace_back([this, id = (int)workers_.size()] { loop(id); });
      fn_ = &fn;
      tasks_ = tasks;
      next_.store(0);
      active_ = threads - 1;
      running_.store(threads - 1);
      // adaptive spin (below): the workers spin after this call only if it came within the spin window of the
      // previous one, i.e. while calls arrive back to back (a serving loop); an occasional caller wakes them
      // through the condition variable and leaves no thread spinning between its calls
      const uint64_t t = now_ns();
      hot_.store(last_call_ns_ != 0 && t - last_call_ns_ < spin_ns(), std::memory_order_relaxed);
      last_call_ns_ = t;
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    drain(fn);
    // the caller's share is done: wait for the workers' tasks (spinning first, briefly; they are short)
    for (int spin = 0; running_.load(std::memory_order_acquire) != 0; ++spin) {
      if (spin < 4000) {
        __builtin_ia32_pause();
      } else {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return running_.load() == 0; });
      }
    }
    std::lock_guard<std::mutex> lk(mu_);
    fn_ = nullptr;
  }

 private:
  void drain(const std::function<void(int)>& fn) {
    for (int i = next_.fetch_add(1); i < tasks_; i = next_.fetch_add(1)) fn(i);
  }
  // A worker may spin on the generation counter for a while after its last task before it sleeps on the condition
  // variable: a condition-variable wake-up measured 1-4 ms on some hosts (the per-image tasks are 0.1-1 ms), and a
  // serving loop calls again within a few ms. Only while calls arrive within the window of each other (hot_), and
  // only the first PEMP_POOL_SPIN_WORKERS workers (default 4): the rest sleep at once, so several ranks or
  // processes on one host do not each keep 15 threads spinning. PEMP_POOL_SPIN_US (default 2000) sets the window,
  // 0 disables spinning.
  static uint64_t spin_ns() {
    static const uint64_t v = [] {
      const char* e = getenv("PEMP_POOL_SPIN_US");
      return (uint64_t)(e ? strtoull(e, nullptr, 10) : 2000) * 1000;
    }();
    return v;
  }
  static int spin_workers() {
    static const int v = [] {
      const char* e = getenv("PEMP_POOL_SPIN_WORKERS");
      return e ? std::max(0, atoi(e)) : 4;
    }();
    return v;
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const uint64_t t_idle = now_ns();
      const uint64_t window = (id < spin_workers() && hot_.load(std::memory_order_relaxed)) ? spin_ns() : 0;
      while (gen_.load(std::memory_order_acquire) == seen && now_ns() - t_idle < window)
        for (int k = 0; k < 64; ++k) __builtin_ia32_pause();
      const std::function<void(int)>* fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_.load() != seen; });
        seen = gen_.load();
        if (id >= active_) continue;   // not needed this call
        fn = fn_;
      }
      drain(*fn);
      if (running_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        std::lock_guard<std::mutex> lk(mu_);
        done_cv_.notify_one();
      }
    }
  }
  static uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;   // never joined: the pool lives as long as the process
  const std::function<void(int)>* fn_ = nullptr;
  std::atomic<int> next_{0};
  std::atomic<int> running_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> hot_{false};
  uint64_t last_call_ns_ = 0;   // (under mu_)
  int tasks_ = 0, active_ = 0;
};

HostPool& host_pool() {
  static HostPool* p = new HostPool();   // (leaked on purpose: no join at exit)
  return *p;
}

void union_join(std::vector<size_t>& parent, size_t a, size_t b) {
  auto find = [&](size_t v) {
    while (parent[v] != v) {
      parent[v] = parent[parent[v]];
      v = parent[v];
    }
    return v;
  };
  a = find(a);
  b = find(b);
  if (a != b) parent[std::max(a, b)] = std::min(a, b);
}

}  // namespace

extern "C" int pemp_pose_edge_weights(const int64_t* edge_index, int64_t E, const float* pred,
                                      const float* node_scores, float th, int use_th, const int64_t* node_off, int B,
                                      int64_t N, int method, int64_t* row_start, float* w, int* flags, void* stream) {
  PEMP_CHECK_ARG(E >= 0 && B >= 1 && N >= 0 && (method == 0 || method == 1), "pemp_pose_edge_weights: bad args");
  PEMP_CHECK_ARG(node_off && flags && (E == 0 || (edge_index && pred && w && row_start && (!use_th || node_scores))),
                 "pemp_pose_edge_weights: null pointer");
  PEMP_HIP(hipMemsetAsync(flags, 0, sizeof(int) * (B + 1), as_stream(stream)));
  if (E == 0) return PEMP_OK;
  ProfScope prof("pose_edge_weights", as_stream(stream));
  hipLaunchKernelGGL(pose_row_start_kernel, dim3((unsigned)((N + 1 + 255) / 256)), dim3(256), 0, as_stream(stream),
                     edge_index, E, N, row_start);
  PEMP_LAUNCH_CHECK();
  const int64_t blocks = std::min<int64_t>((E + 255) / 256, 8192);
  hipLaunchKernelGGL(pose_edge_weights_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), edge_index,
                     E, pred, node_scores, th, use_th, node_off, B, method, row_start, N, w, flags);
  PEMP_LAUNCH_CHECK();
  hipLaunchKernelGGL(pose_image_flags_kernel, dim3(16, B), dim3(256), 0, as_stream(stream), edge_index, E, pred,
                     node_scores, th, use_th, node_off, row_start, N, flags);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

extern "C" int pemp_pose_cluster(int B, const int64_t* node_off, const int64_t* edge_index, int64_t E, const float* w,
                                 const int* flags, int method, int n_threads, int32_t* labels, int32_t* n_comp) {
  PEMP_CHECK_ARG(B >= 1 && E >= 0 && node_off && flags && labels && n_comp && (method == 0 || method == 1),
                 "pemp_pose_cluster: bad args");
  PEMP_CHECK_ARG(E == 0 || (edge_index && w), "pemp_pose_cluster: null edge arrays");
  if (flags[B] & 4) {
    ::pemp::set_error("pemp_pose_cluster: edge_index holds a node index outside [0, N)");
    return PEMP_ERR_INVALID_ARG;
  }
  if (flags[B] & 1) {
    ::pemp::set_error("pemp_pose_cluster: edge_index is not sorted by (src, dst) without duplicates");
    return PEMP_ERR_INVALID_ARG;
  }
  for (int b = 0; b < B; ++b)
    PEMP_CHECK_ARG(node_off[b + 1] >= node_off[b], "pemp_pose_cluster: node_off not monotone");
  size_t dense_max = 2048;  // dense adjacency up to 2048 vertices (54 MB); PEMP_GAEC_DENSE_MAX overrides
  if (const char* env = getenv("PEMP_GAEC_DENSE_MAX")) dense_max = (size_t)strtoull(env, nullptr, 10);
  dense_max = std::min<size_t>(dense_max, 65535);
  const bool exact_only = getenv("PEMP_GAEC_EXACT") != nullptr;   // diagnostics / tests: the full heap always
  std::atomic<int64_t> bad_edge{-1};
  // one task per image: its edges are the contiguous run of the (src, dst)-sorted list whose src lies in the image
  // (found by binary search), bucketed in edge_index order, then clustered
  auto run = [&](int img) {
    const int64_t o = node_off[img], n64 = node_off[img + 1] - o;
    const size_t n = (size_t)n64;
    const int64_t lo = std::lower_bound(edge_index, edge_index + E, o) - edge_index;
    const int64_t hi = std::lower_bound(edge_index + lo, edge_index + E, o + n64) - edge_index;
    // image-local edges, written in place (sized for the whole run, then cut to the surviving count)
    static thread_local std::vector<uint32_t> ua, ub;
    static thread_local std::vector<double> uw;
    const size_t cap = (size_t)(hi - lo);
    if (ua.size() < cap) {
      ua.resize(cap);
      ub.resize(cap);
      uw.resize(cap);
    }
    size_t m = 0;
    uint32_t* pa = ua.data();
    uint32_t* pb = ub.data();
    double* pw = uw.data();
    const bool avg = (flags[img] & 1) != 0;
    for (int64_t e = lo; e < hi; ++e) {
      const float we = w[e];
      if (std::isnan(we)) continue;
      const int64_t d = edge_index[E + e];
      if (d < o || d >= o + n64) {
        int64_t none = -1;
        bad_edge.compare_exchange_strong(none, e);
        return;
      }
      double weight;
      if (method == 0) {
        const float mm = avg ? we * 0.5f : we;   // extract_edge_matrix: average, or M + M^T
        weight = (double)(mm - 0.5f);             // cluster_andres_graph: edge_attr - 0.5 (fp32)
      } else {
        if (!(we > 0.8f)) continue;               // pred_to_person "threshold": pred > 0.8
        weight = 1.0;
      }
      pa[m] = (uint32_t)(edge_index[e] - o);
      pb[m] = (uint32_t)(d - o);
      pw[m] = weight;
      ++m;
    }
    const EdgeList el{pa, pb, pw, m};
    std::vector<size_t> root;
    if (method == 0) {
      if (n <= dense_max) {
        if (exact_only || !gaec_fast(n, el, root)) gaec_dense(n, el, root);
        gaec_release_if_large(n);
      } else {
        gaec(n, el, root);
      }
    } else {
      root.resize(n);
      for (size_t v = 0; v < n; ++v) root[v] = v;
      for (size_t i = 0; i < m; ++i) union_join(root, pa[i], pb[i]);
      for (size_t v = 0; v < n; ++v) {
        size_t r = v;
        while (root[r] != r) r = root[r];
        root[v] = r;
      }
    }
    std::vector<int32_t> lab(n, -1);
    int32_t next = 0;
    int32_t* out = labels + o;
    for (size_t v = 0; v < n; ++v) {  // scipy connected_components: labels in order of first vertex
      if (lab[root[v]] < 0) lab[root[v]] = next++;
      out[v] = lab[root[v]];
    }
    n_comp[img] = next;
  };
  host_pool().run(B, n_threads, run);
  {   // surviving edges whose source lies in no image
    const int64_t lo = std::lower_bound(edge_index, edge_index + E, node_off[0]) - edge_index;
    const int64_t hi = std::lower_bound(edge_index, edge_index + E, node_off[B]) - edge_index;
    auto scan = [&](int64_t a, int64_t b) {
      for (int64_t e = a; e < b; ++e)
        if (!std::isnan(w[e])) {
          int64_t none = -1;
          bad_edge.compare_exchange_strong(none, e);
          return;
        }
    };
    scan(0, lo);
    scan(hi, E);
  }
  if (bad_edge.load() >= 0) {
    ::pemp::set_error("pemp_pose_cluster: edge %lld crosses images", (long long)bad_edge.load());
    return PEMP_ERR_INVALID_ARG;
  }
  return PEMP_OK;
}

extern "C" int pemp_pose_persons(int B, const int64_t* node_off, const int32_t* labels, const int32_t* n_comp,
                                 const int64_t* joint_det, const float* scores, const float* pose_scores,
                                 const float* class_probs, int J, int allow_single, int64_t cap, double* persons,
                                 int32_t* person_count, int32_t* mutants) {
  PEMP_CHECK_ARG(B >= 1 && J >= 1 && cap >= 0 && node_off && n_comp && person_count && mutants &&
                     (cap == 0 || persons),
                 "pemp_pose_persons: bad args");
  PEMP_CHECK_ARG(node_off[B] == 0 || (labels && joint_det && scores), "pemp_pose_persons: null node arrays");
  int64_t out = 0;
  for (int b = 0; b < B; ++b) {
    const int64_t o = node_off[b], n = node_off[b + 1] - o;
    std::vector<std::vector<int64_t>> members(n_comp[b]);
    for (int64_t v = 0; v < n; ++v) {
      const int32_t l = labels[o + v];
      PEMP_CHECK_ARG(l >= 0 && l < n_comp[b], "pemp_pose_persons: label out of range");
      members[l].push_back(o + v);
    }
    int32_t count = 0;
    mutants[b] = 0;
    // each node's type once: its detection type, or the first argmax of its class probabilities (np.argmax)
    std::vector<int64_t> types((size_t)n);
    for (int64_t v = 0; v < n; ++v) {
      const int64_t g = o + v;
      if (!class_probs) {
        types[v] = joint_det[g * 3 + 2];
        continue;
      }
      const float* c = class_probs + g * J;
      int best = 0;
      for (int j = 1; j < J; ++j)
        if (c[j] > c[best]) best = j;  // np.argmax: first maximum
      types[v] = best;
    }
    for (const auto& m : members) {
      if ((int64_t)m.size() > J) mutants[b] = 1;
      auto type_of = [&](int64_t g) -> int64_t { return types[g - o]; };
      double kp[64 * 3];
      PEMP_CHECK_ARG(J <= 64, "pemp_pose_persons: J > 64");
      std::fill(kp, kp + J * 3, 0.0);
      bool emit = false;
      if (m.size() > 1) {
        for (int t = 0; t < J; ++t) {
          int64_t best = -1;
          for (int64_t g : m)
            if (type_of(g) == t && (best < 0 || scores[g] > scores[best])) best = g;
          if (best < 0) continue;
          kp[t * 3 + 0] = (double)joint_det[best * 3 + 0];
          kp[t * 3 + 1] = (double)joint_det[best * 3 + 1];
          kp[t * 3 + 2] = pose_scores ? (double)pose_scores[best] : (double)scores[best];
        }
        for (int t = 0; t < J; ++t) emit |= kp[t * 3 + 2] > 0.0;
      } else if (m.size() == 1 && allow_single) {
        const int64_t g = m[0];
        if (scores[g] < 0.1f) continue;
        const int64_t t = type_of(g);
        for (int j = 0; j < J; ++j) {
          kp[j * 3 + 0] = (double)joint_det[g * 3 + 0];
          kp[j * 3 + 1] = (double)joint_det[g * 3 + 1];
        }
        kp[t * 3 + 2] = (double)scores[g];
        emit = true;
      }
      if (!emit) continue;
      if (out >= cap) {
        ::pemp::set_error("pemp_pose_persons: more than cap = %lld persons", (long long)cap);
        return PEMP_ERR_WORKSPACE;
      }
      std::copy(kp, kp + J * 3, persons + out * J * 3);
      ++out;
      ++count;
    }
    person_count[b] = count;
  }
  return PEMP_OK;
}

// ------------------------------------------------------------------------------------------------
// refine (Utils.py:1026-1104) and adjust (Utils.py:917-936)
// ------------------------------------------------------------------------------------------------
namespace {


// numpy's float32 add.reduce of k values: pairwise_sum for a contiguous run (F = 1: n < 8 sequential,
// else 8 strided partial sums combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus the tail); for F = 2 the
// reduction axis is the outer one and numpy adds row by row (sequential).
__device__ float np_sum_f32(const float* v, int n, bool pairwise) {
  if (!pairwise || n < 8) {
    float r = 0.f;
    for (int i = 0; i < n; ++i) r += v[i];
    return r;
  }
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = v[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += v[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += v[i];
  return res;
}

// prev_tag[p] = np.mean(tags at the detected joints of person p, axis=0) (float32). One wave per person:
// lane j loads joint j's flag and tag values (all loads in flight together), lane 0 sums in numpy's order.
// Batched form (pemp_pose_finish_batch): pimg[p] is person p's image, whose maps start at image * J H W (F) and
// which is refined only where ref[image] != 0; pimg == nullptr: one image, refined.
__global__ __launch_bounds__(64) void refine_mean_tag_kernel(const double* __restrict__ kp, int P, int J,
                                                             const float* __restrict__ tag, int H, int W, int F,
                                                             float* __restrict__ mean_tag,
                                                             const int32_t* __restrict__ pimg,
                                                             const uint8_t* __restrict__ ref) {
  const int p = blockIdx.x, j = threadIdx.x;
  if (pimg) {
    const int b = pimg[p];
    if (!ref[b]) return;
    tag += (size_t)b * J * H * W * F;
  }
  bool det = false;
  float v0 = 0.f, v1 = 0.f;
  if (j < J) {
    const double* q = kp + ((size_t)p * J + j) * 3;
    det = q[2] > 0.0;
    const int x = (int)q[0], y = (int)q[1];  // astype(np.int32): truncation
    // (the host wrapper rejects detected joints outside the map; here they are only kept from faulting)
    det = det && x >= 0 && x < W && y >= 0 && y < H;
    if (det) {
      const size_t o = (((size_t)j * H + y) * W + x) * F;
      v0 = tag[o];
      if (F == 2) v1 = tag[o + 1];
    }
  }
  __shared__ float vals[2][64];
  __shared__ int flag[64];
  vals[0][j] = v0;
  vals[1][j] = v1;
  flag[j] = det;
  __syncthreads();
  if (j == 0) {
    float c[2][64];
    int k = 0;
    for (int i = 0; i < J; ++i)
      if (flag[i]) {
        c[0][k] = vals[0][i];
        c[1][k] = vals[1][i];
        ++k;
      }
    for (int f = 0; f < F; ++f) mean_tag[p * F + f] = np_sum_f32(c[f], k, F == 1) / (float)k;
  }
}

// np.argmax order as a 64-bit key: NaN above everything (argmax returns the first NaN), -0.0 equal to
// +0.0 (canonicalised), then the lower flat index among equal values
__device__ __forceinline__ unsigned long long refine_key(float v, uint32_t idx) {
  const uint32_t u = __float_as_uint(v == 0.f ? 0.f : v);
  const uint32_t o = v != v ? 0xFFFFFFFFu : (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)o << 32) | (0xFFFFFFFFu - idx);  // max: larger v, then lower flat index
}

// ordered 64-bit key: larger value first, then the lower flat index
// partial keys[i][block][p] = max over the block's pixels of key(s - rint(||tag - prev_tag[p]||), pixel):
// np.argmax(tmp2), first max. grid: (pixel blocks, J, person chunks of PC). Straight-line code: persons
// beyond P in the last chunk are computed on a copy of a real mean tag and never stored; pixels past the
// end are clamped to the last pixel (a true candidate with its own index). A thread visits its pixels in
// increasing order, so a strict > keeps the first maximum; (value, index) pairs become ordered 64-bit keys
// only for the cross-thread reduction.
// Only (person, joint) pairs whose joint is not detected (keypoints[p, i, 2] == 0) are searched: the reference
// computes the argmax for every pair but keeps it only for those (Utils.py:1096-1101), so the others are skipped
// (block-uniform branches; a chunk with every person's joint i detected returns at once and stores nothing --
// refine_finish_kernel reads keys only for the pairs searched).
template <int PC, int F>
__global__ __launch_bounds__(256) void refine_argmax_kernel(const float* __restrict__ s, const float* __restrict__ tag,
                                                            int H, int W, const float* __restrict__ mean_tag,
                                                            int P, unsigned long long* __restrict__ keys, int J,
                                                            const double* __restrict__ kp,
                                                            const int32_t* __restrict__ chunks) {
  const int i = blockIdx.y;
  int p0 = blockIdx.z * PC, np_ = min(PC, P - p0);
  if (chunks) {   // batched: chunk z = (first person, persons, image); a chunk never spans two images
    const int b = chunks[3 * blockIdx.z + 2];
    p0 = chunks[3 * blockIdx.z];
    np_ = chunks[3 * blockIdx.z + 1];
    s += (size_t)b * J * H * W;
    tag += (size_t)b * J * H * W * F;
  }
  bool need[PC];
  bool any = false;
#pragma unroll
  for (int q = 0; q < PC; ++q) {
    need[q] = q < np_ && kp[((size_t)(p0 + q) * J + i) * 3 + 2] == 0.0;
    any |= need[q];
  }
  if (!any) return;
  float mt0[PC], mt1[PC], bv[PC];
  uint32_t bi[PC];
  const size_t HW = (size_t)H * W;
  const size_t first = min((size_t)blockIdx.x * blockDim.x + threadIdx.x, HW - 1);
#pragma unroll
  for (int q = 0; q < PC; ++q) {
    const int pq = p0 + min(q, np_ - 1);
    mt0[q] = mean_tag[pq * F];
    mt1[q] = F == 2 ? mean_tag[pq * F + 1] : 0.f;
    bv[q] = -INFINITY;
    bi[q] = (uint32_t)first;
  }
  const float* sp = s + (size_t)i * HW;
  const float* tp = tag + (size_t)i * HW * F;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t base = (size_t)blockIdx.x * blockDim.x + threadIdx.x; base < HW; base += 4 * stride) {
    float sv[4], t0[4], t1[4];
    uint32_t pxs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t px = min(base + u * stride, HW - 1);
      pxs[u] = (uint32_t)px;
      sv[u] = sp[px];
      t0[u] = tp[px * F];
      t1[u] = F == 2 ? tp[px * F + 1] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int q = 0; q < PC; ++q) {
        if (!need[q]) continue;                  // (block-uniform)
        const float d0 = __fsub_rn(t0[u], mt0[q]);
        float k;
        if (F == 2) {
          const float d1 = __fsub_rn(t1[u], mt1[q]);
          // sqrtf is the correctly rounded square root (numpy's); __fsqrt_rn lowers to the 1-ulp v_sqrt_f32
          k = rintf(sqrtf(__fadd_rn(__fmul_rn(d0, d0), __fmul_rn(d1, d1))));
        } else {
          // F = 1: in binary floating point with round-to-nearest, sqrt(RN(d * d)) == |d| whenever d * d
          // neither overflows nor underflows (an underflow only happens for |d| < 2^-63, where both round
          // to 0), so rint(sqrt(d^2)) = rint(|d|) with no square root; d^2 = inf gives inf as in numpy
          k = isinf(__fmul_rn(d0, d0)) ? INFINITY : rintf(fabsf(d0));
        }
        const float v = __fsub_rn(sv[u], k);
        const bool better = v > bv[q] || (v != v && bv[q] == bv[q]);   // first NaN wins, as np.argmax
        bv[q] = better ? v : bv[q];
        bi[q] = better ? pxs[u] : bi[q];
      }
    }
  }
  unsigned long long best[PC];
#pragma unroll
  for (int q = 0; q < PC; ++q) best[q] = refine_key(bv[q], bi[q]);
  __shared__ unsigned long long red[4][PC];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int q = 0; q < PC; ++q) {
    unsigned long long k = best[q];
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long other = __shfl_xor(k, o);
      k = other > k ? other : k;
    }
    if (lane == 0) red[wv][q] = k;
  }
  __syncthreads();
  bool mine = false;   // this thread's person (q = threadIdx.x) was searched
#pragma unroll
  for (int q = 0; q < PC; ++q) mine |= need[q] && (int)threadIdx.x == q;
  if (mine) {  // per-block partial: no cross-XCD atomics on the same few addresses
    const int q = threadIdx.x;
    unsigned long long k = red[0][q];
    for (int w2 = 1; w2 < (int)(blockDim.x >> 6); ++w2) k = red[w2][q] > k ? red[w2][q] : k;
    keys[((size_t)i * gridDim.x + blockIdx.x) * P + p0 + q] = k;
  }
}

// ans[p][i] = (x + 0.5 +- 0.25, y + 0.5 +- 0.25, val) as Utils.py:1075-1092, then the fill rule of
// :1096-1101: keypoints[p, i] = (ans x, ans y, 0.001) where ans val > 0 and keypoints[p, i, 2] == 0.
// One wave per (person, joint): the lanes reduce the per-block partial keys, lane 0 finishes.
__global__ __launch_bounds__(64) void refine_finish_kernel(const float* __restrict__ s, int H, int W,
                                                           const unsigned long long* __restrict__ keys, int nblk,
                                                           int P, int J, double* __restrict__ kp,
                                                           const int32_t* __restrict__ pimg,
                                                           const uint8_t* __restrict__ ref) {
  const int t = blockIdx.x;
  const int i = t % J, p = t / J;
  if (kp[(size_t)t * 3 + 2] != 0.0) return;   // a detected joint: nothing searched, nothing changes
  if (pimg) {
    const int b = pimg[p];
    if (!ref[b]) return;                         // an image that is not refined
    s += (size_t)b * J * H * W;
  }
  unsigned long long key = 0ull;
  for (int b = threadIdx.x; b < nblk; b += 64) {
    const unsigned long long k = keys[((size_t)i * nblk + b) * P + p];
    key = k > key ? k : key;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(key, o);
    key = other > key ? other : key;
  }
  if (threadIdx.x != 0) return;
  const uint32_t idx = 0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull);
  const int yy = idx / W, xx = idx % W;
  const float* tmp = s + (size_t)i * H * W;
  const float val = tmp[(size_t)yy * W + xx];
  double x = xx + 0.5, y = yy + 0.5;
  x += tmp[(size_t)yy * W + min(xx + 1, W - 1)] > tmp[(size_t)yy * W + max(xx - 1, 0)] ? 0.25 : -0.25;
  y += tmp[(size_t)min(yy + 1, H - 1) * W + xx] > tmp[(size_t)max(yy - 1, 0) * W + xx] ? 0.25 : -0.25;
  double* q = kp + (size_t)t * 3;
  if ((double)val > 0.0 && q[2] == 0.0) {
    q[0] = x;
    q[1] = y;
    q[2] = 0.001;
  }
}

// adjust (Utils.py:917-936): for joints with score > 0, quarter-pixel shift toward the larger neighbour of
// det[joint_id] (indexed [int(kp[1]), int(kp[0])]), then + 0.5.
__global__ void adjust_kernel(const float* __restrict__ det, int H, int W, int P, int J, double* __restrict__ kp,
                              const int32_t* __restrict__ pimg) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= P * J) return;
  double* q = kp + (size_t)t * 3;
  if (!(q[2] > 0.0)) return;
  const int j = t % J;
  if (pimg) det += (size_t)pimg[t / J] * J * H * W;
  double y = q[0], x = q[1];
  const int xx = (int)x, yy = (int)y;
  if (xx < 0 || xx >= H || yy < 0 || yy >= W) return;   // rejected by the host wrapper; kept from faulting
  const float* tmp = det + (size_t)j * H * W;
  y += tmp[(size_t)xx * W + min(yy + 1, W - 1)] > tmp[(size_t)xx * W + max(yy - 1, 0)] ? 0.25 : -0.25;
  x += tmp[(size_t)min(xx + 1, H - 1) * W + yy] > tmp[(size_t)max(0, xx - 1) * W + yy] ? 0.25 : -0.25;
  q[1] = x + 0.5;
  q[0] = y + 0.5;
}

}  // namespace

static int refine_blocks(int J, int H, int W) {
  return (int)std::min<size_t>(((size_t)H * W + 1023) / 1024, (size_t)std::max(1, 4096 / J));
}

extern "C" size_t pemp_pose_refine_workspace_size(int P, int J, int H, int W, int F) {
  if (P <= 0 || J <= 0 || H <= 0 || W <= 0) return 0;
  return align_up((size_t)P * F * sizeof(float), 256) + (size_t)J * refine_blocks(J, H, W) * P * 8;
}

// persons per argmax thread: the smallest instantiated width covering an even split of P into <= 16-wide chunks
static int refine_pc(int P) {
  const int chunks = (P + 15) / 16, per = (P + chunks - 1) / chunks;
  return per <= 2 ? 2 : per <= 4 ? 4 : per <= 6 ? 6 : per <= 8 ? 8 : per <= 10 ? 10 : per <= 12 ? 12 : 16;
}

// The three refine launches (mean tags, per-block argmax keys, finish) over P persons; pimg / chunks / ref null:
// one image, n_chunks = ceil(P / pc) chunks of pc persons; else the batched plan of pemp_pose_finish_plan.
static int refine_launch(const float* scoremaps, const float* tag, int J, int H, int W, int F, double* keypoints,
                         int P, const int32_t* pimg, const int32_t* chunks, int n_chunks, int pc, const uint8_t* ref,
                         void* workspace, hipStream_t st) {
  float* mean_tag = reinterpret_cast<float*>(workspace);
  unsigned long long* keys =
      reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(workspace) + align_up((size_t)P * F * 4, 256));
  ProfScope prof("pose_refine", st);
  hipLaunchKernelGGL(refine_mean_tag_kernel, dim3(P), dim3(64), 0, st, keypoints, P, J, tag, H, W, F,
                     mean_tag, pimg, ref);
  PEMP_LAUNCH_CHECK();
  const int bx = refine_blocks(J, H, W);
  const dim3 grid(bx, J, n_chunks);
#define PEMP_REFINE_LAUNCH(N)                                                                                   \
  case N:                                                                                                       \
    if (F == 1)                                                                                                 \
      hipLaunchKernelGGL((refine_argmax_kernel<N, 1>), grid, dim3(256), 0, st, scoremaps, tag, H, W, mean_tag, P,  \
                         keys, J, keypoints, chunks);                                                           \
    else                                                                                                        \
      hipLaunchKernelGGL((refine_argmax_kernel<N, 2>), grid, dim3(256), 0, st, scoremaps, tag, H, W, mean_tag, P,  \
                         keys, J, keypoints, chunks);                                                           \
    break;
  switch (pc) {
    PEMP_REFINE_LAUNCH(2)
    PEMP_REFINE_LAUNCH(4)
    PEMP_REFINE_LAUNCH(6)
    PEMP_REFINE_LAUNCH(8)
    PEMP_REFINE_LAUNCH(10)
    PEMP_REFINE_LAUNCH(12)
    PEMP_REFINE_LAUNCH(16)
    default: set_error("pose refine: persons per chunk %d not instantiated", pc); return PEMP_ERR_INVALID_ARG;
  }
#undef PEMP_REFINE_LAUNCH
  PEMP_LAUNCH_CHECK();
  hipLaunchKernelGGL(refine_finish_kernel, dim3(P * J), dim3(64), 0, st, scoremaps, H, W, keys, bx, P, J, keypoints,
                     pimg, ref);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

extern "C" int pemp_pose_refine(const float* scoremaps, const float* tag, int J, int H, int W, int F, double* keypoints,
                                int P, void* workspace, size_t workspace_bytes, void* stream) {
  PEMP_CHECK_ARG(J >= 1 && J <= 64 && H >= 1 && W >= 1 && (F == 1 || F == 2) && P >= 0,
                 "pemp_pose_refine: bad args (J <= 64, F in {1, 2})");
  PEMP_CHECK_ARG((size_t)H * W < 0xFFFFFFFFull, "pemp_pose_refine: map too large");
  if (P == 0) return PEMP_OK;
  PEMP_CHECK_ARG(scoremaps && tag && keypoints, "pemp_pose_refine: null pointer");
  const size_t need = pemp_pose_refine_workspace_size(P, J, H, W, F);
  PEMP_CHECK_ARG(workspace && workspace_bytes >= need, "pemp_pose_refine: workspace %zu < %zu", workspace_bytes,
                 need);
  const int pc = refine_pc(P);
  return refine_launch(scoremaps, tag, J, H, W, F, keypoints, P, nullptr, nullptr, (P + pc - 1) / pc, pc, nullptr,
                       workspace, as_stream(stream));
}

extern "C" int pemp_pose_finish_plan(int B, const int32_t* counts, const uint8_t* ref, int32_t* pimg, int32_t* chunks,
                                     int max_chunks, int32_t* out2) {
  PEMP_CHECK_ARG(B >= 0 && (B == 0 || (counts && ref)) && out2, "pemp_pose_finish_plan: bad args");
  int pmax = 0;
  int64_t P = 0;
  for (int b = 0; b < B; ++b) {
    PEMP_CHECK_ARG(counts[b] >= 0, "pemp_pose_finish_plan: counts[%d] < 0", b);
    if (ref[b]) pmax = std::max(pmax, (int)counts[b]);
    P += counts[b];
  }
  PEMP_CHECK_ARG(P == 0 || pimg, "pemp_pose_finish_plan: null pimg");
  const int pc = refine_pc(std::max(pmax, 1));
  int64_t p = 0;
  int nc = 0;
  for (int b = 0; b < B; ++b) {
    for (int k = 0; k < counts[b]; ++k) pimg[p + k] = b;
    if (ref[b])
      for (int q = 0; q < counts[b]; q += pc) {
        PEMP_CHECK_ARG(nc < max_chunks && chunks, "pemp_pose_finish_plan: more than %d chunks", max_chunks);
        chunks[3 * nc] = (int32_t)(p + q);
        chunks[3 * nc + 1] = std::min(pc, (int)counts[b] - q);
        chunks[3 * nc + 2] = b;
        ++nc;
      }
    p += counts[b];
  }
  out2[0] = nc;
  out2[1] = pc;
  return PEMP_OK;
}

extern "C" int pemp_pose_finish_batch(const float* scoremaps, const float* tags, int B, int J, int H, int W, int F,
                                      double* keypoints, int P, const int32_t* pimg, const int32_t* chunks,
                                      int n_chunks, int pc, const uint8_t* ref, int adjust, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  PEMP_CHECK_ARG(B >= 1 && J >= 1 && J <= 64 && H >= 1 && W >= 1 && (F == 1 || F == 2) && P >= 0 && n_chunks >= 0,
                 "pemp_pose_finish_batch: bad args (J <= 64, F in {1, 2})");
  PEMP_CHECK_ARG((size_t)H * W < 0xFFFFFFFFull, "pemp_pose_finish_batch: map too large");
  if (P == 0) return PEMP_OK;
  PEMP_CHECK_ARG(scoremaps && keypoints && pimg && ref, "pemp_pose_finish_batch: null pointer");
  hipStream_t st = as_stream(stream);
  if (n_chunks > 0) {
    PEMP_CHECK_ARG(tags && chunks, "pemp_pose_finish_batch: refine needs tags and chunks");
    const size_t need = pemp_pose_refine_workspace_size(P, J, H, W, F);
    PEMP_CHECK_ARG(workspace && workspace_bytes >= need, "pemp_pose_finish_batch: workspace %zu < %zu",
                   workspace_bytes, need);
    const int r = refine_launch(scoremaps, tags, J, H, W, F, keypoints, P, pimg, chunks, n_chunks, pc, ref,
                                workspace, st);
    if (r) return r;
  }
  if (adjust) {
    hipLaunchKernelGGL(adjust_kernel, dim3((P * J + 255) / 256), dim3(256), 0, st, scoremaps, H, W, P, J, keypoints,
                       pimg);
    PEMP_LAUNCH_CHECK();
  }
  return PEMP_OK;
}

// ---- pemp_pack_to_host: several device regions gathered into one staging buffer, then one copy to the host ----
namespace {
constexpr int PACK_MAX = 16;
struct PackArgs {
  const uint8_t* src[PACK_MAX];
  uint64_t bytes[PACK_MAX];
  uint64_t off[PACK_MAX];
  uint8_t* dst;
};

// blockIdx.y = region; 16-byte moves where the region's source, destination and size allow, else 4 / 1 bytes
__global__ __launch_bounds__(256) void pack_kernel(PackArgs a) {
  const int i = blockIdx.y;
  const uint8_t* src = a.src[i];
  uint8_t* dst = a.dst + a.off[i];
  const uint64_t n = a.bytes[i];
  const uint64_t t0 = (uint64_t)blockIdx.x * 256 + threadIdx.x, step = (uint64_t)gridDim.x * 256;
  const uint64_t al = (reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | n);
  if ((al & 15) == 0) {
    for (uint64_t k = t0; k < n / 16; k += step)
      reinterpret_cast<uint4*>(dst)[k] = reinterpret_cast<const uint4*>(src)[k];
  } else if ((al & 3) == 0) {
    for (uint64_t k = t0; k < n / 4; k += step)
      reinterpret_cast<uint32_t*>(dst)[k] = reinterpret_cast<const uint32_t*>(src)[k];
  } else {
    for (uint64_t k = t0; k < n; k += step) dst[k] = src[k];
  }
}
}  // namespace

extern "C" int pemp_pack_to_host(int n, const void* const* src, const size_t* bytes, const size_t* off, size_t total,
                                 void* staging, void* host_dst, void* stream) {
  PEMP_CHECK_ARG(n >= 0 && n <= PACK_MAX && (n == 0 || (src && bytes && off)), "pemp_pack_to_host: bad args (n <= %d)",
                 PACK_MAX);
  if (total == 0) return PEMP_OK;
  PEMP_CHECK_ARG(staging, "pemp_pack_to_host: null staging buffer");
  PackArgs a{};
  uint64_t most = 0;
  for (int i = 0; i < n; ++i) {
    PEMP_CHECK_ARG(off[i] % 16 == 0 && off[i] + bytes[i] <= total && (bytes[i] == 0 || src[i]),
                   "pemp_pack_to_host: region %d (offset %zu, %zu bytes) outside [0, %zu) or unaligned", i, off[i],
                   bytes[i], total);
    a.src[i] = static_cast<const uint8_t*>(src[i]);
    a.bytes[i] = bytes[i];
    a.off[i] = off[i];
    most = std::max<uint64_t>(most, bytes[i]);
  }
  a.dst = static_cast<uint8_t*>(staging);
  hipStream_t st = as_stream(stream);
  if (n > 0 && most > 0) {
    const unsigned gx = (unsigned)std::min<uint64_t>((most / 16 + 255) / 256 + 1, 1024);
    hipLaunchKernelGGL(pack_kernel, dim3(gx, n), dim3(256), 0, st, a);
    PEMP_LAUNCH_CHECK();
  }
  // host_dst NULL: gather only (the caller copies staging itself, e.g. with torch, whose pinned-memory cache then
  // records the copy's event before the block can be reused)
  if (host_dst) PEMP_HIP(hipMemcpyAsync(host_dst, staging, total, hipMemcpyDeviceToHost, st));
  return PEMP_OK;
}

extern "C" int pemp_pose_adjust(const float* det, int J, int H, int W, double* keypoints, int P, void* stream) {
  PEMP_CHECK_ARG(J >= 1 && H >= 1 && W >= 1 && P >= 0, "pemp_pose_adjust: bad args");
  if (P == 0) return PEMP_OK;
  PEMP_CHECK_ARG(det && keypoints, "pemp_pose_adjust: null pointer");
  hipLaunchKernelGGL(adjust_kernel, dim3((P * J + 255) / 256), dim3(256), 0, as_stream(stream), det, H, W, P, J,
                     keypoints, nullptr);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

// fill_mean (Utils.py:1468-1470), host: joints with score == 0 take the mean (x, y) of the person's joints
// with score != 0 (float64, numpy's row-by-row axis-0 sum from 0, then / count; NaN when none).
extern "C" int pemp_pose_fill_mean(double* keypoints, int P, int J) {
  PEMP_CHECK_ARG(P >= 0 && J >= 1 && (P == 0 || keypoints), "pemp_pose_fill_mean: bad args");
  for (int p = 0; p < P; ++p) {
    double* kp = keypoints + (size_t)p * J * 3;
    double sx = 0.0, sy = 0.0;
    int k = 0;
    for (int j = 0; j < J; ++j)
      if (kp[j * 3 + 2] != 0.0) {
        sx += kp[j * 3 + 0];
        sy += kp[j * 3 + 1];
        ++k;
      }
    const double mx = sx / (double)k, my = sy / (double)k;
    for (int j = 0; j < J; ++j)
      if (kp[j * 3 + 2] == 0.0) {
        kp[j * 3 + 0] = mx;
        kp[j * 3 + 1] = my;
      }
  }
  return PEMP_OK;
}

// greedy_person_construction (Utils.py:517-626), host, per image: class re-typing (first argmax), the
// float64 symmetric adjacency (adj + adj^T) / 2 of the surviving edges (w = pred, NaN = dropped; the
// output of pemp_pose_edge_weights method 1), then type-major seeding: a free joint with node score >= 0.5
// becomes a core and claims, per other type, its strongest neighbour (first maximum), taking it over from
// an earlier core unless that core's edge is strictly stronger. Clusters are the joints claimed by one core
// (cores in node order); persons as graph_cluster_to_persons without class re-typing of the keypoint rows.
// taken[ΣN]: core node (image-local) or -1.
extern "C" int pemp_pose_greedy(int B, const int64_t* node_off, const int64_t* edge_index, int64_t E, const float* w,
                                const int64_t* joint_det, const float* scores, const float* class_probs, int J,
                                int32_t* taken, int64_t cap, double* persons, int32_t* person_count) {
  PEMP_CHECK_ARG(B >= 1 && J >= 1 && J <= 64 && E >= 0 && cap >= 0 && node_off && person_count &&
                     (E == 0 || (edge_index && w)) && (cap == 0 || persons),
                 "pemp_pose_greedy: bad args");
  PEMP_CHECK_ARG(node_off[B] == 0 || (joint_det && scores && taken), "pemp_pose_greedy: null node arrays");
  int64_t out = 0;
  int64_t e = 0;
  for (int b = 0; b < B; ++b) {
    const int64_t o = node_off[b], n = node_off[b + 1] - o;
    std::vector<double> adj((size_t)(n * n), 0.0);
    for (; e < E && edge_index[e] < node_off[b + 1]; ++e) {
      if (std::isnan(w[e])) continue;
      const int64_t s = edge_index[e] - o, d = edge_index[E + e] - o;
      PEMP_CHECK_ARG(s >= 0 && d >= 0 && d < n, "pemp_pose_greedy: edge %lld crosses images", (long long)e);
      adj[s * n + d] = (double)w[e];
    }
    std::vector<double> sym((size_t)(n * n));
    for (int64_t i = 0; i < n; ++i)
      for (int64_t k = 0; k < n; ++k) sym[i * n + k] = (adj[k * n + i] + adj[i * n + k]) / 2.0;
    for (int64_t i = 0; i < n; ++i) sym[i * n + i] = 1.0;
    std::vector<int> type(n);
    for (int64_t i = 0; i < n; ++i) {
      if (class_probs) {
        const float* c = class_probs + (o + i) * J;
        int best = 0;
        for (int j = 1; j < J; ++j)
          if (c[j] > c[best]) best = j;
        type[i] = best;
      } else {
        type[i] = (int)joint_det[(o + i) * 3 + 2];
      }
    }
    int32_t* tk = taken + o;
    for (int64_t i = 0; i < n; ++i) tk[i] = -1;
    for (int t = 0; t < J; ++t) {
      for (int64_t i = 0; i < n; ++i) {
        if (type[i] != t || tk[i] != -1) continue;
        if (scores[o + i] < 0.5f) continue;
        tk[i] = (int32_t)i;
        for (int j = 0; j < J; ++j) {
          if (j == t) continue;
          double best = 0.0;  // np.max / np.argmax (first maximum) of the row with other types zeroed
          int64_t idx = 0;
          for (int64_t k = 0; k < n; ++k) {
            const double v = type[k] == j ? sym[i * n + k] : 0.0;
            if (k == 0 || v > best) {
              best = v;
              idx = k;
            }
          }
          if (best == 0.0 || idx == i) continue;
          if (tk[idx] != -1) {
            if (sym[(int64_t)tk[idx] * n + idx] > best) continue;
            tk[idx] = (int32_t)i;
          } else {
            tk[idx] = (int32_t)i;
          }
        }
      }
    }
    int32_t mx = -1;
    for (int64_t i = 0; i < n; ++i) mx = std::max(mx, tk[i]);
    int32_t count = 0;
    for (int32_t c = 0; c <= mx; ++c) {
      std::vector<int64_t> m;
      for (int64_t i = 0; i < n; ++i)
        if (tk[i] == c) m.push_back(i);
      if (m.size() <= 1) continue;
      double kp[64 * 3];
      std::fill(kp, kp + J * 3, 0.0);
      for (int t = 0; t < J; ++t) {
        int64_t bsel = -1;
        for (int64_t i : m)
          if (type[i] == t && (bsel < 0 || scores[o + i] > scores[o + bsel])) bsel = i;
        if (bsel < 0) continue;
        kp[t * 3 + 0] = (double)joint_det[(o + bsel) * 3 + 0];
        kp[t * 3 + 1] = (double)joint_det[(o + bsel) * 3 + 1];
        kp[t * 3 + 2] = (double)scores[o + bsel];
      }
      bool emit = false;
      for (int t = 0; t < J; ++t) emit |= kp[t * 3 + 2] > 0.0;
      if (!emit) continue;
      if (out >= cap) {
        ::pemp::set_error("pemp_pose_greedy: more than cap = %lld persons", (long long)cap);
        return PEMP_ERR_WORKSPACE;
      }
      std::copy(kp, kp + J * 3, persons + out * J * 3);
      ++out;
      ++count;
    }
    person_count[b] = count;
  }
  return PEMP_OK;
}
