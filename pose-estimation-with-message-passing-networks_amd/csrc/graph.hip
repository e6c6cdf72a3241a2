// Graph construction for gfx950 — restates:
//   ConstructGraph.py:100-103,262-269  node features x = features[:, y, x].T, joint tags
//   ConstructGraph.py:206-231          batching (node offsets added to edge_index, cat)
//   ConstructGraph.py:376-381          fully_connected_mpn_graph: all i != j sorted by (src, dst)
//   ConstructGraph.py:363-368          knn_mpn_graph: knn_graph(k) -> to_undirected -> no self loops
//   ConstructGraph.py:405-422          score_based_graph: k best-scoring roots, every edge touching one
//   ConstructGraph.py:289-359          edge_attr = [dx, dy, onehot(type_src) | onehot(type_dst)]
// All integer outputs are bit-exact; dx/dy are IEEE fp32 divisions of exact integer differences.
#include <math.h>

#include "pemp_common.h"

namespace pemp {
namespace {

__device__ __forceinline__ int find_segment(const int64_t* off, int n, int64_t v) {
  // largest b in [0, n) with off[b] <= v  (off non-decreasing, off[0] = 0)
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= v) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// ---- edge_attr (ConstructGraph.py:289-357) --------------------------------------------------
// Per edge the kernels stage dx, dy, the endpoint types and one extra scalar `aux`: theta for the
// angle mode, the tag term for the associative-embedding modes. ef_value() then lays out column f.

// ||tag[dst] - tag[src]||_2 rounded as the reference's CPU torch.norm: sqrt(fma(d1, d1, d0 * d0))
// (F = 2); F = 1 is |d| exactly. Contraction is spelled out so the compiler cannot re-fuse it.
// sqrtf, not __fsqrt_rn: on gfx950 the latter lowers to the bare 1-ulp v_sqrt_f32, while sqrtf
// gets the correctly rounded sequence.
__device__ __forceinline__ float tag_distance(const float* ts, const float* td, int F) {
  const float d0 = __fsub_rn(td[0], ts[0]);
  if (F == 1) return fabsf(d0);
  const float d1 = __fsub_rn(td[1], ts[1]);
  return sqrtf(fmaf(d1, d1, __fmul_rn(d0, d0)));
}

// ConstructGraph.py:337-357: ae -> dist; ae_normed -> round(dist) * 100 - score[src];
// ae_tracking_1 -> (t_a - dist) / t_a with t_a = 1.8425 (fp32 ops, no contraction)
__device__ __forceinline__ float ae_term(int mode, float dist, float score_src) {
  if (mode == PEMP_EF_AE_NORMED) return __fsub_rn(__fmul_rn(rintf(dist), 100.0f), score_src);
  if (mode == PEMP_EF_AE_TRACKING) return div_rn(__fsub_rn(1.8425f, dist), 1.8425f);
  return dist;
}

__device__ __forceinline__ bool ef_uses_tags(int mode) {
  return mode == PEMP_EF_POSITION_CONNECTION_AE || mode == PEMP_EF_AE || mode == PEMP_EF_AE_NORMED ||
         mode == PEMP_EF_AE_TRACKING;
}

// theta (angle mode) from the integer endpoint coordinates, ConstructGraph.py:319-321
__device__ __forceinline__ float edge_theta(int64_t sx, int64_t sy, int64_t dx, int64_t dy) {
  const float ax = (float)(sx - dx), ay = (float)(sy - dy);
  const float th = fabsf(acosf(ax * (1.0f / sqrtf(ax * ax + ay * ay))));
  return isnan(th) ? 0.0f : th;
}

__device__ __forceinline__ float ef_value(int mode, int f, int J, float dx, float dy, float aux, int ts, int td) {
  int oh = -1;   // one-hot column index, or -1
  float v = 0.0f;
  switch (mode) {
    case PEMP_EF_POSITION_CONNECTION:
      if (f == 0) v = dx; else if (f == 1) v = dy; else oh = f - 2;
      break;
    case PEMP_EF_CONNECTION: oh = f; break;
    case PEMP_EF_NOTHING: break;
    case PEMP_EF_POSITION: v = f == 0 ? dx : dy; break;
    case PEMP_EF_POSITION_ANGLE_CONNECTION:
      if (f == 0) v = dx; else if (f == 1) v = dy; else if (f == 2) v = aux; else oh = f - 3;
      break;
    case PEMP_EF_POSITION_CONNECTION_AE:
      if (f == 0) v = dx; else if (f == 1) v = dy; else if (f == J + 2) v = aux; else oh = f - 2;
      break;
    default: v = aux; break;   // AE, AE_NORMED, AE_TRACKING: one column
  }
  if (oh >= 0) v = (ts == oh || td == oh) ? 1.0f : 0.0f;
  return v;
}

// Granlund-Montgomery constants of an unsigned division by d >= 1 for dividends below 2^31:
// q = (umulhi(n, m) + n) >> l (3 instructions instead of a 32-bit division's ~15, a 64-bit one's ~100)
__host__ __device__ inline void graph_fastdiv_consts(unsigned d, uint32_t& m, int& l) {
  l = 0;
  while ((1ull << l) < d) ++l;
  m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
}
__device__ __forceinline__ int graph_fastdiv(int n, uint32_t m, int l) {
  return (int)((__umulhi((unsigned)n, m) + (unsigned)n) >> l);
}

__global__ __launch_bounds__(256) void pack_nodes_kernel(
    const float* __restrict__ feat, int C, const float* __restrict__ tags, int F, int B, int J, int H, int W,
    const int64_t* __restrict__ det, const float* __restrict__ det_sc, int cap, const int64_t* __restrict__ node_off,
    int64_t n_total, float* __restrict__ x, int64_t* __restrict__ jdet, float* __restrict__ jsc,
    int64_t* __restrict__ bidx, float* __restrict__ jtag) {
  const int64_t total = n_total * C;
  uint32_t mC;
  int lC;
  graph_fastdiv_consts((unsigned)C, mC, lC);
  const bool small = total + (int64_t)gridDim.x * blockDim.x < ((int64_t)1 << 31);   // (uniform)
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = small ? graph_fastdiv((int)idx, mC, lC) : idx / C;
    const int c = (int)(idx - g * C);
    const int b = find_segment(node_off, B, g);
    const int64_t i = g - node_off[b];
    const int64_t* d = det + ((size_t)b * cap + i) * 3;
    const int64_t px = d[0], py = d[1], pt = d[2];
    if (feat) x[idx] = feat[(((size_t)b * C + c) * H + py) * W + px];   // NULL: pemp_gather_projected fills x
    if (c == 0) {
      jdet[g * 3 + 0] = px; jdet[g * 3 + 1] = py; jdet[g * 3 + 2] = pt;
      jsc[g] = det_sc[(size_t)b * cap + i];
      bidx[g] = b;
    }
    if (tags && c < F) jtag[g * F + c] = tags[((((size_t)b * J + pt) * H + py) * W + px) * F + c];
  }
}

__global__ __launch_bounds__(256) void fully_graph_kernel(const int64_t* __restrict__ node_off,
                                                          const int64_t* __restrict__ edge_off, int B,
                                                          int64_t e_total, int64_t* __restrict__ ei) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < e_total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int b = find_segment(edge_off, B, e);
    const int64_t n = node_off[b + 1] - node_off[b];
    const int64_t el = e - edge_off[b];
    int64_t i, r;
    if (n <= 46340) {   // the image's n (n - 1) edges below 2^31: 32-bit division
      const unsigned nm1 = (unsigned)(n - 1), iu = (unsigned)el / nm1;
      i = iu;
      r = (unsigned)el - iu * nm1;
    } else {
      i = el / (n - 1);
      r = el - i * (n - 1);
    }
    const int64_t j = r < i ? r : r + 1;
    ei[e] = node_off[b] + i;
    ei[e_total + e] = node_off[b] + j;
  }
}

// 256 edges per step: per-edge values (dx, dy, theta, the two types) go to LDS once, then the
// block writes the 256 x A output rows as one contiguous, coalesced range.
__global__ __launch_bounds__(256) void edge_features_kernel(const int64_t* __restrict__ jdet,
                                                            const float* __restrict__ jtag, int F,
                                                            const float* __restrict__ jsc,
                                                            const int64_t* __restrict__ ei, int64_t E, int J,
                                                            float norm, int mode, int A, float* __restrict__ out,
                                                            const int64_t* __restrict__ e_dev = nullptr) {
  __shared__ float dx_s[256], dy_s[256], aux_s[256];
  __shared__ int ts_s[256], td_s[256];
  if (e_dev) {   // the edge total known only on the device (pemp_knn_graph_build); E = the capacity
    const int64_t e = *e_dev;
    if (e > E) return;
    E = e;
  }
  uint32_t mA;
  int lA;
  graph_fastdiv_consts((unsigned)A, mA, lA);
  for (int64_t base = (int64_t)blockIdx.x * 256; base < E; base += (int64_t)gridDim.x * 256) {
    const int64_t e = base + threadIdx.x;
    if (e < E) {
      const int64_t s = ei[e], d = ei[E + e];
      const int64_t sx = jdet[s * 3 + 0], sy = jdet[s * 3 + 1], dx = jdet[d * 3 + 0], dy = jdet[d * 3 + 1];
      dx_s[threadIdx.x] = (float)(dx - sx) / norm;            // ConstructGraph.py:311-317 (IEEE division)
      dy_s[threadIdx.x] = (float)(dy - sy) / norm;
      ts_s[threadIdx.x] = (int)jdet[s * 3 + 2];
      td_s[threadIdx.x] = (int)jdet[d * 3 + 2];
      if (mode == PEMP_EF_POSITION_ANGLE_CONNECTION) aux_s[threadIdx.x] = edge_theta(sx, sy, dx, dy);
      else if (ef_uses_tags(mode)) aux_s[threadIdx.x] = ae_term(mode, tag_distance(jtag + s * F, jtag + d * F, F), jsc[s]);
    }
    __syncthreads();
    const int n = (int)min<int64_t>(256, E - base), total = n * A;
    float* o = out + base * A;
    for (int k = threadIdx.x; k < total; k += 256) {
      const int el = graph_fastdiv(k, mA, lA), f = k - el * A;
      o[k] = ef_value(mode, f, J, dx_s[el], dy_s[el], aux_s[el], ts_s[el], td_s[el]);
    }
    __syncthreads();
  }
}

// ---- knn ----
struct KnnWs {
  unsigned long long* adj;   // per image: n_b rows x words_b  (A: j among i's nearest)
  unsigned long long* adjt;  // transpose                      (T[j][i] = A[i][j])
  int64_t* mat_off;          // [B+1] word offsets (device copy)
  int64_t* ecount;           // [B] edges per image (pemp_knn_graph_build)
  int64_t* edge_off;         // [B+1] exclusive scan of ecount; [B] = the batch's edge total
  unsigned long long* arow;  // fast path: A (the k+1 nearest of each node), 8 words per node
  unsigned long long* rows;  // fast path: R = A | A^T, 8 words per node
  int* rowstart;             // LDS path: degree prefix of each row inside its image
  int64_t* doff;             // feature_knn: [B+1] offsets of the per-image n_b x n_b key matrices
  unsigned* dkey;            // feature_knn: squared feature distances as ordered fp32 bit patterns
};

static size_t knn_words(const int64_t* node_off_host, int B, int64_t* mat_off_host) {
  size_t w = 0;
  for (int b = 0; b < B; ++b) {
    if (mat_off_host) mat_off_host[b] = (int64_t)w;
    const int64_t n = node_off_host[b + 1] - node_off_host[b];
    w += (size_t)n * ((n + 63) / 64);
  }
  if (mat_off_host) mat_off_host[B] = (int64_t)w;
  return w;
}

static KnnWs knn_carve(void* base, const int64_t* node_off_host, int B, size_t* bytes, bool feat = false) {
  Carver c(base);
  const size_t w = knn_words(node_off_host, B, nullptr);
  KnnWs k;
  k.adj = c.take<unsigned long long>(w);
  k.adjt = c.take<unsigned long long>(w);
  k.mat_off = c.take<int64_t>(B + 1);
  k.ecount = c.take<int64_t>(B);
  k.edge_off = c.take<int64_t>(B + 1);
  // LDS path (pemp_knn_graph_build, every n_b <= 512): rows at a fixed stride of 8 words per node
  const int64_t nt = node_off_host[B];
  k.arow = c.take<unsigned long long>((size_t)nt * 8);
  k.rows = c.take<unsigned long long>((size_t)nt * 8);
  k.rowstart = c.take<int>((size_t)nt);
  k.doff = nullptr;
  k.dkey = nullptr;
  if (feat) {
    size_t nn = 0;
    for (int b = 0; b < B; ++b) {
      const int64_t n = node_off_host[b + 1] - node_off_host[b];
      nn += (size_t)n * (size_t)n;
    }
    k.doff = c.take<int64_t>(B + 1);
    k.dkey = c.take<unsigned>(nn);
  }
  if (bytes) *bytes = c.used;
  return k;
}

// The distance a selection kernel ranks by. Positions (knn_mpn_graph, ConstructGraph.py:363-368):
// the squared integer pixel distance. Features (feature_knn_mpn_graph, ConstructGraph.py:370-374):
// the key matrix of fknn_dist_kernel, row i of image b at dkey + doff[b] + i n.
struct KnnDist {
  const int64_t* jdet;
  const unsigned* dkey;   // null: positions
  const int64_t* doff;
  __device__ __forceinline__ long long operator()(int64_t base, int b, int n, int i, int j) const {
    if (dkey) return (long long)dkey[doff[b] + (int64_t)i * n + j];
    const long long dx = jdet[(base + j) * 3 + 0] - jdet[(base + i) * 3 + 0];
    const long long dy = jdet[(base + j) * 3 + 1] - jdet[(base + i) * 3 + 1];
    return dx * dx + dy * dy;
  }
};

// feature_knn keys: torch_cluster 1.5.4's CUDA knn (the reference's knn_graph(features, k=50) on the
// device) ranks candidates by tmp_dist += (x_j[c] - x_i[c]) * (x_j[c] - x_i[c]) over c in order, fp32,
// which nvcc contracts to one fma per channel; restated here as that fma chain. A non-negative fp32
// orders as its bit pattern; NaN (a NaN feature) becomes the largest key. Block per query node,
// candidates across the threads, the query row broadcast from LDS.
__global__ __launch_bounds__(256) void fknn_dist_kernel(const float* __restrict__ x, int C,
                                                        const int64_t* __restrict__ node_off, int B,
                                                        const int64_t* __restrict__ doff,
                                                        unsigned* __restrict__ dkey) {
  extern __shared__ float xq[];
  const int64_t g = blockIdx.x;
  const int b = find_segment(node_off, B, g);
  const int64_t base = node_off[b];
  const int n = (int)(node_off[b + 1] - base), i = (int)(g - base);
  for (int c = threadIdx.x; c < C; c += blockDim.x) xq[c] = x[g * C + c];
  __syncthreads();
  unsigned* row = dkey + doff[b] + (int64_t)i * n;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const float* xj = x + (base + j) * C;
    float acc = 0.f;
    int c = 0;
    if ((C & 3) == 0) {
      for (; c < C; c += 4) {
        const float4 v = *reinterpret_cast<const float4*>(xj + c);
        float t = v.x - xq[c];
        acc = __fmaf_rn(t, t, acc);
        t = v.y - xq[c + 1];
        acc = __fmaf_rn(t, t, acc);
        t = v.z - xq[c + 2];
        acc = __fmaf_rn(t, t, acc);
        t = v.w - xq[c + 3];
        acc = __fmaf_rn(t, t, acc);
      }
    }
    for (; c < C; ++c) {
      const float t = xj[c] - xq[c];
      acc = __fmaf_rn(t, t, acc);
    }
    row[j] = acc != acc ? 0xffffffffu : __float_as_uint(acc);
  }
}

__global__ void fknn_doff_kernel(const int64_t* __restrict__ node_off, int B, int64_t* __restrict__ doff) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t w = 0;
  for (int b = 0; b < B; ++b) {
    doff[b] = w;
    const int64_t n = node_off[b + 1] - node_off[b];
    w += n * n;
  }
  doff[B] = w;
}

// One wave per query node i: the k+1 nearest (distance, then index), self dropped.
__global__ __launch_bounds__(256) void knn_adj_kernel(KnnDist dist,
                                                      const int64_t* __restrict__ node_off, int B, int64_t n_total,
                                                      int kq, const int64_t* __restrict__ mat_off,
                                                      unsigned long long* __restrict__ adj,
                                                      unsigned long long* __restrict__ adjt) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= n_total) return;
  const int b = find_segment(node_off, B, g);
  const int64_t base = node_off[b];
  const int n = (int)(node_off[b + 1] - base);
  const int i = (int)(g - base);
  const int wpr = (n + 63) / 64;
  unsigned long long* A = adj + mat_off[b];
  unsigned long long* T = adjt + mat_off[b];
  auto d2 = [&](int j) -> int64_t { return dist(base, b, n, i, j); };
  const int chunk = (n + 63) / 64;
  const int j0 = lane * chunk, j1 = min(n, j0 + chunk);
  if (n <= kq) {   // every node is among the k+1 nearest
    for (int j = j0; j < j1; ++j) {
      if (j == i) continue;
      atomicOr(&A[(size_t)i * wpr + j / 64], 1ull << (j & 63));
      atomicOr(&T[(size_t)j * wpr + i / 64], 1ull << (i & 63));
    }
    return;
  }
  // smallest tau with #{d2 <= tau} >= kq (binary search over the integer distance / key)
  int64_t lo = 0, hi = 0;
  for (int j = j0; j < j1; ++j) hi = max(hi, d2(j));
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) hi = max(hi, (int64_t)__shfl_xor((long long)hi, off));
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    int c = 0;
    for (int j = j0; j < j1; ++j) c += d2(j) <= mid;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off);
    if (c >= kq) hi = mid; else lo = mid + 1;
  }
  const int64_t tau = lo;
  int less = 0, ties = 0;
  for (int j = j0; j < j1; ++j) { const int64_t d = d2(j); less += d < tau; ties += d == tau; }
  int less_all = less;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) less_all += __shfl_xor(less_all, off);
  int tie_pre = ties;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(tie_pre, off);
    if (lane >= off) tie_pre += o;
  }
  int tie_rank = tie_pre - ties;   // ties in lower-index lanes
  const int need = kq - less_all;  // ties admitted, lowest index first
  for (int j = j0; j < j1; ++j) {
    const int64_t d = d2(j);
    bool take = d < tau;
    if (d == tau) { take = tie_rank < need; ++tie_rank; }
    if (take && j != i) {
      atomicOr(&A[(size_t)i * wpr + j / 64], 1ull << (j & 63));
      atomicOr(&T[(size_t)j * wpr + i / 64], 1ull << (i & 63));
    }
  }
}

__global__ void knn_matoff_kernel(const int64_t* __restrict__ node_off, int B, int64_t* __restrict__ mat_off) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t w = 0;
  for (int b = 0; b < B; ++b) {
    mat_off[b] = w;
    const int64_t n = node_off[b + 1] - node_off[b];
    w += n * ((n + 63) / 64);
  }
  mat_off[B] = w;
}

__device__ __forceinline__ int row_degree(const unsigned long long* A, const unsigned long long* T, int a, int wpr) {
  int c = 0;
  for (int w = 0; w < wpr; ++w) c += __popcll(A[(size_t)a * wpr + w] | T[(size_t)a * wpr + w]);
  return c;
}

__global__ __launch_bounds__(256) void knn_count_kernel(const int64_t* __restrict__ node_off, int B,
                                                        const int64_t* __restrict__ mat_off,
                                                        const unsigned long long* __restrict__ adj,
                                                        const unsigned long long* __restrict__ adjt,
                                                        int64_t* __restrict__ edge_count) {
  const int b = blockIdx.x;
  const int n = (int)(node_off[b + 1] - node_off[b]);
  const int wpr = (n + 63) / 64;
  __shared__ int64_t sh[4];
  int64_t c = 0;
  for (int a = threadIdx.x; a < n; a += blockDim.x) c += row_degree(adj + mat_off[b], adjt + mat_off[b], a, wpr);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor((long long)c, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) edge_count[b] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ __launch_bounds__(1024) void knn_emit_kernel(const int64_t* __restrict__ node_off, int B,
                                                        const int64_t* __restrict__ mat_off,
                                                        const unsigned long long* __restrict__ adj,
                                                        const unsigned long long* __restrict__ adjt,
                                                        const int64_t* __restrict__ edge_off, int64_t e_total,
                                                        int64_t e_cap, int64_t* __restrict__ ei) {
  // e_total < 0: the total is edge_off[B], known only on the device (pemp_knn_graph_build); the
  // destination row starts right after the source row, at ei + e_total (a contiguous [2, E] view)
  if (e_total < 0) e_total = edge_off[B];
  if (e_total > e_cap) return;   // reported by the host (the total exceeds the buffer)
  const int b = blockIdx.x;
  const int64_t base = node_off[b];
  const int n = (int)(node_off[b + 1] - base);
  const int wpr = (n + 63) / 64;
  const unsigned long long* A = adj + mat_off[b];
  const unsigned long long* T = adjt + mat_off[b];
  __shared__ int64_t carry;
  __shared__ int64_t wsum[16];
  if (threadIdx.x == 0) carry = edge_off[b];
  __syncthreads();
  for (int a0 = 0; a0 < n; a0 += 1024) {
    const int a = a0 + threadIdx.x;
    const int deg = a < n ? row_degree(A, T, a, wpr) : 0;
    int64_t x = deg;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t o = __shfl_up((long long)x, off);
      if (lane >= off) x += o;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int64_t pre = carry;
    for (int w = 0; w < wave; ++w) pre += wsum[w];
    pre += x - deg;
    if (a < n) {
      int64_t pos = pre;
      for (int w = 0; w < wpr; ++w) {
        unsigned long long word = A[(size_t)a * wpr + w] | T[(size_t)a * wpr + w];
        while (word) {
          const int bit = __ffsll((long long)word) - 1;
          word &= word - 1;
          ei[pos] = base + a;
          ei[e_total + pos] = base + w * 64 + bit;
          ++pos;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t s = 0;
      for (int w = 0; w < 16; ++w) s += wsum[w];
      carry += s;
    }
    __syncthreads();
  }
}

// ---- knn, fast path (every image with n <= KNN_LDS_MAXN nodes) ------------------------------
// Three launches, no atomics in global memory and no memsets:
//   knn_select_kernel: wave per query node i (all images at once), candidates j = lane + 64 r in
//     registers, the k+1 nearest by squared integer distance with ties admitted lowest index first
//     (the rule of knn_adj_kernel); the counts of the threshold search are ballots + popcounts (no
//     cross-lane shuffles). Row i of A goes to global memory at a fixed stride of KNN_W words.
//   knn_rows_kernel: one workgroup per image: A^T in LDS, R = A | A^T, each row's degree prefix inside
//     its image, the image's edge count.
//   knn_emit_rows_kernel: wave per row (below).
constexpr int KNN_LDS_MAXN = 512, KNN_W = KNN_LDS_MAXN / 64;

__device__ __forceinline__ int ballot_count(bool p) { return __popcll(__ballot(p)); }

__global__ __launch_bounds__(1024) void knn_select_kernel(KnnDist dist,
                                                          const int64_t* __restrict__ node_off, int B,
                                                          int64_t n_total, int kq,
                                                          unsigned long long* __restrict__ Arow) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  if (g >= n_total) return;
  const int b = find_segment(node_off, B, g);
  const int64_t base = node_off[b];
  const int n = (int)(node_off[b + 1] - base), i = (int)(g - base);
  const int wpr = (n + 63) / 64;
  long long d[KNN_W];
  long long dmax = 0;
#pragma unroll
  for (int r = 0; r < KNN_W; ++r) {
    const int j = lane + 64 * r;
    d[r] = 0x7fffffffffffffffll;
    if (r < wpr && j < n) {
      d[r] = dist(base, b, n, i, j);
      dmax = max(dmax, d[r]);
    }
  }
  long long tau = 0x7fffffffffffffffll;
  int need = 0;   // n <= kq: every node is among the k+1 nearest
  if (n > kq) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) dmax = max(dmax, (long long)__shfl_xor(dmax, off));
    long long lo = 0, hi = dmax;   // smallest tau with #{d <= tau} >= kq
    while (lo < hi) {
      const long long mid = lo + (hi - lo) / 2;
      int c = 0;
      for (int r = 0; r < wpr; ++r) c += ballot_count(d[r] <= mid);
      if (c >= kq) hi = mid; else lo = mid + 1;
    }
    tau = lo;
    int less = 0;
    for (int r = 0; r < wpr; ++r) less += ballot_count(d[r] < tau);
    need = kq - less;
  }
  int ties_before = 0;   // ties at lower indices (j = lane + 64 r: r-major, then lane)
  for (int r = 0; r < wpr; ++r) {
    const int j = lane + 64 * r;
    bool take = j < n && d[r] <= tau;
    if (n > kq) {
      const unsigned long long tm = __ballot(d[r] == tau);
      const int rank = ties_before + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(tm >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((unsigned)tm, 0u));
      if (d[r] == tau) take = rank < need;
      ties_before += __popcll(tm);
    }
    const unsigned long long word = __ballot(take && j != i);
    if (lane == 0) Arow[g * KNN_W + r] = word;
  }
}

__global__ __launch_bounds__(1024) void knn_rows_kernel(const int64_t* __restrict__ node_off,
                                                        const unsigned long long* __restrict__ Arow,
                                                        unsigned long long* __restrict__ R, int* __restrict__ rowstart,
                                                        int64_t* __restrict__ ecount) {
  __shared__ unsigned long long T[KNN_LDS_MAXN * KNN_W];
  __shared__ int wsum[16];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t base = node_off[b];
  const int n = (int)(node_off[b + 1] - base);
  const int wpr = (n + 63) / 64;
  for (int t = tid; t < n * KNN_W; t += 1024) T[t] = 0ull;
  __syncthreads();
  for (int t = tid; t < n * wpr; t += 1024) {   // T[j] |= bit i for every j in A[i]
    const int i = t / wpr, w = t - i * wpr;
    unsigned long long word = Arow[(base + i) * KNN_W + w];
    while (word) {
      const int j = 64 * w + __builtin_ctzll(word);
      word &= word - 1;
      atomicOr(&T[j * KNN_W + (i >> 6)], 1ull << (i & 63));
    }
  }
  __syncthreads();
  int deg = 0;
  if (tid < n) {
    for (int w = 0; w < wpr; ++w) {
      const unsigned long long v = Arow[(base + tid) * KNN_W + w] | T[tid * KNN_W + w];
      R[(base + tid) * KNN_W + w] = v;
      deg += __popcll(v);
    }
  }
  int x = deg;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(x, off);
    if (lane >= off) x += o;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int pre = 0;
  for (int w = 0; w < wave; ++w) pre += wsum[w];
  if (tid < n) rowstart[base + tid] = pre + x - deg;
  if (tid == 1023) ecount[b] = pre + x;
}

// Wave per row: the row's edges (src = the row, dst ascending) at image base + row prefix; the
// destination row of edge_index starts at the batch total. With edge_attr != NULL the wave also writes
// the edges' features (edge_features_kernel's values), staged in LDS so that each word's edges leave
// as one contiguous range. Block (0, 0) publishes the total (edge_off[B], the mapped host word).
struct KnnEmitArgs {
  const int64_t* node_off;
  int B;
  const unsigned long long* R;
  const int* rowstart;
  const int64_t* ecount;
  int64_t e_cap;
  int64_t* edge_off;
  int* e_host;
  int64_t* ei;
  // edge features (ConstructGraph.py:289-357)
  const int64_t* jdet;
  const float* jtag;
  int F;
  const float* jsc;
  int J, mode, A;
  float norm;
  float* edge_attr;
};

__global__ __launch_bounds__(1024) void knn_emit_rows_kernel(KnnEmitArgs k) {
  __shared__ long long red[2][16];
  __shared__ float fdx[16][64], fdy[16][64], faux[16][64];
  __shared__ int fts[16][64], ftd[16][64];
  __shared__ int nx[KNN_LDS_MAXN], ny[KNN_LDS_MAXN], nt[KNN_LDS_MAXN];   // the image's nodes (features)
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, B = k.B;
  long long before = 0, all = 0;
  for (int q = tid; q < B; q += 1024) {
    const long long e = k.ecount[q];
    all += e;
    if (q < b) before += e;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    before += __shfl_xor(before, off);
    all += __shfl_xor(all, off);
  }
  if (lane == 0) { red[0][wave] = before; red[1][wave] = all; }
  __syncthreads();
  before = 0; all = 0;
  for (int w = 0; w < 16; ++w) { before += red[0][w]; all += red[1][w]; }
  if (b == 0 && blockIdx.y == 0 && tid == 0) {
    k.edge_off[B] = all;
    if (k.e_host) __hip_atomic_store(k.e_host, (int)(all < 0x7fffffffll ? all : 0x7fffffffll), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (all > k.e_cap) return;   // reported by the host
  const int64_t base = k.node_off[b];
  const int n = (int)(k.node_off[b + 1] - base);
  if (k.edge_attr) {   // (uniform) node coordinates and types once per block
    for (int t = tid; t < n; t += 1024) {
      nx[t] = (int)k.jdet[(base + t) * 3];
      ny[t] = (int)k.jdet[(base + t) * 3 + 1];
      nt[t] = (int)k.jdet[(base + t) * 3 + 2];
    }
    __syncthreads();
  }
  const int a = blockIdx.y * 16 + wave;
  if (a >= n) return;
  const int wpr = (n + 63) / 64;
  const int64_t src = base + a;
  int64_t pos = before + k.rowstart[src];
  int64_t sx = 0, sy = 0;
  int ts = 0;
  float tsrc = 0.f;
  if (k.edge_attr) { sx = nx[a]; sy = ny[a]; ts = nt[a]; }
  for (int w = 0; w < wpr; ++w) {
    const unsigned long long word = k.R[src * KNN_W + w];
    const int cnt = __popcll(word);
    const int r = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(word >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)word, 0u));
    const bool has = (word >> lane) & 1ull;
    const int64_t dst = base + 64 * w + lane;
    if (has) {
      k.ei[pos + r] = src;
      k.ei[all + pos + r] = dst;
    }
    if (k.edge_attr) {   // (uniform)
      if (has) {
        const int jl = 64 * w + lane;
        const int64_t dx = nx[jl], dy = ny[jl];
        fdx[wave][r] = (float)(dx - sx) / k.norm;             // ConstructGraph.py:311-317 (IEEE division)
        fdy[wave][r] = (float)(dy - sy) / k.norm;
        fts[wave][r] = ts;
        ftd[wave][r] = nt[jl];
        if (k.mode == PEMP_EF_POSITION_ANGLE_CONNECTION) faux[wave][r] = edge_theta(sx, sy, dx, dy);
        else if (ef_uses_tags(k.mode))
          faux[wave][r] = ae_term(k.mode, tag_distance(k.jtag + src * k.F, k.jtag + dst * k.F, k.F), k.jsc[src]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float* o = k.edge_attr + pos * k.A;
      for (int q = lane; q < cnt * k.A; q += 64) {
        const int el = q / k.A, f = q - el * k.A;
        o[q] = ef_value(k.mode, f, k.J, fdx[wave][el], fdy[wave][el], faux[wave][el], fts[wave][el], ftd[wave][el]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    pos += cnt;
  }
}

// edge_off = exclusive scan of ecount, edge_off[B] = total; the total also goes straight into the
// caller's mapped host word (system-scope store), like pemp_detect's counts
__global__ __launch_bounds__(64) void knn_offsets_kernel(const int64_t* __restrict__ ecount, int B,
                                                         int64_t* __restrict__ edge_off, int* __restrict__ e_host) {
  const int lane = threadIdx.x;
  long long c = 0;
  for (int c0 = 0; c0 < B; c0 += 64) {
    const int b = c0 + lane;
    const long long e = b < B ? ecount[b] : 0;
    long long x = e;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const long long o = __shfl_up(x, off);
      if (lane >= off) x += o;
    }
    if (b < B) edge_off[b] = c + x - e;
    c += __shfl(x, 63);
  }
  if (lane == 0) {
    edge_off[B] = c;
    if (e_host) __hip_atomic_store(e_host, (int)(c < 0x7fffffffll ? c : 0x7fffffffll), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static int grid_for(int64_t total, int block, int cap_blocks = 65536) {
  int64_t g = (total + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap_blocks) g = cap_blocks;
  return (int)g;
}

}  // namespace
}  // namespace pemp

using namespace pemp;

extern "C" int pemp_pack_nodes(const float* features, int C, const float* tagmaps, int F, int B, int J, int H, int W,
                               const int64_t* det_xyt, const float* det_scores, int cap, const int64_t* node_off,
                               int64_t n_total, float* x, int64_t* joint_det, float* joint_scores,
                               int64_t* batch_index, float* joint_tags, void* stream) {
  PEMP_CHECK_ARG(det_xyt && det_scores && node_off && x && joint_det && joint_scores && batch_index,
                 "pemp_pack_nodes: null pointer");
  PEMP_CHECK_ARG(C > 0 && B > 0 && J > 0 && H > 0 && W > 0 && n_total >= 0, "pemp_pack_nodes: bad shape");
  PEMP_CHECK_ARG(!tagmaps || (joint_tags && F > 0 && F <= C), "pemp_pack_nodes: tags need F in [1, C]");
  if (n_total == 0) return PEMP_OK;
  ProfScope prof("pack_nodes", as_stream(stream));
  hipLaunchKernelGGL(pack_nodes_kernel, dim3(grid_for(n_total * C, 256)), dim3(256), 0, as_stream(stream), features,
                     C, tagmaps, F, B, J, H, W, det_xyt, det_scores, cap, node_off, n_total, x, joint_det,
                     joint_scores, batch_index, joint_tags);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

namespace pemp {
namespace {
constexpr int FUSED_MAXB = 1024;   // images per batch handled by the fused build (offsets in LDS)

struct FusedGraphArgs {
  const int32_t* n_det;
  int B, cap, C, F, J, H, W, mode, A;
  const int64_t* det;
  const float *det_sc, *feat, *tags;
  float norm;
  int64_t n_total, e_total;   // exact totals, or capacities (capacity mode)
  int capacity;               // 1: totals come from n_det on the device; nothing is written if they exceed
  int write_counts;           // capacity mode, PEMP_BUILD_WRITE_COUNTS: (N, E, overflow) at node_off_out[B + 1 ..]
  int node_blocks;
  float *x, *jsc, *jtag, *edge_attr;
  int64_t *jdet, *bidx, *ei;
  int64_t* node_off_out;      // [B + 1] or NULL
  uint32_t mC, mA;            // unsigned division by C and by A for dividends below 2^31 (graph_fastdiv)
  int lC, lA;
};


// One launch for the whole fully-connected graph after the count read-back: every block derives
// the per-image node / edge offsets from n_det in LDS; blocks [0, node_blocks) pack nodes
// (pack_nodes_kernel), the rest emit 256 edges each: (src, dst) of the fully graph
// (fully_graph_kernel) and their edge_attr rows (edge_features_kernel), the endpoints read
// straight from the detections.
__global__ __launch_bounds__(256) void fused_fully_graph_kernel(FusedGraphArgs a) {
  __shared__ long long noff[FUSED_MAXB + 1], eoff[FUSED_MAXB + 1];
  __shared__ float dx_s[256], dy_s[256], aux_s[256];
  __shared__ int ts_s[256], td_s[256];
  __shared__ int over_cap;
  const int B = a.B;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    long long cn = 0, ce = 0;
    int over = 0;
    for (int c0 = 0; c0 < B; c0 += 64) {
      const int b = c0 + lane;
      const long long n = b < B ? a.n_det[b] : 0, e = n * (n > 0 ? n - 1 : 0);
      over |= n > a.cap;   // an image with more detections than the detection buffer holds
      long long xn = n, xe = e;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const long long on = __shfl_up(xn, off), oe = __shfl_up(xe, off);
        if (lane >= off) { xn += on; xe += oe; }
      }
      if (b < B) { noff[b] = cn + xn - n; eoff[b] = ce + xe - e; }
      cn += __shfl(xn, 63);
      ce += __shfl(xe, 63);
    }
    over = __any(over);
    if (lane == 0) { noff[B] = cn; eoff[B] = ce; over_cap = over; }
  }
  __syncthreads();
  // capacity mode (launched before the host has read the counts back): device totals; a batch that
  // does not fit (totals over the capacities, or an image over the detection cap: its detections past
  // the cap were never written) writes nothing and the host rebuilds it with exact sizes
  const int64_t n_total = a.capacity ? (int64_t)noff[B] : a.n_total;
  const int64_t e_total = a.capacity ? (int64_t)eoff[B] : a.e_total;
  if (a.write_counts && blockIdx.x == 0 && threadIdx.x == 0) {   // (N, E, overflow) for the capacity-mode MPN
    const bool over = n_total > a.n_total || e_total > a.e_total || over_cap;
    a.node_off_out[B + 1] = over ? 0 : n_total;
    a.node_off_out[B + 2] = over ? 0 : e_total;
    a.node_off_out[B + 3] = over ? 1 : 0;
  }
  if (a.capacity && (n_total > a.n_total || e_total > a.e_total || over_cap)) return;
  if (a.node_off_out && blockIdx.x == 0)   // per-image node offsets for pemp_mpn_forward_fully
    for (int i = threadIdx.x; i <= B; i += blockDim.x) a.node_off_out[i] = noff[i];
  auto seg = [&](const long long* off, long long v) {
    int lo = 0, hi = B - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off[mid] <= v) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  if ((int)blockIdx.x < a.node_blocks) {   // ---- nodes ----
    // (32-bit index arithmetic: the host takes this kernel only for n_total * C < 2^30)
    const int total = (int)(n_total * a.C);
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += a.node_blocks * 256) {
      const int g = graph_fastdiv(idx, a.mC, a.lC);
      const int c = idx - g * a.C;
      const int b = seg(noff, g);
      const int64_t i = g - noff[b];
      const int64_t* d = a.det + ((size_t)b * a.cap + i) * 3;
      const int64_t px = d[0], py = d[1], pt = d[2];
      if (a.feat) a.x[idx] = a.feat[(((size_t)b * a.C + c) * a.H + py) * a.W + px];
      if (c == 0) {
        a.jdet[g * 3 + 0] = px; a.jdet[g * 3 + 1] = py; a.jdet[g * 3 + 2] = pt;
        a.jsc[g] = a.det_sc[(size_t)b * a.cap + i];
        a.bidx[g] = b;
      }
      if (a.tags && c < a.F) a.jtag[g * a.F + c] = a.tags[((((size_t)b * a.J + pt) * a.H + py) * a.W + px) * a.F + c];
    }
    return;
  }
  // ---- edges ----
  const int eb = blockIdx.x - a.node_blocks, nbe = gridDim.x - a.node_blocks;
  for (int64_t base = (int64_t)eb * 256; base < e_total; base += (int64_t)nbe * 256) {
    const int64_t e = base + threadIdx.x;
    if (e < e_total) {
      const int b = seg(eoff, e);
      const int64_t n = noff[b + 1] - noff[b];
      const int64_t el = e - eoff[b];
      int64_t i, r;
      if (n <= 46340) {   // the image's n (n - 1) edges below 2^31: 32-bit division (the 64-bit one is ~10x longer)
        const unsigned nm1 = (unsigned)(n - 1), iu = (unsigned)el / nm1;
        i = iu;
        r = (unsigned)el - iu * nm1;
      } else {
        i = el / (n - 1);
        r = el - i * (n - 1);
      }
      const int64_t j = r < i ? r : r + 1;                 // all (i, j), i != j, sorted by (i, j)
      a.ei[e] = noff[b] + i;
      a.ei[e_total + e] = noff[b] + j;
      const int64_t* ds = a.det + ((size_t)b * a.cap + i) * 3;   // source = edge_index[0]
      const int64_t* dd = a.det + ((size_t)b * a.cap + j) * 3;   // target = edge_index[1]
      const int64_t sx = ds[0], sy = ds[1], dx = dd[0], dy = dd[1];
      dx_s[threadIdx.x] = (float)(dx - sx) / a.norm;            // ConstructGraph.py:311-317
      dy_s[threadIdx.x] = (float)(dy - sy) / a.norm;
      ts_s[threadIdx.x] = (int)ds[2];
      td_s[threadIdx.x] = (int)dd[2];
      if (a.mode == PEMP_EF_POSITION_ANGLE_CONNECTION) {
        aux_s[threadIdx.x] = edge_theta(sx, sy, dx, dy);
      } else if (ef_uses_tags(a.mode)) {   // tags straight from the tag maps [B, J, H, W, F]
        const float* tg = a.tags + (size_t)b * a.J * a.H * a.W * a.F;
        const float* t_s = tg + (((size_t)ds[2] * a.H + sy) * a.W + sx) * a.F;
        const float* t_d = tg + (((size_t)dd[2] * a.H + dy) * a.W + dx) * a.F;
        aux_s[threadIdx.x] = ae_term(a.mode, tag_distance(t_s, t_d, a.F), a.det_sc[(size_t)b * a.cap + i]);
      }
    }
    __syncthreads();
    const int cnt = (int)min<int64_t>(256, e_total - base), total = cnt * a.A;
    float* o = a.edge_attr + base * a.A;
    for (int k = threadIdx.x; k < total; k += 256) {
      const int el = graph_fastdiv(k, a.mA, a.lA), f = k - el * a.A;
      o[k] = ef_value(a.mode, f, a.J, dx_s[el], dy_s[el], aux_s[el], ts_s[el], td_s[el]);
    }
    __syncthreads();
  }
}
}  // namespace
}  // namespace pemp

static int ef_width(int mode, int J) {
  switch (mode) {
    case PEMP_EF_POSITION_CONNECTION: return J + 2;
    case PEMP_EF_CONNECTION: return J;
    case PEMP_EF_NOTHING: return 1;
    case PEMP_EF_POSITION: return 2;
    case PEMP_EF_POSITION_ANGLE_CONNECTION: return J + 3;
    case PEMP_EF_POSITION_CONNECTION_AE: return J + 3;
    case PEMP_EF_AE: case PEMP_EF_AE_NORMED: case PEMP_EF_AE_TRACKING: return 1;
    default: return -1;
  }
}

// The associative-embedding modes need the tags; F = 1 or 2 (torch.norm's rounding is pinned for
// those); ae needs F = 1 and ae_normed F = 2 (the reference fails otherwise, :337-341).
static int ef_tag_check(int mode, const float* tags, int F, const char* fn) {
  if (mode != PEMP_EF_POSITION_CONNECTION_AE && mode != PEMP_EF_AE && mode != PEMP_EF_AE_NORMED &&
      mode != PEMP_EF_AE_TRACKING)
    return 0;
  if (!tags) { set_error("%s: edge feature mode %d needs the tags", fn, mode); return PEMP_ERR_INVALID_ARG; }
  if (F < 1 || F > 2 || (mode == PEMP_EF_AE && F != 1) || (mode == PEMP_EF_AE_NORMED && F != 2)) {
    set_error("%s: edge feature mode %d with %d tag dims is not supported", fn, mode, F);
    return PEMP_ERR_UNSUPPORTED;
  }
  return 0;
}

static int fully_graph_build(const int32_t* n_det, int B, const int64_t* det_xyt, const float* det_scores, int cap,
                             const float* features, int C, const float* tagmaps, int F, int J, int H, int W,
                             int64_t n_total, int64_t e_total, float norm_factor, int mode, float* x,
                             int64_t* joint_det, float* joint_scores, int64_t* batch_index, float* joint_tags,
                             int64_t* edge_index, float* edge_attr, int64_t* node_off_out, int capacity, void* stream);

extern "C" int pemp_fully_graph_build(const int32_t* n_det, int B, const int64_t* det_xyt, const float* det_scores,
                                      int cap, const float* features, int C, const float* tagmaps, int F, int J,
                                      int H, int W, int64_t n_total, int64_t e_total, float norm_factor, int mode,
                                      float* x, int64_t* joint_det, float* joint_scores, int64_t* batch_index,
                                      float* joint_tags, int64_t* edge_index, float* edge_attr, int64_t* node_off,
                                      void* stream) {
  return fully_graph_build(n_det, B, det_xyt, det_scores, cap, features, C, tagmaps, F, J, H, W, n_total, e_total,
                           norm_factor, mode, x, joint_det, joint_scores, batch_index, joint_tags, edge_index,
                           edge_attr, node_off, 0, stream);
}

extern "C" int pemp_fully_graph_build_cap(const int32_t* n_det, int B, const int64_t* det_xyt, const float* det_scores,
                                          int cap, const float* features, int C, const float* tagmaps, int F, int J,
                                          int H, int W, int64_t n_cap, int64_t e_cap, float norm_factor, int mode,
                                          float* x, int64_t* joint_det, float* joint_scores, int64_t* batch_index,
                                          float* joint_tags, int64_t* edge_index, float* edge_attr,
                                          int64_t* node_off, void* stream) {
  return fully_graph_build(n_det, B, det_xyt, det_scores, cap, features, C, tagmaps, F, J, H, W, n_cap, e_cap,
                           norm_factor, mode, x, joint_det, joint_scores, batch_index, joint_tags, edge_index,
                           edge_attr, node_off, 1, stream);
}

static int fully_graph_build(const int32_t* n_det, int B, const int64_t* det_xyt, const float* det_scores, int cap,
                             const float* features, int C, const float* tagmaps, int F, int J, int H, int W,
                             int64_t n_total, int64_t e_total, float norm_factor, int mode, float* x,
                             int64_t* joint_det, float* joint_scores, int64_t* batch_index, float* joint_tags,
                             int64_t* edge_index, float* edge_attr, int64_t* node_off_out, int capacity,
                             void* stream) {
  PEMP_CHECK_ARG(n_det && det_xyt && det_scores && x && joint_det && joint_scores && batch_index,
                 "pemp_fully_graph_build: null pointer");
  PEMP_CHECK_ARG(B > 0 && B <= FUSED_MAXB && C > 0 && J > 0 && H > 0 && W > 0 && n_total >= 0 && e_total >= 0,
                 "pemp_fully_graph_build: bad shape (B must be in [1, %d])", FUSED_MAXB);
  PEMP_CHECK_ARG(!tagmaps || (joint_tags && F > 0 && F <= C), "pemp_fully_graph_build: tags need F in [1, C]");
  PEMP_CHECK_ARG(e_total == 0 || (edge_index && edge_attr), "pemp_fully_graph_build: null edge outputs");
  const int write_counts = (mode & PEMP_BUILD_WRITE_COUNTS) ? 1 : 0;
  mode &= ~PEMP_BUILD_WRITE_COUNTS;
  PEMP_CHECK_ARG(!write_counts || (capacity && node_off_out),
                 "pemp_fully_graph_build: PEMP_BUILD_WRITE_COUNTS needs the capacity build and node_off");
  const int A = ef_width(mode, J);
  if (A < 0) { set_error("pemp_fully_graph_build: unknown edge feature mode %d", mode); return PEMP_ERR_INVALID_ARG; }
  if (const int rc = ef_tag_check(mode, tagmaps, F, "pemp_fully_graph_build")) return rc;
  if (n_total == 0) return PEMP_OK;
  FusedGraphArgs a{};
  a.n_det = n_det; a.B = B; a.cap = cap; a.C = C; a.F = F; a.J = J; a.H = H; a.W = W; a.mode = mode; a.A = A;
  a.det = det_xyt; a.det_sc = det_scores; a.feat = features; a.tags = tagmaps; a.norm = norm_factor;
  a.n_total = n_total; a.e_total = e_total; a.capacity = capacity; a.write_counts = write_counts;
  a.node_blocks = grid_for(n_total * C, 256, 4096);
  const int edge_blocks = e_total > 0 ? grid_for(e_total, 256, 8192) : 0;
  a.x = x; a.jsc = joint_scores; a.jtag = joint_tags; a.edge_attr = edge_attr;
  a.jdet = joint_det; a.bidx = batch_index; a.ei = edge_index; a.node_off_out = node_off_out;
  // the kernel's 32-bit node index arithmetic (below 2^30 elements)
  PEMP_CHECK_ARG(n_total * (int64_t)C < ((int64_t)1 << 30),
                 "pemp_fully_graph_build: %lld nodes x %d features past the 32-bit range", (long long)n_total, C);
  graph_fastdiv_consts((unsigned)C, a.mC, a.lC);
  graph_fastdiv_consts((unsigned)A, a.mA, a.lA);
  ProfScope prof("graph_build", as_stream(stream));
  hipLaunchKernelGGL(fused_fully_graph_kernel, dim3(a.node_blocks + edge_blocks), dim3(256), 0, as_stream(stream), a);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

namespace pemp {
namespace {
// node_off[b] = sum_{b'<b} n_det[b'], fully_edge_off[b] = sum_{b'<b} n (n - 1): one wave, chunks of 64
__global__ __launch_bounds__(64) void graph_offsets_kernel(const int32_t* __restrict__ n_det, int B,
                                                           int64_t* __restrict__ node_off,
                                                           int64_t* __restrict__ edge_off) {
  const int lane = threadIdx.x;
  long long cn = 0, ce = 0;
  for (int c0 = 0; c0 < B; c0 += 64) {
    const int b = c0 + lane;
    const long long n = b < B ? n_det[b] : 0, e = n * (n > 0 ? n - 1 : 0);
    long long xn = n, xe = e;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const long long on = __shfl_up(xn, off), oe = __shfl_up(xe, off);
      if (lane >= off) { xn += on; xe += oe; }
    }
    if (b < B) {
      node_off[b] = cn + xn - n;
      if (edge_off) edge_off[b] = ce + xe - e;
    }
    cn += __shfl(xn, 63);
    ce += __shfl(xe, 63);
  }
  if (lane == 0) {
    node_off[B] = cn;
    if (edge_off) edge_off[B] = ce;
  }
}
// ---- node features sampled from projected maps -----------------------------
// The test front-end projects every scale's gathered features to the image size
// (PoseEstimation.py:426-452: interpolate(bilinear, align_corners=False)), sums the scales and
// divides by their count (multi_scales_testing.py:182-190, PoseEstimation.py:244), then
// construct_graph reads x = features[:, y, x].T. Here only the N detections are interpolated:
// nothing of size [C, H, W] is materialised. Source index as torch's area_pixel_compute_source_index:
// s = (h / H) * (y + 0.5) - 0.5 clamped at 0, y1 = y0 + (y0 < h - 1), weights 1 - l, l.
constexpr int PROJ_MAXS = 8;
struct ProjMaps {
  const float* p[PROJ_MAXS];   // [B][C][h_s][w_s]
  int h[PROJ_MAXS], w[PROJ_MAXS];
  int S;
};

__device__ __forceinline__ void proj_src(int dst, int out_size, int in_size, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in_size / (float)out_size;
  float src = __fsub_rn(__fmul_rn(scale, __fadd_rn((float)dst, 0.5f)), 0.5f);
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  i1 = i0 + (i0 < in_size - 1 ? 1 : 0);
  l1 = fminf(fmaxf(__fsub_rn(src, (float)i0), 0.f), 1.f);
  l0 = __fsub_rn(1.f, l1);
}

__global__ __launch_bounds__(256) void gather_projected_kernel(ProjMaps m, int C, int H, int W, float divisor,
                                                               const int64_t* __restrict__ jdet,
                                                               const int64_t* __restrict__ bidx, int64_t N,
                                                               float* __restrict__ x) {
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < N * C;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = idx / C;
    const int c = (int)(idx - n * C);
    const int px = (int)jdet[n * 3 + 0], py = (int)jdet[n * 3 + 1];
    const int64_t b = bidx[n];
    float acc = 0.f;
    for (int s = 0; s < m.S; ++s) {
      const int h = m.h[s], w = m.w[s];
      int y0, y1, x0, x1;
      float ly0, ly1, lx0, lx1;
      proj_src(py, H, h, y0, y1, ly0, ly1);
      proj_src(px, W, w, x0, x1, lx0, lx1);
      const float* pl = m.p[s] + ((size_t)b * C + c) * h * w;
      const float t0 = __fadd_rn(__fmul_rn(pl[y0 * w + x0], lx0), __fmul_rn(pl[y0 * w + x1], lx1));
      const float t1 = __fadd_rn(__fmul_rn(pl[y1 * w + x0], lx0), __fmul_rn(pl[y1 * w + x1], lx1));
      const float v = __fadd_rn(__fmul_rn(t0, ly0), __fmul_rn(t1, ly1));
      acc = s == 0 ? v : __fadd_rn(acc, v);
    }
    x[idx] = div_rn(acc, divisor);
  }
}

// The same projection with the model's feature_gather Conv2d in front of it (PoseEstimation.py:64-66, 341,
// 426-452: interpolate(feature_gather(feat)) per scale): the conv output is needed only at the 4 bilinear taps
// of each detection, so one workgroup per detection stages the (k+1) x (k+1) x Cin input patch under the taps
// in LDS (zero padding outside the map) and each thread computes the 4 tap values of its output channels
// (weights transposed on the host to [Cin][k][k][Cout]: one coalesced load per tap weight).
constexpr int PCONV_THREADS = 128, PCONV_MAXQ = 4;   // Cout <= 512
__global__ __launch_bounds__(PCONV_THREADS) void gather_projected_conv_kernel(
    ProjMaps m, const float* __restrict__ wt, const float* __restrict__ bias, int Cin, int Cout, int k, int pad, int H,
    int W, float divisor, const int64_t* __restrict__ jdet, const int64_t* __restrict__ bidx, float* __restrict__ x) {
  extern __shared__ float patch[];   // [Cin][P][P]
  const int P = k + 1, PP = P * P, tid = threadIdx.x;
  const int64_t n = blockIdx.x;
  const int px = (int)jdet[n * 3 + 0], py = (int)jdet[n * 3 + 1];
  const int64_t b = bidx[n];
  float acc[PCONV_MAXQ] = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < m.S; ++s) {
    const int h = m.h[s], w = m.w[s], ho = h + 2 * pad - k + 1, wo = w + 2 * pad - k + 1;
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    proj_src(py, H, ho, y0, y1, ly0, ly1);
    proj_src(px, W, wo, x0, x1, lx0, lx1);
    const int dy1 = y1 - y0, dx1 = x1 - x0;
    const float* f = m.p[s] + (size_t)b * Cin * h * w;
    __syncthreads();   // the previous scale's patch is consumed
    for (int i = tid; i < Cin * PP; i += PCONV_THREADS) {
      const int ci = i / PP, r = (i - ci * PP) / P, q = i - ci * PP - r * P;
      const int yy = y0 - pad + r, xx = x0 - pad + q;
      patch[i] = (yy >= 0 && yy < h && xx >= 0 && xx < w) ? f[((size_t)ci * h + yy) * w + xx] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PCONV_MAXQ; ++q) {
      const int co = tid + PCONV_THREADS * q;
      if (co >= Cout) break;
      float c00 = 0.f, c01 = 0.f, c10 = 0.f, c11 = 0.f;
      const float* wp = wt + co;
      for (int ci = 0; ci < Cin; ++ci)
        for (int dy = 0; dy < k; ++dy) {
          const float* pr = patch + ci * PP + dy * P;
          for (int dx = 0; dx < k; ++dx, wp += Cout) {
            const float wv = *wp;
            c00 = fmaf(wv, pr[dx], c00);
            c01 = fmaf(wv, pr[dx + dx1], c01);
            c10 = fmaf(wv, pr[dx + dy1 * P], c10);
            c11 = fmaf(wv, pr[dx + dy1 * P + dx1], c11);
          }
        }
      const float bb = bias ? bias[co] : 0.0f;
      c00 += bb; c01 += bb; c10 += bb; c11 += bb;
      const float t0 = __fadd_rn(__fmul_rn(c00, lx0), __fmul_rn(c01, lx1));
      const float t1 = __fadd_rn(__fmul_rn(c10, lx0), __fmul_rn(c11, lx1));
      const float v = __fadd_rn(__fmul_rn(t0, ly0), __fmul_rn(t1, ly1));
      acc[q] = s == 0 ? v : __fadd_rn(acc[q], v);
    }
  }
#pragma unroll
  for (int q = 0; q < PCONV_MAXQ; ++q) {
    const int co = tid + PCONV_THREADS * q;
    if (co < Cout) x[n * Cout + co] = div_rn(acc[q], divisor);
  }
}

// ---- score_based_graph (ConstructGraph.py:405-422) -------------------------------------------
// Roots are the k best-scoring nodes of an image (ties: lower node index). Edge (a, b), a != b,
// exists iff a or b is a root, sorted by (a, b): a root row lists every other node, a non-root row
// lists the roots in index order. Row a starts at  a*k + roots_before(a)*(n-1-k)  in its image.
constexpr int SCORE_LDS = 8192;   // scores of an image staged in LDS up to this many nodes

struct ScoreWs {
  int* rinfo;     // [N]    2 * roots_before(node) + is_root
  int* roots;     // [B*k]  local indices of the roots, ascending
  int64_t* eoff;  // [B]    first edge of each image
};

inline size_t score_ws_bytes(int64_t n_total, int B, int k) {
  return align_up((size_t)n_total * 4, 256) + align_up((size_t)B * k * 4, 256) + align_up((size_t)B * 8, 256);
}

inline ScoreWs score_carve(void* ws, int64_t n_total, int B, int k) {
  char* p = static_cast<char*>(ws);
  ScoreWs w;
  w.rinfo = reinterpret_cast<int*>(p); p += align_up((size_t)n_total * 4, 256);
  w.roots = reinterpret_cast<int*>(p); p += align_up((size_t)B * k * 4, 256);
  w.eoff = reinterpret_cast<int64_t*>(p);
  return w;
}

__global__ __launch_bounds__(256) void score_roots_kernel(const float* __restrict__ scores,
                                                          const int64_t* __restrict__ node_off, int B, int k,
                                                          ScoreWs w) {
  __shared__ float sl[SCORE_LDS];
  __shared__ int wcnt[4];
  __shared__ int64_t wsum[4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t base = node_off[b];
  const int n = (int)(node_off[b + 1] - base);
  // first edge of this image: sum over the images before it of k (2 n - k - 1)
  int64_t acc = 0;
  for (int q = threadIdx.x; q < b; q += 256) {
    const int64_t m = node_off[q + 1] - node_off[q];
    acc += m > 0 ? (int64_t)k * (2 * m - k - 1) : 0;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor((long long)acc, off);
  if (lane == 0) wsum[wave] = acc;
  const float* s = scores + base;
  const bool in_lds = n <= SCORE_LDS;
  if (in_lds)
    for (int i = threadIdx.x; i < n; i += 256) sl[i] = s[i];
  __syncthreads();
  if (threadIdx.x == 0) w.eoff[b] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  const float* sv = in_lds ? sl : s;
  int carry = 0;
  for (int i0 = 0; i0 < n; i0 += 256) {
    const int i = i0 + threadIdx.x;
    bool root = false;
    if (i < n) {
      const float si = sv[i];
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        const float sj = sv[j];
        rank += (sj > si) || (sj == si && j < i);
      }
      root = rank < k;
    }
    const unsigned long long m = __ballot(root);
    const int pos = __popcll(m & ((1ull << lane) - 1));
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int pre = carry;
    for (int q = 0; q < wave; ++q) pre += wcnt[q];
    pre += pos;
    if (i < n) {
      w.rinfo[base + i] = 2 * pre + (root ? 1 : 0);
      if (root) w.roots[(int64_t)b * k + pre] = i;
    }
    carry += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
}

// one wave per row; consecutive lanes write consecutive edges
__global__ __launch_bounds__(256) void score_emit_kernel(const int64_t* __restrict__ node_off, int B, int k,
                                                         const ScoreWs w, int64_t n_total, int64_t e_total,
                                                         int64_t* __restrict__ ei) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n_total; r += stride) {
    const int b = find_segment(node_off, B, r);
    const int64_t base = node_off[b];
    const int n = (int)(node_off[b + 1] - base), i = (int)(r - base);
    const int v = w.rinfo[r];
    const bool root = v & 1;
    const int64_t e0 = w.eoff[b] + (int64_t)i * k + (int64_t)(v >> 1) * (n - 1 - k);
    const int cnt = root ? n - 1 : k;
    const int* rl = w.roots + (int64_t)b * k;
    for (int c = lane; c < cnt; c += 64) {
      const int col = root ? c + (c >= i) : rl[c];
      ei[e0 + c] = r;
      ei[e_total + e0 + c] = base + col;
    }
  }
}

}  // namespace
}  // namespace pemp

extern "C" int pemp_graph_offsets(const int32_t* n_det, int B, int64_t* node_off, int64_t* fully_edge_off,
                                  void* stream) {
  PEMP_CHECK_ARG(n_det && node_off && B > 0, "pemp_graph_offsets: bad args");
  hipLaunchKernelGGL(graph_offsets_kernel, dim3(1), dim3(64), 0, as_stream(stream), n_det, B, node_off,
                     fully_edge_off);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

extern "C" int pemp_fully_graph(const int64_t* node_off, const int64_t* edge_off, int B, int64_t e_total,
                                int64_t* edge_index, void* stream) {
  PEMP_CHECK_ARG(node_off && edge_off && edge_index && B > 0 && e_total >= 0, "pemp_fully_graph: bad args");
  if (e_total == 0) return PEMP_OK;
  ProfScope prof("fully_graph", as_stream(stream));
  hipLaunchKernelGGL(fully_graph_kernel, dim3(grid_for(e_total, 256)), dim3(256), 0, as_stream(stream), node_off,
                     edge_off, B, e_total, edge_index);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

extern "C" int pemp_edge_features(const int64_t* joint_det, const float* joint_tags, int F, const float* joint_scores,
                                  const int64_t* edge_index, int64_t e_total, int J, float norm_factor, int mode,
                                  float* edge_attr, void* stream) {
  PEMP_CHECK_ARG(joint_det && edge_index && edge_attr && J > 0 && e_total >= 0, "pemp_edge_features: bad args");
  const int A = ef_width(mode, J);
  if (A < 0) { set_error("pemp_edge_features: unknown mode %d", mode); return PEMP_ERR_INVALID_ARG; }
  if (const int rc = ef_tag_check(mode, joint_tags, F, "pemp_edge_features")) return rc;
  PEMP_CHECK_ARG(mode != PEMP_EF_AE_NORMED || joint_scores, "pemp_edge_features: ae_normed needs joint_scores");
  if (e_total == 0) return PEMP_OK;
  ProfScope prof("edge_features", as_stream(stream));
  hipLaunchKernelGGL(edge_features_kernel, dim3(grid_for(e_total, 256)), dim3(256), 0, as_stream(stream),
                     joint_det, joint_tags, F, joint_scores, edge_index, e_total, J, norm_factor, mode, A, edge_attr);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

extern "C" size_t pemp_knn_workspace_size(const int64_t* node_off_host, int B) {
  if (!node_off_host || B <= 0) return 0;
  size_t bytes = 0;
  knn_carve(nullptr, node_off_host, B, &bytes);
  return bytes;
}

extern "C" int pemp_knn_graph_count(const int64_t* joint_det, const int64_t* node_off, const int64_t* node_off_host,
                                    int B, int k, void* workspace, size_t workspace_bytes, int64_t* edge_count,
                                    void* stream) {
  PEMP_CHECK_ARG(joint_det && node_off && node_off_host && workspace && edge_count && B > 0 && k >= 1,
                 "pemp_knn_graph_count: bad args");
  size_t need = 0;
  knn_carve(nullptr, node_off_host, B, &need);
  if (workspace_bytes < need) {
    set_error("pemp_knn_graph_count: workspace %zu < %zu", workspace_bytes, need);
    return PEMP_ERR_WORKSPACE;
  }
  const KnnWs w = knn_carve(workspace, node_off_host, B, nullptr);
  const hipStream_t st = as_stream(stream);
  const size_t words = knn_words(node_off_host, B, nullptr);
  hipLaunchKernelGGL(knn_matoff_kernel, dim3(1), dim3(64), 0, st, node_off, B, w.mat_off);
  PEMP_LAUNCH_CHECK();
  PEMP_HIP(hipMemsetAsync(w.adj, 0, words * sizeof(unsigned long long), st));
  PEMP_HIP(hipMemsetAsync(w.adjt, 0, words * sizeof(unsigned long long), st));
  const int64_t n_total = node_off_host[B];
  if (n_total > 0) {
    ProfScope prof("knn_adj", st);
    hipLaunchKernelGGL(knn_adj_kernel, dim3((unsigned)((n_total + 3) / 4)), dim3(256), 0, st,
                       KnnDist{joint_det, nullptr, nullptr}, node_off, B, n_total, k + 1, w.mat_off, w.adj, w.adjt);
    PEMP_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(knn_count_kernel, dim3(B), dim3(256), 0, st, node_off, B, w.mat_off, w.adj, w.adjt, edge_count);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

extern "C" int pemp_knn_graph_emit(const int64_t* node_off, const int64_t* node_off_host, int B,
                                   const int64_t* edge_off, int64_t e_total, void* workspace,
                                   size_t workspace_bytes, int64_t* edge_index, void* stream) {
  PEMP_CHECK_ARG(node_off && node_off_host && edge_off && workspace && edge_index && B > 0 && e_total >= 0,
                 "pemp_knn_graph_emit: bad args");
  size_t need = 0;
  knn_carve(nullptr, node_off_host, B, &need);
  if (workspace_bytes < need) {
    set_error("pemp_knn_graph_emit: workspace %zu < %zu", workspace_bytes, need);
    return PEMP_ERR_WORKSPACE;
  }
  const KnnWs w = knn_carve(workspace, node_off_host, B, nullptr);
  if (e_total == 0) return PEMP_OK;
  ProfScope prof("knn_emit", as_stream(stream));
  hipLaunchKernelGGL(knn_emit_kernel, dim3(B), dim3(1024), 0, as_stream(stream), node_off, B, w.mat_off, w.adj,
                     w.adjt, edge_off, e_total, e_total, edge_index);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

// The whole knn graph without a host round trip in the middle: adjacency, per-image counts, their scan
// and the emit are queued back to back; the edge total reaches the host through mapped memory
// (e_total_host, written by the scan kernel while the emit runs). edge_buf holds 2 * e_cap int64: the
// graph is its leading [2, E] block (source row at 0, destination row at E).
static int knn_build(const char* who, const float* feat, int C, const int64_t* joint_det, const int64_t* node_off,
                     const int64_t* node_off_host, int B, int k, void* workspace, size_t workspace_bytes,
                     int64_t e_cap, int64_t* edge_buf, int32_t* e_total_host, const float* joint_tags, int F,
                     const float* joint_scores, int J, float norm_factor, int mode, float* edge_attr,
                     void* stream) {
  PEMP_CHECK_ARG(joint_det && node_off && node_off_host && workspace && edge_buf && B > 0 && k >= 1 && e_cap >= 0,
                 "%s: bad args", who);
  int A = 0;
  if (edge_attr) {
    PEMP_CHECK_ARG(J > 0, "%s: J <= 0", who);
    A = ef_width(mode, J);
    if (A < 0) { set_error("%s: unknown mode %d", who, mode); return PEMP_ERR_INVALID_ARG; }
    if (const int rc = ef_tag_check(mode, joint_tags, F, who)) return rc;
    PEMP_CHECK_ARG(mode != PEMP_EF_AE_NORMED || joint_scores, "%s: ae_normed needs joint_scores", who);
  }
  const bool fk = feat != nullptr;
  size_t need = 0;
  knn_carve(nullptr, node_off_host, B, &need, fk);
  if (workspace_bytes < need) {
    set_error("%s: workspace %zu < %zu", who, workspace_bytes, need);
    return PEMP_ERR_WORKSPACE;
  }
  int64_t bound = 0;   // every node keeps min(k, n - 1) nearest; the union with the reverse at most doubles it
  for (int b = 0; b < B; ++b) {
    const int64_t n = node_off_host[b + 1] - node_off_host[b];
    PEMP_CHECK_ARG(n >= 0, "%s: decreasing node offsets", who);
    bound += std::min<int64_t>(n * (n > 0 ? n - 1 : 0), 2 * (int64_t)k * n);
  }
  PEMP_CHECK_ARG(e_cap >= bound, "%s: e_cap %lld < bound %lld", who, (long long)e_cap, (long long)bound);
  const KnnWs w = knn_carve(workspace, node_off_host, B, nullptr, fk);
  const hipStream_t st = as_stream(stream);
  KnnDist dist{joint_det, nullptr, nullptr};
  if (fk && node_off_host[B] > 0) {   // the n_b x n_b feature-distance keys of every image
    ProfScope prof("fknn_dist", st);
    hipLaunchKernelGGL(fknn_doff_kernel, dim3(1), dim3(64), 0, st, node_off, B, w.doff);
    PEMP_LAUNCH_CHECK();
    hipLaunchKernelGGL(fknn_dist_kernel, dim3((unsigned)node_off_host[B]), dim3(256), (size_t)C * sizeof(float), st,
                       feat, C, node_off, B, w.doff, w.dkey);
    PEMP_LAUNCH_CHECK();
    dist = KnnDist{joint_det, w.dkey, w.doff};
  }
  int* e_dev_host = nullptr;   // device address of the caller's mapped host word
  if (e_total_host) PEMP_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&e_dev_host), e_total_host, 0));
  int64_t nmax = 0;
  for (int b = 0; b < B; ++b) nmax = std::max<int64_t>(nmax, node_off_host[b + 1] - node_off_host[b]);
  if (nmax <= KNN_LDS_MAXN) {   // three launches: selection, rows, emit
    ProfScope prof("knn_build", st);
    const int64_t n_all = node_off_host[B];
    if (n_all > 0) {
      hipLaunchKernelGGL(knn_select_kernel, dim3((unsigned)((n_all + 15) / 16)), dim3(1024), 0, st, dist, node_off, B,
                         n_all, k + 1, w.arow);
      PEMP_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(knn_rows_kernel, dim3(B), dim3(1024), 0, st, node_off, w.arow, w.rows, w.rowstart, w.ecount);
    PEMP_LAUNCH_CHECK();
    KnnEmitArgs ka{node_off, B, w.rows, w.rowstart, w.ecount, e_cap, w.edge_off, e_dev_host, edge_buf,
                   joint_det, joint_tags, F, joint_scores, J, mode, A, norm_factor, edge_attr};
    hipLaunchKernelGGL(knn_emit_rows_kernel, dim3(B, (unsigned)std::max<int64_t>(1, (nmax + 15) / 16)), dim3(1024), 0,
                       st, ka);
    PEMP_LAUNCH_CHECK();
    return PEMP_OK;
  }
  const size_t words = knn_words(node_off_host, B, nullptr);
  hipLaunchKernelGGL(knn_matoff_kernel, dim3(1), dim3(64), 0, st, node_off, B, w.mat_off);
  PEMP_LAUNCH_CHECK();
  if (words) {
    PEMP_HIP(hipMemsetAsync(w.adj, 0, words * sizeof(unsigned long long), st));
    PEMP_HIP(hipMemsetAsync(w.adjt, 0, words * sizeof(unsigned long long), st));
  }
  const int64_t n_total = node_off_host[B];
  ProfScope prof("knn_build", st);
  if (n_total > 0) {
    hipLaunchKernelGGL(knn_adj_kernel, dim3((unsigned)((n_total + 3) / 4)), dim3(256), 0, st, dist, node_off, B,
                       n_total, k + 1, w.mat_off, w.adj, w.adjt);
    PEMP_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(knn_count_kernel, dim3(B), dim3(256), 0, st, node_off, B, w.mat_off, w.adj, w.adjt, w.ecount);
  PEMP_LAUNCH_CHECK();
  hipLaunchKernelGGL(knn_offsets_kernel, dim3(1), dim3(64), 0, st, w.ecount, B, w.edge_off, e_dev_host);
  PEMP_LAUNCH_CHECK();
  if (bound > 0) {
    hipLaunchKernelGGL(knn_emit_kernel, dim3(B), dim3(1024), 0, st, node_off, B, w.mat_off, w.adj, w.adjt,
                       w.edge_off, (int64_t)-1, e_cap, edge_buf);
    PEMP_LAUNCH_CHECK();
    if (edge_attr) {
      // edge_index's destination row starts at the device-side total: the features kernel reads it too
      hipLaunchKernelGGL(edge_features_kernel, dim3(grid_for(e_cap, 256)), dim3(256), 0, st, joint_det, joint_tags, F,
                         joint_scores, edge_buf, e_cap, J, norm_factor, mode, A, edge_attr, w.edge_off + B);
      PEMP_LAUNCH_CHECK();
    }
  }
  return PEMP_OK;
}

extern "C" int pemp_knn_graph_build(const int64_t* joint_det, const int64_t* node_off, const int64_t* node_off_host,
                                    int B, int k, void* workspace, size_t workspace_bytes, int64_t e_cap,
                                    int64_t* edge_buf, int32_t* e_total_host, const float* joint_tags, int F,
                                    const float* joint_scores, int J, float norm_factor, int mode, float* edge_attr,
                                    void* stream) {
  return knn_build("pemp_knn_graph_build", nullptr, 0, joint_det, node_off, node_off_host, B, k, workspace,
                   workspace_bytes, e_cap, edge_buf, e_total_host, joint_tags, F, joint_scores, J, norm_factor, mode,
                   edge_attr, stream);
}

extern "C" size_t pemp_feature_knn_workspace_size(const int64_t* node_off_host, int B) {
  if (!node_off_host || B <= 0) return 0;
  size_t bytes = 0;
  knn_carve(nullptr, node_off_host, B, &bytes, true);
  return bytes;
}

extern "C" int pemp_knn_rows_layout(const int64_t* node_off_host, int B, int feature, size_t* offs) {
  PEMP_CHECK_ARG(node_off_host && B > 0 && offs, "pemp_knn_rows_layout: bad args");
  for (int b = 0; b < B; ++b)
    if (node_off_host[b + 1] - node_off_host[b] > KNN_LDS_MAXN) {
      set_error("pemp_knn_rows_layout: image %d over %d nodes (no bit rows)", b, KNN_LDS_MAXN);
      return PEMP_ERR_UNSUPPORTED;
    }
  char* const base = reinterpret_cast<char*>(4096);   // (any aligned base: offsets only)
  const KnnWs w = knn_carve(base, node_off_host, B, nullptr, feature != 0);
  offs[0] = (size_t)(reinterpret_cast<char*>(w.rows) - base);
  offs[1] = (size_t)(reinterpret_cast<char*>(w.rowstart) - base);
  offs[2] = (size_t)(reinterpret_cast<char*>(w.ecount) - base);
  return PEMP_OK;
}

extern "C" int pemp_feature_knn_graph_build(const float* x, int C, const int64_t* joint_det, const int64_t* node_off,
                                            const int64_t* node_off_host, int B, int k, void* workspace,
                                            size_t workspace_bytes, int64_t e_cap, int64_t* edge_buf,
                                            int32_t* e_total_host, const float* joint_tags, int F,
                                            const float* joint_scores, int J, float norm_factor, int mode,
                                            float* edge_attr, void* stream) {
  PEMP_CHECK_ARG(x && C > 0 && C <= 8192, "pemp_feature_knn_graph_build: x null or C %d out of (0, 8192]", C);
  PEMP_CHECK_ARG((reinterpret_cast<uintptr_t>(x) & 15) == 0 || (C & 3) != 0,
                 "pemp_feature_knn_graph_build: x not 16-byte aligned");
  return knn_build("pemp_feature_knn_graph_build", x, C, joint_det, node_off, node_off_host, B, k, workspace,
                   workspace_bytes, e_cap, edge_buf, e_total_host, joint_tags, F, joint_scores, J, norm_factor, mode,
                   edge_attr, stream);
}

extern "C" size_t pemp_score_graph_workspace_size(const int64_t* node_off_host, int B, int k) {
  if (!node_off_host || B <= 0 || k < 1) return 0;
  return score_ws_bytes(node_off_host[B], B, k);
}

extern "C" int pemp_score_graph(const float* joint_scores, const int64_t* node_off, const int64_t* node_off_host,
                                int B, int k, int64_t e_total, void* workspace, size_t workspace_bytes,
                                int64_t* edge_index, void* stream) {
  PEMP_CHECK_ARG(joint_scores && node_off && node_off_host && workspace && B > 0 && k >= 1,
                 "pemp_score_graph: bad args");
  int64_t e_need = 0;
  for (int b = 0; b < B; ++b) {
    const int64_t n = node_off_host[b + 1] - node_off_host[b];
    if (n < k) {   // the reference's joint_scores.topk(k) raises (ConstructGraph.py:414)
      set_error("pemp_score_graph: image %d has %lld detections < k = %d", b, (long long)n, k);
      return PEMP_ERR_INVALID_ARG;
    }
    e_need += (int64_t)k * (2 * n - k - 1);
  }
  PEMP_CHECK_ARG(e_total == e_need, "pemp_score_graph: e_total does not match k (2 n - k - 1) per image");
  PEMP_CHECK_ARG(e_total == 0 || edge_index, "pemp_score_graph: null edge_index");
  const int64_t n_total = node_off_host[B];
  if (workspace_bytes < score_ws_bytes(n_total, B, k)) {
    set_error("pemp_score_graph: workspace %zu < %zu", workspace_bytes, score_ws_bytes(n_total, B, k));
    return PEMP_ERR_WORKSPACE;
  }
  if (e_total == 0) return PEMP_OK;
  const ScoreWs w = score_carve(workspace, n_total, B, k);
  const hipStream_t st = as_stream(stream);
  ProfScope prof("score_graph", st);
  hipLaunchKernelGGL(score_roots_kernel, dim3(B), dim3(256), 0, st, joint_scores, node_off, B, k, w);
  PEMP_LAUNCH_CHECK();
  const int64_t blocks = std::min<int64_t>((n_total + 3) / 4, 4096);
  hipLaunchKernelGGL(score_emit_kernel, dim3((unsigned)blocks), dim3(256), 0, st, node_off, B, k, w, n_total,
                     e_total, edge_index);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

extern "C" int pemp_gather_projected(const float* const* maps, const int* map_h, const int* map_w, int S, int C,
                                     int H, int W, float divisor, const int64_t* joint_det,
                                     const int64_t* batch_index, int64_t N, float* x, void* stream) {
  PEMP_CHECK_ARG(maps && map_h && map_w && S >= 1 && S <= PROJ_MAXS && C > 0 && H > 0 && W > 0 && N >= 0 &&
                     divisor > 0.f,
                 "pemp_gather_projected: bad args (S in [1, %d])", PROJ_MAXS);
  PEMP_CHECK_ARG(N == 0 || (joint_det && batch_index && x), "pemp_gather_projected: null node arrays");
  ProjMaps m{};
  m.S = S;
  for (int s = 0; s < S; ++s) {
    PEMP_CHECK_ARG(maps[s] && map_h[s] > 0 && map_w[s] > 0, "pemp_gather_projected: bad map %d", s);
    m.p[s] = maps[s];
    m.h[s] = map_h[s];
    m.w[s] = map_w[s];
  }
  if (N == 0) return PEMP_OK;
  ProfScope prof("gather_projected", as_stream(stream));
  hipLaunchKernelGGL(gather_projected_kernel, dim3(grid_for(N * C, 256, 4096)), dim3(256), 0, as_stream(stream), m, C,
                     H, W, divisor, joint_det, batch_index, N, x);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

extern "C" int pemp_gather_projected_conv(const float* const* maps, const int* map_h, const int* map_w, int S, int Cin,
                                          const float* weight_t, const float* bias, int Cout, int ksize, int pad, int H,
                                          int W, float divisor, const int64_t* joint_det, const int64_t* batch_index,
                                          int64_t N, float* x, void* stream) {
  PEMP_CHECK_ARG(maps && map_h && map_w && S >= 1 && S <= PROJ_MAXS && Cin > 0 && H > 0 && W > 0 && N >= 0 &&
                     divisor > 0.f && weight_t && Cout > 0 && Cout <= PCONV_THREADS * PCONV_MAXQ && ksize >= 1 &&
                     ksize <= 7 && pad >= 0 && pad < ksize,
                 "pemp_gather_projected_conv: bad args (S in [1, %d], Cout <= %d, k <= 7, 0 <= pad < k)", PROJ_MAXS,
                 PCONV_THREADS * PCONV_MAXQ);
  PEMP_CHECK_ARG((size_t)Cin * (ksize + 1) * (ksize + 1) * 4 <= 64 * 1024,
                 "pemp_gather_projected_conv: Cin * (k+1)^2 patch exceeds 64 KB of LDS");
  PEMP_CHECK_ARG(N == 0 || (joint_det && batch_index && x), "pemp_gather_projected_conv: null node arrays");
  ProjMaps m{};
  m.S = S;
  for (int s = 0; s < S; ++s) {
    PEMP_CHECK_ARG(maps[s] && map_h[s] + 2 * pad - ksize + 1 > 0 && map_w[s] + 2 * pad - ksize + 1 > 0,
                   "pemp_gather_projected_conv: bad map %d (conv output empty)", s);
    m.p[s] = maps[s];
    m.h[s] = map_h[s];
    m.w[s] = map_w[s];
  }
  if (N == 0) return PEMP_OK;
  PEMP_CHECK_ARG(N < (1ll << 31), "pemp_gather_projected_conv: N exceeds the grid");
  ProfScope prof("gather_projected_conv", as_stream(stream));
  const size_t lds = (size_t)Cin * (ksize + 1) * (ksize + 1) * sizeof(float);
  hipLaunchKernelGGL(gather_projected_conv_kernel, dim3((unsigned)N), dim3(PCONV_THREADS), lds, as_stream(stream), m,
                     weight_t, bias, Cin, Cout, ksize, pad, H, W, divisor, joint_det, batch_index, x);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}
