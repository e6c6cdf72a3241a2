// Keypoint detection from heatmaps — restates, for gfx950:
//   Utils/Utils.py:15-20          non_maximum_suppression: MaxPool2d(k,1,k//2) == s (-inf padding)
//   ConstructGraph.py:1161-1196   joint_det_from_scoremap: s *= maxima (* mask); per-type top-k;
//                                 threshold set; (DETECT_THRESHOLD > 1.5: top-20 + 1e-10)
//   ConstructGraph.py:1199-1209   cat_unique ordering
//
// Stage 1 (nms_tiles_kernel, HBM-bound): one workgroup per 32x128 tile of one (image, type)
//   plane. Tile + halo staged in LDS, separable max, then per pixel v = s * jm. Emits, per tile:
//   each wave's k best (v, flat index) candidates (ties -> lower index), the tile's count of
//   threshold pixels, and the threshold bitmask (row-major, one bit per pixel, 64-px words).
// Stage 2 (select_kernel): one workgroup per image. Merges the candidates into the exact
//   per-type top-k, scans per-strip counts, and emits detections in the reference's order.
#include <math.h>

#include "pemp_common.h"

namespace pemp {
namespace {

constexpr int TR = 32;    // tile rows (= strip height)
constexpr int TC = 128;   // tile cols (multiple of 64: a tile owns whole bitmask words)
constexpr int NT1 = 256;  // stage-1 threads: 32 rows x 8 threads x 16 px
#ifndef NMS_MIN_WAVES
#define NMS_MIN_WAVES 4
#endif
constexpr int MAXR = 4;   // max pool radius (POOL_KERNEL_SIZE <= 9)
constexpr int NT2 = 1024; // stage-2 threads
constexpr int MAXJ = 32;

__device__ __forceinline__ bool better(float v1, int i1, float v2, int i2) {
  return v1 > v2 || (v1 == v2 && i1 < i2);
}

struct DetectGeom {
  int B, J, H, W, p, K, tiles_x, tiles_y, tiles, WW, S;
};

static DetectGeom geom(int B, int J, int H, int W, int pool_k, int K) {
  DetectGeom g;
  g.B = B; g.J = J; g.H = H; g.W = W; g.p = pool_k / 2; g.K = K;
  g.tiles_x = (W + TC - 1) / TC;
  g.tiles_y = (H + TR - 1) / TR;
  g.tiles = g.tiles_x * g.tiles_y;
  g.WW = (W + 63) / 64;
  g.S = g.tiles_y;
  return g;
}

struct DetectWs {
  float *cand_v, *neg_v; int *cand_i, *neg_i, *tile_count, *tile_nonneg; unsigned long long* bits;
};

static DetectWs carve(void* base, const DetectGeom& g, size_t* bytes) {
  Carver c(base);
  DetectWs w;
  size_t ncand = (size_t)g.B * g.J * g.tiles * 4 * g.K;
  w.cand_v = c.take<float>(ncand);
  w.cand_i = c.take<int>(ncand);
  w.neg_v = c.take<float>(ncand);
  w.neg_i = c.take<int>(ncand);
  w.tile_count = c.take<int>((size_t)g.B * g.J * g.tiles * 4);
  w.tile_nonneg = c.take<int>((size_t)g.B * g.J * g.tiles * 4);
  w.bits = c.take<unsigned long long>((size_t)g.B * g.J * g.H * g.WW);
  if (bytes) *bytes = c.used;
  return w;
}

// Stage 1 (persistent): a workgroup walks tiles tl = blockIdx.x, +gridDim.x, ...; the next tile's
// global loads are issued into registers before the current tile is processed. Tile = 32 rows x
// 128 cols of one plane; LDS holds rows y0-P..y0+31+P, columns x0-4..x0+131 (P <= 4) at a
// conflict-free row stride. A thread owns 16 consecutive pixels of one row.
//
// Candidates (exact):
//   MODE_POS (threshold set in use): per tile the top-K of the POSITIVE values. Zero-valued top-k
//     entries are never emitted, and negatives can enter a plane's top-k only when the plane has
//     fewer than K non-negative pixels, so the tile also reports its non-negative count and, when
//     that count is below K, the top-K of its negative values.
//   MODE_ALL (DETECT_THRESHOLD > 1.5: every top-k entry is emitted as value + 1e-10): the exact
//     top-K of all pixels.
constexpr int HALO = 4;                   // staged columns on each side (>= P)
constexpr int LQ = (TC + 2 * HALO) / 4;   // 34 float4 quads per staged row
constexpr int LS = 140;                   // LDS row stride (floats): ds_read_b128 conflict-free here
constexpr int INV = 0x7fffffff;
enum { MODE_POS = 0, MODE_ALL = 1 };

template <int CTRL>
__device__ __forceinline__ void dpp_better(float& v, int& i) {
  const float ov = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
  const int oi = __builtin_amdgcn_update_dpp(i, i, CTRL, 0xF, 0xF, false);
  if (better(ov, oi, v, i)) { v = ov; i = oi; }
}

// wave-wide argmax under (value desc, index asc); result is wave-uniform
__device__ __forceinline__ void wave_best(float& v, int& i) {
  dpp_better<0xB1>(v, i);    // quad_perm [1,0,3,2]
  dpp_better<0x4E>(v, i);    // quad_perm [2,3,0,1]
  dpp_better<0x141>(v, i);   // row_half_mirror
  dpp_better<0x140>(v, i);   // row_mirror  -> every lane holds its 16-lane row's best
  float bv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
  for (int r = 1; r < 4; ++r) {
    const float rv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16 * r));
    const int ri = __builtin_amdgcn_readlane(i, 16 * r);
    if (better(rv, ri, bv, bi)) { bv = rv; bi = ri; }
  }
  v = bv;
  i = bi;
}

// K rounds: pop the wave's best among the lane's 16 values that pass `keep`; the winner lane
// removes the value and rescans. Writes out_v/out_i[k] (sentinels once exhausted).
template <typename Keep>
__device__ __forceinline__ void wave_topk(float (&v)[16], int base_id, int K, Keep keep, float* out_v, int* out_i) {
  const int lane = threadIdx.x & 63;
  float lbv = -INFINITY;
  int lbj = -1;
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (keep(v[j]) && (lbj < 0 || v[j] > lbv)) { lbv = v[j]; lbj = j; }
  for (int k = 0; k < K; ++k) {
    float bv = lbj < 0 ? -INFINITY : lbv;
    int bi = lbj < 0 ? INV : base_id + lbj;
    wave_best(bv, bi);
    if (lane == 0) { out_v[k] = bv; out_i[k] = bi; }
    if (bi == INV) {                               // wave exhausted: fill with sentinels
      for (int k2 = k + 1; k2 < K; ++k2)
        if (lane == 0) { out_v[k2] = -INFINITY; out_i[k2] = INV; }
      break;
    }
    if (lbj >= 0 && bi == base_id + lbj) {        // this lane owned the winner
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j == lbj) v[j] = NAN;                  // removed (fails every keep predicate)
      lbj = -1;
      lbv = -INFINITY;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (keep(v[j]) && (lbj < 0 || v[j] > lbv)) { lbv = v[j]; lbj = j; }
    }
  }
}

template <int P, bool VEC>
__device__ __forceinline__ void load_tile(const float* __restrict__ s, const DetectGeom& g, int tl,
                                          float4 (&q)[((TR + 2 * P) * LQ + NT1 - 1) / NT1]) {
  constexpr int LH = TR + 2 * P;
  constexpr int NQ = (LH * LQ + NT1 - 1) / NT1;
  const int tile = tl % g.tiles, plane_i = tl / g.tiles;
  const int ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
  const int y0 = ty * TR, x0 = tx * TC, H = g.H, W = g.W;
  const float* plane = s + (size_t)plane_i * H * W;
#pragma unroll
  for (int u = 0; u < NQ; ++u) {
    const int idx = threadIdx.x + u * NT1;
    const int r = idx / LQ, c4 = idx - r * LQ;
    const int y = y0 - P + r, x = x0 - HALO + 4 * c4;
    const bool yok = idx < LH * LQ && y >= 0 && y < H;
    const float* row = plane + (size_t)min(max(y, 0), H - 1) * W;   // clamped: always a valid address
    float4 v;
    if (VEC) {
      // W % 4 == 0: a quad is entirely inside or entirely outside the row
      v = *reinterpret_cast<const float4*>(row + min(max(x, 0), W - 4));
      const bool ok = yok && x >= 0 && x < W;
      if (!ok) v = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    } else {
      const float a0 = row[min(max(x, 0), W - 1)], a1 = row[min(max(x + 1, 0), W - 1)];
      const float a2 = row[min(max(x + 2, 0), W - 1)], a3 = row[min(max(x + 3, 0), W - 1)];
      v.x = (yok && x >= 0 && x < W) ? a0 : -INFINITY;
      v.y = (yok && x + 1 >= 0 && x + 1 < W) ? a1 : -INFINITY;
      v.z = (yok && x + 2 >= 0 && x + 2 < W) ? a2 : -INFINITY;
      v.w = (yok && x + 3 >= 0 && x + 3 < W) ? a3 : -INFINITY;
    }
    q[u] = v;
  }
}

// Per tile: two block barriers (stage the tile, then each wave works on its own 8-row strip:
// vertical max, horizontal max, v, threshold bits, top-k). Each wave writes its own candidate
// list (K entries) and counts: per tile 4 lists.
template <int P, int MODE, bool VEC, bool MASKED>
__global__ __launch_bounds__(NT1, NMS_MIN_WAVES) void nms_tiles_kernel(
    const float* __restrict__ s, const float* __restrict__ masks, DetectGeom g, float thr, int use_thr,
    float* __restrict__ cand_v, int* __restrict__ cand_i, float* __restrict__ neg_v, int* __restrict__ neg_i,
    int* __restrict__ tile_count, int* __restrict__ tile_nonneg, unsigned long long* __restrict__ bits) {
  constexpr int LH = TR + 2 * P;
  constexpr int NQ = (LH * LQ + NT1 - 1) / NT1;
  __shared__ __attribute__((aligned(16))) float in[LH * LS];
  __shared__ __attribute__((aligned(16))) float vmax[TR * LS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int total = g.B * g.J * g.tiles;
  const int H = g.H, W = g.W, K = g.K;
  int tl = blockIdx.x;
  float4 q[NQ];
  if (tl < total) load_tile<P, VEC>(s, g, tl, q);
  for (; tl < total; tl += gridDim.x) {
    const int tile = tl % g.tiles, plane_i = tl / g.tiles, b = plane_i / g.J;
    const int ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
    const int y0 = ty * TR, x0 = tx * TC;
    __syncthreads();                               // previous tile's readers of `in` are done
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int idx = threadIdx.x + u * NT1;
      if (idx < LH * LQ) {
        const int r = idx / LQ, c4 = idx - r * LQ;
        *reinterpret_cast<float4*>(&in[r * LS + 4 * c4]) = q[u];
      }
    }
    if (tl + (int)gridDim.x < total) load_tile<P, VEC>(s, g, tl + gridDim.x, q);   // prefetch next tile
    __syncthreads();
    // vertical max of this wave's rows 8w..8w+7: lane = column quad, sliding window in registers
    if (lane < LQ) {
      float4 col[8 + 2 * P];
#pragma unroll
      for (int i = 0; i < 8 + 2 * P; ++i) col[i] = *reinterpret_cast<const float4*>(&in[(wave * 8 + i) * LS + 4 * lane]);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float4 m = col[i];
#pragma unroll
        for (int d = 1; d <= 2 * P; ++d) {
          m.x = fmaxf(m.x, col[i + d].x); m.y = fmaxf(m.y, col[i + d].y);
          m.z = fmaxf(m.z, col[i + d].z); m.w = fmaxf(m.w, col[i + d].w);
        }
        *reinterpret_cast<float4*>(&vmax[(wave * 8 + i) * LS + 4 * lane]) = m;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int r = threadIdx.x >> 3, cb = (threadIdx.x & 7) * 16;
    const int y = y0 + r;
    const bool row_ok = y < H;
    float vm[24], sc[16], mk[MASKED ? 16 : 1];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const float4 m = *reinterpret_cast<const float4*>(&vmax[r * LS + cb + 4 * k]);
      vm[4 * k] = m.x; vm[4 * k + 1] = m.y; vm[4 * k + 2] = m.z; vm[4 * k + 3] = m.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 o = *reinterpret_cast<const float4*>(&in[(r + P) * LS + cb + HALO + 4 * k]);
      sc[4 * k] = o.x; sc[4 * k + 1] = o.y; sc[4 * k + 2] = o.z; sc[4 * k + 3] = o.w;
    }
    if (MASKED) {
      const float* mrow = masks + ((size_t)b * H + min(y, H - 1)) * W;
#pragma unroll
      for (int j = 0; j < (MASKED ? 16 : 1); ++j) mk[j] = mrow[min(x0 + cb + j, W - 1)];
    }
    // v = s * jm (ConstructGraph.py:1162-1165); NaN marks pixels outside the plane
    float v[16];
    unsigned int mybits = 0;
    int nonneg = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float m = vm[j + HALO - P];
#pragma unroll
      for (int d = 1; d <= 2 * P; ++d) m = fmaxf(m, vm[j + HALO - P + d]);
      float jm = (m == sc[j]) ? 1.0f : 0.0f;
      if (MASKED) jm = jm * mk[MASKED ? j : 0];
      const float vj = sc[j] * jm;
      const bool ok = row_ok && x0 + cb + j < W;
      v[j] = ok ? vj : NAN;
      mybits |= (unsigned)(ok && use_thr && !(vj < thr) && (vj != 0.0f)) << j;
      nonneg += ok && vj >= 0.0f;
    }
    const int base_id = y * W + x0 + cb;
    const size_t wl = (size_t)tl * 4 + wave;     // this wave's list
    if (MODE == MODE_POS)
      wave_topk(v, base_id, K, [](float x) { return x > 0.0f; }, cand_v + wl * K, cand_i + wl * K);
    else
      wave_topk(v, base_id, K, [](float x) { return x == x; }, cand_v + wl * K, cand_i + wl * K);

    // threshold bitmask: 4 consecutive threads x 16 px = one 64-px word
    unsigned int lo = (threadIdx.x & 3) < 2 ? (mybits << (16 * (threadIdx.x & 1))) : 0u;
    unsigned int hi = (threadIdx.x & 3) >= 2 ? (mybits << (16 * (threadIdx.x & 1))) : 0u;
    lo |= __shfl_xor(lo, 1); hi |= __shfl_xor(hi, 1);
    lo |= __shfl_xor(lo, 2); hi |= __shfl_xor(hi, 2);
    const int word = x0 / 64 + ((threadIdx.x & 7) >> 2);
    if ((threadIdx.x & 3) == 0 && row_ok && word < g.WW)
      bits[((size_t)plane_i * H + y) * g.WW + word] = ((unsigned long long)hi << 32) | lo;
    int cnt = __popc(mybits);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      cnt += __shfl_xor(cnt, off);
      nonneg += __shfl_xor(nonneg, off);
    }
    if (lane == 0) { tile_count[wl] = cnt; tile_nonneg[wl] = nonneg; }
    if (MODE == MODE_POS) {
      if (nonneg < K)      // degenerate strip: also keep its best negatives (see stage 2)
        wave_topk(v, base_id, K, [](float x) { return x < 0.0f; }, neg_v + wl * K, neg_i + wl * K);
      else if (lane < K) { neg_v[wl * K + lane] = -INFINITY; neg_i[wl * K + lane] = INV; }
    }
  }
}

__device__ __forceinline__ int block_excl_scan(int v, int* sh, int* total) {
  // 1024-thread exclusive scan; sh: >= 16 ints
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(x, off);
    if (lane >= off) x += o;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  if (threadIdx.x < 64) {
    int w = threadIdx.x < (int)(blockDim.x >> 6) ? sh[threadIdx.x] : 0;
    int inc = w;
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(inc, off);
      if (threadIdx.x >= off) inc += o;
    }
    if (threadIdx.x < (int)(blockDim.x >> 6)) sh[threadIdx.x] = inc - w;
    if (threadIdx.x == (int)(blockDim.x >> 6) - 1) sh[32] = inc;
  }
  __syncthreads();
  const int res = sh[wave] + x - v;
  *total = sh[32];
  __syncthreads();
  return res;
}

// Wave-level exact top-`take` of n candidates (value desc, index asc) into out (lane 0 writes);
// returns the number of valid entries written.
template <int KMAX>
__device__ __forceinline__ int merge_candidates(const float* __restrict__ cv, const int* __restrict__ ci, int n,
                                                int take, float* out_v, int* out_i) {
  const int lane = threadIdx.x & 63;
  float lv[KMAX];
  int li[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) { lv[k] = -INFINITY; li[k] = INV; }
  for (int c = lane; c < n; c += 64) {
    float v = cv[c];
    int i = ci[c];
    if (i != INV && better(v, i, lv[KMAX - 1], li[KMAX - 1])) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (better(v, i, lv[k], li[k])) {
          const float s2 = lv[k]; const int i2 = li[k];
          lv[k] = v; li[k] = i; v = s2; i = i2;
        }
      }
    }
  }
  int got = 0;
  for (int q = 0; q < take; ++q) {
    float bv = lv[0];
    int bi = li[0];
    wave_best(bv, bi);
    if (bi == INV) break;
    if (lane == 0) { out_v[q] = bv; out_i[q] = bi; }
    ++got;
    if (li[0] == bi) {
#pragma unroll
      for (int k = 0; k < KMAX - 1; ++k) { lv[k] = lv[k + 1]; li[k] = li[k + 1]; }
      lv[KMAX - 1] = -INFINITY; li[KMAX - 1] = INV;
    }
  }
  return got;
}

template <int KMAX>
__global__ __launch_bounds__(NT2) void select_kernel(
    const float* __restrict__ s, const float* __restrict__ masks, DetectGeom g, float thr, int use_thr,
    const float* __restrict__ cand_v, const int* __restrict__ cand_i, const float* __restrict__ neg_v,
    const int* __restrict__ neg_i, const int* __restrict__ tile_count, const int* __restrict__ tile_nonneg,
    const unsigned long long* __restrict__ bits, int64_t* __restrict__ det, float* __restrict__ scores,
    int* __restrict__ n_det, int cap) {
  extern __shared__ int sh_strip[];            // [J*S] counts, then [J*S] offsets
  __shared__ float top_v[MAXJ][2 * KMAX];
  __shared__ float top_sc[MAXJ][KMAX];
  __shared__ int top_i[MAXJ][2 * KMAX];
  __shared__ int top_bit[MAXJ][KMAX];
  __shared__ int n_top[MAXJ];
  __shared__ int scan_sh[40];
  const int b = blockIdx.x;
  const int J = g.J, H = g.H, W = g.W, K = g.K, S = g.S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = NT2 / 64;
  int* strip_cnt = sh_strip;
  int* strip_off = sh_strip + J * S;

  // (a) exact per-type top-k from the per-tile candidates: each lane keeps a sorted local list of
  //     its candidates, then rounds of wave argmax pop the global order.
  for (int t = wave; t < J; t += nwaves) {
    const size_t pt = (size_t)(b * J + t) * g.tiles * 4;      // first wave list of the plane
    int n = merge_candidates<KMAX>(cand_v + pt * K, cand_i + pt * K, g.tiles * 4 * K, K, top_v[t], top_i[t]);
    if (use_thr) {
      // degenerate plane (fewer than K non-negative pixels): its top-k also holds negatives
      int nn = 0;
      for (int c = lane; c < g.tiles * 4; c += 64) nn += tile_nonneg[pt + c];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) nn += __shfl_xor(nn, off);
      if (nn < K)
        n += merge_candidates<KMAX>(neg_v + pt * K, neg_i + pt * K, g.tiles * 4 * K, K - nn, top_v[t] + n,
                                    top_i[t] + n);
    }
    if (lane == 0) {
      // keep value != 0 (ConstructGraph.py:1174 nonzero), then order by flat index (y, x)
      int m = 0;
      for (int q = 0; q < n; ++q) {
        const float v = top_v[t][q];
        const float sc = use_thr ? v : v + 1e-10f;
        if (sc != 0.0f && top_i[t][q] != 0x7fffffff) {
          top_v[t][m] = v; top_sc[t][m] = sc; top_i[t][m] = top_i[t][q];
          ++m;
        }
      }
      for (int a2 = 1; a2 < m; ++a2) {            // insertion sort by index
        const float v = top_v[t][a2], sc = top_sc[t][a2];
        const int i = top_i[t][a2];
        int c = a2 - 1;
        while (c >= 0 && top_i[t][c] > i) {
          top_v[t][c + 1] = top_v[t][c]; top_sc[t][c + 1] = top_sc[t][c]; top_i[t][c + 1] = top_i[t][c];
          --c;
        }
        top_v[t][c + 1] = v; top_sc[t][c + 1] = sc; top_i[t][c + 1] = i;
      }
      for (int q = 0; q < m; ++q)
        top_bit[t][q] = use_thr && !(top_v[t][q] < thr) && top_v[t][q] != 0.0f;
      n_top[t] = m;
    }
  }
  __syncthreads();

  // (b) per-strip threshold counts minus top-k entries already listed (cat_unique)
  for (int e = threadIdx.x; e < J * S; e += NT2) {
    const int t = e / S, st = e - t * S;
    int c = 0;
    if (use_thr) {
      const int* tc = tile_count + ((size_t)(b * J + t) * g.tiles + st * g.tiles_x) * 4;
      for (int x = 0; x < 4 * g.tiles_x; ++x) c += tc[x];
      for (int q = 0; q < n_top[t]; ++q)
        if (top_bit[t][q] && top_i[t][q] / W / TR == st) --c;
    }
    strip_cnt[e] = c;
  }
  __syncthreads();

  // (c) offsets: [top dets of all types] ++ [threshold dets, type-major, strip order]
  int n_top_all = 0;
  for (int t = 0; t < J; ++t) n_top_all += n_top[t];
  const int per = (J * S + NT2 - 1) / NT2;
  int local = 0;
  for (int k = 0; k < per; ++k) {
    const int e = threadIdx.x * per + k;
    if (e < J * S) local += strip_cnt[e];
  }
  int total_thr;
  int base = block_excl_scan(local, scan_sh, &total_thr);
  for (int k = 0; k < per; ++k) {
    const int e = threadIdx.x * per + k;
    if (e < J * S) { strip_off[e] = n_top_all + base; base += strip_cnt[e]; }
  }
  __syncthreads();
  const int N = n_top_all + total_thr;

  int64_t* dout = det + (size_t)b * cap * 3;
  float* sout = scores + (size_t)b * cap;
  // (d) top-k detections
  for (int e = threadIdx.x; e < J * KMAX; e += NT2) {
    const int t = e / KMAX, q = e - t * KMAX;
    if (t < J && q < n_top[t]) {
      int pos = q;
      for (int t2 = 0; t2 < t; ++t2) pos += n_top[t2];
      if (pos < cap) {
        const int idx = top_i[t][q];
        dout[pos * 3 + 0] = idx % W;
        dout[pos * 3 + 1] = idx / W;
        dout[pos * 3 + 2] = t;
        sout[pos] = top_sc[t][q];
      }
    }
  }
  // (e) threshold detections, one wave per non-empty strip
  for (int e = wave; e < J * S; e += nwaves) {
    if (strip_cnt[e] == 0) continue;             // wave-uniform
    const int t = e / S, st = e - t * S;
    const int ry0 = st * TR, rows = min(TR, H - ry0);
    const int nw = rows * g.WW;
    const int chunk = (nw + 63) / 64;
    const unsigned long long* wsrc = bits + ((size_t)(b * J + t) * H + ry0) * g.WW;
    int cnt = 0;
    for (int k = 0; k < chunk; ++k) {
      const int wi = lane * chunk + k;
      if (wi >= nw) break;
      unsigned long long word = wsrc[wi];
      if (word) {
        for (int q = 0; q < n_top[t]; ++q) {
          if (!top_bit[t][q]) continue;
          const int idx = top_i[t][q], yy = idx / W, xx = idx - yy * W;
          if ((yy - ry0) * g.WW + xx / 64 == wi) word &= ~(1ull << (xx & 63));
        }
      }
      cnt += __popcll(word);
    }
    int pre = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(pre, off);
      if (lane >= off) pre += o;
    }
    int pos = strip_off[e] + pre - cnt;
    const float* plane = s + (size_t)(b * J + t) * H * W;
    for (int k = 0; k < chunk; ++k) {
      const int wi = lane * chunk + k;
      if (wi >= nw) break;
      unsigned long long word = wsrc[wi];
      if (!word) continue;
      for (int q = 0; q < n_top[t]; ++q) {
        if (!top_bit[t][q]) continue;
        const int idx = top_i[t][q], yy = idx / W, xx = idx - yy * W;
        if ((yy - ry0) * g.WW + xx / 64 == wi) word &= ~(1ull << (xx & 63));
      }
      const int yy = ry0 + wi / g.WW, xw = (wi % g.WW) * 64;
      while (word) {
        const int bit = __ffsll((long long)word) - 1;
        word &= word - 1;
        const int xx = xw + bit;
        if (pos < cap) {
          const float sv = plane[(size_t)yy * W + xx];
          float jm = 1.0f;
          if (masks) jm = jm * masks[((size_t)b * H + yy) * W + xx];
          dout[pos * 3 + 0] = xx;
          dout[pos * 3 + 1] = yy;
          dout[pos * 3 + 2] = t;
          sout[pos] = sv * jm;
        }
        ++pos;
      }
    }
  }
  if (threadIdx.x == 0) n_det[b] = N;
}

static int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) return 256;
    return v;
  }();
  return n;
}

template <int P, int MODE, bool VEC>
static void launch_nms(const float* s, const float* masks, const DetectGeom& g, float thr, int use_thr,
                       const DetectWs& w, hipStream_t st) {
  const int total = g.B * g.J * g.tiles;
  const int grid = total < 4 * num_cus() ? total : 4 * num_cus();
  if (masks)
    hipLaunchKernelGGL((nms_tiles_kernel<P, MODE, VEC, true>), dim3(grid), dim3(NT1), 0, st, s, masks, g, thr, use_thr,
                       w.cand_v, w.cand_i, w.neg_v, w.neg_i, w.tile_count, w.tile_nonneg, w.bits);
  else
    hipLaunchKernelGGL((nms_tiles_kernel<P, MODE, VEC, false>), dim3(grid), dim3(NT1), 0, st, s, masks, g, thr,
                       use_thr, w.cand_v, w.cand_i, w.neg_v, w.neg_i, w.tile_count, w.tile_nonneg, w.bits);
}

template <int MODE, bool VEC>
static void dispatch_nms(const float* s, const float* masks, const DetectGeom& g, float thr, int use_thr,
                         const DetectWs& w, hipStream_t st) {
  switch (g.p) {
    case 0: launch_nms<0, MODE, VEC>(s, masks, g, thr, use_thr, w, st); break;
    case 1: launch_nms<1, MODE, VEC>(s, masks, g, thr, use_thr, w, st); break;
    case 2: launch_nms<2, MODE, VEC>(s, masks, g, thr, use_thr, w, st); break;
    case 3: launch_nms<3, MODE, VEC>(s, masks, g, thr, use_thr, w, st); break;
    default: launch_nms<4, MODE, VEC>(s, masks, g, thr, use_thr, w, st); break;
  }
}

template <int KMAX>
static int launch_detect(const float* s, const float* masks, const DetectGeom& g, float thr, int use_thr,
                         int stages, const DetectWs& w, int64_t* det, float* scores, int32_t* n_det, int cap,
                         hipStream_t st) {
  if (stages & PEMP_DETECT_NMS) {
    ProfScope prof("detect_nms", st);
    const bool vec = (g.W % 4) == 0 && (reinterpret_cast<uintptr_t>(s) % 16) == 0 &&
                     (!masks || (reinterpret_cast<uintptr_t>(masks) % 16) == 0);
    if (use_thr) {
      if (vec) dispatch_nms<MODE_POS, true>(s, masks, g, thr, use_thr, w, st);
      else dispatch_nms<MODE_POS, false>(s, masks, g, thr, use_thr, w, st);
    } else {
      if (vec) dispatch_nms<MODE_ALL, true>(s, masks, g, thr, use_thr, w, st);
      else dispatch_nms<MODE_ALL, false>(s, masks, g, thr, use_thr, w, st);
    }
    PEMP_LAUNCH_CHECK();
  }
  if (stages & PEMP_DETECT_SELECT) {
    const size_t lds = (size_t)2 * g.J * g.S * sizeof(int);
    ProfScope prof("detect_select", st);
    hipLaunchKernelGGL(select_kernel<KMAX>, dim3(g.B), dim3(NT2), lds, st, s, masks, g, thr, use_thr, w.cand_v,
                       w.cand_i, w.neg_v, w.neg_i, w.tile_count, w.tile_nonneg, w.bits, det, scores, (int*)n_det, cap);
    PEMP_LAUNCH_CHECK();
  }
  return PEMP_OK;
}

}  // namespace
}  // namespace pemp

using namespace pemp;

extern "C" size_t pemp_detect_workspace_size(int B, int J, int H, int W, int topk) {
  if (B <= 0 || J <= 0 || H <= 0 || W <= 0) return 0;
  const int K = topk < H * W ? topk : H * W;
  size_t bytes = 0;
  carve(nullptr, geom(B, J, H, W, 1, K), &bytes);
  return bytes;
}

extern "C" int pemp_detect(const float* scoremaps, const float* masks, int B, int J, int H, int W, int pool_kernel,
                           float threshold, int use_threshold, int topk, int stages, void* workspace,
                           size_t workspace_bytes, int64_t* det_xyt, float* det_scores, int32_t* n_det, int cap,
                           void* stream) {
  PEMP_CHECK_ARG(scoremaps && workspace && det_xyt && det_scores && n_det, "pemp_detect: null pointer");
  PEMP_CHECK_ARG(B > 0 && J > 0 && J <= MAXJ && H > 0 && W > 0, "pemp_detect: bad shape B=%d J=%d H=%d W=%d", B, J, H, W);
  PEMP_CHECK_ARG(pool_kernel % 2 == 1 && pool_kernel >= 1 && pool_kernel / 2 <= MAXR,
                 "pemp_detect: pool_kernel must be odd and <= %d (got %d)", 2 * MAXR + 1, pool_kernel);
  PEMP_CHECK_ARG(topk >= 1 && topk <= 32, "pemp_detect: topk must be in [1, 32] (got %d)", topk);
  PEMP_CHECK_ARG(cap >= 0, "pemp_detect: cap < 0");
  PEMP_CHECK_ARG((size_t)H * W < 0x7fffffffull, "pemp_detect: plane too large");
  const int K = topk < H * W ? topk : H * W;
  const DetectGeom g = geom(B, J, H, W, pool_kernel, K);
  PEMP_CHECK_ARG(g.S * J * 2 * sizeof(int) <= 48 * 1024, "pemp_detect: H too large for the select stage");
  size_t need = 0;
  carve(nullptr, g, &need);
  if (workspace_bytes < need) {
    set_error("pemp_detect: workspace %zu < %zu bytes", workspace_bytes, need);
    return PEMP_ERR_WORKSPACE;
  }
  const DetectWs w = carve(workspace, g, nullptr);
  const hipStream_t st = as_stream(stream);
  if (K <= 8)
    return launch_detect<8>(scoremaps, masks, g, threshold, use_threshold, stages, w, det_xyt, det_scores, n_det,
                            cap, st);
  return launch_detect<32>(scoremaps, masks, g, threshold, use_threshold, stages, w, det_xyt, det_scores, n_det,
                           cap, st);
}
