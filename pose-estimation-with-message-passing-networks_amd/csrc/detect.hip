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
// Stage 2a (plane_top_kernel): one workgroup per plane. Merges the candidates into the exact
//   per-type top-k and counts threshold detections per 32-row strip.
// Stage 2b (emit_kernel): one workgroup per plane. Offsets from the image's per-plane counts;
//   emits detections in the reference's order.
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

constexpr int KCAP = 32;   // max top-k (pemp_detect checks topk <= 32)

struct DetectWs {
  float *cand_v, *neg_v; int *cand_i, *neg_i, *tile_count, *tile_nonneg; unsigned long long* bits;
  // per plane (image, type): sorted top-k list, threshold-set counts per strip and in-plane offsets
  float* ptop_sc; int *ptop_i, *ptop_bit, *pn_top, *pn_thr, *pstrip, *pstrip_off;
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
  const size_t np = (size_t)g.B * g.J;
  w.ptop_sc = c.take<float>(np * KCAP);
  w.ptop_i = c.take<int>(np * KCAP);
  w.ptop_bit = c.take<int>(np * KCAP);
  w.pn_top = c.take<int>(np);
  w.pn_thr = c.take<int>(np);
  w.pstrip = c.take<int>(np * g.S);
  w.pstrip_off = c.take<int>(np * g.S);
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

// Block-level exact top-`take` (take <= KMAX) of n candidates: each of the 4 waves reduces a
// quarter to its own top-`take` in LDS, wave 0 merges those. Returns the count (all threads).
template <int KMAX>
__device__ int block_topk(const float* __restrict__ cv, const int* __restrict__ ci, int n, int take, float* out_v,
                          int* out_i, float (*lv)[KMAX], int (*li)[KMAX], int* cnt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = (n + 3) / 4, lo = min(n, wave * q), hi = min(n, lo + q);
  const int got = merge_candidates<KMAX>(cv + lo, ci + lo, hi - lo, take, lv[wave], li[wave]);
  for (int k = got + lane; k < KMAX; k += 64) li[wave][k] = INV;
  __syncthreads();
  if (wave == 0) {
    const int m = merge_candidates<KMAX>(&lv[0][0], &li[0][0], 4 * KMAX, take, out_v, out_i);
    if (lane == 0) *cnt = m;
  }
  __syncthreads();
  const int m = *cnt;
  __syncthreads();
  return m;
}

// Stage 2a: one 256-thread workgroup per plane (image, type). Exact top-k from the stage-1 wave
// lists (ConstructGraph.py:1166-1174: top-k, nonzero, ordered by flat index), plus per-strip
// counts of threshold pixels not already in the top-k (cat_unique, ConstructGraph.py:1199-1209).
template <int KMAX>
__global__ __launch_bounds__(256) void plane_top_kernel(DetectGeom g, float thr, int use_thr,
                                                        const float* __restrict__ cand_v,
                                                        const int* __restrict__ cand_i,
                                                        const float* __restrict__ neg_v,
                                                        const int* __restrict__ neg_i,
                                                        const int* __restrict__ tile_count,
                                                        const int* __restrict__ tile_nonneg, DetectWs w) {
  __shared__ float lv[4][KMAX];
  __shared__ int li[4][KMAX];
  __shared__ float top_v[2 * KMAX], top_sc[KMAX];
  __shared__ int top_i[2 * KMAX], top_bit[KMAX], sh[8];
  const int pl = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = g.K, W = g.W, S = g.S, nl = g.tiles * 4;
  const size_t pt = (size_t)pl * nl;                  // first wave list of the plane
  int n = block_topk<KMAX>(cand_v + pt * K, cand_i + pt * K, nl * K, K, top_v, top_i, lv, li, &sh[0]);
  if (use_thr) {
    // degenerate plane (fewer than K non-negative pixels): its top-k also holds negatives
    int nn = 0;
    for (int c = threadIdx.x; c < nl; c += 256) nn += tile_nonneg[pt + c];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) nn += __shfl_xor(nn, off);
    if (lane == 0) sh[4 + wave] = nn;
    __syncthreads();
    nn = sh[4] + sh[5] + sh[6] + sh[7];
    if (nn < K) n += block_topk<KMAX>(neg_v + pt * K, neg_i + pt * K, nl * K, K - nn, top_v + n, top_i + n, lv, li, &sh[1]);
  }
  if (threadIdx.x == 0) {
    int m = 0;
    for (int q = 0; q < n; ++q) {
      const float v = top_v[q];
      const float sc = use_thr ? v : v + 1e-10f;
      if (sc != 0.0f && top_i[q] != INV) { top_v[m] = v; top_sc[m] = sc; top_i[m] = top_i[q]; ++m; }
    }
    for (int a2 = 1; a2 < m; ++a2) {            // insertion sort by flat index
      const float v = top_v[a2], sc = top_sc[a2];
      const int i = top_i[a2];
      int c = a2 - 1;
      while (c >= 0 && top_i[c] > i) { top_v[c + 1] = top_v[c]; top_sc[c + 1] = top_sc[c]; top_i[c + 1] = top_i[c]; --c; }
      top_v[c + 1] = v; top_sc[c + 1] = sc; top_i[c + 1] = i;
    }
    for (int q = 0; q < m; ++q) {
      top_bit[q] = use_thr && !(top_v[q] < thr) && top_v[q] != 0.0f;
      w.ptop_i[(size_t)pl * KCAP + q] = top_i[q];
      w.ptop_sc[(size_t)pl * KCAP + q] = top_sc[q];
      w.ptop_bit[(size_t)pl * KCAP + q] = top_bit[q];
    }
    w.pn_top[pl] = m;
    sh[0] = m;
  }
  __syncthreads();
  const int m = sh[0];
  // per-strip threshold counts minus the top-k entries already listed
  for (int st = threadIdx.x; st < S; st += 256) {
    int c = 0;
    if (use_thr) {
      const int* tc = tile_count + pt + (size_t)st * g.tiles_x * 4;
      for (int x = 0; x < 4 * g.tiles_x; ++x) c += tc[x];
      for (int q = 0; q < m; ++q)
        if (top_bit[q] && top_i[q] / W / TR == st) --c;
    }
    w.pstrip[(size_t)pl * S + st] = c;
  }
  __syncthreads();
  // in-plane exclusive scan over strips (wave 0, chunks of 64)
  if (wave == 0) {
    int carry = 0;
    for (int c0 = 0; c0 < S; c0 += 64) {
      const int st = c0 + lane;
      const int v = st < S ? w.pstrip[(size_t)pl * S + st] : 0;
      int x = v;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(x, off);
        if (lane >= off) x += o;
      }
      if (st < S) w.pstrip_off[(size_t)pl * S + st] = carry + x - v;
      carry += __shfl(x, 63);
    }
    if (lane == 0) w.pn_thr[pl] = carry;
  }
}

// Stage 2b: one workgroup per plane. The plane's output offsets follow from the per-plane counts
// of its image: [top-k dets of types 0..J-1] ++ [threshold dets, type-major, strip order].
__global__ __launch_bounds__(256) void emit_kernel(const float* __restrict__ s, const float* __restrict__ masks,
                                                   DetectGeom g, const unsigned long long* __restrict__ bits,
                                                   DetectWs w, int64_t* __restrict__ det,
                                                   float* __restrict__ scores, int* __restrict__ n_det, int cap) {
  __shared__ int top_i[KCAP], top_bit[KCAP], sh[4];
  const int pl = blockIdx.x, J = g.J, b = pl / J, t = pl - b * J;
  const int H = g.H, W = g.W, S = g.S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave == 0) {
    // J <= 32: one lane per type of this image
    const int nt = lane < J ? w.pn_top[b * J + lane] : 0, nh = lane < J ? w.pn_thr[b * J + lane] : 0;
    int top_before = lane < t ? nt : 0, thr_before = lane < t ? nh : 0, top_all = nt, thr_all = nh;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      top_before += __shfl_xor(top_before, off); thr_before += __shfl_xor(thr_before, off);
      top_all += __shfl_xor(top_all, off); thr_all += __shfl_xor(thr_all, off);
    }
    const int ntop = __shfl(nt, t);
    if (lane == 0) {
      sh[0] = top_before; sh[1] = top_all + thr_before; sh[2] = ntop;
      if (t == 0) n_det[b] = top_all + thr_all;
    }
    if (lane < ntop) { top_i[lane] = w.ptop_i[(size_t)pl * KCAP + lane]; top_bit[lane] = w.ptop_bit[(size_t)pl * KCAP + lane]; }
  }
  __syncthreads();
  const int ntop = sh[2], top_base = sh[0], thr_base = sh[1];
  int64_t* dout = det + (size_t)b * cap * 3;
  float* sout = scores + (size_t)b * cap;
  if ((int)threadIdx.x < ntop) {
    const int pos = top_base + threadIdx.x;
    if (pos < cap) {
      const int idx = top_i[threadIdx.x];
      dout[pos * 3 + 0] = idx % W;
      dout[pos * 3 + 1] = idx / W;
      dout[pos * 3 + 2] = t;
      sout[pos] = w.ptop_sc[(size_t)pl * KCAP + threadIdx.x];
    }
  }
  // threshold detections, one wave per non-empty strip
  for (int st = wave; st < S; st += 4) {
    if (w.pstrip[(size_t)pl * S + st] == 0) continue;     // wave-uniform
    const int ry0 = st * TR, rows = min(TR, H - ry0);
    const int nw = rows * g.WW;
    const int chunk = (nw + 63) / 64;
    const unsigned long long* wsrc = bits + ((size_t)pl * H + ry0) * g.WW;
    int cnt = 0;
    for (int k = 0; k < chunk; ++k) {
      const int wi = lane * chunk + k;
      if (wi >= nw) break;
      unsigned long long word = wsrc[wi];
      if (word) {
        for (int q = 0; q < ntop; ++q) {
          if (!top_bit[q]) continue;
          const int idx = top_i[q], yy = idx / W, xx = idx - yy * W;
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
    int pos = thr_base + w.pstrip_off[(size_t)pl * S + st] + pre - cnt;
    const float* plane = s + (size_t)pl * H * W;
    for (int k = 0; k < chunk; ++k) {
      const int wi = lane * chunk + k;
      if (wi >= nw) break;
      unsigned long long word = wsrc[wi];
      if (!word) continue;
      for (int q = 0; q < ntop; ++q) {
        if (!top_bit[q]) continue;
        const int idx = top_i[q], yy = idx / W, xx = idx - yy * W;
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
    {
      ProfScope prof("detect_top", st);
      hipLaunchKernelGGL(plane_top_kernel<KMAX>, dim3(g.B * g.J), dim3(256), 0, st, g, thr, use_thr, w.cand_v,
                         w.cand_i, w.neg_v, w.neg_i, w.tile_count, w.tile_nonneg, w);
      PEMP_LAUNCH_CHECK();
    }
    ProfScope prof("detect_emit", st);
    hipLaunchKernelGGL(emit_kernel, dim3(g.B * g.J), dim3(256), 0, st, s, masks, g, w.bits, w, det, scores,
                       (int*)n_det, cap);
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
