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
constexpr int MAXR = 7;   // max pool radius (POOL_KERNEL_SIZE <= 15)
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
  float* cand_v; int* cand_i; int* tile_count; unsigned long long* bits;
};

static DetectWs carve(void* base, const DetectGeom& g, size_t* bytes) {
  Carver c(base);
  DetectWs w;
  size_t ncand = (size_t)g.B * g.J * g.tiles * 4 * g.K;
  w.cand_v = c.take<float>(ncand);
  w.cand_i = c.take<int>(ncand);
  w.tile_count = c.take<int>((size_t)g.B * g.J * g.tiles);
  w.bits = c.take<unsigned long long>((size_t)g.B * g.J * g.H * g.WW);
  if (bytes) *bytes = c.used;
  return w;
}

template <int KMAX>
__global__ __launch_bounds__(NT1) void nms_tiles_kernel(
    const float* __restrict__ s, const float* __restrict__ masks, DetectGeom g, float thr, int use_thr,
    float* __restrict__ cand_v, int* __restrict__ cand_i, int* __restrict__ tile_count,
    unsigned long long* __restrict__ bits) {
  extern __shared__ float lds[];
  __shared__ int wave_cnt[NT1 / 64];
  const int tile = blockIdx.x, t = blockIdx.y, b = blockIdx.z;
  const int ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
  const int y0 = ty * TR, x0 = tx * TC;
  const int p = g.p, H = g.H, W = g.W;
  const int LW = TC + 2 * p, LH = TR + 2 * p;
  float* in = lds;
  float* vm = lds + LH * LW;
  const float* plane = s + (size_t)(b * g.J + t) * H * W;

  // stage tile + halo (-inf outside the plane, as MaxPool2d's implicit padding)
  for (int idx = threadIdx.x; idx < LH * LW; idx += NT1) {
    const int r = idx / LW, c = idx - r * LW;
    const int y = y0 - p + r, x = x0 - p + c;
    in[idx] = (y >= 0 && y < H && x >= 0 && x < W) ? plane[(size_t)y * W + x] : -INFINITY;
  }
  __syncthreads();
  // vertical max over 2p+1 rows
  for (int idx = threadIdx.x; idx < TR * LW; idx += NT1) {
    const int r = idx / LW, c = idx - r * LW;
    float m = in[r * LW + c];
    for (int d = 1; d <= 2 * p; ++d) m = fmaxf(m, in[(r + d) * LW + c]);
    vm[idx] = m;
  }
  __syncthreads();

  const int r = threadIdx.x >> 3, cb = (threadIdx.x & 7) * 16;
  const int y = y0 + r;
  float tv[KMAX];
  int ti[KMAX];
#pragma unroll
  for (int q = 0; q < KMAX; ++q) { tv[q] = -INFINITY; ti[q] = 0x7fffffff; }
  unsigned int mybits = 0;
  if (y < H) {
    const float* mrow = masks ? masks + ((size_t)b * H + y) * W : nullptr;
    for (int j = 0; j < 16; ++j) {
      const int c = cb + j, x = x0 + c;
      if (x >= W) break;
      float m = vm[r * LW + c];
      for (int d = 1; d <= 2 * p; ++d) m = fmaxf(m, vm[r * LW + c + d]);
      const float sv = in[(r + p) * LW + c + p];
      float jm = (m == sv) ? 1.0f : 0.0f;
      if (mrow) jm = jm * mrow[x];
      const float v = sv * jm;
      const bool bit = use_thr && !(v < thr) && (v != 0.0f);
      mybits |= (unsigned)bit << j;
      float cv = v;
      int ci = y * W + x;
#pragma unroll
      for (int q = 0; q < KMAX; ++q) {
        if (better(cv, ci, tv[q], ti[q])) {
          const float sv2 = tv[q]; const int si2 = ti[q];
          tv[q] = cv; ti[q] = ci; cv = sv2; ci = si2;
        }
      }
    }
  }

  // wave-level exact top-K of the wave's pixels -> candidates
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t plane_tile = (size_t)(b * g.J + t) * g.tiles + tile;
  float* cv_out = cand_v + plane_tile * 4 * g.K + wave * g.K;
  int* ci_out = cand_i + plane_tile * 4 * g.K + wave * g.K;
  for (int q = 0; q < g.K; ++q) {
    float bv = tv[0];
    int bi = ti[0];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float ov = __shfl_xor(bv, off);
      const int oi = __shfl_xor(bi, off);
      if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { cv_out[q] = bv; ci_out[q] = bi; }
    if (ti[0] == bi && tv[0] == bv && bi != 0x7fffffff) {   // owner pops its head
#pragma unroll
      for (int k = 0; k < KMAX - 1; ++k) { tv[k] = tv[k + 1]; ti[k] = ti[k + 1]; }
      tv[KMAX - 1] = -INFINITY; ti[KMAX - 1] = 0x7fffffff;
    }
  }

  // threshold bitmask: 4 consecutive threads x 16 px = one 64-px word
  unsigned int lo = (threadIdx.x & 3) < 2 ? (mybits << (16 * (threadIdx.x & 1))) : 0u;
  unsigned int hi = (threadIdx.x & 3) >= 2 ? (mybits << (16 * (threadIdx.x & 1))) : 0u;
  lo |= __shfl_xor(lo, 1); hi |= __shfl_xor(hi, 1);
  lo |= __shfl_xor(lo, 2); hi |= __shfl_xor(hi, 2);
  const int word = x0 / 64 + ((threadIdx.x & 7) >> 2);
  if ((threadIdx.x & 3) == 0 && y < H && word < g.WW)
    bits[((size_t)(b * g.J + t) * H + y) * g.WW + word] = ((unsigned long long)hi << 32) | lo;

  int cnt = __popc(mybits);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
  if (lane == 0) wave_cnt[wave] = cnt;
  __syncthreads();
  if (threadIdx.x == 0)
    tile_count[plane_tile] = wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
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

template <int KMAX>
__global__ __launch_bounds__(NT2) void select_kernel(
    const float* __restrict__ s, const float* __restrict__ masks, DetectGeom g, float thr, int use_thr,
    const float* __restrict__ cand_v, const int* __restrict__ cand_i, const int* __restrict__ tile_count,
    const unsigned long long* __restrict__ bits, int64_t* __restrict__ det, float* __restrict__ scores,
    int* __restrict__ n_det, int cap) {
  extern __shared__ int sh_strip[];            // [J*S] counts, then [J*S] offsets
  __shared__ float top_v[MAXJ][KMAX];
  __shared__ float top_sc[MAXJ][KMAX];
  __shared__ int top_i[MAXJ][KMAX];
  __shared__ int top_bit[MAXJ][KMAX];
  __shared__ int n_top[MAXJ];
  __shared__ int scan_sh[40];
  const int b = blockIdx.x;
  const int J = g.J, H = g.H, W = g.W, K = g.K, S = g.S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = NT2 / 64;
  int* strip_cnt = sh_strip;
  int* strip_off = sh_strip + J * S;

  // (a) exact per-type top-K from the tile candidates
  const int ncand = g.tiles * 4 * K;
  for (int t = wave; t < J; t += nwaves) {
    const float* cv = cand_v + (size_t)(b * J + t) * ncand;
    const int* ci = cand_i + (size_t)(b * J + t) * ncand;
    float pv = INFINITY;
    int pi = -1;
    for (int q = 0; q < K; ++q) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int c = lane; c < ncand; c += 64) {
        const float v = cv[c];
        const int i = ci[c];
        if (better(pv, pi, v, i) && better(v, i, bv, bi)) { bv = v; bi = i; }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const float ov = __shfl_xor(bv, off);
        const int oi = __shfl_xor(bi, off);
        if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
      }
      if (lane == 0) { top_v[t][q] = bv; top_i[t][q] = bi; }
      pv = bv; pi = bi;
    }
    if (lane == 0) {
      // keep value != 0 (ConstructGraph.py:1174 nonzero), then order by flat index (y, x)
      int n = 0;
      for (int q = 0; q < K; ++q) {
        const float v = top_v[t][q];
        const float sc = use_thr ? v : v + 1e-10f;
        if (sc != 0.0f && top_i[t][q] != 0x7fffffff) {
          top_v[t][n] = v; top_sc[t][n] = sc; top_i[t][n] = top_i[t][q];
          ++n;
        }
      }
      for (int a = 1; a < n; ++a) {            // insertion sort by index
        const float v = top_v[t][a], sc = top_sc[t][a];
        const int i = top_i[t][a];
        int c = a - 1;
        while (c >= 0 && top_i[t][c] > i) {
          top_v[t][c + 1] = top_v[t][c]; top_sc[t][c + 1] = top_sc[t][c]; top_i[t][c + 1] = top_i[t][c];
          --c;
        }
        top_v[t][c + 1] = v; top_sc[t][c + 1] = sc; top_i[t][c + 1] = i;
      }
      for (int q = 0; q < n; ++q)
        top_bit[t][q] = use_thr && !(top_v[t][q] < thr) && top_v[t][q] != 0.0f;
      n_top[t] = n;
    }
  }
  __syncthreads();

  // (b) per-strip threshold counts minus top-k entries already listed (cat_unique)
  for (int e = threadIdx.x; e < J * S; e += NT2) {
    const int t = e / S, st = e - t * S;
    int c = 0;
    if (use_thr) {
      const int* tc = tile_count + (size_t)(b * J + t) * g.tiles + st * g.tiles_x;
      for (int x = 0; x < g.tiles_x; ++x) c += tc[x];
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

template <int KMAX>
static int launch_detect(const float* s, const float* masks, const DetectGeom& g, float thr, int use_thr,
                         int stages, const DetectWs& w, int64_t* det, float* scores, int32_t* n_det, int cap,
                         hipStream_t st) {
  if (stages & PEMP_DETECT_NMS) {
    const size_t lds = (size_t)((TR + 2 * g.p) + TR) * (TC + 2 * g.p) * sizeof(float);
    ProfScope prof("detect_nms", st);
    hipLaunchKernelGGL(nms_tiles_kernel<KMAX>, dim3(g.tiles, g.J, g.B), dim3(NT1), lds, st, s, masks, g, thr,
                       use_thr, w.cand_v, w.cand_i, w.tile_count, w.bits);
    PEMP_LAUNCH_CHECK();
  }
  if (stages & PEMP_DETECT_SELECT) {
    const size_t lds = (size_t)2 * g.J * g.S * sizeof(int);
    ProfScope prof("detect_select", st);
    hipLaunchKernelGGL(select_kernel<KMAX>, dim3(g.B), dim3(NT2), lds, st, s, masks, g, thr, use_thr, w.cand_v,
                       w.cand_i, w.tile_count, w.bits, det, scores, (int*)n_det, cap);
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
