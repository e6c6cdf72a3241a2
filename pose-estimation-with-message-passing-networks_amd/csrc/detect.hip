// Keypoint detection from heatmaps — restates, for gfx950:
//   Utils/Utils.py:15-20          non_maximum_suppression: MaxPool2d(k,1,k//2) == s (-inf padding)
//   ConstructGraph.py:1161-1196   joint_det_from_scoremap: s *= maxima (* mask); per-type top-k;
//                                 threshold set; (DETECT_THRESHOLD > 1.5: top-20 + 1e-10)
//   ConstructGraph.py:1199-1209   cat_unique ordering
//
// Stage 1 (nms_strips_kernel, HBM-bound, no LDS): one WAVE per unit = 16 rows x (64 - 2P)
//   columns of one (image, type) plane; lane c owns column x0 - P + c (lanes < P and >= 64 - P
//   are the halo). The lane's column is loaded once (16 + 2P rows, coalesced across lanes, the
//   next unit's rows already in flight), the vertical max runs in registers, the horizontal max
//   with DPP whole-wave lane shifts; per-row predicates accumulate as per-lane row bitmasks
//   (counts are popcounts). Emits per unit: the K best (v, flat index) candidates (ties -> lower
//   index), threshold / non-negative counts, and the lanes' 16-bit threshold column masks.
// Stage 2a (plane_top_kernel): one workgroup per plane. Merges the candidates into the exact
//   per-type top-k and counts threshold detections per 16-row band.
// Stage 2b (emit_kernel): one workgroup per plane. Offsets from the image's per-plane counts;
//   emits detections in the reference's order.
#include <math.h>
#include <cmath>
#include <atomic>

#include <type_traits>

#include "pemp_common.h"

namespace pemp {
namespace {

#ifndef NMS_SR
#define NMS_SR 16
#endif
#ifndef NMS_PREFETCH
#define NMS_PREFETCH 1
#endif
#ifndef NMS_XCD_MAP
#define NMS_XCD_MAP 1   // XCD-sliced unit windows (1.0x HBM fetch vs 1.5x without)
#endif
#ifndef NMS_RESERVE_CUS
#define NMS_RESERVE_CUS 0   // CUs the strip kernel leaves free (PEMP_NMS_RESERVE_CUS overrides)
#endif
#ifndef NMS_PER_CU
#define NMS_PER_CU 5
#endif
#ifndef PEMP_DETECT_CLOCKS
#define PEMP_DETECT_CLOCKS 0
#endif   // diagnostics: phase clocks of the fused select + emit stage (printf)
#ifndef NMS_THR_POS
#define NMS_THR_POS 1   // positive thresholds take the one-compare threshold test (nms_strips_kernel TP)
#endif
#ifndef NMS_CLAMPED_LOADS
#define NMS_CLAMPED_LOADS 1
#endif
constexpr int SR = NMS_SR;  // rows per unit (= band height of the threshold bitmask)
static_assert(SR <= 32, "column masks are at most 32-bit");
// a lane's threshold bits over the SR rows of its unit column
using cmask_t = typename std::conditional<(SR > 16), uint32_t, uint16_t>::type;
constexpr int MAXR = 4;   // max pool radius (POOL_KERNEL_SIZE <= 9)
constexpr int MAXJ = 32;
constexpr int MAXB = 256;   // max bands per plane (H <= 4096)
constexpr int NT1 = 256;  // stage-1 workgroup: 4 independent waves
constexpr int INV = 0x7fffffff;
enum { MODE_POS = 0, MODE_ALL = 1 };

__device__ __forceinline__ bool better(float v1, int i1, float v2, int i2) {
  return v1 > v2 || (v1 == v2 && i1 < i2);
}

// Unit grid: nb bands of SR rows x nsx strips of sc = 64 - 2p columns per plane; lane c of a
// unit owns column x = strip * sc - p + c.
//
// Quad layout (NMS_QUAD, dense MODE_POS detection without masks; nms_quad_kernel): units are 16 rows x 64 columns
// with no halo lanes (sc = 64, p = 0: lane c of a unit <-> column strip * 64 + c), and the pool radius is pr. The NMS
// pass walks blocks of 16 rows x 256 columns (4 units side by side, 4 columns per lane), nbx per band.
struct DetectGeom {
  int B, J, H, W, p, K, sc, nsx, nb, units, S;
  unsigned mu, mn;   // unsigned division by units / nsx: q = (umulhi(n, m) + n) >> l (n < 2^31)
  int lu, ln;
  int pr, quad, nbx, blocks;   // pool radius; quad layout; blocks per band / per plane (quad layout)
  unsigned mq, mx;             // division by blocks / nbx
  int lq, lx;
};

// Granlund-Montgomery constants of an unsigned division by d >= 1 for dividends below 2^31
static void fastdiv_consts(unsigned d, unsigned& m, int& l) {
  l = 0;
  while ((1ull << l) < d) ++l;
  m = (unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
}

__device__ __forceinline__ int fastdiv(int n, unsigned m, int l) {
  return (int)((__umulhi((unsigned)n, m) + (unsigned)n) >> l);
}

// plane, band and strip of unit u (wave-uniform; a few scalar instructions instead of two divisions)
struct UnitPos {
  int plane, band, strip;
};
__device__ __forceinline__ UnitPos unit_pos(const DetectGeom& g, int u) {
  UnitPos q;
  q.plane = fastdiv(u, g.mu, g.lu);
  const int rem = u - q.plane * g.units;
  q.band = fastdiv(rem, g.mn, g.ln);
  q.strip = rem - q.band * g.nsx;
  return q;
}

static DetectGeom geom(int B, int J, int H, int W, int pool_k, int K, bool quad = false) {
  DetectGeom g;
  g.B = B; g.J = J; g.H = H; g.W = W; g.p = pool_k / 2; g.K = K;
  g.pr = pool_k / 2;
  g.quad = quad ? 1 : 0;
  if (quad) g.p = 0;
  g.sc = 64 - 2 * g.p;
  g.nsx = (W + g.sc - 1) / g.sc;
  g.nb = (H + SR - 1) / SR;
  g.units = g.nb * g.nsx;
  g.S = g.nb;
  fastdiv_consts((unsigned)g.units, g.mu, g.lu);
  fastdiv_consts((unsigned)g.nsx, g.mn, g.ln);
  g.nbx = (g.nsx + 3) / 4;
  g.blocks = g.nb * g.nbx;
  fastdiv_consts((unsigned)g.blocks, g.mq, g.lq);
  fastdiv_consts((unsigned)g.nbx, g.mx, g.lx);
  return g;
}

constexpr int KCAP = 32;   // max top-k (pemp_detect checks topk <= 32)

struct DetectWs {
  float *cand_v, *neg_v; int *cand_i, *neg_i, *tile_count, *tile_nonneg;
  cmask_t* cbits;    // threshold bits per (unit, lane): bit j <-> row y0 + j of the lane's column
  // per plane (image, type): sorted top-k list, threshold-set counts per band and in-plane offsets
  float* ptop_sc; int *ptop_i, *ptop_bit, *pn_top, *pn_thr, *pstrip, *pstrip_off;
  // per plane, the fused stage's publication: bit 63 set once published, bits 32..47 the top-k count, bits 0..31
  // the threshold count -- one 64-bit word, so one relaxed device-scope atomic carries all of it (zeroed by stage 1)
  unsigned long long* pflag;
};

static DetectWs carve(void* base, const DetectGeom& g, size_t* bytes) {
  Carver c(base);
  DetectWs w;
  const size_t nu = (size_t)g.B * g.J * g.units;
  w.cand_v = c.take<float>(nu * g.K);
  w.cand_i = c.take<int>(nu * g.K);
  w.neg_v = c.take<float>(nu * g.K);
  w.neg_i = c.take<int>(nu * g.K);
  w.tile_count = c.take<int>(nu);
  w.tile_nonneg = c.take<int>(nu);
  w.cbits = c.take<cmask_t>(nu * 64);
  const size_t np = (size_t)g.B * g.J;
  w.ptop_sc = c.take<float>(np * KCAP);
  w.ptop_i = c.take<int>(np * KCAP);
  w.ptop_bit = c.take<int>(np * KCAP);
  w.pn_top = c.take<int>(np);
  w.pn_thr = c.take<int>(np);
  w.pstrip = c.take<int>(np * g.S);
  w.pstrip_off = c.take<int>(np * g.S);
  w.pflag = c.take<unsigned long long>(np);
  if (bytes) *bytes = c.used;
  return w;
}

// Candidates (exact):
//   MODE_POS (threshold set in use): per unit the top-K of the POSITIVE values. Zero-valued top-k
//     entries are never emitted, and negatives can enter a plane's top-k only when the plane has
//     fewer than K non-negative pixels, so the unit also reports its non-negative count and, when
//     that count is below K, the top-K of its negative values.
//   MODE_ALL (DETECT_THRESHOLD > 1.5: every top-k entry is emitted as value + 1e-10): the exact
//     top-K of all pixels.

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

// K rounds: pop the wave's best among the lane's SR values that pass `keep` (value j has flat index
// base_id + j * stride, increasing in j); the winner lane removes the value and rescans. Writes
// out_v/out_i[k] (sentinels once exhausted).
template <typename Keep>
__device__ __forceinline__ void wave_topk(float (&v)[SR], int base_id, int stride, int K, Keep keep, float* out_v,
                                          int* out_i) {
  const int lane = threadIdx.x & 63;
  float lbv = -INFINITY;
  int lbj = -1;
#pragma unroll
  for (int j = 0; j < SR; ++j)
    if (keep(v[j]) && (lbj < 0 || v[j] > lbv)) { lbv = v[j]; lbj = j; }
  for (int k = 0; k < K; ++k) {
    float bv = lbj < 0 ? -INFINITY : lbv;
    int bi = lbj < 0 ? INV : base_id + lbj * stride;
    wave_best(bv, bi);
    if (lane == 0) { out_v[k] = bv; out_i[k] = bi; }
    if (bi == INV) {                               // wave exhausted: fill with sentinels
      for (int k2 = k + 1; k2 < K; ++k2)
        if (lane == 0) { out_v[k2] = -INFINITY; out_i[k2] = INV; }
      break;
    }
    if (lbj >= 0 && bi == base_id + lbj * stride) {   // this lane owned the winner
#pragma unroll
      for (int j = 0; j < SR; ++j)
        if (j == lbj) v[j] = NAN;                  // removed (fails every keep predicate)
      lbj = -1;
      lbv = -INFINITY;
#pragma unroll
      for (int j = 0; j < SR; ++j)
        if (keep(v[j]) && (lbj < 0 || v[j] > lbv)) { lbv = v[j]; lbj = j; }
    }
  }
}

__device__ __forceinline__ void write_sentinels(float* out_v, int* out_i, int K) {
  const int lane = threadIdx.x & 63;
  if (lane < K) { out_v[lane] = -INFINITY; out_i[lane] = INV; }
}

// whole-wave lane shifts (gfx9 DPP wave_shr:1 / wave_shl:1); lanes without a source get 0 —
// only halo lanes see that, and their outputs are discarded.
__device__ __forceinline__ float wave_shr1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_shl1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xF, 0xF, true));
}

// ---- test-time front-end evaluated on demand (pemp_detect_projected) -------------
// s[b, j, Y, X] = (sum_s avg_s) / divisor, avg_s = (up(maps_s)[b, j] + up(flip(flip_maps_s))[b, fi[j]]) / 2
// (or up(maps_s)[b, j] without a flipped pass). up = bilinear to H x W, align_corners=False, torch's
// source index (area_pixel_compute_source_index); every product and sum rounded in fp32 in the order
// t0 = a lx0 + b lx1, t1 = c lx0 + d lx1, v = t0 ly0 + t1 ly1 (as pemp_gather_projected). flip mirrors
// the columns of the low-resolution map (torch.flip(output, [3]) before the interpolation).
struct ProjArgs {
  int S, C;                            // scales; channels of every map
  const float* m[PEMP_PROJ_MAXS];      // [B][C][h][w]
  const float* f[PEMP_PROJ_MAXS];      // flipped pass, or NULL
  int h[PEMP_PROJ_MAXS], w[PEMP_PROJ_MAXS];
  const int* fi;                       // [J] or NULL
  float divisor;
  float rdiv;                          // 1 / divisor when that is exact (a power of two), else 0
  int ch0;                             // first channel read (0: heatmaps; J: tags)
};

// v / divisor: a product with the exact reciprocal when the divisor is a power of two (the same real, so the
// same rounding, for every v), the IEEE division otherwise (~10 instructions: the single-scale front-end's
// divisor 1 took 20 of them per lane and unit)
__device__ __forceinline__ float proj_div(const ProjArgs& pj, float v) {
  return pj.rdiv != 0.f ? __fmul_rn(v, pj.rdiv) : div_rn(v, pj.divisor);
}

struct ProjTaps {   // one axis of the bilinear source index
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ ProjTaps proj_taps(int dst, int out_size, int in_size) {
  ProjTaps t;
  const float scale = (float)in_size / (float)out_size;
  float src = __fsub_rn(__fmul_rn(scale, __fadd_rn((float)dst, 0.5f)), 0.5f);
  if (src < 0.f) src = 0.f;
  t.i0 = (int)src;
  t.i1 = t.i0 + (t.i0 < in_size - 1 ? 1 : 0);
  t.l1 = fminf(fmaxf(__fsub_rn(src, (float)t.i0), 0.f), 1.f);
  t.l0 = __fsub_rn(1.f, t.l1);
  return t;
}

__device__ __forceinline__ float bilerp(const float* pl, int w, const ProjTaps& ty, int x0, int x1, float lx0,
                                        float lx1) {
  const float a = pl[ty.i0 * w + x0], b = pl[ty.i0 * w + x1];
  const float c = pl[ty.i1 * w + x0], d = pl[ty.i1 * w + x1];
  const float t0 = __fadd_rn(__fmul_rn(a, lx0), __fmul_rn(b, lx1));
  const float t1 = __fadd_rn(__fmul_rn(c, lx0), __fmul_rn(d, lx1));
  return __fadd_rn(__fmul_rn(t0, ty.l0), __fmul_rn(t1, ty.l1));
}

// one scale's (flip-averaged) value at row taps ty and the column's taps tx (tx of the unflipped map)
__device__ __forceinline__ float proj_scale(const ProjArgs& pj, int s, int b, int j, const ProjTaps& ty,
                                            const ProjTaps& tx) {
  const int h = pj.h[s], w = pj.w[s];
  const float v0 = bilerp(pj.m[s] + ((size_t)b * pj.C + pj.ch0 + j) * h * w, w, ty, tx.i0, tx.i1, tx.l0, tx.l1);
  if (!pj.f[s]) return v0;
  const int jf = pj.fi ? pj.fi[j] : j;
  const float v1 = bilerp(pj.f[s] + ((size_t)b * pj.C + pj.ch0 + jf) * h * w, w, ty, w - 1 - tx.i0, w - 1 - tx.i1,
                          tx.l0, tx.l1);
  return __fmul_rn(__fadd_rn(v0, v1), 0.5f);   // (a + b) / 2.0: the division by 2 is exact
}

__device__ float proj_pixel(const ProjArgs& pj, int b, int j, int Y, int X, int H, int W) {
  float acc = 0.f;
  for (int s = 0; s < pj.S; ++s) {
    const float v = proj_scale(pj, s, b, j, proj_taps(Y, H, pj.h[s]), proj_taps(X, W, pj.w[s]));
    acc = s == 0 ? v : __fadd_rn(acc, v);
  }
  return proj_div(pj, acc);
}

// r / divisor, -inf outside the plane; the divisor's form decided once per unit, not per row (uniform)
template <int P>
__device__ __forceinline__ void proj_finish(const ProjArgs& pj, const DetectGeom& g, int y0, bool xok,
                                            float (&r)[SR + 2 * P]) {
  if (pj.rdiv != 0.f) {
#pragma unroll
    for (int i = 0; i < SR + 2 * P; ++i) {
      const int y = y0 - P + i;
      r[i] = (xok && y >= 0 && y < g.H) ? __fmul_rn(r[i], pj.rdiv) : -INFINITY;
    }
  } else {
#pragma unroll
    for (int i = 0; i < SR + 2 * P; ++i) {
      const int y = y0 - P + i;
      r[i] = (xok && y >= 0 && y < g.H) ? div_rn(r[i], pj.divisor) : -INFINITY;
    }
  }
}

// rows y0 - P .. y0 + SR - 1 + P of the lane's column from the projected maps; -inf outside the plane
template <int P>
__device__ __forceinline__ void load_unit_proj(const ProjArgs& pj, const DetectGeom& g, int u, float (&r)[SR + 2 * P]) {
  const int lane = threadIdx.x & 63;
  const int plane = u / g.units, rem = u - plane * g.units, band = rem / g.nsx, strip = rem - band * g.nsx;
  const int b = plane / g.J, j = plane - b * g.J;
  const int y0 = band * SR, x = strip * g.sc - P + lane;
  const bool xok = x >= 0 && x < g.W;
  const int xc = min(max(x, 0), g.W - 1);
#pragma unroll
  for (int i = 0; i < SR + 2 * P; ++i) r[i] = 0.f;
  for (int s = 0; s < pj.S; ++s) {
    const ProjTaps tx = proj_taps(xc, g.W, pj.w[s]);
#pragma unroll
    for (int i = 0; i < SR + 2 * P; ++i) {
      const int yc = min(max(y0 - P + i, 0), g.H - 1);
      const float v = proj_scale(pj, s, b, j, proj_taps(yc, g.H, pj.h[s]), tx);
      r[i] = s == 0 ? v : __fadd_rn(r[i], v);
    }
  }
  proj_finish<P>(pj, g, y0, xok, r);
}

// The same rows, separably: per scale and map, the horizontal interpolation of every low-resolution row
// the unit's output rows touch (at most PROJ_LR - 1 of them: upsampling) is computed once per lane and
// staged in the wave's LDS rows; the vertical interpolation of each output row then reads its two staged
// rows. The values are bitwise those of proj_pixel (same operations on the same operands). Ratios needing
// more rows take load_unit_proj.
// Loads: one SGPR buffer descriptor per map, the lane's two source columns as its only VGPR offsets and
// the (clamped, uniform) source row as the scalar offset -- no per-load address arithmetic. The staged
// rows run one past the unit's last source row (clamped to the map), so a row's second tap is always the
// next stage row (i1 = i0 + 1, or at the bottom border the duplicate of row h - 1, whose horizontal value
// is the same operands'): one ds_read2 per map and output row.
constexpr int PROJ_LR = 16;
#ifndef PROJ_X2
#define PROJ_X2 1   // the register-only loader for interior bands of an exact 2x upsampling (proj_x2_first)
#endif

// horizontal interpolation of rows lo .. lo + nl - 1 (clamped to the map) of the forward pass and, FLIP,
// the flipped pass into the wave's stage rows; groups of 4 rows of both maps (16 loads) under one wait
template <bool FLIP>
__device__ __forceinline__ void proj_rows_maps(const float* pl0, const float* pl1, int w, int h, int lo, int nl,
                                               int x0, int x1, float lx0, float lx1, float* __restrict__ st0,
                                               float* __restrict__ st1) {
  const int lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(pl0), 0, h * w * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(FLIP ? pl1 : pl0), 0, h * w * 4, 0x00020000);
  const int va = 4 * x0, vb = 4 * x1, vc = 4 * (w - 1 - x0), vd = 4 * (w - 1 - x1);   // flipped: mirrored columns
  const int rowb = 4 * w;
#pragma unroll
  for (int k0 = 0; k0 < PROJ_LR; k0 += 4) {
    if (k0 < nl) {   // (uniform)
      float a[4], b[4], c[4], d[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int so = min(lo + k0 + k, h - 1) * rowb;   // rows past the range: loaded, never read
        a[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r0, va, so, 0));
        b[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r0, vb, so, 0));
        if constexpr (FLIP) {
          c[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r1, vc, so, 0));
          d[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r1, vd, so, 0));
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        st0[(k0 + k) * 64 + lane] = __fadd_rn(__fmul_rn(a[k], lx0), __fmul_rn(b[k], lx1));
        if constexpr (FLIP) st1[(k0 + k) * 64 + lane] = __fadd_rn(__fmul_rn(c[k], lx0), __fmul_rn(d[k], lx1));
      }
    }
  }
}

// (the host checks that every unit's rows span at most PROJ_LR - 1 low-resolution rows: proj_sep_ok)
template <int P, bool FLIP, bool FIRST>
__device__ __forceinline__ void proj_sep_scale(const ProjArgs& pj, const DetectGeom& g, int s, int b, int j, int y0,
                                               int xc, float (&r)[SR + 2 * P], float* __restrict__ stage) {
  const int lane = threadIdx.x & 63;
  const int h = pj.h[s], w = pj.w[s];
  const int ya = min(max(y0 - P, 0), g.H - 1), yb = min(max(y0 + SR + P - 1, 0), g.H - 1);
  const int lo = proj_taps(ya, g.H, h).i0, nl = proj_taps(yb, g.H, h).i1 - lo + 2;
  const ProjTaps tx = proj_taps(xc, g.W, w);
  float* st0 = stage;                    // forward pass rows
  float* st1 = stage + PROJ_LR * 64;     // flipped pass rows
  __builtin_amdgcn_wave_barrier();   // the previous readers of the wave's rows are done
  proj_rows_maps<FLIP>(pj.m[s] + ((size_t)b * pj.C + pj.ch0 + j) * h * w,
                       FLIP ? pj.f[s] + ((size_t)b * pj.C + pj.ch0 + (pj.fi ? pj.fi[j] : j)) * h * w : nullptr, w, h,
                       lo, nl, tx.i0, tx.i1, tx.l0, tx.l1, st0, st1);
  // the rows' taps (uniform per row) computed once per unit by lanes 0 .. SR + 2P - 1 and read back as LDS
  // broadcasts: (byte offset of the first source row in the stage, weights)
  float4* tap = reinterpret_cast<float4*>(stage + 2 * PROJ_LR * 64);
  if (lane < SR + 2 * P) {
    const ProjTaps t = proj_taps(min(max(y0 - P + lane, 0), g.H - 1), g.H, h);
    tap[lane] = make_float4(__int_as_float((t.i0 - lo) * 256), 0.f, t.l0, t.l1);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const char* b0 = reinterpret_cast<const char*>(st0 + lane);
  const char* b1 = reinterpret_cast<const char*>(st1 + lane);
#pragma unroll
  for (int i = 0; i < SR + 2 * P; ++i) {
    const float4 t = tap[i];
    const float* p0 = reinterpret_cast<const float*>(b0 + __float_as_int(t.x));
    float v = __fadd_rn(__fmul_rn(p0[0], t.z), __fmul_rn(p0[64], t.w));
    if constexpr (FLIP) {
      const float* p1 = reinterpret_cast<const float*>(b1 + __float_as_int(t.x));
      v = __fmul_rn(__fadd_rn(v, __fadd_rn(__fmul_rn(p1[0], t.z), __fmul_rn(p1[64], t.w))), 0.5f);
    }
    r[i] = FIRST ? v : __fadd_rn(r[i], v);
  }
}

// Exact 2x upsampling (h * 2 == H, the single-scale test front-end of a stride-2 output): out row Y's
// source index is Y / 2 - 0.25 in fp32 with no rounding, so an even Y reads rows (Y / 2 - 1, Y / 2) with
// weights (0.25, 0.75) and an odd Y rows ((Y - 1) / 2, (Y + 1) / 2) with (0.75, 0.25) -- what proj_taps
// computes, as constants. Since y0 is even, the row of every output row i relative to y0 / 2 is a
// compile-time constant, so a band whose rows need no clamping (y0 - P >= 1, y0 + SR - 1 + P <= H - 3)
// keeps its NL source rows' horizontal values in registers: no LDS stage, no tap table, no waits on LDS.
template <int P>
__host__ __device__ constexpr int x2_row(int i) {   // source row of output row i (tap 0), relative to y0 / 2
  return ((i - P) & 1) == 0 ? (i - P) / 2 - 1 : (i - P - 1) / 2;
}

template <int P, bool FLIP>
__device__ __forceinline__ void proj_x2_first(const ProjArgs& pj, const DetectGeom& g, int b, int j, int y0, int xc,
                                              float (&r)[SR + 2 * P]) {
  constexpr int NR = SR + 2 * P, LO = x2_row<P>(0), NL = x2_row<P>(NR - 1) + 2 - LO;
  const int h = pj.h[0], w = pj.w[0];
  const ProjTaps tx = proj_taps(xc, g.W, w);
  const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(pj.m[0] + ((size_t)b * pj.C + pj.ch0 + j) * h * w), 0, h * w * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(FLIP ? pj.f[0] + ((size_t)b * pj.C + pj.ch0 + (pj.fi ? pj.fi[j] : j)) * h * w : pj.m[0]), 0,
      h * w * 4, 0x00020000);
  const int va = 4 * tx.i0, vb = 4 * tx.i1, vc = 4 * (w - 1 - tx.i0), vd = 4 * (w - 1 - tx.i1);
  const int rowb = 4 * w;
  int so = (y0 / 2 + LO) * rowb;
  float a[NL], bb[NL], c[NL], d[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    a[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r0, va, so, 0));
    bb[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r0, vb, so, 0));
    if constexpr (FLIP) {
      c[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r1, vc, so, 0));
      d[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r1, vd, so, 0));
    }
    so += rowb;
  }
  float h0[NL], h1[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    h0[k] = __fadd_rn(__fmul_rn(a[k], tx.l0), __fmul_rn(bb[k], tx.l1));
    if constexpr (FLIP) h1[k] = __fadd_rn(__fmul_rn(c[k], tx.l0), __fmul_rn(d[k], tx.l1));
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    constexpr float q = 0.25f, t = 0.75f;
    const int k = x2_row<P>(i) - LO;
    const bool even = ((i - P) & 1) == 0;
    const float w0 = even ? q : t, w1 = even ? t : q;
    float v = __fadd_rn(__fmul_rn(h0[k], w0), __fmul_rn(h0[k + 1], w1));
    if constexpr (FLIP) v = __fmul_rn(__fadd_rn(v, __fadd_rn(__fmul_rn(h1[k], w0), __fmul_rn(h1[k + 1], w1))), 0.5f);
    r[i] = v;
  }
}

template <int P>
__device__ __forceinline__ void load_unit_proj_sep(const ProjArgs& pj, const DetectGeom& g, int u,
                                                   float (&r)[SR + 2 * P], float* __restrict__ stage) {
  const int lane = threadIdx.x & 63;
  const UnitPos q = unit_pos(g, u);
  const int b = q.plane / g.J, j = q.plane - b * g.J;
  const int y0 = q.band * SR, x = q.strip * g.sc - P + lane;
  const bool xok = x >= 0 && x < g.W;
  const int xc = min(max(x, 0), g.W - 1);
  if (PROJ_X2 && pj.h[0] * 2 == g.H && y0 - P >= 1 && y0 + SR - 1 + P <= g.H - 3) {   // (uniform)
    if (pj.f[0]) proj_x2_first<P, true>(pj, g, b, j, y0, xc, r);
    else proj_x2_first<P, false>(pj, g, b, j, y0, xc, r);
  } else if (pj.f[0]) {
    proj_sep_scale<P, true, true>(pj, g, 0, b, j, y0, xc, r, stage);
  } else {
    proj_sep_scale<P, false, true>(pj, g, 0, b, j, y0, xc, r, stage);
  }
  for (int s = 1; s < pj.S; ++s) {
    if (pj.f[s]) proj_sep_scale<P, true, false>(pj, g, s, b, j, y0, xc, r, stage);
    else proj_sep_scale<P, false, false>(pj, g, s, b, j, y0, xc, r, stage);
  }
  proj_finish<P>(pj, g, y0, xok, r);
}

// rows y0 - P .. y0 + SR - 1 + P of the lane's column, rows and columns outside the plane CLAMPED to
// the border: a window that reaches past the border always contains that border row / column, so the
// duplicates leave every window maximum -- and with it MaxPool2d's -inf padding -- unchanged, and the
// loads need no masks. One SGPR buffer descriptor per plane, the row offsets in SGPRs (soffset), the
// lane's column as the only VGPR offset.
template <int P>
__device__ __forceinline__ void load_unit_clamped(const float* __restrict__ s, const DetectGeom& g, int u,
                                                  float (&r)[SR + 2 * P]) {
  const int lane = threadIdx.x & 63;
  const UnitPos q = unit_pos(g, u);
  const int y0 = q.band * SR, x = q.strip * g.sc - P + lane;
  const int xo = min(max(x, 0), g.W - 1);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(s + (size_t)q.plane * g.H * g.W), 0, g.H * g.W * 4, 0x00020000);
  const int rowb = g.W * 4;
  if (y0 - P >= 0 && y0 + SR + P <= g.H) {   // interior band (uniform): one running row offset
    int so = (y0 - P) * rowb;
#pragma unroll
    for (int i = 0; i < SR + 2 * P; ++i) {
      r[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, 4 * xo, so, 0));
      so += rowb;
    }
  } else {
#pragma unroll
    for (int i = 0; i < SR + 2 * P; ++i) {
      const int yc = min(max(y0 - P + i, 0), g.H - 1);
      r[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, 4 * xo, yc * rowb, 0));
    }
  }
}

// rows y0 - P .. y0 + SR - 1 + P of the lane's column; -inf outside the plane (MaxPool padding)
template <int P>
__device__ __forceinline__ void load_unit(const float* __restrict__ s, const DetectGeom& g, int u,
                                          float (&r)[SR + 2 * P]) {
  const int lane = threadIdx.x & 63;
  const int plane = u / g.units, rem = u - plane * g.units, band = rem / g.nsx, strip = rem - band * g.nsx;
  const int y0 = band * SR, x = strip * g.sc - P + lane;
  const bool xok = x >= 0 && x < g.W;
  const int xo = min(max(x, 0), g.W - 1);
  const int* pl = reinterpret_cast<const int*>(s) + (size_t)plane * g.H * g.W;
  // Loads are unconditional (clamped addresses) and the -inf padding is applied with integer bit
  // masks: a select would let the compiler sink each load into a divergent branch with its own
  // vmcnt(0) wait, serialising the 16 + 2P loads of a unit.
  const int xmask = xok ? -1 : 0;
  if (y0 - P >= 0 && y0 + SR + P <= g.H) {                    // interior band: one running pointer
    const int* p = pl + (y0 - P) * g.W + xo;
#pragma unroll
    for (int i = 0; i < SR + 2 * P; ++i) {
      const int bits_v = p[0];
      p += g.W;
      r[i] = __int_as_float((bits_v & xmask) | (int)(0xff800000u & ~(unsigned)xmask));
    }
  } else {
#pragma unroll
    for (int i = 0; i < SR + 2 * P; ++i) {
      const int y = y0 - P + i;
      const int off = min(max(y, 0), g.H - 1) * g.W + xo;    // clamped: always a valid address
      const int m = (y >= 0 && y < g.H) ? xmask : 0;
      const int bits_v = pl[off];
      r[i] = __int_as_float((bits_v & m) | (int)(0xff800000u & ~(unsigned)m));
    }
  }
}

// PROJ: 0 dense maps, 1 projected, 2 projected separable. TP: the threshold is positive, so !(v < thr) alone
// decides a threshold pixel (v = 0 fails it; NaN passes both forms): one compare per pixel fewer.
template <int P, int MODE, bool MASKED, int PROJ, bool TP = false>
__global__ __launch_bounds__(NT1) void nms_strips_kernel(
    const float* __restrict__ s, const float* __restrict__ masks, DetectGeom g, float thr, int use_thr,
    float* __restrict__ cand_v, int* __restrict__ cand_i, float* __restrict__ neg_v, int* __restrict__ neg_i,
    int* __restrict__ tile_count, int* __restrict__ tile_nonneg, cmask_t* __restrict__ cbits, ProjArgs pj,
    unsigned long long* __restrict__ pflag) {
  const int lane = threadIdx.x & 63;
  const int total = g.B * g.J * g.units;
  if (blockIdx.x == 0)   // the fused select + emit stage's publish flags, for this detection
    for (int i = threadIdx.x; i < g.B * g.J; i += NT1) pflag[i] = 0ull;
  const int H = g.H, W = g.W, K = g.K;
  // Grid-stride over windows of G x 4 consecutive units; inside a window the units are dealt by XCD
  // (blocks b and b + 8 share one): XCD x takes the x-th eighth of the window, a contiguous run of bands
  // whose halo rows and columns its neighbours fetch at the same time into the same L2, instead of every
  // neighbour sitting on another XCD and reading its halo from HBM again.
  const int G = gridDim.x;
  const int slot = (NMS_XCD_MAP && (G & 7) == 0) ? ((int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3)) : (int)blockIdx.x;
  const int stride_u = G * (NT1 / 64), u_hi = total;
  // the unit index is wave-uniform: keep it (and all address math derived from it) scalar
  int u = __builtin_amdgcn_readfirstlane(slot * (NT1 / 64) + (threadIdx.x >> 6));
  float r[SR + 2 * P];
  __shared__ __attribute__((aligned(16))) float proj_stage[PROJ == 2 ? NT1 / 64 : 1]
                                                          [PROJ == 2 ? 2 * PROJ_LR * 64 + 4 * (SR + 2 * MAXR) : 1];
  auto load = [&](int uu) {
    if constexpr (PROJ) {
      if constexpr (PROJ == 2) load_unit_proj_sep<P>(pj, g, uu, r, proj_stage[threadIdx.x >> 6]);
      else load_unit_proj<P>(pj, g, uu, r);
    }
    else if constexpr (NMS_CLAMPED_LOADS) load_unit_clamped<P>(s, g, uu, r);
    else load_unit<P>(s, g, uu, r);
  };
  // (the projected loader computes its values as it loads: nothing to overlap, no prefetch)
  constexpr bool PF = NMS_PREFETCH && PROJ == 0;
  if (PF && u < u_hi) load(u);
  for (; u < u_hi; u += stride_u) {
    if (!PF) load(u);
    const UnitPos up = unit_pos(g, u);
    const int plane = up.plane, band = up.band, strip = up.strip;
    const int b = plane / g.J;
    const int y0 = band * SR, x = strip * g.sc - P + lane;
    const bool lane_ok = lane >= P && lane < 64 - P && x < W;
    float cur[SR + 2 * P];
#pragma unroll
    for (int i = 0; i < SR + 2 * P; ++i) cur[i] = r[i];
    if (PF && u + stride_u < u_hi) load(u + stride_u);   // next unit's rows in flight
    float vm[SR], c[SR];
#pragma unroll
    for (int j = 0; j < SR; ++j) {
      float m = cur[j];
#pragma unroll
      for (int d = 1; d <= 2 * P; ++d) m = fmaxf(m, cur[j + d]);
      vm[j] = m;
      c[j] = cur[j + P];
    }
    // horizontal: P rounds of a 3-wide max over neighbouring lanes -> window [x - P, x + P]
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
      for (int j = 0; j < SR; ++j) {
        const float t = fmaxf(vm[j], wave_shr1(vm[j]));
        vm[j] = fmaxf(t, wave_shl1(vm[j]));
      }
    // per lane: threshold bits and non-negative bits over the unit's rows, the largest value
    // (per-row ballots + scalar popcounts for the counts measured slower: 91 vs 67 us)
    // the row / lane validity applied once to the per-row bits (rows past the plane: last band only)
    const int rows = min(SR, H - y0);
    const unsigned vmask = lane_ok ? (rows >= 32 ? 0xffffffffu : ((1u << rows) - 1u)) : 0u;
    float v[SR];
    unsigned int tbits = 0, nnbits = 0;
    // the lane's largest value (a positive one marks the unit for ranking): one max per pixel instead of a
    // compare, a select and an or of a per-row bit. Rows past the plane (last band only) are included: a value
    // there can only mark a unit whose ranking then finds nothing valid (it masks those rows) and writes the
    // same sentinel list as an unmarked unit.
    float pmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < SR; ++j) {
      float jm = (vm[j] == c[j]) ? 1.0f : 0.0f;
      if (MASKED) jm = jm * masks[((size_t)b * H + min(y0 + j, H - 1)) * W + min(max(x, 0), W - 1)];
      const float vj = c[j] * jm;                       // ConstructGraph.py:1162-1165
      v[j] = vj;
      tbits |= (unsigned)(TP ? !(vj < thr) : (!(vj < thr) && vj != 0.0f)) << j;
      nnbits |= (unsigned)(vj >= 0.0f) << j;
      pmax = fmaxf(pmax, vj);                            // (fmaxf skips a NaN operand)
    }
    tbits &= vmask;
    nnbits &= vmask;
    if (!use_thr) tbits = 0;
    cbits[(size_t)u * 64 + lane] = (cmask_t)tbits;
    // both counts (<= 16 x 64 each) in one word, summed over the wave without the LDS pipe
    const int both = wave_sum_i32((__popc(tbits) << 16) | __popc(nnbits));
    const int cnt = both >> 16, nonneg = both & 0xffff;
    const bool anypos = __ballot(lane_ok && pmax > 0.0f) != 0;
    if (lane == 0) { tile_count[u] = cnt; tile_nonneg[u] = nonneg; }
    const int base_id = y0 * W + x;
    if (MODE == MODE_ALL || anypos || nonneg < K) {   // (uniform; rare with MODE_POS) invalid rows -> NaN
#pragma unroll
      for (int j = 0; j < SR; ++j)
        if (!((vmask >> j) & 1u)) v[j] = NAN;
    }
    if (MODE == MODE_POS) {
      if (anypos) wave_topk(v, base_id, W, K, [](float a) { return a > 0.0f; }, cand_v + (size_t)u * K, cand_i + (size_t)u * K);
      else write_sentinels(cand_v + (size_t)u * K, cand_i + (size_t)u * K, K);
      if (nonneg < K)      // degenerate unit: also keep its best negatives (see stage 2)
        wave_topk(v, base_id, W, K, [](float a) { return a < 0.0f; }, neg_v + (size_t)u * K, neg_i + (size_t)u * K);
      else write_sentinels(neg_v + (size_t)u * K, neg_i + (size_t)u * K, K);
    } else {
      wave_topk(v, base_id, W, K, [](float a) { return a == a; }, cand_v + (size_t)u * K, cand_i + (size_t)u * K);
    }
  }
}

// ---- split dense NMS (quad layout, round 6) ------------------------------------------------------------------------
// nms_quad_kernel: one wave per block of SR rows x 256 columns = 4 units of 16 x 64; lane L owns the columns x0 + 4L ..
// x0 + 4L + 3 (one buffer_load_dwordx4 per row, columns past the plane set to -inf; a clamped dword per column when
// W % 4 != 0). The P
// columns either side of the block come from one more P-dword load per row into the same registers of every lane, of
// which lanes 0 (left: x0 - P ..) and 63 (right: x0 + 256 ..) are the ones read: the DPP wave shifts that bring the
// neighbours' columns leave those two lanes' `old` operand in place. Per row the horizontal 2P + 1 window first (6
// v_max3 for P = 2), then the vertical one over the 2P + 1 row maxima; per pixel v = c * (window max == c), and the
// threshold, non-negative and maximum bits (shift-add accumulation) and the lane's largest v. No ranking in the loop:
// a unit holding a positive v (or with fewer than K non-negative pixels) is re-read one column per lane, its maximum
// bits from LDS, and ranked by nms_strips_kernel's wave top-k; every other unit writes a sentinel candidate list. The
// negative lists are written only for units with fewer than K non-negative pixels (readers gate them on tile_nonneg).
#ifndef NMS_QUAD
#define NMS_QUAD 0   // opt-in (PEMP_NMS_QUAD=1): measured no faster than the strip kernel, see DESIGN.md section 4
#endif
#ifndef NMS_QUAD_PER_CU
#define NMS_QUAD_PER_CU 8
#endif
#ifndef NMS_QUAD_PF
#define NMS_QUAD_PF 6   // rows of a block in flight ahead of the row being reduced
#endif

template <int P>
__device__ __forceinline__ void quad_hmax(const float (&q)[4], const float (&h)[P > 0 ? P : 1], float (&o)[4]) {
  if constexpr (P == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = q[k];
  } else {
    float e[4 + 2 * P];
#pragma unroll
    for (int i = 0; i < P; ++i) {   // wave_shr:1 / wave_shl:1 with bound_ctrl off: lanes 0 / 63 keep the halo load
      e[i] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(h[i]), __float_as_int(q[4 - P + i]), 0x138,
                                                        0xF, 0xF, false));
      e[P + 4 + i] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(h[i]), __float_as_int(q[i]), 0x130, 0xF,
                                                                0xF, false));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) e[P + k] = q[k];
    if constexpr (P == 2) {
      const float a = fmaxf(fmaxf(q[0], q[1]), q[2]), b = fmaxf(fmaxf(q[1], q[2]), q[3]);
      o[0] = fmaxf(fmaxf(e[0], e[1]), a);
      o[1] = fmaxf(fmaxf(e[1], a), q[3]);
      o[2] = fmaxf(fmaxf(q[0], b), e[6]);
      o[3] = fmaxf(fmaxf(b, e[6]), e[7]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float m = e[k];
#pragma unroll
        for (int d = 1; d <= 2 * P; ++d) m = fmaxf(m, e[k + d]);
        o[k] = m;
      }
    }
  }
}

template <int P>
__device__ __forceinline__ void quad_halo_load(__amdgpu_buffer_rsrc_t rs, int vo, int so, float (&h)[P > 0 ? P : 1]) {
  if constexpr (P == 1) {
    h[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, 0));
  } else if constexpr (P == 2) {
    const auto t = __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, 0);
    h[0] = __uint_as_float(t[0]); h[1] = __uint_as_float(t[1]);
  } else if constexpr (P == 3) {
    const auto t = __builtin_amdgcn_raw_buffer_load_b96(rs, vo, so, 0);
    h[0] = __uint_as_float(t[0]); h[1] = __uint_as_float(t[1]); h[2] = __uint_as_float(t[2]);
  } else if constexpr (P == 4) {
    const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0);
    h[0] = __uint_as_float(t[0]); h[1] = __uint_as_float(t[1]); h[2] = __uint_as_float(t[2]); h[3] = __uint_as_float(t[3]);
  }
}

// One pixel's bits: v = (m == c) ? c : c * 0 (exactly c * (maximum ? 1 : 0)); ab, tb, nb shifted left by one with the
// maximum, threshold (TP: !(v < thr); else !(v < thr) && v != 0) and non-negative (v >= 0) predicates as the carry-in
// of v_addc (t + t + carry: one instruction per bit, where the compiler spends a select, a shift and an or).
template <bool TP>
__device__ __forceinline__ void quad_px_bits(float c, float m, float thr, float& v, unsigned& ab, unsigned& tb,
                                             unsigned& nb) {
  float z;
  if constexpr (TP) {
    asm("v_mul_f32_e32 %[z], 0, %[c]\n\t"
        "v_cmp_eq_f32_e32 vcc, %[m], %[c]\n\t"
        "v_cndmask_b32_e32 %[v], %[z], %[c], vcc\n\t"
        "v_addc_co_u32_e32 %[ab], vcc, %[ab], %[ab], vcc\n\t"
        "v_cmp_nlt_f32_e32 vcc, %[v], %[thr]\n\t"
        "v_addc_co_u32_e32 %[tb], vcc, %[tb], %[tb], vcc\n\t"
        "v_cmp_le_f32_e32 vcc, 0, %[v]\n\t"
        "v_addc_co_u32_e32 %[nb], vcc, %[nb], %[nb], vcc"
        : [v] "=&v"(v), [z] "=&v"(z), [ab] "+v"(ab), [tb] "+v"(tb), [nb] "+v"(nb)
        : [c] "v"(c), [m] "v"(m), [thr] "v"(thr)
        : "vcc");
  } else {
    unsigned long long nz;
    asm("v_mul_f32_e32 %[z], 0, %[c]\n\t"
        "v_cmp_eq_f32_e32 vcc, %[m], %[c]\n\t"
        "v_cndmask_b32_e32 %[v], %[z], %[c], vcc\n\t"
        "v_addc_co_u32_e32 %[ab], vcc, %[ab], %[ab], vcc\n\t"
        "v_cmp_neq_f32_e64 %[nz], 0, %[v]\n\t"
        "v_cmp_nlt_f32_e32 vcc, %[v], %[thr]\n\t"
        "s_and_b64 vcc, vcc, %[nz]\n\t"
        "v_addc_co_u32_e32 %[tb], vcc, %[tb], %[tb], vcc\n\t"
        "v_cmp_le_f32_e32 vcc, 0, %[v]\n\t"
        "v_addc_co_u32_e32 %[nb], vcc, %[nb], %[nb], vcc"
        : [v] "=&v"(v), [z] "=&v"(z), [ab] "+v"(ab), [tb] "+v"(tb), [nb] "+v"(nb), [nz] "=&s"(nz)
        : [c] "v"(c), [m] "v"(m), [thr] "v"(thr)
        : "vcc", "scc");
  }
}

// LM: 0 the block lies inside the plane (16-byte loads), 1 it reaches past it and W % 4 == 0 (16-byte loads; the
// columns past the plane become -inf, MaxPool's padding), 2 W % 4 != 0 (clamped dword per column)
template <int P, bool TP, int LM>
__device__ __forceinline__ void quad_block(__amdgpu_buffer_rsrc_t rs, const DetectGeom& g, int y0, int x0, float thr,
                                           unsigned (&tb)[4], unsigned (&nb)[4], unsigned (&ab)[4], float& pmax) {
  constexpr int NR = SR + 2 * P, HP = P > 0 ? P : 1, PF = NMS_QUAD_PF < NR ? NMS_QUAD_PF : NR;
  const int lane = threadIdx.x & 63, H = g.H, W = g.W, rowb = W * 4;
  // the lane's columns and its halo columns (read in lanes 0 and 63)
  constexpr bool FAST = LM < 2;
  const int xq = x0 + 4 * lane;
  const bool xin = xq < W;
  int vq[4], vh[HP];
  if constexpr (FAST) {
    vq[0] = 4 * xq;
    vh[0] = 4 * (lane == 63 ? min(x0 + 256, W - P) : max(x0 - P, 0));
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) vq[k] = 4 * min(xq + k, W - 1);
#pragma unroll
    for (int i = 0; i < HP; ++i) vh[i] = 4 * (lane == 63 ? min(x0 + 256 + i, W - 1) : max(x0 - P + i, 0));
  }
  float qr[NR][4], hr[NR][HP];
  auto load_row = [&](int r) {
    const int so = min(max(y0 - P + r, 0), H - 1) * rowb;   // clamped rows: duplicates leave every window max as is
    if constexpr (FAST) {
      const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, vq[0], so, 0);
      qr[r][0] = __uint_as_float(t[0]); qr[r][1] = __uint_as_float(t[1]);
      qr[r][2] = __uint_as_float(t[2]); qr[r][3] = __uint_as_float(t[3]);
      if constexpr (LM == 1) {
#pragma unroll
        for (int k = 0; k < 4; ++k) qr[r][k] = xin ? qr[r][k] : -INFINITY;
      }
      quad_halo_load<P>(rs, vh[0], so, hr[r]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) qr[r][k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vq[k], so, 0));
#pragma unroll
      for (int i = 0; i < P; ++i) hr[r][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vh[i], so, 0));
    }
  };
#pragma unroll
  for (int r = 0; r < PF; ++r) load_row(r);
  float hm[NR][4];
  // output row j: window max m, centre c = row j + P of the lane's column k
  auto pixel = [&](int j, int k, float m) {
    const float c = qr[j + P][k];
    float v;
    quad_px_bits<TP>(c, m, thr, v, ab[k], tb[k], nb[k]);   // row j ends at bit 15 - j (reversed by the caller)
    pmax = fmaxf(pmax, v);
  };
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    if (r + PF < NR) load_row(r + PF);   // the row PF ahead goes out before this row's wait
    __builtin_amdgcn_sched_barrier(0);
    quad_hmax<P>(qr[r], hr[r], hm[r]);
    if constexpr (P > 0) {
      // rows in pairs: the two windows share their middle 2P - 1 rows (3 v_max3 per 2 outputs for P = 2)
      if (r >= 2 * P + 1 && ((r - 2 * P) & 1)) {
        const int j = r - 2 * P - 1;
        float t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          t[k] = hm[j + 1][k];
#pragma unroll
          for (int d = 2; d < 2 * P; ++d) t[k] = fmaxf(t[k], hm[j + d][k]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) pixel(j, k, fmaxf(fmaxf(hm[j][k], t[k]), hm[j + 2 * P][k]));
#pragma unroll
        for (int k = 0; k < 4; ++k) pixel(j + 1, k, fmaxf(fmaxf(t[k], hm[j + 2 * P][k]), hm[j + 2 * P + 1][k]));
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) pixel(r, k, hm[r][k]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

#ifndef NMS_QUAD_WAVES
#define NMS_QUAD_WAVES 4   // waves per SIMD the register allocation targets (the pass is latency-bound: 3 -> 4 waves
#endif                     // took it from 69 to 49 us at c3)
template <int P, bool TP>
__global__ __launch_bounds__(NT1) __attribute__((amdgpu_waves_per_eu(NMS_QUAD_WAVES, 8))) void nms_quad_kernel(
    const float* __restrict__ s, DetectGeom g, float thr, float* __restrict__ cand_v, int* __restrict__ cand_i,
    float* __restrict__ neg_v, int* __restrict__ neg_i, int* __restrict__ tile_count, int* __restrict__ tile_nonneg,
    cmask_t* __restrict__ cbits, unsigned long long* __restrict__ pflag) {
  static_assert(SR == 16, "quad layout: 16-row units");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int H = g.H, W = g.W, K = g.K;
  __shared__ __attribute__((aligned(16))) unsigned short abits_sh[NT1 / 64][4 * 64];
  if (blockIdx.x == 0)   // the fused select + emit stage's publish flags, for this detection
    for (int i = threadIdx.x; i < g.B * g.J; i += NT1) pflag[i] = 0ull;
  const int total = g.B * g.J * g.blocks;
  const int G = gridDim.x;
  const int slot = (NMS_XCD_MAP && (G & 7) == 0) ? ((int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3)) : (int)blockIdx.x;
  const int stride = G * (NT1 / 64);
  for (int q = __builtin_amdgcn_readfirstlane(slot * (NT1 / 64) + wave); q < total; q += stride) {
    const int plane = fastdiv(q, g.mq, g.lq), rem = q - plane * g.blocks;
    const int band = fastdiv(rem, g.mx, g.lx), bx = rem - band * g.nbx;
    const int y0 = band * SR;
    const int su = 4 * bx;   // first unit of the block
    const int x0 = su * 64;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s + (size_t)plane * H * W), 0, H * W * 4, 0x00020000);
    unsigned tb[4] = {0u, 0u, 0u, 0u}, nb[4] = {0u, 0u, 0u, 0u}, ab[4] = {0u, 0u, 0u, 0u};
    float pmax = -INFINITY;
    if ((W & 3) != 0) quad_block<P, TP, 2>(rs, g, y0, x0, thr, tb, nb, ab, pmax);
    else if (x0 + 256 <= W) quad_block<P, TP, 0>(rs, g, y0, x0, thr, tb, nb, ab, pmax);
    else quad_block<P, TP, 1>(rs, g, y0, x0, thr, tb, nb, ab, pmax);
    // validity: rows past the plane (last band), columns and units past it (last block of a band)
    const int rows = min(SR, H - y0);
    const unsigned rmask = rows >= 16 ? 0xffffu : ((1u << rows) - 1u);
    const int ul = lane >> 4, u = su + ul;
    const bool uok = u < g.nsx;
    unsigned tk[4], ak[4];
    int tcnt = 0, ncnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned m = (uok && x0 + 4 * lane + k < W) ? rmask : 0u;
      tk[k] = (__builtin_bitreverse32(tb[k]) >> 16) & m;
      ak[k] = (__builtin_bitreverse32(ab[k]) >> 16) & m;
      tcnt += __popc(tk[k]);
      ncnt += __popc((__builtin_bitreverse32(nb[k]) >> 16) & m);
    }
    // both counts of the lane's unit (its 16-lane DPP row): threshold << 16 | non-negative (each <= 1024)
    int both = (tcnt << 16) | ncnt;
    both += __builtin_amdgcn_update_dpp(0, both, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    both += __builtin_amdgcn_update_dpp(0, both, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    both += __builtin_amdgcn_update_dpp(0, both, 0x141, 0xF, 0xF, false);   // row_half_mirror
    both += __builtin_amdgcn_update_dpp(0, both, 0x140, 0xF, 0xF, false);   // row_mirror
    const size_t ub = ((size_t)plane * g.nb + band) * g.nsx;   // first unit of the band
    if (uok) {
      uint2 pk;
      pk.x = tk[0] | (tk[1] << 16);
      pk.y = tk[2] | (tk[3] << 16);
      *reinterpret_cast<uint2*>(cbits + (ub + u) * 64 + (lane & 15) * 4) = pk;
      if ((lane & 15) == 0) { tile_count[ub + u] = both >> 16; tile_nonneg[ub + u] = both & 0xffff; }
    }
    // ranking: units holding a positive v (top-K positives) or with fewer than K non-negative pixels (top-K negatives)
    const unsigned long long posm = __ballot(pmax > 0.0f);
    unsigned live = 0u, negl = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ui = su + i;
      if (ui >= g.nsx) continue;   // (uniform)
      if ((posm >> (16 * i)) & 0xffffull) live |= 1u << i;
      if ((__builtin_amdgcn_readlane(both, 16 * i) & 0xffff) < K) negl |= 1u << i;
      if (!((live >> i) & 1u) && lane < K) {     // a unit without a positive value: sentinel list
        cand_v[(ub + ui) * K + lane] = -INFINITY;
        cand_i[(ub + ui) * K + lane] = INV;
      }
    }
    if (live | negl) {   // (uniform; MODE_POS: the units around the peaks)
      uint2 pa;
      pa.x = ak[0] | (ak[1] << 16);
      pa.y = ak[2] | (ak[3] << 16);
      *reinterpret_cast<uint2*>(&abits_sh[wave][ul * 64 + (lane & 15) * 4]) = pa;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int rowb = W * 4;
#pragma unroll 1
      for (int i = 0; i < 4; ++i) {
        if (!(((live | negl) >> i) & 1u)) continue;   // (uniform)
        const int xu = (su + i) * 64 + lane;
        const bool xok = xu < W;
        const int vo = 4 * min(xu, W - 1);
        const unsigned a = abits_sh[wave][i * 64 + lane];
        float v[SR];
#pragma unroll
        for (int j = 0; j < SR; ++j)
          v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, min(y0 + j, H - 1) * rowb, 0));
#pragma unroll
        for (int j = 0; j < SR; ++j) {
          const float c = v[j];
          v[j] = ((a >> j) & 1u) ? c : c * 0.0f;
          if (!xok || y0 + j >= H) v[j] = NAN;
        }
        const int base_id = y0 * W + xu;
        const size_t ui = ub + su + i;
        if ((live >> i) & 1u)
          wave_topk(v, base_id, W, K, [](float x) { return x > 0.0f; }, cand_v + ui * K, cand_i + ui * K);
        if ((negl >> i) & 1u)
          wave_topk(v, base_id, W, K, [](float x) { return x < 0.0f; }, neg_v + ui * K, neg_i + ui * K);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

// Wave-level exact top-`take` of n candidates (value desc, index asc) into out (lane 0 writes);
// returns the number of valid entries written. gate (optional): candidate c belongs to list c / K of the plane, which
// holds entries only when gate[c / K] < K (the negative lists: a unit's non-negative count).
template <int KMAX>
__device__ __forceinline__ int merge_candidates(const float* __restrict__ cv, const int* __restrict__ ci, int n,
                                                int take, float* out_v, int* out_i, const int* __restrict__ gate = nullptr,
                                                int gk = 1, int goff = 0) {
  const int lane = threadIdx.x & 63;
  float lv[KMAX];
  int li[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) { lv[k] = -INFINITY; li[k] = INV; }
  // 16 candidates per lane per round: their loads are issued together (clamped addresses, masked
  // values), so a wave's whole list usually costs one memory round trip
  constexpr int PER = 16;
  for (int c0 = lane; c0 < n; c0 += 64 * PER) {
    float vq[PER];
    int iq[PER], gq[PER];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int c = min(c0 + 64 * r, n - 1);
      vq[r] = cv[c];
      iq[r] = ci[c];
      gq[r] = gate ? gate[(goff + c) / gk] : 0;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      if (c0 + 64 * r >= n || gq[r] >= gk) iq[r] = INV;
    }
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      float v = vq[r];
      int i = iq[r];
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
                          int* out_i, float (*lv)[KMAX], int (*li)[KMAX], int* cnt, const int* __restrict__ gate = nullptr,
                          int gk = 1) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = (n + 3) / 4, lo = min(n, wave * q), hi = min(n, lo + q);
  const int got = merge_candidates<KMAX>(cv + lo, ci + lo, hi - lo, take, lv[wave], li[wave], gate, gk, lo);
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
  const int K = g.K, W = g.W, S = g.S, nl = g.units;
  const size_t pt = (size_t)pl * nl;                  // first wave list of the plane
  // the plane's per-unit counts (first UPT x 256 units) are loaded together with the candidates
  constexpr int UPT = 4;
  int tc[UPT], tn[UPT];
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    const int c = min((int)threadIdx.x + 256 * k, nl - 1);
    tc[k] = tile_count[pt + c];
    tn[k] = tile_nonneg[pt + c];
  }
  int n = block_topk<KMAX>(cand_v + pt * K, cand_i + pt * K, nl * K, K, top_v, top_i, lv, li, &sh[0]);
  if (use_thr) {
    // degenerate plane (fewer than K non-negative pixels): its top-k also holds negatives
    int nn = 0;
#pragma unroll
    for (int k = 0; k < UPT; ++k) nn += (int)threadIdx.x + 256 * k < nl ? tn[k] : 0;
    for (int c = threadIdx.x + 256 * UPT; c < nl; c += 256) nn += tile_nonneg[pt + c];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) nn += __shfl_xor(nn, off);
    if (lane == 0) sh[4 + wave] = nn;
    __syncthreads();
    nn = sh[4] + sh[5] + sh[6] + sh[7];
    if (nn < K)   // (a unit's negative list holds entries only when its non-negative count is below K)
      n += block_topk<KMAX>(neg_v + pt * K, neg_i + pt * K, nl * K, K - nn, top_v + n, top_i + n, lv, li, &sh[1],
                            tile_nonneg + pt, K);
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
  // per-band threshold counts (all units of the plane in parallel, integer LDS atomics) minus the
  // top-k entries already listed
  __shared__ int band_cnt[MAXB];
  for (int st = threadIdx.x; st < S; st += 256) band_cnt[st] = 0;
  __syncthreads();
  if (use_thr) {
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int idx = threadIdx.x + 256 * k;
      if (idx < nl && tc[k]) atomicAdd(&band_cnt[idx / g.nsx], tc[k]);
    }
    for (int idx = threadIdx.x + 256 * UPT; idx < nl; idx += 256) {
      const int v = tile_count[pt + idx];
      if (v) atomicAdd(&band_cnt[idx / g.nsx], v);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 0; q < m; ++q)
      if (top_bit[q]) band_cnt[top_i[q] / W / SR] -= 1;
  }
  __syncthreads();
  // in-plane exclusive scan over bands (wave 0, chunks of 64)
  if (wave == 0) {
    int carry = 0;
    for (int c0 = 0; c0 < S; c0 += 64) {
      const int st = c0 + lane;
      const int v = st < S ? band_cnt[st] : 0;
      int x = v;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(x, off);
        if (lane >= off) x += o;
      }
      if (st < S) {
        w.pstrip[(size_t)pl * S + st] = v;
        w.pstrip_off[(size_t)pl * S + st] = carry + x - v;
      }
      carry += __shfl(x, 63);
    }
    if (lane == 0) w.pn_thr[pl] = carry;
  }
}

// Stage 2b: one workgroup per plane. The plane's output offsets follow from the per-plane counts
// of its image: [top-k dets of types 0..J-1] ++ [threshold dets, type-major, strip order].
__global__ __launch_bounds__(256) void emit_kernel(const float* __restrict__ s, const float* __restrict__ masks,
                                                   DetectGeom g, const cmask_t* __restrict__ cbits,
                                                   DetectWs w, int64_t* __restrict__ det,
                                                   float* __restrict__ scores, int* __restrict__ n_det, int cap,
                                                   int* __restrict__ n_host, ProjArgs pj) {
  __shared__ int top_i[KCAP], top_bit[KCAP], sh[4];
  __shared__ int band_n[MAXB], band_off[MAXB];
  __shared__ unsigned band_nz[MAXB][2];      // non-empty strips of each band (bit = strip, nsx <= 64)
  const int pl = blockIdx.x, J = g.J, b = pl / J, t = pl - b * J;
  const int H = g.H, W = g.W, S = g.S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // every per-plane input is requested up front (one memory round trip): band counts and offsets,
  // unit counts (first 4 x 256 units), then the image's per-type counts (wave 0)
  const size_t pt = (size_t)pl * g.units;
  constexpr int UPT = 4;
  int tc[UPT];
#pragma unroll
  for (int k = 0; k < UPT; ++k) tc[k] = w.tile_count[pt + min((int)threadIdx.x + 256 * k, g.units - 1)];
  const int bn = (int)threadIdx.x < S ? w.pstrip[(size_t)pl * S + threadIdx.x] : 0;
  const int bo = (int)threadIdx.x < S ? w.pstrip_off[(size_t)pl * S + threadIdx.x] : 0;
  if ((int)threadIdx.x < S) {
    band_n[threadIdx.x] = bn;
    band_off[threadIdx.x] = bo;
    band_nz[threadIdx.x][0] = 0u;
    band_nz[threadIdx.x][1] = 0u;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    const int idx = threadIdx.x + 256 * k;
    if (idx < g.units && tc[k] > 0) {
      const int band = idx / g.nsx, sx = idx - band * g.nsx;
      atomicOr(&band_nz[band][sx >> 5], 1u << (sx & 31));
    }
  }
  for (int idx = threadIdx.x + 256 * UPT; idx < g.units; idx += 256) {
    if (w.tile_count[pt + idx] > 0) {
      const int band = idx / g.nsx, sx = idx - band * g.nsx;
      atomicOr(&band_nz[band][sx >> 5], 1u << (sx & 31));
    }
  }
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
      if (t == 0) {
        n_det[b] = top_all + thr_all;
        // straight into the caller's mapped host memory: the host reads the count while this
        // kernel writes the detections and the graph kernels run (no copy, no event wait)
        if (n_host) __hip_atomic_store(&n_host[b], top_all + thr_all, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
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
  // threshold detections, one wave per non-empty band. The band's non-empty units (strips) are
  // found from their counts; their column masks go to LDS; row words are rebuilt with one ballot
  // per (row, non-empty strip), visited in (y, x) order; a lane's output slot is the running base
  // plus the set bits below it (mbcnt).
  __shared__ cmask_t cm_sh[4][64][64];
  __shared__ int nz_sh[4][64];
  // non-empty bands, round-robin over the waves (the wave's k-th band is the (4k + wave)-th one)
  int kb = 0;
  for (int st = 0; st < S; ++st) {
    if (band_n[st] == 0) continue;                       // uniform
    if ((kb++ & 3) != wave) continue;
    const int ry0 = st * SR, rows = min(SR, H - ry0);
    int pos = thr_base + band_off[st];
    const float* plane = s + (size_t)pl * H * W;
    const size_t u0 = ((size_t)pl * g.nb + st) * g.nsx;   // first unit of the band (nsx <= 64)
    const unsigned long long nzm = (unsigned long long)band_nz[st][0] | ((unsigned long long)band_nz[st][1] << 32);
    int nnz = 0;
    unsigned rows_any = 0;
    unsigned cms[4];
    {                                                    // the first 4 strips' column masks together
      unsigned long long m = nzm;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int sx = m ? __builtin_ctzll(m) : 0;
        cms[k] = cbits[(u0 + sx) * 64 + lane];
        if (m) m &= m - 1;
      }
    }
    for (unsigned long long m = nzm; m; m &= m - 1) {
      const int sx = __builtin_ctzll(m);
      const unsigned cm = nnz < 4 ? cms[nnz & 3] : cbits[(u0 + sx) * 64 + lane];
      cm_sh[wave][nnz][lane] = (cmask_t)cm;
      if (lane == 0) nz_sh[wave][nnz] = sx;
      unsigned ra = cm;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) ra |= __shfl_xor(ra, off);
      rows_any |= ra;
      ++nnz;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (unsigned rm = rows_any & (rows >= 32 ? ~0u : (1u << rows) - 1u); rm; rm &= rm - 1) {
      const int j = __builtin_ctz(rm), yy = ry0 + j;
      for (int k = 0; k < nnz; ++k) {
        const int sx = nz_sh[wave][k];
        unsigned long long word = __ballot((cm_sh[wave][k][lane] >> j) & 1u);
        if (!word) continue;
        for (int q = 0; q < ntop; ++q) {               // already listed as a top-k detection
          if (!top_bit[q]) continue;
          const int idx = top_i[q], ty = idx / W, tx = idx - ty * W, tsx = tx / g.sc;
          if (ty == yy && tsx == sx) word &= ~(1ull << (tx - tsx * g.sc + g.p));
        }
        if ((word >> lane) & 1ull) {
          const int xx = sx * g.sc - g.p + lane;
          const int o = pos + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(word >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((unsigned)word, 0u));
          if (o < cap) {
            const float sv = pj.S ? proj_pixel(pj, b, t, yy, xx, H, W) : plane[(size_t)yy * W + xx];
            float jm = 1.0f;
            if (masks) jm = jm * masks[((size_t)b * H + yy) * W + xx];
            dout[o * 3 + 0] = xx;
            dout[o * 3 + 1] = yy;
            dout[o * 3 + 2] = t;
            sout[o] = sv * jm;
          }
        }
        pos += __popcll(word);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

constexpr int SEL_GATHER = 2048;   // candidates of live units gathered into LDS by the fused stage
constexpr int SEL_UNITS = 1024;    // units per plane the fused stage handles (4 per thread); more: the two kernels

// Stages 2a + 2b in one launch (PEMP_DETECT_FUSED, the default; planes of at most SEL_UNITS units): one workgroup per
// plane. Every phase is shaped for latency (136 workgroups at C3, each a chain of dependent steps):
//   A  one round trip: the plane's unit counts and the first candidate of every unit list (live = not a sentinel);
//   B  band counts (LDS atomics), the non-negative total, and the live lists' candidates gathered into LDS (a second
//      round trip; MODE_POS: a handful of units per plane instead of all of them);
//   C  exact top-k from LDS (block_topk; the degenerate negative lists from global memory when needed);
//   D  wave 0, one lane per entry: drop zero / empty entries, order by flat index (ranks by readlane, no serial
//      loop), threshold bits, the band counts minus the entries already listed, the entries' emission positions;
//   E  in-plane band scan, publish (release store of the plane's flag, agent scope), wait for the image's other
//      planes (acquire polls; they are consecutive workgroups, dispatched together), output bases;
//   F  emission as emit_kernel, except that a wave queues its detections (position, output slot) in LDS and then
//      reads all their scores in one batch of loads.
template <int KMAX>
__global__ __launch_bounds__(256) void plane_emit_kernel(const float* __restrict__ s, const float* __restrict__ masks,
                                                         DetectGeom g, float thr, int use_thr,
                                                         const cmask_t* __restrict__ cbits, DetectWs w,
                                                         int64_t* __restrict__ det, float* __restrict__ scores,
                                                         int* __restrict__ n_det, int cap, int* __restrict__ n_host,
                                                         ProjArgs pj) {
  static_assert(2 * KMAX <= 64, "phase D: one lane per candidate");
  __shared__ float lv[4][KMAX];
  __shared__ int li[4][KMAX];
  __shared__ float top_v[2 * KMAX], top_sc[KMAX];
  __shared__ int top_i[2 * KMAX], sh[8];
  __shared__ int ex_y[KMAX], ex_sx[KMAX], ex_lane[KMAX];   // listed threshold entries: row, strip, lane (y -1: none)
  __shared__ int band_n[MAXB], band_off[MAXB];
  __shared__ unsigned band_nz[MAXB][2];      // non-empty strips of each band (bit = strip, nsx <= 64)
  __shared__ float gv[SEL_GATHER];
  __shared__ int gi[SEL_GATHER], glive[4][4], gnn[4];
  const int pl = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int J = g.J, b = pl / J, t = pl - b * J;
  const int K = g.K, H = g.H, W = g.W, S = g.S, nl = g.units;
  const size_t pt = (size_t)pl * nl;
#if PEMP_DETECT_CLOCKS   // diagnostics: per-phase wall clock (100 MHz) of one plane per image, printed
  long long clk[6];
  clk[0] = wall_clock64();
#define PEMP_CLK(i) clk[i] = wall_clock64()
#else
#define PEMP_CLK(i) (void)0
#endif
  // ---- A: counts and list heads of the plane's units (4 per thread) ----
  constexpr int UPT = SEL_UNITS / 256;
  int tc[UPT], tn[UPT];
  bool live[UPT];
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    const int c = min((int)threadIdx.x + 256 * k, nl - 1);
    tc[k] = w.tile_count[pt + c];
    tn[k] = w.tile_nonneg[pt + c];
    live[k] = w.cand_v[(pt + c) * K] != -INFINITY;
  }
  for (int st = threadIdx.x; st < S; st += 256) {
    band_n[st] = 0;
    band_nz[st][0] = 0u;
    band_nz[st][1] = 0u;
  }
  __syncthreads();
  // ---- B: band counts, non-negative total, live lists ----
  int nn = 0;
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    const int idx = threadIdx.x + 256 * k;
    const bool in = idx < nl;
    live[k] = live[k] && in && use_thr;
    nn += in ? tn[k] : 0;
    if (in && tc[k] && use_thr) {
      const int band = fastdiv(idx, g.mn, g.ln), sx = idx - band * g.nsx;
      atomicAdd(&band_n[band], tc[k]);
      atomicOr(&band_nz[band][sx >> 5], 1u << (sx & 31));
    }
    const unsigned long long bal = __ballot(live[k]);
    if (lane == 0) glive[k][wave] = __popcll(bal);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) nn += __shfl_xor(nn, off);
  if (lane == 0) gnn[wave] = nn;
  __syncthreads();
  nn = gnn[0] + gnn[1] + gnn[2] + gnn[3];
  int live_total = 0;
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    int before = live_total;
    for (int w2 = 0; w2 < wave; ++w2) before += glive[k][w2];
    live_total += glive[k][0] + glive[k][1] + glive[k][2] + glive[k][3];
    if (live[k]) {
      const unsigned long long bal = __ballot(true);   // (the live lanes of this wave: exec mask)
      const int slot = before + (int)__popcll(bal & ((1ull << lane) - 1ull));
      const size_t src = (pt + threadIdx.x + 256 * k) * K;
      if ((slot + 1) * K <= SEL_GATHER)
        for (int q = 0; q < K; ++q) {
          gv[slot * K + q] = w.cand_v[src + q];
          gi[slot * K + q] = w.cand_i[src + q];
        }
    }
  }
  __syncthreads();
  PEMP_CLK(1);
  // ---- C: exact top-k ----
  int n;
  if (use_thr && live_total * K <= 256) {
    // one gathered candidate per thread: its rank = the candidates better than it (distinct flat indices), the K
    // best go to their rank's slot
    const int nc = live_total * K;
    const bool mine = (int)threadIdx.x < nc;
    const float v = mine ? gv[threadIdx.x] : -INFINITY;
    const int i = mine ? gi[threadIdx.x] : INV;
    int rank = 0, valid = 0;
    for (int r = 0; r < nc; ++r) {                 // (LDS broadcast reads)
      const float vr = gv[r];
      const int ir = gi[r];
      rank += better(vr, ir, v, i) && ir != INV ? 1 : 0;
    }
    if (mine && i != INV && rank < K) { top_v[rank] = v; top_i[rank] = i; }
    const unsigned long long bal = __ballot(mine && i != INV);
    if (lane == 0) glive[0][wave] = __popcll(bal);
    __syncthreads();
    valid = glive[0][0] + glive[0][1] + glive[0][2] + glive[0][3];
    n = min(K, valid);
  } else if (use_thr && live_total * K <= SEL_GATHER)
    n = block_topk<KMAX>(gv, gi, live_total * K, K, top_v, top_i, lv, li, &sh[0]);
  else
    n = block_topk<KMAX>(w.cand_v + pt * K, w.cand_i + pt * K, nl * K, K, top_v, top_i, lv, li, &sh[0]);
  if (use_thr && nn < K)   // degenerate plane (fewer than K non-negative pixels): its top-k also holds negatives
    n += block_topk<KMAX>(w.neg_v + pt * K, w.neg_i + pt * K, nl * K, K - nn, top_v + n, top_i + n, lv, li, &sh[1],
                          w.tile_nonneg + pt, K);
  PEMP_CLK(2);
  // ---- D: the listed entries (wave 0, one lane per entry) ----
  if (wave == 0) {
    const bool has = lane < n;
    const float v = has ? top_v[lane] : 0.0f;
    const int i = has ? top_i[lane] : INV;
    const float sc = use_thr ? v : v + 1e-10f;
    const bool keep = has && sc != 0.0f && i != INV;
    const unsigned long long km = __ballot(keep);
    int rank = 0;                                  // position in flat-index order among the kept entries
    for (int r = 0; r < n; ++r) {                  // (n uniform)
      const int ir = __builtin_amdgcn_readlane(i, r);
      rank += ((km >> r) & 1ull) && ir < i ? 1 : 0;
    }
    if (keep) {
      const bool bit = use_thr && !(v < thr) && v != 0.0f;
      const int ty = i / W, tx = i - ty * W, tsx = tx / g.sc;
      top_i[KMAX + rank] = i;                      // (upper half: the lower one may still be read by other lanes)
      top_sc[rank] = sc;
      ex_y[rank] = bit ? ty : -1;
      ex_sx[rank] = tsx;
      ex_lane[rank] = tx - tsx * g.sc + g.p;
      if (bit) atomicSub(&band_n[ty / SR], 1);     // already listed as a top-k detection
    }
    if (lane == 0) sh[4] = __popcll(km);
  }
  __syncthreads();
  const int ntop = sh[4];
  PEMP_CLK(3);
  // ---- E: band offsets, publish, the image's per-type counts ----
  if (wave == 0) {
    int carry = 0;
    for (int c0 = 0; c0 < S; c0 += 64) {
      const int st = c0 + lane;
      const int v = st < S ? band_n[st] : 0;
      int x = v;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(x, off);
        if (lane >= off) x += o;
      }
      if (st < S) band_off[st] = carry + x - v;
      carry += __shfl(x, 63);
    }
    // publish both counts and the flag as one word: a relaxed device-scope atomic, no release / acquire fences
    // (which would write back / invalidate the whole L2 of this XCD)
    if (lane == 0)
      __hip_atomic_store(&w.pflag[pl], (1ull << 63) | ((unsigned long long)ntop << 32) | (unsigned)carry,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long word = 1ull << 63;
    for (;;) {
      if (lane < J) word = __hip_atomic_load(&w.pflag[b * J + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all(word >> 63)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    const int nt = lane < J ? (int)((word >> 32) & 0xffff) : 0;
    const int nh = lane < J ? (int)(word & 0xffffffffu) : 0;
    int top_before = lane < t ? nt : 0, thr_before = lane < t ? nh : 0, top_all = nt, thr_all = nh;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      top_before += __shfl_xor(top_before, off); thr_before += __shfl_xor(thr_before, off);
      top_all += __shfl_xor(top_all, off); thr_all += __shfl_xor(thr_all, off);
    }
    if (lane == 0) {
      sh[5] = top_before; sh[6] = top_all + thr_before;
      if (t == 0) {
        n_det[b] = top_all + thr_all;
        if (n_host) __hip_atomic_store(&n_host[b], top_all + thr_all, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  __syncthreads();
  PEMP_CLK(4);
  // ---- F: emission ----
  const int top_base = sh[5], thr_base = sh[6];
  int64_t* dout = det + (size_t)b * cap * 3;
  float* sout = scores + (size_t)b * cap;
  if ((int)threadIdx.x < ntop) {
    const int pos = top_base + threadIdx.x;
    if (pos < cap) {
      const int idx = top_i[KMAX + threadIdx.x];
      dout[pos * 3 + 0] = idx % W;
      dout[pos * 3 + 1] = idx / W;
      dout[pos * 3 + 2] = t;
      sout[pos] = top_sc[threadIdx.x];
    }
  }
  __shared__ cmask_t cm_sh[4][64][64];
  __shared__ int nz_sh[4][64];
  __shared__ int q_xy[4][64], q_o[4][64];          // a wave's queued detections: y * W + x, output slot
  const float* plane = s + (size_t)pl * H * W;
  int qn = 0;                                      // (wave-uniform)
  auto flush = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < qn && q_xy[wave][lane] >= 0) {
      const int xy = q_xy[wave][lane], o = q_o[wave][lane];
      const int yy = xy / W, xx = xy - yy * W;
      const float sv = pj.S ? proj_pixel(pj, b, t, yy, xx, H, W) : plane[xy];
      float jm = 1.0f;
      if (masks) jm = jm * masks[((size_t)b * H + yy) * W + xx];
      dout[o * 3 + 0] = xx;
      dout[o * 3 + 1] = yy;
      dout[o * 3 + 2] = t;
      sout[o] = sv * jm;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    qn = 0;
  };
  int kb = 0;
  for (int st = 0; st < S; ++st) {
    if (band_n[st] == 0) continue;                       // uniform
    if ((kb++ & 3) != wave) continue;
    const int ry0 = st * SR, rows = min(SR, H - ry0);
    int pos = thr_base + band_off[st];
    const size_t u0 = ((size_t)pl * g.nb + st) * g.nsx;   // first unit of the band (nsx <= 64)
    const unsigned long long nzm = (unsigned long long)band_nz[st][0] | ((unsigned long long)band_nz[st][1] << 32);
    int nnz = 0;
    unsigned rows_any = 0;
    unsigned cms[4];
    {                                                    // the first 4 strips' column masks together
      unsigned long long m = nzm;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int sx = m ? __builtin_ctzll(m) : 0;
        cms[k] = cbits[(u0 + sx) * 64 + lane];
        if (m) m &= m - 1;
      }
    }
    for (unsigned long long m = nzm; m; m &= m - 1) {
      const int sx = __builtin_ctzll(m);
      const unsigned cm = nnz < 4 ? cms[nnz & 3] : cbits[(u0 + sx) * 64 + lane];
      cm_sh[wave][nnz][lane] = (cmask_t)cm;
      if (lane == 0) nz_sh[wave][nnz] = sx;
      unsigned ra = cm;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) ra |= __shfl_xor(ra, off);
      rows_any |= ra;
      ++nnz;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (unsigned rm = rows_any & (rows >= 32 ? ~0u : (1u << rows) - 1u); rm; rm &= rm - 1) {
      const int j = __builtin_ctz(rm), yy = ry0 + j;
      for (int k = 0; k < nnz; ++k) {
        const int sx = nz_sh[wave][k];
        unsigned long long word = __ballot((cm_sh[wave][k][lane] >> j) & 1u);
        if (!word) continue;
        for (int q = 0; q < ntop; ++q)                   // already listed as a top-k detection
          if (ex_y[q] == yy && ex_sx[q] == sx) word &= ~(1ull << ex_lane[q]);
        const int cnt = __popcll(word);
        if (qn + cnt > 64) flush();
        if ((word >> lane) & 1ull) {
          const int below = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(word >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((unsigned)word, 0u));
          const int o = pos + below;
          if (o < cap) {
            q_xy[wave][qn + below] = yy * W + sx * g.sc - g.p + lane;
            q_o[wave][qn + below] = o;
          } else {
            q_xy[wave][qn + below] = -1;
          }
        }
        qn += cnt;
        pos += cnt;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (qn) flush();
#if PEMP_DETECT_CLOCKS
  __syncthreads();
  PEMP_CLK(5);
  if (threadIdx.x == 0 && t == 0)
    printf("clk plane %d: start %lld gathered +%lld selected +%lld listed +%lld published +%lld emitted +%lld\n", pl,
           clk[0], clk[1] - clk[0], clk[2] - clk[0], clk[3] - clk[0], clk[4] - clk[0], clk[5] - clk[0]);
#endif
#undef PEMP_CLK
}

#ifndef PEMP_DETECT_FUSED
#define PEMP_DETECT_FUSED 1
#endif

template <int P, int MODE, int PROJ>
static void launch_nms(const float* s, const float* masks, const DetectGeom& g, float thr, int use_thr,
                       const DetectWs& w, const ProjArgs& pj, hipStream_t st) {
  const int total = g.B * g.J * g.units;
  const int want = (total + NT1 / 64 - 1) / (NT1 / 64);
  // resident workgroups per CU: 5 (the kernel fits 91 VGPRs: 5 waves per SIMD; measured 59-60 vs 61-63 us at 4);
  // the 32-row units need ~190 VGPRs: 2
  // The grid-stride loop assumes every workgroup is resident: size the grid by the kernel's own occupancy
  // (the projected loaders need ~140 VGPRs: 3 workgroups per CU, not 4; a fourth row of workgroups
  // would only start once the first ones finish)
  auto launch = [&](auto kern) {
    int per_cu = SR > 16 ? 2 : NMS_PER_CU, occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, NT1, 0) == hipSuccess && occ > 0)
      per_cu = std::min(per_cu, occ);
    static const int cus = [] {   // CUs the strips spread over (PEMP_NMS_RESERVE_CUS left to another batch in flight)
      const char* e = getenv("PEMP_NMS_RESERVE_CUS");
      const int r = e ? (atoi(e) & ~7) : NMS_RESERVE_CUS;
      return std::max(8, num_cus() - std::max(r, 0));
    }();
    const int grid = want < per_cu * cus ? want : per_cu * cus;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT1), 0, st, s, masks, g, thr, use_thr, w.cand_v, w.cand_i, w.neg_v,
                       w.neg_i, w.tile_count, w.tile_nonneg, w.cbits, pj, w.pflag);
  };
  const bool tp = MODE == MODE_POS && thr > 0.0f && NMS_THR_POS;
  if (masks) {
    if (tp) launch(nms_strips_kernel<P, MODE, true, PROJ, MODE == MODE_POS>);
    else launch(nms_strips_kernel<P, MODE, true, PROJ, false>);
  } else {
    if (tp) launch(nms_strips_kernel<P, MODE, false, PROJ, MODE == MODE_POS>);
    else launch(nms_strips_kernel<P, MODE, false, PROJ, false>);
  }
}

template <int P>
static void launch_quad(const float* s, const DetectGeom& g, float thr, const DetectWs& w, hipStream_t st) {
  const int total = g.B * g.J * g.blocks;
  const int want = (total + NT1 / 64 - 1) / (NT1 / 64);
  auto launch = [&](auto kern) {
    int per_cu = NMS_QUAD_PER_CU, occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, NT1, 0) == hipSuccess && occ > 0)
      per_cu = std::min(per_cu, occ);
    static const int cus = [] {
      const char* e = getenv("PEMP_NMS_RESERVE_CUS");
      const int r = e ? (atoi(e) & ~7) : NMS_RESERVE_CUS;
      return std::max(8, num_cus() - std::max(r, 0));
    }();
    const int grid = want < per_cu * cus ? want : per_cu * cus;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT1), 0, st, s, g, thr, w.cand_v, w.cand_i, w.neg_v, w.neg_i,
                       w.tile_count, w.tile_nonneg, w.cbits, w.pflag);
  };
  if (thr > 0.0f && NMS_THR_POS) launch(nms_quad_kernel<P, true>);
  else launch(nms_quad_kernel<P, false>);
}

static void dispatch_quad(const float* s, const DetectGeom& g, float thr, const DetectWs& w, hipStream_t st) {
  switch (g.pr) {
    case 0: launch_quad<0>(s, g, thr, w, st); break;
    case 1: launch_quad<1>(s, g, thr, w, st); break;
    case 2: launch_quad<2>(s, g, thr, w, st); break;
    case 3: launch_quad<3>(s, g, thr, w, st); break;
    default: launch_quad<4>(s, g, thr, w, st); break;
  }
}

// the quad layout takes dense MODE_POS detection without masks (PEMP_NMS_QUAD=0: the strip kernel, A/B runs); the
// choice depends only on the call's arguments, so a SELECT-only call on the same workspace sees the same layout
static bool use_quad(bool projected, bool masked, int use_thr) {
  static const bool on = [] {
    const char* e = getenv("PEMP_NMS_QUAD");
    return e ? atoi(e) != 0 : NMS_QUAD != 0;
  }();
  return on && !projected && !masked && use_thr;
}

template <int MODE, int PROJ>
static void dispatch_nms(const float* s, const float* masks, const DetectGeom& g, float thr, int use_thr,
                         const DetectWs& w, const ProjArgs& pj, hipStream_t st) {
  switch (g.p) {
    case 0: launch_nms<0, MODE, PROJ>(s, masks, g, thr, use_thr, w, pj, st); break;
    case 1: launch_nms<1, MODE, PROJ>(s, masks, g, thr, use_thr, w, pj, st); break;
    case 2: launch_nms<2, MODE, PROJ>(s, masks, g, thr, use_thr, w, pj, st); break;
    case 3: launch_nms<3, MODE, PROJ>(s, masks, g, thr, use_thr, w, pj, st); break;
    default: launch_nms<4, MODE, PROJ>(s, masks, g, thr, use_thr, w, pj, st); break;
  }
}

// host restatement of proj_taps (same fp32 operations, round to nearest): does every unit's row span
// fit the separable loader's PROJ_LR staged rows (with the one past them)?
static int proj_taps_host(int dst, int out_size, int in_size, bool upper) {
  const float scale = (float)in_size / (float)out_size;
  volatile float t = (float)dst + 0.5f;   // volatile: one rounded operation each, as on the device
  volatile float m = scale * t;
  float src = m - 0.5f;
  if (src < 0.f) src = 0.f;
  const int i0 = (int)src;
  return upper ? i0 + (i0 < in_size - 1 ? 1 : 0) : i0;
}

static bool proj_sep_ok(const ProjArgs& pj, const DetectGeom& g) {
  const int P = g.p;
  for (int s = 0; s < pj.S; ++s) {
    if ((size_t)pj.h[s] * pj.w[s] * 4 >= 0x7fffffffull) return false;   // the buffer descriptors' 32-bit extent
    for (int band = 0; band < g.nb; ++band) {
      const int y0 = band * SR;
      const int ya = std::min(std::max(y0 - P, 0), g.H - 1), yb = std::min(std::max(y0 + SR + P - 1, 0), g.H - 1);
      // the unit's source rows plus the one staged past them (the second tap of the bottom border's rows)
      if (proj_taps_host(yb, g.H, pj.h[s], true) - proj_taps_host(ya, g.H, pj.h[s], false) + 2 > PROJ_LR) return false;
    }
  }
  return true;
}

template <int KMAX>
static int launch_detect(const float* s, const float* masks, const DetectGeom& g, float thr, int use_thr,
                         int stages, const DetectWs& w, int64_t* det, float* scores, int32_t* n_det, int cap,
                         int32_t* n_host, const ProjArgs& pj, hipStream_t st) {
  if (stages & PEMP_DETECT_NMS) {
    ProfScope prof(pj.S ? "detect_nms_projected" : "detect_nms", st);
    if (g.quad) {
      dispatch_quad(s, g, thr, w, st);
    } else if (pj.S && proj_sep_ok(pj, g)) {
      if (use_thr) dispatch_nms<MODE_POS, 2>(s, masks, g, thr, use_thr, w, pj, st);
      else dispatch_nms<MODE_ALL, 2>(s, masks, g, thr, use_thr, w, pj, st);
    } else if (pj.S) {
      if (use_thr) dispatch_nms<MODE_POS, 1>(s, masks, g, thr, use_thr, w, pj, st);
      else dispatch_nms<MODE_ALL, 1>(s, masks, g, thr, use_thr, w, pj, st);
    } else {
      if (use_thr) dispatch_nms<MODE_POS, 0>(s, masks, g, thr, use_thr, w, pj, st);
      else dispatch_nms<MODE_ALL, 0>(s, masks, g, thr, use_thr, w, pj, st);
    }
    PEMP_LAUNCH_CHECK();
  }
  // The fused stage's workgroups wait for their image's other J - 1 planes to publish: it needs at least J of its
  // workgroups resident at once (workgroups are dispatched in order, so complete images drain and make room for the
  // next). Checked once per device from the kernel's own occupancy; a device (partition) that cannot hold J takes
  // the two-kernel path, which has no inter-workgroup wait.
  auto fused_fits = [&]() {
    // (relaxed atomics: several host threads may launch detection at once; a race only recomputes the same value)
    static std::atomic<int> cap_wg[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) { (void)hipGetLastError(); return false; }
    int cap = cap_wg[dev].load(std::memory_order_relaxed);
    if (!cap) {
      int occ = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, plane_emit_kernel<KMAX>, 256, 0) != hipSuccess) {
        (void)hipGetLastError();
        occ = 0;
      }
      cap = std::max(occ, 0) * num_cus() + 1;   // (+1: computed)
      cap_wg[dev].store(cap, std::memory_order_relaxed);
    }
    return cap - 1 >= g.J;
  };
  if ((stages & PEMP_DETECT_SELECT) && PEMP_DETECT_FUSED && g.units <= SEL_UNITS && fused_fits()) {
    if (!(stages & PEMP_DETECT_NMS)) PEMP_HIP(hipMemsetAsync(w.pflag, 0, sizeof(unsigned long long) * g.B * g.J, st));
    ProfScope prof("detect_select_emit", st);
    hipLaunchKernelGGL(plane_emit_kernel<KMAX>, dim3(g.B * g.J), dim3(256), 0, st, s, masks, g, thr, use_thr, w.cbits,
                       w, det, scores, (int*)n_det, cap, (int*)n_host, pj);
    PEMP_LAUNCH_CHECK();
  } else if (stages & PEMP_DETECT_SELECT) {
    {
      ProfScope prof("detect_top", st);
      hipLaunchKernelGGL(plane_top_kernel<KMAX>, dim3(g.B * g.J), dim3(256), 0, st, g, thr, use_thr, w.cand_v,
                         w.cand_i, w.neg_v, w.neg_i, w.tile_count, w.tile_nonneg, w);
      PEMP_LAUNCH_CHECK();
    }
    ProfScope prof("detect_emit", st);
    hipLaunchKernelGGL(emit_kernel, dim3(g.B * g.J), dim3(256), 0, st, s, masks, g, w.cbits, w, det, scores,
                       (int*)n_det, cap, (int*)n_host, pj);
    PEMP_LAUNCH_CHECK();
  }
  return PEMP_OK;
}

// tags of the detections from the projected maps (channels J + type): joint_tags[n] = [up(maps_s)(y, x),
// up(flip(flip_maps_s))(y, x) at channel J + fi[type]] for the tag scale s (F = 1 without a flipped pass)
__global__ __launch_bounds__(256) void gather_proj_tags_kernel(ProjArgs pj, int s, int H, int W,
                                                               const int64_t* __restrict__ jdet,
                                                               const int64_t* __restrict__ bidx, int64_t N,
                                                               float* __restrict__ tags) {
  const int F = pj.f[s] ? 2 : 1;
  for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < N; n += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)jdet[n * 3], y = (int)jdet[n * 3 + 1], j = (int)jdet[n * 3 + 2];
    const int b = (int)bidx[n];
    const int h = pj.h[s], w = pj.w[s];
    const ProjTaps ty = proj_taps(y, H, h), tx = proj_taps(x, W, w);
    tags[n * F] = bilerp(pj.m[s] + ((size_t)b * pj.C + pj.ch0 + j) * h * w, w, ty, tx.i0, tx.i1, tx.l0, tx.l1);
    if (F == 2) {
      const int jf = pj.fi ? pj.fi[j] : j;
      tags[n * F + 1] = bilerp(pj.f[s] + ((size_t)b * pj.C + pj.ch0 + jf) * h * w, w, ty, w - 1 - tx.i0,
                               w - 1 - tx.i1, tx.l0, tx.l1);
    }
  }
}

// the projected scoremaps (or, ch0 = J, one tag plane f of the tags) materialised at [B, J, H, W]
__global__ __launch_bounds__(256) void proj_materialize_kernel(ProjArgs pj, int B, int J, int H, int W, int tags_f,
                                                               float* __restrict__ out) {
  const int64_t total = (int64_t)B * J * H * W;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int X = (int)(idx % W);
    const int64_t r = idx / W;
    const int Y = (int)(r % H), plane = (int)(r / H), b = plane / J, j = plane - b * J;
    if (tags_f < 0) {
      out[idx] = proj_pixel(pj, b, j, Y, X, H, W);
    } else {   // tags of scale 0 of pj (the caller selects the scale): f = 0 forward, 1 flipped
      const ProjTaps ty = proj_taps(Y, H, pj.h[0]), tx = proj_taps(X, W, pj.w[0]);
      const int h = pj.h[0], w = pj.w[0];
      float v;
      if (tags_f == 0) {
        v = bilerp(pj.m[0] + ((size_t)b * pj.C + pj.ch0 + j) * h * w, w, ty, tx.i0, tx.i1, tx.l0, tx.l1);
      } else {
        const int jf = pj.fi ? pj.fi[j] : j;
        v = bilerp(pj.f[0] + ((size_t)b * pj.C + pj.ch0 + jf) * h * w, w, ty, w - 1 - tx.i0, w - 1 - tx.i1, tx.l0,
                   tx.l1);
      }
      out[idx] = v;
    }
  }
}

// HigherHRNet's multi-stage merge at the last stage's resolution (_get_multi_stage_outputs, PoseEstimation.py:338-364
// for the forward pass, :380-412 for the flipped one, TEST.WITH_HEATMAPS [True, True] / WITH_AE [True, False]):
// up = bilinear stage 0 (h0 x w0) -> stage 1's h1 x w1 (align_corners=False, the projection's taps and fp32 order);
// out[b, c] = (up(s0)[b, c] + s1[b, c]) / 2 for c < J (heatmaps_avg = 0 + up(s0) + s1, / num_heatmaps = 2),
// out[b, c] = up(s0)[b, c] for J <= c < C0 (the tags: stage 0 only). One thread per output pixel, the channels in a
// loop (the taps are the pixel's): every row of every plane is read and written by consecutive lanes.
__global__ __launch_bounds__(256) void stage_merge_kernel(const float* __restrict__ s0, int C0, int h0, int w0,
                                                          const float* __restrict__ s1, int C1, int h1, int w1, int B,
                                                          int J, float* __restrict__ out) {
  const int64_t npix = (int64_t)B * h1 * w1, plane0 = (int64_t)h0 * w0, plane1 = (int64_t)h1 * w1;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < npix;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(idx % w1);
    const int64_t r = idx / w1;
    const int y = (int)(r % h1), b = (int)(r / h1);
    const ProjTaps ty = proj_taps(y, h1, h0), tx = proj_taps(x, w1, w0);
    const float* p0 = s0 + (size_t)b * C0 * plane0;
    const float* p1 = s1 + (size_t)b * C1 * plane1 + (size_t)y * w1 + x;
    float* po = out + (size_t)b * C0 * plane1 + (size_t)y * w1 + x;
    for (int c = 0; c < C0; ++c) {
      const float u = bilerp(p0 + c * plane0, w0, ty, tx.i0, tx.i1, tx.l0, tx.l1);
      po[c * plane1] = c < J ? __fmul_rn(__fadd_rn(u, p1[c * plane1]), 0.5f) : u;
    }
  }
}

static int proj_args(const pemp_proj_maps* m, int J, ProjArgs* pj, const char* fn) {
  PEMP_CHECK_ARG(m && m->num_scales >= 1 && m->num_scales <= PEMP_PROJ_MAXS && m->channels >= J && m->divisor > 0.f,
                 "%s: bad projected maps (1..%d scales, channels >= J, divisor > 0)", fn, PEMP_PROJ_MAXS);
  ProjArgs a{};
  a.S = m->num_scales;
  a.C = m->channels;
  for (int s = 0; s < a.S; ++s) {
    PEMP_CHECK_ARG(m->maps[s] && m->h[s] > 0 && m->w[s] > 0, "%s: scale %d: null map or empty size", fn, s);
    PEMP_CHECK_ARG((size_t)m->h[s] * m->w[s] < 0x7fffffffull, "%s: scale %d map too large", fn, s);
    a.m[s] = m->maps[s];
    a.f[s] = m->flip_maps[s];
    a.h[s] = m->h[s];
    a.w[s] = m->w[s];
  }
  a.fi = m->flip_index;
  a.divisor = m->divisor;
  int ex;
  a.rdiv = std::frexp(m->divisor, &ex) == 0.5f && ex >= -125 && ex <= 126 ? std::ldexp(1.0f, 1 - ex) : 0.f;
  a.ch0 = 0;
  *pj = a;
  return PEMP_OK;
}

}  // namespace
}  // namespace pemp

using namespace pemp;

extern "C" size_t pemp_detect_workspace_size(int B, int J, int H, int W, int topk) {
  if (B <= 0 || J <= 0 || H <= 0 || W <= 0) return 0;
  const int K = topk < H * W ? topk : H * W;
  size_t bytes = 0;
  carve(nullptr, geom(B, J, H, W, 2 * MAXR + 1, K), &bytes);   // widest halo = most strips (upper bound)
  return bytes;
}

static int detect_impl(const float* scoremaps, const ProjArgs* proj, const float* masks, int B, int J, int H, int W,
                       int pool_kernel, float threshold, int use_threshold, int topk, int stages, void* workspace,
                       size_t workspace_bytes, int64_t* det_xyt, float* det_scores, int32_t* n_det, int cap,
                       int32_t* n_det_host, void* stream) {
  PEMP_CHECK_ARG(workspace && det_xyt && det_scores && n_det, "pemp_detect: null pointer");
  PEMP_CHECK_ARG(B > 0 && J > 0 && J <= MAXJ && H > 0 && W > 0, "pemp_detect: bad shape B=%d J=%d H=%d W=%d", B, J, H, W);
  PEMP_CHECK_ARG(pool_kernel % 2 == 1 && pool_kernel >= 1 && pool_kernel / 2 <= MAXR,
                 "pemp_detect: pool_kernel must be odd and <= %d (got %d)", 2 * MAXR + 1, pool_kernel);
  PEMP_CHECK_ARG(topk >= 1 && topk <= 32, "pemp_detect: topk must be in [1, 32] (got %d)", topk);
  PEMP_CHECK_ARG(cap >= 0, "pemp_detect: cap < 0");
  PEMP_CHECK_ARG((size_t)H * W * 4 < 0x7fffffffull, "pemp_detect: plane too large (H * W * 4 >= 2^31)");
  const int K = topk < H * W ? topk : H * W;
  const DetectGeom g = geom(B, J, H, W, pool_kernel, K, use_quad(proj != nullptr, masks != nullptr, use_threshold));
  PEMP_CHECK_ARG(g.nsx <= 64, "pemp_detect: W=%d too wide (max %d for pool_kernel %d)", W, 64 * g.sc, pool_kernel);
  PEMP_CHECK_ARG(g.nb <= MAXB, "pemp_detect: H=%d too tall (max %d)", H, MAXB * SR);
  size_t need = 0;
  carve(nullptr, g, &need);
  if (workspace_bytes < need) {
    set_error("pemp_detect: workspace %zu < %zu bytes", workspace_bytes, need);
    return PEMP_ERR_WORKSPACE;
  }
  const DetectWs w = carve(workspace, g, nullptr);
  const hipStream_t st = as_stream(stream);
  int32_t* n_host = nullptr;   // device address of the caller's mapped host counts
  if (n_det_host) {
    PEMP_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&n_host), n_det_host, 0));
  }
  const ProjArgs pj = proj ? *proj : ProjArgs{};
  if (K <= 8)
    return launch_detect<8>(scoremaps, masks, g, threshold, use_threshold, stages, w, det_xyt, det_scores, n_det,
                            cap, n_host, pj, st);
  return launch_detect<32>(scoremaps, masks, g, threshold, use_threshold, stages, w, det_xyt, det_scores, n_det,
                           cap, n_host, pj, st);
}

extern "C" int pemp_detect(const float* scoremaps, const float* masks, int B, int J, int H, int W, int pool_kernel,
                           float threshold, int use_threshold, int topk, int stages, void* workspace,
                           size_t workspace_bytes, int64_t* det_xyt, float* det_scores, int32_t* n_det, int cap,
                           int32_t* n_det_host, void* stream) {
  PEMP_CHECK_ARG(scoremaps, "pemp_detect: null pointer");
  return detect_impl(scoremaps, nullptr, masks, B, J, H, W, pool_kernel, threshold, use_threshold, topk, stages,
                     workspace, workspace_bytes, det_xyt, det_scores, n_det, cap, n_det_host, stream);
}

extern "C" int pemp_detect_projected(const pemp_proj_maps* maps, const float* masks, int B, int J, int H, int W,
                                     int pool_kernel, float threshold, int use_threshold, int topk, int stages,
                                     void* workspace, size_t workspace_bytes, int64_t* det_xyt, float* det_scores,
                                     int32_t* n_det, int cap, int32_t* n_det_host, void* stream) {
  ProjArgs pj;
  if (const int rc = proj_args(maps, J, &pj, "pemp_detect_projected")) return rc;
  return detect_impl(nullptr, &pj, masks, B, J, H, W, pool_kernel, threshold, use_threshold, topk, stages, workspace,
                     workspace_bytes, det_xyt, det_scores, n_det, cap, n_det_host, stream);
}

extern "C" int pemp_project_maps(const pemp_proj_maps* maps, int B, int J, int H, int W, int tag_scale,
                                 float* scoremaps, float* tags, void* stream) {
  ProjArgs pj;
  if (const int rc = proj_args(maps, J, &pj, "pemp_project_maps")) return rc;
  PEMP_CHECK_ARG(B > 0 && J > 0 && H > 0 && W > 0 && (scoremaps || tags), "pemp_project_maps: bad args");
  const hipStream_t st = as_stream(stream);
  const int64_t total = (int64_t)B * J * H * W;
  const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
  ProfScope prof("project_maps", st);
  if (scoremaps) {
    hipLaunchKernelGGL(proj_materialize_kernel, dim3(grid), dim3(256), 0, st, pj, B, J, H, W, -1, scoremaps);
    PEMP_LAUNCH_CHECK();
  }
  if (tags) {   // [B, J, H, W, F] interleaved: materialise each f plane, then interleave on the host side
    PEMP_CHECK_ARG(tag_scale >= 0 && tag_scale < pj.S && maps->channels >= 2 * J, "pemp_project_maps: no tag channels");
    ProjArgs pt = pj;
    pt.S = 1;
    pt.m[0] = pj.m[tag_scale]; pt.f[0] = pj.f[tag_scale]; pt.h[0] = pj.h[tag_scale]; pt.w[0] = pj.w[tag_scale];
    pt.ch0 = J;
    const int F = pt.f[0] ? 2 : 1;
    for (int f = 0; f < F; ++f) {
      hipLaunchKernelGGL(proj_materialize_kernel, dim3(grid), dim3(256), 0, st, pt, B, J, H, W, f, tags + f * total);
      PEMP_LAUNCH_CHECK();
    }
  }
  return PEMP_OK;
}

extern "C" int pemp_stage_merge(const float* stage0, int C0, int h0, int w0, const float* stage1, int C1, int h1,
                                int w1, int B, int J, float* out, void* stream) {
  PEMP_CHECK_ARG(B > 0 && J > 0 && C0 >= J && C1 >= J && h0 > 0 && w0 > 0 && h1 > 0 && w1 > 0,
                 "pemp_stage_merge: bad shapes (B=%d J=%d C0=%d C1=%d)", B, J, C0, C1);
  PEMP_CHECK_ARG(stage0 && stage1 && out, "pemp_stage_merge: null pointer");
  PEMP_CHECK_ARG((size_t)h0 * w0 < 0x7fffffffull && (size_t)h1 * w1 < 0x7fffffffull, "pemp_stage_merge: map too large");
  const hipStream_t st = as_stream(stream);
  const int64_t npix = (int64_t)B * h1 * w1;
  ProfScope prof("stage_merge", st);
  hipLaunchKernelGGL(stage_merge_kernel, dim3((unsigned)std::min<int64_t>((npix + 255) / 256, 16384)), dim3(256), 0, st,
                     stage0, C0, h0, w0, stage1, C1, h1, w1, B, J, out);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

extern "C" int pemp_gather_projected_tags(const pemp_proj_maps* maps, int tag_scale, int J, int H, int W,
                                          const int64_t* joint_det, const int64_t* batch_index, int64_t N,
                                          float* joint_tags, void* stream) {
  ProjArgs pj;
  if (const int rc = proj_args(maps, 2 * J, &pj, "pemp_gather_projected_tags")) return rc;
  PEMP_CHECK_ARG(tag_scale >= 0 && tag_scale < pj.S && H > 0 && W > 0 && N >= 0,
                 "pemp_gather_projected_tags: bad args");
  PEMP_CHECK_ARG(N == 0 || (joint_det && batch_index && joint_tags), "pemp_gather_projected_tags: null pointer");
  if (N == 0) return PEMP_OK;
  pj.ch0 = J;
  const hipStream_t st = as_stream(stream);
  ProfScope prof("gather_proj_tags", st);
  hipLaunchKernelGGL(gather_proj_tags_kernel, dim3((unsigned)std::min<int64_t>((N + 255) / 256, 1024)), dim3(256), 0,
                     st, pj, tag_scale, H, W, joint_det, batch_index, N, joint_tags);
  PEMP_LAUNCH_CHECK();
  return PEMP_OK;
}

// Mapped, coherent host memory for pemp_detect's n_det_host (the kernels store into it directly).
extern "C" void* pemp_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 4, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    set_error("pemp_host_alloc: hipHostMalloc(%zu) failed", bytes);
    return nullptr;
  }
  return p;
}

extern "C" int pemp_host_free(void* p) {
  if (p) PEMP_HIP(hipHostFree(p));
  return PEMP_OK;
}
