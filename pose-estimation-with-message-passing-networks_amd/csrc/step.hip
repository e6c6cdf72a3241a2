// One batch of the inference path in one C-ABI call (pemp_step_fully_cap, include/pemp.h): the detection, the
// capacity graph build and the capacity-mode MPN forward queued back to back, every output carved from one caller
// buffer at offsets computed once per plan. Host code only (the kernels are those of detect.hip, graph.hip and
// mpn.hip, reached through their C entry points). It replaces, per batch, construct_graph_start's three
// argument lists and dozen output allocations (graph_constructor.py; ConstructGraph.py:1161-1209, 206-231, 376-381,
// NodeClassificationMPNSimple.py:62-97).
#include "pemp_common.h"

using namespace pemp;

namespace {

// the three logit arrays of a forward over (n_cap, e_cap): edge [max(n_rec, 1)][e_cap], node [n_rec + 1][n_cap] and
// class [n_rec + 1][n_cap][J], each starting on a 64-element boundary (as mpn/model.py lays them out)
int64_t logits_layout(const pemp_step_plan* p, int64_t* nlog_off, int64_t* clog_off) {
  const int64_t ne = (int64_t)std::max(p->n_rec, 1) * p->e_cap, nn = (int64_t)(p->n_rec + 1) * p->n_cap;
  *nlog_off = (ne + 63) / 64 * 64;
  *clog_off = *nlog_off + (nn + 63) / 64 * 64;
  return *clog_off + nn * p->desc->num_joints;
}

}  // namespace

extern "C" size_t pemp_step_layout(pemp_step_plan* p) {
  if (!p) {
    set_error("pemp_step_layout: null plan");
    return 0;
  }
  if (p->B <= 0 || p->J <= 0 || p->H <= 0 || p->W <= 0 || p->det_cap < 0 || p->C <= 0 || p->F < 0 || p->A <= 0 ||
      p->n_cap < 0 || p->e_cap < 0) {
    set_error("pemp_step_layout: bad plan (B=%d J=%d H=%d W=%d det_cap=%d C=%d F=%d A=%d n_cap=%lld e_cap=%lld)", p->B,
              p->J, p->H, p->W, p->det_cap, p->C, p->F, p->A, (long long)p->n_cap, (long long)p->e_cap);
    return 0;
  }
  if (p->desc) {
    const int st = p->desc->steps, aux = p->desc->aux_loss_steps;
    int n = 0;
    for (int i = 0; i < st; ++i) n += i >= st - aux - 1 ? 1 : 0;   // NodeClassificationMPNSimple.py:81-94
    p->n_rec = n;
  } else {
    p->n_rec = 0;
  }
  const size_t B = (size_t)p->B, cap = (size_t)p->det_cap, nc = (size_t)p->n_cap, ec = (size_t)p->e_cap;
  const size_t sizes[PEMP_STEP_NOUT] = {
      B * cap * 3 * 8,                    // DET
      B * cap * 4,                        // DSC
      B * 4,                              // NDET
      nc * (size_t)p->C * 4,              // X
      nc * 3 * 8,                         // JDET
      nc * 4,                             // JSC
      nc * 8,                             // BIDX
      nc * (size_t)p->F * 4,              // JTAGS
      2 * ec * 8,                         // EIDX
      ec * (size_t)p->A * 4,              // EATTR
      (B + 4) * 8,                        // NOFF
      0,                                  // LOGITS
  };
  size_t used = 0;
  for (int i = 0; i < PEMP_STEP_NOUT; ++i) {
    used = align_up(used, 256);
    p->off[i] = used;
    size_t n = sizes[i];
    if (i == PEMP_STEP_LOGITS && p->desc) {
      int64_t a1 = 0, a2 = 0;
      n = (size_t)logits_layout(p, &a1, &a2) * 4;
      p->elog_n = (int64_t)std::max(p->n_rec, 1) * p->e_cap;
      p->nlog_off = a1;
      p->clog_off = a2;
    }
    used += n;
  }
  if (!p->desc) p->elog_n = p->nlog_off = p->clog_off = 0;
  p->bytes = align_up(used, 256);
  return p->bytes;
}

extern "C" int pemp_step_fully_cap(const pemp_step_plan* p, const void* scoremaps, const float* masks,
                                   const float* features, const float* tagmaps, void* out, int32_t* n_det_host,
                                   void* stream) {
  PEMP_CHECK_ARG(p && scoremaps && features && out && p->bytes > 0, "pemp_step_fully_cap: null argument or plan "
                 "without a layout (pemp_step_layout)");
  PEMP_CHECK_ARG((p->F > 0) == (tagmaps != nullptr), "pemp_step_fully_cap: tagmaps %s but plan F = %d",
                 tagmaps ? "given" : "NULL", p->F);
  char* o = static_cast<char*>(out);
  auto at = [&](int i) { return o + p->off[i]; };
  int64_t* det = reinterpret_cast<int64_t*>(at(PEMP_STEP_DET));
  float* dsc = reinterpret_cast<float*>(at(PEMP_STEP_DSC));
  int32_t* n_det = reinterpret_cast<int32_t*>(at(PEMP_STEP_NDET));
  int rc;
  if (p->projected)
    rc = pemp_detect_projected(static_cast<const pemp_proj_maps*>(scoremaps), masks, p->B, p->J, p->H, p->W,
                               p->pool_kernel, p->threshold, p->use_threshold, p->topk, PEMP_DETECT_ALL,
                               p->det_workspace, p->det_workspace_bytes, det, dsc, n_det, p->det_cap, n_det_host,
                               stream);
  else
    rc = pemp_detect(static_cast<const float*>(scoremaps), masks, p->B, p->J, p->H, p->W, p->pool_kernel, p->threshold,
                     p->use_threshold, p->topk, PEMP_DETECT_ALL, p->det_workspace, p->det_workspace_bytes, det, dsc,
                     n_det, p->det_cap, n_det_host, stream);
  if (rc != PEMP_OK) return rc;
  float* x = reinterpret_cast<float*>(at(PEMP_STEP_X));
  int64_t* jdet = reinterpret_cast<int64_t*>(at(PEMP_STEP_JDET));
  int64_t* noff = reinterpret_cast<int64_t*>(at(PEMP_STEP_NOFF));
  float* eattr = reinterpret_cast<float*>(at(PEMP_STEP_EATTR));
  rc = pemp_fully_graph_build_cap(n_det, p->B, det, dsc, p->det_cap, features, p->C, tagmaps, p->F ? p->F : 1, p->J,
                                  p->H, p->W, p->n_cap, p->e_cap, p->norm_factor, p->mode | PEMP_BUILD_WRITE_COUNTS, x,
                                  jdet, reinterpret_cast<float*>(at(PEMP_STEP_JSC)),
                                  reinterpret_cast<int64_t*>(at(PEMP_STEP_BIDX)),
                                  p->F ? reinterpret_cast<float*>(at(PEMP_STEP_JTAGS)) : nullptr,
                                  reinterpret_cast<int64_t*>(at(PEMP_STEP_EIDX)), eattr, noff, stream);
  if (rc != PEMP_OK || !p->desc) return rc;
  PEMP_CHECK_ARG(p->desc->flags & PEMP_MPN_COUNTS_IN_OFFSETS,
                 "pemp_step_fully_cap: the forward reads the build's counts (desc flags PEMP_MPN_COUNTS_IN_OFFSETS)");
  float* lg = reinterpret_cast<float*>(at(PEMP_STEP_LOGITS));
  return pemp_mpn_forward_fully_cap(p->desc, p->weights, x, eattr, jdet + 2, p->n_cap, p->e_cap, n_det, p->det_cap,
                                    noff, p->B, lg, lg + p->nlog_off, lg + p->clog_off, p->mpn_workspace,
                                    p->mpn_workspace_bytes, stream);
}
