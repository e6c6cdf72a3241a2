/*
 * pemp.h — C-ABI of libpemp.so, the MI355X (gfx950) kernels of the keypoint-graph hot path of
 * nibox/Pose-Estimation-with-Message-Passing-Networks.
 *
 * Every function takes caller-owned DEVICE pointers (except where marked host), plain sizes and
 * a hipStream_t passed as void*. Work is stream-ordered; nothing synchronises the host. The
 * library owns no returned memory: outputs go to caller-allocated buffers, scratch goes to a
 * caller-allocated workspace sized by the matching *_workspace_size() query.
 * Return value: 0 (PEMP_OK) or a negative PEMP_ERR_*; pemp_last_error() gives a message
 * (thread-local).
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo):
 *   pemp_detect          ConstructGraph.py:1161-1209 joint_det_from_scoremap + cat_unique,
 *                        Utils/Utils.py:15-20 non_maximum_suppression
 *   pemp_pack_nodes      ConstructGraph.py:100-103,206-231 (node features, tags, batching)
 *   pemp_graph_offsets   ConstructGraph.py:222-223 (per-image node/edge offsets, on the device)
 *   pemp_fully_graph_build  the four above fused for GRAPH_TYPE fully (one launch)
 *   pemp_fully_graph     ConstructGraph.py:376-381 fully_connected_mpn_graph (+ batch offsets :222-223)
 *   pemp_knn_graph_*     ConstructGraph.py:363-368 knn_mpn_graph (torch_cluster knn_graph k=50,
 *                        PyG to_undirected, remove_self_loops)
 *   pemp_score_graph     ConstructGraph.py:405-422 score_based_graph (k = 75 roots)
 *   pemp_edge_features   ConstructGraph.py:289-359 (edge_attr)
 *   pemp_gather_projected  PoseEstimation.py:426-452 feature projection, sampled at the detections only
 *   pemp_gather_projected_conv  the same with feature_gather (PoseEstimation.py:64-66, 341) at the taps only
 *   pemp_pose_*          Utils.py:499-514,672-743,1445-1455 pose grouping (pred_to_ann prefix, pred_to_person,
 *                        GAEC of correlation_clustering_utils.py:187-245, graph_cluster_to_persons)
 *   pemp_mpn_forward     Models/MessagePassingNetwork/NodeClassificationMPNSimple.py:62-97 with
 *                        layers.py:32-86 (MPLayer) / :157-274 (TypeAwareMPNLayer)
 */
#ifndef PEMP_H_
#define PEMP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PEMP_ABI_VERSION 20

enum {
  PEMP_OK = 0,
  PEMP_ERR_INVALID_ARG = -1,
  PEMP_ERR_HIP = -2,
  PEMP_ERR_WORKSPACE = -3,
  PEMP_ERR_UNSUPPORTED = -4,
};

int pemp_abi_version(void);
const char* pemp_last_error(void);
/* 0 if the current HIP device is a gfx950 (MI355X); PEMP_ERR_UNSUPPORTED otherwise. */
int pemp_device_check(void);

/* ------------------------------------------------------------------------------------------
 * Detection: NMS maxima (MaxPool2d(k,1,k//2) == s, -inf padding), s *= maxima (* mask),
 * per-type top-k (ties: lower flat index first) + threshold set, cat_unique ordering:
 *   [top-k dets of type 0..J-1, each sorted by (y,x), value != 0]
 *   ++ [dets with s >= threshold not already listed, type-major then (y,x)].
 * use_threshold = 0 restates the DETECT_THRESHOLD > 1.5 branch (top-20, +1e-10).
 * Writes det_xyt[b][i] = (x, y, type) int64 and det_scores[b][i] for i < min(n, cap), and
 * n_det[b] = n (the true count, which may exceed cap: re-run with stages = PEMP_DETECT_SELECT
 * and a larger cap; the NMS stage's workspace is reused).
 * n_det_host (optional): host memory from pemp_host_alloc. Each n is stored into it by the device
 * when the selection stage starts writing the detections: the caller sets it to -1, launches, and
 * reads it while the stream keeps running (the one count read-back of ConstructGraph.py's
 * nonzero calls, without a copy or an event wait).
 * ---------------------------------------------------------------------------------------- */
enum { PEMP_DETECT_NMS = 1, PEMP_DETECT_SELECT = 2, PEMP_DETECT_ALL = 3 };
size_t pemp_detect_workspace_size(int B, int J, int H, int W, int topk);
int pemp_detect(const float* scoremaps /*[B,J,H,W]*/, const float* masks /*[B,H,W] or NULL*/,
                int B, int J, int H, int W, int pool_kernel, float threshold, int use_threshold,
                int topk, int stages, void* workspace, size_t workspace_bytes,
                int64_t* det_xyt /*[B,cap,3]*/, float* det_scores /*[B,cap]*/,
                int32_t* n_det /*[B]*/, int cap, int32_t* n_det_host /*[B] or NULL*/, void* stream);
/* The test-time front-end evaluated inside the detection instead of materialising [B,J,H,W] maps
 * (PoseEstimation.py:329-452 _get_multi_stage_outputs with flip + project2image,
 * multi_scales_testing.py:144-195 aggregate_results_mpn, PoseEstimation.py:227):
 *   s[b,j,Y,X] = (sum_s avg_s[b,j,Y,X]) / divisor,
 *   avg_s = flip_maps[s] ? (up(maps[s])[b,j] + up(flip(flip_maps[s]))[b,flip_index[j]]) / 2
 *                        : up(maps[s])[b,j],
 * up = bilinear to H x W, align_corners = False (torch's source-index rule), each product and sum rounded
 * in fp32 in the order t0 = a lx0 + b lx1, t1 = c lx0 + d lx1, v = t0 ly0 + t1 ly1; flip mirrors the
 * columns of the low-resolution map. maps[s] / flip_maps[s]: the network's outputs for scale s as it
 * produced them ([B][channels][h][w]: heatmaps in channels 0..J-1, per-joint tags in J..2J-1; the
 * flipped pass NOT un-flipped), flip_maps NULL without flip test. flip_index: device [J] int32 (the
 * FLIP_CONFIG permutation) or NULL for the identity. Scales summed in the caller's order (the reference
 * visits them in descending scale). */
#define PEMP_PROJ_MAXS 4
typedef struct pemp_proj_maps {
  int num_scales;
  int channels;
  const float* maps[PEMP_PROJ_MAXS];
  const float* flip_maps[PEMP_PROJ_MAXS];
  int h[PEMP_PROJ_MAXS], w[PEMP_PROJ_MAXS];
  const int32_t* flip_index;
  float divisor;                        /* len(TEST.SCALE_FACTOR) */
} pemp_proj_maps;
/* pemp_detect on the projected maps (same outputs, workspace and stages; the values are sampled on
 * demand in the NMS loads and at the emitted detections). */
int pemp_detect_projected(const pemp_proj_maps* maps, const float* masks, int B, int J, int H, int W,
                          int pool_kernel, float threshold, int use_threshold, int topk, int stages,
                          void* workspace, size_t workspace_bytes, int64_t* det_xyt, float* det_scores,
                          int32_t* n_det, int cap, int32_t* n_det_host, void* stream);
/* The same maps materialised (refine / adjust need the image-size maps; checks): scoremaps [B,J,H,W]
 * (or NULL) and tags (or NULL) as F planes [F][B,J,H,W] (f = 0 forward, 1 flipped pass), F = 2 with a
 * flipped pass. Values identical to the ones the detection samples. */
int pemp_project_maps(const pemp_proj_maps* maps, int B, int J, int H, int W, int tag_scale, float* scoremaps,
                      float* tags, void* stream);

/* HigherHRNet's multi-stage merge (_get_multi_stage_outputs, PoseEstimation.py:338-364 forward pass, :380-412 the
 * flipped pass before its flip, with TEST.WITH_HEATMAPS [True, True] / TEST.WITH_AE [True, False] of the published
 * configs): stage0 [B, C0, h0, w0] (heatmaps in channels 0..J-1, per-joint tags in J..C0-1), stage1 [B, C1, h1, w1]
 * (heatmaps in 0..J-1) -> out [B, C0, h1, w1]: (up(stage0) + stage1) / 2 in channels 0..J-1, up(stage0) in J..C0-1,
 * up = bilinear to h1 x w1 with align_corners=False (the rounding of pemp_project_maps). The merged maps of every
 * scale and pass are what pemp_proj_maps takes (a flipped pass merged in the network's orientation: the projection
 * applies the flip). Device pointers, stream-ordered. */
int pemp_stage_merge(const float* stage0, int C0, int h0, int w0, const float* stage1, int C1, int h1, int w1, int B,
                     int J, float* out, void* stream);
/* joint_tags [N, F] of the detections from the tag channels (J + type) of scale tag_scale: F = 2
 * (up(maps), up(flip(flip_maps)) at channel J + flip_index[type]) with a flipped pass, else F = 1
 * (aggregate_results_mpn's tags_list of that scale, ConstructGraph.py:103). channels >= 2 J. */
int pemp_gather_projected_tags(const pemp_proj_maps* maps, int tag_scale, int J, int H, int W,
                               const int64_t* joint_det, const int64_t* batch_index, int64_t N,
                               float* joint_tags, void* stream);
/* Mapped, coherent host memory (hipHostMalloc) that kernels may store into; NULL on failure. */
void* pemp_host_alloc(size_t bytes);
int pemp_host_free(void* p);

/* ------------------------------------------------------------------------------------------
 * Node packing into the batched layout: x[g] = features[b,:,y,x], joint_det[g], joint_scores[g],
 * batch_index[g] = b, joint_tags[g,:] = tagmaps[b,type,y,x,:] for g = node_off[b] + i.
 * node_off: device [B+1] int64. tagmaps may be NULL (then joint_tags is not written).
 * ---------------------------------------------------------------------------------------- */
int pemp_pack_nodes(const float* features /*[B,C,H,W]*/, int C, const float* tagmaps /*[B,J,H,W,F]*/,
                    int F, int B, int J, int H, int W, const int64_t* det_xyt, const float* det_scores,
                    int cap, const int64_t* node_off, int64_t n_total, float* x /*[N,C]*/,
                    int64_t* joint_det /*[N,3]*/, float* joint_scores /*[N]*/,
                    int64_t* batch_index /*[N]*/, float* joint_tags /*[N,F]*/, void* stream);

/* Batch offsets on the device from pemp_detect's per-image counts (replaces the host cumsum +
 * upload of ConstructGraph.py:222-223): node_off[b] = sum_{b'<b} n_det[b'] ([B+1] int64) and, if
 * fully_edge_off != NULL, fully_edge_off[b] = sum_{b'<b} n_b' (n_b' - 1) ([B+1] int64). */
int pemp_graph_offsets(const int32_t* n_det, int B, int64_t* node_off, int64_t* fully_edge_off, void* stream);

/* The whole fully-connected graph in ONE launch after the count read-back (equivalent to
 * pemp_graph_offsets + pemp_pack_nodes + pemp_fully_graph + pemp_edge_features, same outputs
 * bit for bit): node offsets from n_det, node packing, edge_index of every image, edge_attr
 * (mode = PEMP_EF_*; the AE modes read the tags from tagmaps). B <= 1024.
 * n_total = sum n_det, e_total = sum n (n - 1). tagmaps / joint_tags may be NULL. */
int pemp_fully_graph_build(const int32_t* n_det, int B, const int64_t* det_xyt, const float* det_scores, int cap,
                           const float* features, int C, const float* tagmaps, int F, int J, int H, int W,
                           int64_t n_total, int64_t e_total, float norm_factor, int mode, float* x,
                           int64_t* joint_det, float* joint_scores, int64_t* batch_index, float* joint_tags,
                           int64_t* edge_index, float* edge_attr, int64_t* node_off /*[B+1] or NULL*/,
                           void* stream);

/* Capacity mode of pemp_fully_graph_build, launched BEFORE the host reads the counts back (the
 * reference's nonzero/cat syncs, ConstructGraph.py:1170-1196, become one host read that overlaps
 * this launch): the totals come from n_det on the device; x / joint_* hold n_cap rows, edge_attr
 * e_cap rows and edge_index 2 * e_cap entries written as a contiguous [2, E] array. When the batch
 * exceeds either capacity nothing is written: the caller compares its read-back totals with the
 * capacities and then calls pemp_fully_graph_build with exact sizes. */
/* mode | PEMP_BUILD_WRITE_COUNTS (capacity mode): node_off holds B + 4 entries and the build also writes the batch's
 * (N, E, overflow) at node_off[B + 1 .. B + 3] -- (0, 0, 1) for a batch past a capacity -- for
 * pemp_mpn_forward_fully_cap with PEMP_MPN_COUNTS_IN_OFFSETS */
#define PEMP_BUILD_WRITE_COUNTS 0x100
int pemp_fully_graph_build_cap(const int32_t* n_det, int B, const int64_t* det_xyt, const float* det_scores, int cap,
                               const float* features, int C, const float* tagmaps, int F, int J, int H, int W,
                               int64_t n_cap, int64_t e_cap, float norm_factor, int mode, float* x,
                               int64_t* joint_det, float* joint_scores, int64_t* batch_index, float* joint_tags,
                               int64_t* edge_index, float* edge_attr, int64_t* node_off /*[B+1] or NULL*/,
                               void* stream);

/* Fully connected graph per image: all (i,j), i != j, sorted by (src,dst), node-offset per image.
 * node_off / edge_off: device [B+1] int64 with edge_off[b+1]-edge_off[b] = n_b (n_b - 1). */
int pemp_fully_graph(const int64_t* node_off, const int64_t* edge_off, int B, int64_t e_total,
                     int64_t* edge_index /*[2,E]*/, void* stream);

/* knn graph per image (k nearest by squared integer distance, ties by node index; k+1 queried
 * with self removed), symmetrised and sorted by (src,dst).
 * Stage 1 (count): writes edge_count[b] (device int64 [B]). Host then sizes E and edge_off.
 * Stage 2 (emit): writes edge_index with per-image offsets edge_off (device [B+1]).
 * node_off_host: HOST [B+1] copy of node_off (grid sizing). Workspace is shared by both stages. */
size_t pemp_knn_workspace_size(const int64_t* node_off_host, int B);
int pemp_knn_graph_count(const int64_t* joint_det, const int64_t* node_off, const int64_t* node_off_host,
                         int B, int k, void* workspace, size_t workspace_bytes, int64_t* edge_count,
                         void* stream);
int pemp_knn_graph_emit(const int64_t* node_off, const int64_t* node_off_host, int B,
                        const int64_t* edge_off, int64_t e_total, void* workspace,
                        size_t workspace_bytes, int64_t* edge_index, void* stream);
/* Both stages in one call, no host round trip between them (replaces ConstructGraph.py:363-368 +
 * the count read-back): adjacency, per-image counts, their device scan and the emit, back to back.
 * edge_buf: device int64 [2 * e_cap], e_cap >= sum_b min(n_b (n_b - 1), 2 k n_b) (checked); the graph
 * is its leading [2, E] block (sources at 0, destinations at E). e_total_host: mapped host int32
 * (pemp_host_alloc), set to E by the device once the counts are scanned (the emit may still run);
 * the host spins on it (initialise it to -1). Batches whose images all have <= 512 nodes take the
 * fast path (3 launches: selection, LDS transpose, emit with the edge features; node coordinates must
 * fit int32), others the global-memory kernels above + the features kernel. */
int pemp_knn_graph_build(const int64_t* joint_det, const int64_t* node_off, const int64_t* node_off_host,
                         int B, int k, void* workspace, size_t workspace_bytes, int64_t e_cap,
                         int64_t* edge_buf, int32_t* e_total_host, const float* joint_tags, int F,
                         const float* joint_scores, int J, float norm_factor, int mode,
                         float* edge_attr /*[e_cap, A] or NULL: pemp_edge_features' values, leading E rows*/,
                         void* stream);

/* feature_knn graph per image (replaces ConstructGraph.py:370-374 feature_knn_mpn_graph:
 * knn_graph(x, k=50) over the node features -> to_undirected -> remove_self_loops), with the edge
 * features, in one queued call. Same contract as pemp_knn_graph_build (edge_buf, e_cap bound, mapped
 * e_total_host, fast path for images of <= 512 nodes), plus x: device [N, C] fp32 node features
 * (construct_graph's x; 16-byte aligned when C % 4 == 0; C <= 8192). Candidates are ranked by the
 * fp32 sum over c in order of (x_j[c] - x_i[c])^2 as one fma per channel (torch_cluster's CUDA knn
 * as nvcc compiles it), ties by node index; a NaN distance ranks last. The workspace also holds the
 * sum_b n_b^2 distance keys (pemp_feature_knn_workspace_size). */
size_t pemp_feature_knn_workspace_size(const int64_t* node_off_host, int B);
/* Byte offsets, inside a knn build's workspace, of the fast path's bit rows ([N][8] uint64), row starts ([N]
 * int32) and per-image edge counts ([B] int64) (offs[0..2]), for pemp_mpn_forward_knn; feature != 0 for a
 * pemp_feature_knn_graph_build workspace. Returns PEMP_ERR_UNSUPPORTED when the batch would not take the fast
 * path (an image over 512 nodes). */
int pemp_knn_rows_layout(const int64_t* node_off_host, int B, int feature, size_t* offs);
int pemp_feature_knn_graph_build(const float* x, int C, const int64_t* joint_det, const int64_t* node_off,
                                 const int64_t* node_off_host, int B, int k, void* workspace,
                                 size_t workspace_bytes, int64_t e_cap, int64_t* edge_buf,
                                 int32_t* e_total_host, const float* joint_tags, int F,
                                 const float* joint_scores, int J, float norm_factor, int mode,
                                 float* edge_attr, void* stream);

/* Node features from maps projected to the image size on demand (the test front-end's bilinear
 * projection, PoseEstimation.py:426-452, summed over scales and divided, multi_scales_testing.py:182-190
 * / PoseEstimation.py:244): x[n][c] = sum_s bilinear(maps[s][b_n][c], (y_n, x_n); H x W) / divisor,
 * align_corners = False, torch's source-index rule. maps: host array of S (<= 8) device pointers to
 * [B][C][map_h[s]][map_w[s]] fp32. Pairs with pemp_fully_graph_build / pemp_pack_nodes called with
 * features = NULL (they then leave x to this call). */
int pemp_gather_projected(const float* const* maps, const int* map_h, const int* map_w, int S, int C, int H, int W,
                          float divisor, const int64_t* joint_det, const int64_t* batch_index, int64_t N, float* x,
                          void* stream);
/* The same with the model's feature_gather Conv2d applied before the projection (PoseEstimation.py:64-66
 * nn.Conv2d(KP_OUTPUT_DIM, NODE_INPUT_DIM, FEATURE_GATHER_KERNEL, 1, FEATURE_GATHER_PADDING), applied per scale
 * at :341 and projected at :426-452): x[n][co] = sum_s bilinear(conv_s[b_n][co], (y_n, x_n); H x W) / divisor,
 * conv_s = bias + weight * maps[s] (stride 1, zero padding `pad`, output (h + 2 pad - k + 1) x (w + ...)),
 * evaluated only at the 4 taps of each detection. maps: S device pointers to [B][Cin][h_s][w_s] fp32;
 * weight_t: the Conv2d weight transposed to [Cin][k][k][Cout] (device fp32); bias: [Cout] or NULL.
 * Cout <= 512, k <= 7, Cin (k+1)^2 floats <= 64 KB. */
int pemp_gather_projected_conv(const float* const* maps, const int* map_h, const int* map_w, int S, int Cin,
                               const float* weight_t, const float* bias, int Cout, int ksize, int pad, int H, int W,
                               float divisor, const int64_t* joint_det, const int64_t* batch_index, int64_t N,
                               float* x, void* stream);

/* score_based graph per image (ConstructGraph.py:405-422 score_based_graph, k = 75 there): the k
 * highest-scoring nodes are roots (ties: lower node index; torch.topk leaves them unspecified);
 * edge (a, b), a != b, exists iff a or b is a root, sorted by (src, dst) with the per-image node
 * offsets added. Every image needs n >= k (the reference's topk raises otherwise: INVALID_ARG);
 * e_total must be sum over images of k (2 n - k - 1). */
size_t pemp_score_graph_workspace_size(const int64_t* node_off_host, int B, int k);
int pemp_score_graph(const float* joint_scores, const int64_t* node_off, const int64_t* node_off_host, int B, int k,
                     int64_t e_total, void* workspace, size_t workspace_bytes, int64_t* edge_index, void* stream);

/* Edge features. mode: */
enum {
  PEMP_EF_POSITION_CONNECTION = 0, /* [dx, dy, onehot(J)]       (J+2) */
  PEMP_EF_CONNECTION = 1,          /* [onehot(J)]               (J)   */
  PEMP_EF_NOTHING = 2,             /* [0]                       (1)   */
  PEMP_EF_POSITION = 3,            /* [dx, dy]                  (2)   */
  PEMP_EF_POSITION_ANGLE_CONNECTION = 4, /* [dx, dy, theta, onehot(J)] (J+3) */
  /* associative-embedding modes (ConstructGraph.py:337-357); dist = ||tag[dst] - tag[src]||_2 over
   * F = 1 or 2 tag dims, rounded as torch.norm on CPU: sqrt(fma(d1, d1, d0 * d0)) */
  PEMP_EF_POSITION_CONNECTION_AE = 5,    /* {position, connection_type, ae_normed}: [dx, dy, onehot(J), dist] (J+3) */
  PEMP_EF_AE = 6,                        /* {ae}: [dist] (1), F = 1 */
  PEMP_EF_AE_NORMED = 7,                 /* {ae_normed}: [round(dist) * 100 - score[src]] (1), F = 2 */
  PEMP_EF_AE_TRACKING = 8                /* {ae_tracking_1}: [(1.8425 - dist) / 1.8425] (1) */
};
/* joint_tags [N,F] / joint_scores [N] are read by the AE modes only (may be NULL otherwise). */
int pemp_edge_features(const int64_t* joint_det /*[N,3]*/, const float* joint_tags, int F, const float* joint_scores,
                       const int64_t* edge_index /*[2,E]*/, int64_t e_total, int J, float norm_factor, int mode,
                       float* edge_attr, void* stream);

/* ------------------------------------------------------------------------------------------
 * Pose grouping: Utils.py:1445-1455 (pred_to_ann: node threshold + subgraph),
 * Utils.py:499-514 (pred_to_person), correlation_clustering_utils.py:99-151,187-245 (edge matrix
 * symmetrisation, cluster_andres_graph with GAEC), Utils.py:672-743 (graph_cluster_to_persons).
 *
 * 1. pemp_pose_edge_weights (GPU, stream-ordered): edge_index [2,E] int64 must be strictly sorted by
 *    (src, dst) (construct_graph's output is). An edge survives iff use_th == 0 or both
 *    node_scores[end] > th. method 0 (GAEC): w[e] = fl32(pred[e] + pred[reverse(e)]) (0 if the reverse
 *    is absent) for surviving edges with src < dst; method 1 (threshold): w[e] = pred[e] for every
 *    surviving edge; NaN elsewhere. flags[B + 1] (device int32): flags[b] bit 0 = image b has a
 *    surviving src > dst edge with pred != 0 (the reference then averages, else adds), bit 1 = image b
 *    keeps an edge; flags[B] bit 0 = edge_index not sorted.
 * 2. pemp_pose_cluster (HOST arrays, copies of the above): per image, greedy additive edge contraction
 *    (andres graph greedyAdditiveEdgeContraction, weights (w/2 or w) - 0.5 in fp32, then double) or
 *    threshold joins (w > 0.8f); labels[ΣN] = connected-component ids per image in order of each
 *    component's lowest node (scipy connected_components), n_comp[B]. Images run on n_threads threads.
 * 3. pemp_pose_persons (HOST): graph_cluster_to_persons per image from labels: persons[cap][J][3] f64
 *    (x, y, score of the best-scoring joint per (re-)typed joint type; class_probs [ΣN,J] re-types by
 *    first argmax when non-NULL; pose_scores replaces the score when non-NULL), person_count[B],
 *    mutants[B] (a component larger than J). PEMP_ERR_WORKSPACE when more than cap persons. */
int pemp_pose_edge_weights(const int64_t* edge_index, int64_t E, const float* pred, const float* node_scores,
                           float th, int use_th, const int64_t* node_off /*[B+1] device*/, int B, int64_t N,
                           int method, int64_t* row_start /*[N+1] device scratch*/, float* w, int* flags,
                           void* stream);
int pemp_pose_cluster(int B, const int64_t* node_off, const int64_t* edge_index, int64_t E, const float* w,
                      const int* flags, int method, int n_threads, int32_t* labels, int32_t* n_comp);
int pemp_pose_persons(int B, const int64_t* node_off, const int32_t* labels, const int32_t* n_comp,
                      const int64_t* joint_det, const float* scores, const float* pose_scores,
                      const float* class_probs, int J, int allow_single, int64_t cap, double* persons,
                      int32_t* person_count, int32_t* mutants);

/* greedy_person_construction (Utils.py:517-626), HOST, per image over the surviving edges (w from
 * pemp_pose_edge_weights method 1: pred, NaN = dropped; edge_index sorted by src): taken[ΣN] (image-local
 * core node or -1), persons[cap][J][3] f64, person_count[B]. class_probs may be NULL. */
int pemp_pose_greedy(int B, const int64_t* node_off, const int64_t* edge_index, int64_t E, const float* w,
                     const int64_t* joint_det, const float* scores, const float* class_probs, int J, int32_t* taken,
                     int64_t cap, double* persons, int32_t* person_count);

/* Pose finishing, pred_to_ann (Utils.py:1468-1478) per image, keypoints [P][J][3] f64 (x, y, score):
 * pemp_pose_fill_mean (HOST): fill_mean, Utils.py:1468-1470.
 * pemp_pose_refine (GPU, keypoints in device memory, updated in place): refine, Utils.py:1026-1104 -- per
 *   person the float32 mean tag of its detected joints (numpy's summation order), per (person, joint) the
 *   first argmax over the map of s - rint(||tag - mean||) (one pass over the pixels per 8 persons), the
 *   quarter-pixel offset, and the fill of undetected joints with score 0.001. scoremaps [J][H][W] f32,
 *   tag [J][H][W][F] f32 (F = 1 or 2). Workspace: pemp_pose_refine_workspace_size(P, J, H, W, F) bytes.
 * pemp_pose_adjust (GPU, in place): adjust, Utils.py:917-936, det [J][H][W] f32. */
int pemp_pose_fill_mean(double* keypoints, int P, int J);
size_t pemp_pose_refine_workspace_size(int P, int J, int H, int W, int F);
int pemp_pose_refine(const float* scoremaps, const float* tag, int J, int H, int W, int F, double* keypoints, int P,
                     void* workspace, size_t workspace_bytes, void* stream);
int pemp_pose_adjust(const float* det, int J, int H, int W, double* keypoints, int P, void* stream);

/* Batched finishing (finish_batch, the per-image loop of valid.py:101-123 over pred_to_ann's refine / adjust):
 * every image's persons in one keypoints array [P][J][3] f64, person p of image pimg[p].
 * pemp_pose_finish_plan (HOST): from counts[B] persons per image and ref[B] (refine image b or not) fills
 *   pimg[P] and chunks[3 * n] (first person, persons, image; chunks of the refined images only, never across
 *   two images), out2 = {n, persons-per-chunk width}; at most max_chunks (P suffices).
 * pemp_pose_finish_batch (GPU, in place): refine (as pemp_pose_refine) for the persons of the images with
 *   ref[b] != 0, then adjust (adjust != 0) for all, scoremaps [B][J][H][W], tags [B][J][H][W][F] (NULL when
 *   no image is refined); pimg / chunks / ref in device memory. Workspace:
 *   pemp_pose_refine_workspace_size(P, J, H, W, F). Same keypoints as the per-image calls. */
/* pemp_pack_to_host (GPU + copy): the n <= 16 device regions src[i] (bytes[i] bytes each) gathered into the device
 * buffer staging at offsets off[i] (multiples of 16, off[i] + bytes[i] <= total), then one stream-ordered copy of
 * staging[0, total) to host_dst (pinned host memory): the grouping's read-back in one copy instead of one per
 * array. host_dst NULL: the gather only (the caller queues the copy itself). */
int pemp_pack_to_host(int n, const void* const* src, const size_t* bytes, const size_t* off, size_t total,
                      void* staging, void* host_dst, void* stream);
int pemp_pose_finish_plan(int B, const int32_t* counts, const uint8_t* ref, int32_t* pimg, int32_t* chunks,
                          int max_chunks, int32_t* out2);
int pemp_pose_finish_batch(const float* scoremaps, const float* tags, int B, int J, int H, int W, int F,
                           double* keypoints, int P, const int32_t* pimg, const int32_t* chunks, int n_chunks, int pc,
                           const uint8_t* ref, int adjust, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Message-passing network, inference (eval-mode BatchNorm folded into the next Linear by the
 * caller). All hidden widths are 64. Weights are fp32 row-major [out_pad][in_pad], zero padded
 * to multiples of 16 (the caller's folding step; see the Python mirror pemp_amd/mpn/fold.py).
 * ---------------------------------------------------------------------------------------- */
enum { PEMP_AGGR_ATTN = 0, PEMP_AGGR_SUM = 1, PEMP_AGGR_MEAN = 2, PEMP_AGGR_MAX = 3 };

/* Arithmetic of the per-edge GEMMs (edge embedding, edge MLP, message, edge head) and of the node
 * table; the other node-side GEMMs are fp32.
 *   PEMP_PREC_FP32   exact fp32 MFMA (v_mfma_f32_16x16x4_f32)
 *   PEMP_PREC_BF16X3 x·w ~= xh·wh + xl·wh + xh·wl with bf16 hi/lo parts and fp32 accumulation
 *                    (v_mfma_f32_16x16x32_bf16): ~2^-16 relative error per product.
 *   PEMP_PREC_F16X3  x·w ~= xh·wh + 2^-11 (xh·wl + xl·wh) with f16 parts, the low parts scaled by 2^11
 *                    (v_mfma_f32_16x16x32_f16, fp32 accumulation): ~2^-22 relative error per product,
 *                    fp32-level logits; fragments reaching 2^14 are range-scaled by exact powers of two.
 * Both split precisions need the *_bf weight packs, in the matching 16-bit format (the field names
 * keep "bf" for either). */
enum { PEMP_PREC_FP32 = 0, PEMP_PREC_BF16X3 = 1, PEMP_PREC_F16X3 = 2 };

typedef struct pemp_layer {
  const float* w; /* [out_pad][in_pad] */
  const float* b; /* [out_pad] */
  int32_t in_dim, out_dim, relu, pad_;
} pemp_layer;

typedef struct pemp_mlp {
  pemp_layer layer[4];
  int32_t n_layers, pad_;
} pemp_mlp;

typedef struct pemp_mpn_weights {
  pemp_mlp node_emb;   /* NODE_INPUT_DIM -> 64 */
  pemp_mlp edge_emb;   /* EDGE_INPUT_DIM -> 64 */
  const float* pre_w;  /* [128 + T*64][128]: W1[:, x_i], W1[:, x_j], W_t[:, x_i] (t < T) */
  const float* pre_b;  /* [128 + T*64]:      0,          0,          b_t               */
  const float* q0_w;   /* [64][64]  W1[:, e_init] */
  const float* q0_b;   /* [64]      b1            */
  const float* e1_w;   /* [64][64]  W1[:, e_cur]  */
  const float* e2_w;   /* [64][64]  mlp_edge.2    */
  const float* e2_b;   /* [64]                    */
  const float* msg_w;  /* [T][64][64] W_t[:, e'] */
  const float* attn_w; /* [64] attn_net.0.weight (PEMP_AGGR_ATTN); [17][64] when attn_bv is set */
  const float* upd_w;  /* [64][T*64] update_mlp.0.weight, or NULL (x_new = agg) */
  const float* upd_b;  /* [64] */
  pemp_mlp edge_head;  /* 64 -> .. -> 1 */
  pemp_mlp node_head;  /* 64 -> .. -> 1 */
  pemp_mlp class_head; /* 64 -> .. -> J */
  float attn_b;
  int32_t pad_;
  /* split-precision weight packs (16-bit patterns: bf16 hi / lo for PEMP_PREC_BF16X3, f16 hi / f16 lo
   * scaled by 2^11 for PEMP_PREC_F16X3): per matrix [hi | lo][out][64] with the input
   * columns in MFMA slot order: slot 32 kb + 8 g + j holds input 32 kb + 16 (j >> 2) + 4 g + (j & 3). */
  const uint16_t* e1_bf;   /* [2][64][64]    */
  const uint16_t* e2_bf;   /* [2][64][64]    */
  const uint16_t* msg_bf;  /* [T][2][64][64] */
  const uint16_t* head_bf; /* edge head layers 1, 2 (published 64->64->32->1): [2][64][64] then [2][32][64], or NULL */
  const uint16_t* emb_bf;  /* edge embedding layers then the e_init block of mlp_edge.0 (q0): per layer
                              [2][out_pad16][in_pad32], concatenated; or NULL (embedding stays fp32) */
  const uint16_t* upd_bf;  /* per type t: U_t = upd_w[:, 64 t : 64 t + 64] as [T][2][64][64], or NULL */
  const uint16_t* pre_bf;  /* node table weights [2][128 + T*64][128] (K = 128, 4 slot blocks), or NULL */
  const float* node_img;   /* node embedding + head weights in the kernels' LDS layout (pemp_mpn_node_image),
                              or NULL: then every forward builds it in its workspace */
  const float* attn_bv;    /* AGGR_SUB node_edge_attn_per_type (layers.py:199-201, 245-246): [17] attn_net.0.bias;
                              messages from source type t use row t of attn_w and attn_bv[t]. NULL: one shared
                              row attn_w[64] with bias attn_b (node_edge_attn) */
  pemp_mlp upd_mlp;        /* UPDATE_TYPE hierarch_mlp / hierarch_cnn (layers.py:89-154) folded into dense
                              layers over agg[n] flattened to [T*64] (ReLU each; widths % 16 == 0, last 64);
                              n_layers = 0 otherwise. Excludes upd_w. */
  /* EDGE_MLP per_type (TypeAwareEdgeUpdate, layers.py:275-303; attention aggregation), or NULL:
   *   e' = ReLU(O1 ReLU(L1[t_dst] x_dst + c1) + O2 ReLU(L2[t_src] x_src + c2) + e2_w ReLU(q0 + e1_w e) + e2_b)
   * with q0_w / q0_b / e1_w = edge_layer (e_init / e_cur columns), e2_w / e2_b = the e-block of out.1 and
   * the A / B rows of pre_w zero. L1, L2: [T][64][128] on [x_init | x_cur]; c1, c2: [T][64]; O1, O2: [64][64]. */
  const float *ept_l1_w, *ept_l1_b, *ept_l2_w, *ept_l2_b, *ept_o1_w, *ept_o2_w;
  const float* edge_img;   /* edge-pass weight image (pemp_mpn_edge_image for the same desc), or NULL: then every
                              forward builds it in its workspace */
  /* The edge embedding composed with the first edge-MLP layer (PEMP_PREC_F16X3 and the published embedding shape
   * A -> 32 -> 64 -> 64 -> 64, ReLU after all but the last layer), or NULL. The last embedding Linear (W4, b4) has no
   * ReLU, so with h3 the third layer's output: Q0 = Wq h3 + bq, Wq = q0_w W4, bq = q0_w b4 + q0_b, and
   * R0 = Wr h3 + br, Wr = (q0_w + e1_w) W4, br = (q0_w + e1_w) b4 + q0_b, formed by the caller in fp64.
   * emb_comp_bf: [2 (Wq, Wr)][2][64][64] f16x3 packs (as e1_bf); emb_comp_b: [2][64] (bq, br). */
  const uint16_t* emb_comp_bf;
  const float* emb_comp_b;
} pemp_mpn_weights;

typedef struct pemp_mpn_desc {
  int32_t num_types;      /* T: aggregation/message types (NUM_JOINTS, 6, 9) or 1 (MPLayer) */
  int32_t num_joints;     /* J: class-head width */
  int32_t steps;          /* STEPS */
  int32_t aux_loss_steps; /* heads recorded at iterations it >= steps - aux - 1 */
  int32_t aggr;           /* PEMP_AGGR_* */
  int32_t hidden;         /* must be 64 */
  int32_t edge_attr_dim;  /* EDGE_INPUT_DIM */
  int32_t node_in_dim;    /* NODE_INPUT_DIM */
  int32_t precision;      /* PEMP_PREC_* */
  int32_t types_stride;   /* element stride of node_types (e.g. 3 for joint_det[:, 2]); 0 or 1 = dense */
  int32_t flags;          /* PEMP_MPN_PREPARED: pemp_mpn_prepare already ran on this workspace and stream */
} pemp_mpn_desc;

#define PEMP_MPN_PREPARED 1
/* pemp_mpn_forward_fully_cap only: node_off holds B + 4 entries, the last three the batch's (N, E, overflow) as
 * pemp_fully_graph_build_cap wrote them with PEMP_BUILD_WRITE_COUNTS: the forward reads them instead of deriving
 * them from n_det in a launch of its own */
#define PEMP_MPN_COUNTS_IN_OFFSETS 2

size_t pemp_mpn_workspace_size(const pemp_mpn_desc* desc, int64_t N, int64_t E);
/* x [N,node_in_dim], edge_attr [E,edge_attr_dim], edge_index [2,E] (row 0 source j, row 1
 * target i), node_types [N] with element stride desc->types_stride (already mapped by
 * sum_node_types; values < T).
 * Outputs (n_rec = min(aux+1, steps) recorded iterations, NodeClassificationMPNSimple.py:81-94):
 *   edge_logits [n_rec][E]; node_logits [n_rec+1][N] and class_logits [n_rec+1][N][J], whose
 *   last slot is the head evaluation after the loop (:93-94). */
int pemp_mpn_forward(const pemp_mpn_desc* desc, const pemp_mpn_weights* weights, const float* x,
                     const float* edge_attr, const int64_t* edge_index, const int64_t* node_types,
                     int64_t N, int64_t E, float* edge_logits, float* node_logits, float* class_logits,
                     void* workspace, size_t workspace_bytes, void* stream);

/* pemp_mpn_forward for a batch whose edge_index is the fully-connected graph of
 * pemp_fully_graph_build (ConstructGraph.py:376-381) with per-image node offsets node_off (device,
 * [B+1], as written by the build) / node_off_host: the type-major edge order is produced in closed
 * form by one kernel instead of the sorting prepare; results are identical. E must equal
 * sum n_b (n_b - 1) (checked); images above 2048 nodes fall back to the sorting prepare. */
int pemp_mpn_forward_fully(const pemp_mpn_desc* desc, const pemp_mpn_weights* weights, const float* x,
                           const float* edge_attr, const int64_t* edge_index, const int64_t* node_types,
                           int64_t N, int64_t E, const int64_t* node_off, const int64_t* node_off_host, int B,
                           float* edge_logits, float* node_logits, float* class_logits,
                           void* workspace, size_t workspace_bytes, void* stream);

/* Capacity mode of pemp_mpn_forward_fully: queued right behind pemp_fully_graph_build_cap, before the host has the
 * detection counts (replaces the host read-back at ConstructGraph.py:1174,1178 ahead of the MPN). x / edge_attr /
 * node_types (= joint_det + 2, stride 3) / node_off are that build's capacity buffers (n_cap rows, e_cap edges);
 * n_det is the detection's device count array ([B], det_cap detections per image at most). The batch's N and E
 * are derived on the device; the logits are written compactly for those (edge row r at r * E, node / class row r
 * at r * N), inside arrays sized for the capacities. A batch past any capacity (the capacity build then wrote
 * nothing) runs as an empty forward and writes no logits: the caller, which reads the counts back anyway, re-runs
 * the exact path. PEMP_ERR_UNSUPPORTED for models whose node MLPs are not fused (node embedding, heads) or
 * det_cap above the closed-form image limit (2048). Results equal pemp_mpn_forward_fully's. */
int pemp_mpn_forward_fully_cap(const pemp_mpn_desc* desc, const pemp_mpn_weights* weights, const float* x,
                               const float* edge_attr, const int64_t* node_types, int64_t n_cap, int64_t e_cap,
                               const int32_t* n_det, int det_cap, const int64_t* node_off, int B,
                               float* edge_logits, float* node_logits, float* class_logits,
                               void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * One batch of the inference path in one call (no reference counterpart: a serving entry for a repeated batch
 * shape; construct_graph_start's capacity mode, ConstructGraph.py:1161-1209 + 206-231 + 376-381 and
 * NodeClassificationMPNSimple.py:62-97, takes it): pemp_detect (stages ALL, the counts stored into n_det_host) +
 * pemp_fully_graph_build_cap (PEMP_BUILD_WRITE_COUNTS) + pemp_mpn_forward_fully_cap (PEMP_MPN_COUNTS_IN_OFFSETS;
 * desc == NULL: none), queued on one stream. The arguments that repeat from batch to batch live in a plan that
 * pemp_step_layout completes once; every output lives in ONE caller buffer of plan.bytes bytes at the offsets it
 * computes (off[PEMP_STEP_*], 256-byte aligned):
 *   DET [B, det_cap, 3] i64, DSC [B, det_cap] f32, NDET [B] i32 (pemp_detect's outputs); X [n_cap, C],
 *   JDET [n_cap, 3] i64, JSC [n_cap], BIDX [n_cap] i64, JTAGS [n_cap, F] (F > 0), EIDX [2, e_cap] i64 written as a
 *   contiguous [2, E], EATTR [e_cap, A], NOFF [B + 4] i64 (pemp_fully_graph_build_cap's outputs); LOGITS (desc
 *   only): edge [max(n_rec, 1)][e_cap], then node [n_rec + 1][n_cap] at element elog_n rounded up to 64, then class
 *   [n_rec + 1][n_cap][J] likewise (pemp_mpn_forward_fully_cap's three arrays, rows at r * E / r * N).
 * The caller sets n_det_host[0..B) to -1, calls, and reads the counts as with pemp_detect; a batch past a capacity
 * leaves the build's and the forward's outputs unwritten (the caller re-runs the exact path, as with the capacity
 * calls). Returns PEMP_ERR_UNSUPPORTED when only the forward was refused (pemp_mpn_forward_fully_cap's conditions;
 * the detection and the build are queued). Workspaces: det_workspace >= pemp_detect_workspace_size, mpn_workspace
 * >= pemp_mpn_workspace_size(desc with PEMP_MPN_COUNTS_IN_OFFSETS, n_cap, e_cap); both stream-ordered like the
 * outputs. scoremaps: [B, J, H, W] f32, or a pemp_proj_maps* when projected != 0 (pemp_detect_projected). */
enum {
  PEMP_STEP_DET = 0, PEMP_STEP_DSC, PEMP_STEP_NDET, PEMP_STEP_X, PEMP_STEP_JDET, PEMP_STEP_JSC, PEMP_STEP_BIDX,
  PEMP_STEP_JTAGS, PEMP_STEP_EIDX, PEMP_STEP_EATTR, PEMP_STEP_NOFF, PEMP_STEP_LOGITS, PEMP_STEP_NOUT
};
typedef struct pemp_step_plan {
  /* detection */
  int32_t B, J, H, W, pool_kernel, use_threshold, topk, det_cap, projected;
  float threshold;
  void* det_workspace;
  size_t det_workspace_bytes;
  /* capacity graph build */
  int32_t C, F, A, mode;        /* F = 0: no tagmaps; A: edge_attr columns of mode (PEMP_EF_*) */
  float norm_factor;
  int64_t n_cap, e_cap;
  /* forward (desc NULL: none); desc->flags must hold PEMP_MPN_COUNTS_IN_OFFSETS */
  const pemp_mpn_desc* desc;
  const pemp_mpn_weights* weights;
  void* mpn_workspace;
  size_t mpn_workspace_bytes;
  /* pemp_step_layout's results */
  int32_t n_rec;                /* recorded iterations: edge rows max(n_rec, 1), node / class rows n_rec + 1 */
  int64_t elog_n, nlog_off, clog_off;   /* edge / node / class logits: elements from off[PEMP_STEP_LOGITS] (f32) */
  size_t off[PEMP_STEP_NOUT];
  size_t bytes;
} pemp_step_plan;
/* Fills plan->off / bytes / n_rec / elog_n / nlog_off / clog_off from the other fields (host arithmetic, no device
 * call); returns plan->bytes, 0 for an invalid plan (pemp_last_error says why). */
size_t pemp_step_layout(pemp_step_plan* plan);
int pemp_step_fully_cap(const pemp_step_plan* plan, const void* scoremaps, const float* masks, const float* features,
                        const float* tagmaps, void* out, int32_t* n_det_host, void* stream);

/* Counters of pemp_mpn_forward_fully_cap's HIP graphs since the library loaded (no reference counterpart; for
 * tests and servers): out3[0] captures made, out3[1] graph launches (first launch after a capture included),
 * out3[2] captures refused (the forward then ran directly). Graphs are opt-in (PEMP_GRAPHS=1): a repeating argument
 * set is then launched directly the first time, captured the second, replayed from then on; without it, and under
 * PEMP_NO_GRAPHS, PEMP_DEBUG_SYNC or the library profiler, every call runs directly. */
int pemp_mpn_graph_stats(uint64_t* out3);

/* The CU-reservation policy of the edge passes and the edge embedding (no reference counterpart; pure host
 * arithmetic, no device call): the number of CUs a forward over E edges spreads its one-workgroup-per-CU launches
 * over on a device of num_cus CUs when reserve_request CUs are asked to stay free for another batch in flight
 * (reserve_request < 0: the library's setting, PEMP_RESERVE_CUS or 64). Graphs below 65,536 edges keep every CU;
 * above, at most a quarter of the device is reserved (rounded down to a multiple of 8). */
int pemp_edge_cus_policy(int num_cus, int64_t E, int reserve_request);

/* sizeof of the ABI structs as this library was built (host only; bindings check their mirrors against it):
 * which = 0 pemp_mpn_weights, 1 pemp_mpn_desc, 2 pemp_mlp, 3 pemp_proj_maps, 4 pemp_step_plan; 0 for any other
 * value. */
size_t pemp_abi_struct_size(int which);

/* pemp_mpn_forward for an edge_index sorted by (src, dst) without duplicates and symmetric (every s -> d has
 * its d -> s: PyG to_undirected's coalesced output, as knn_mpn_graph / feature_knn_mpn_graph / score_based_graph
 * return it, ConstructGraph.py:363-422): the type-major edge order is read off the rows of the list (segment
 * (t, d) = the type-t entries of row d) instead of the sorting prepare's scatter + segment sort; results are
 * identical. N >= 2^24 falls back to the sorting prepare. A list that breaks the contract is reported by
 * pemp_mpn_status (its logits are then undefined, every index stays in range). The caller's knowledge that a
 * list meets the contract is a hint the library does not verify on this call (the Python mirror tags
 * construct_graph's output and drops the tag on a version-counter change; call pemp_mpn_status to check). */
int pemp_mpn_forward_sym(const pemp_mpn_desc* desc, const pemp_mpn_weights* weights, const float* x,
                         const float* edge_attr, const int64_t* edge_index, const int64_t* node_types,
                         int64_t N, int64_t E, float* edge_logits, float* node_logits, float* class_logits,
                         void* workspace, size_t workspace_bytes, void* stream);

/* pemp_mpn_forward for the knn graph of pemp_knn_graph_build / pemp_feature_knn_graph_build's fast path (every
 * image <= 512 nodes), handed over as the bit rows that build emitted the edges from (pemp_knn_rows_layout):
 * knn_rows [N][8] uint64 (bit j of word w of row n: the edge n -> node 64 w + j of n's image), knn_rowstart [N]
 * int32 (the row's first edge inside its image) and ecount [B] int64 (edges per image), all device, from the
 * same build as edge_index. The edge order then comes from popcounts of the rows in one launch instead of the
 * symmetric prepare's three; results are identical to pemp_mpn_forward_sym's. B <= 64, N <= 4096 and
 * node_off_host[B] == N (checked); rows that do not belong to edge_index break the contract (reported by
 * pemp_mpn_status through the edge total, logits undefined, every index in range). */
int pemp_mpn_forward_knn(const pemp_mpn_desc* desc, const pemp_mpn_weights* weights, const float* x,
                         const float* edge_attr, const int64_t* edge_index, const int64_t* node_types,
                         int64_t N, int64_t E, const void* knn_rows, const int32_t* knn_rowstart,
                         const int64_t* node_off, const int64_t* node_off_host, const int64_t* ecount, int B,
                         float* edge_logits, float* node_logits, float* class_logits,
                         void* workspace, size_t workspace_bytes, void* stream);

/* The edge-ordering part of pemp_mpn_forward (type-major counting sort of edge_index by (source type,
 * target)), callable ahead of it: it needs no weights, so a caller can queue it as soon as the graph
 * exists and then call pemp_mpn_forward with desc->flags |= PEMP_MPN_PREPARED on the same workspace
 * and stream. */
int pemp_mpn_prepare(const pemp_mpn_desc* desc, const int64_t* edge_index, const int64_t* node_types, int64_t N,
                     int64_t E, void* workspace, size_t workspace_bytes, void* stream);

/* The node embedding / node head / class head weights in the node kernels' LDS layout, built once
 * per weight set (stream-ordered) instead of once per forward: image of
 * pemp_mpn_node_image_floats(weights) floats, then weights->node_img = image. */
/* The edge passes' weight image (per type: the pass's 64x64 blocks in the kernels' LDS row layout, bias and
 * attention rows, the published edge head), built once per weight set and precision for `desc`
 * (precision, aggregation, num_types) into a caller buffer of pemp_mpn_edge_image_floats() floats;
 * pass it as pemp_mpn_weights.edge_img. The edge embedding's LDS image (its layers, Q0's layer and W1_e_cur, in the
 * embedding kernel's layout) follows the passes' image in the same buffer, so the embedding stages its weights
 * with one LDS-DMA round. No reference counterpart (replaces per-pass weight staging). */
size_t pemp_mpn_edge_image_floats(const pemp_mpn_desc* desc, const pemp_mpn_weights* w);
int pemp_mpn_edge_image(const pemp_mpn_desc* desc, const pemp_mpn_weights* w, float* image, size_t floats,
                        void* stream);
size_t pemp_mpn_node_image_floats(const pemp_mpn_weights* weights);
int pemp_mpn_node_image(const pemp_mpn_weights* weights, float* image, size_t floats, void* stream);

/* Synchronises `stream` and reports invalid edge_index / node_types seen by the last
 * pemp_mpn_forward on this workspace (those edges were skipped). Optional validation step. */
int pemp_mpn_status(const pemp_mpn_desc* desc, int64_t N, int64_t E, const void* workspace, void* stream);

/* Opt-in profiler: while enabled, hipEvents are recorded on the launch stream around every kernel
 * whose label contains `filter` ("*" = all, NULL or "" = off). pemp_prof_report synchronises those
 * events and writes "label count total_ms" lines into buf (returns the full length), then resets.
 * Labels: detect_nms, detect_top, detect_emit, pack_nodes, fully_graph, edge_features, knn_adj, knn_emit, score_graph,
 * mpn_prepare, node_embed, edge_embed, node_table, edge_step, edge_step_head, node_update, heads.
 * "label@R": launch sites that are idempotent (the edge passes) issue their launch R times between
 * one event pair, so the per-launch average excludes the event-record overhead (count += R). */
int pemp_prof_enable(const char* filter);
int pemp_prof_report(char* buf, size_t len);

#ifdef __cplusplus
}
#endif
#endif /* PEMP_H_ */
