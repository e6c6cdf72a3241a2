"""CPU restatement of the keypoint-graph hot path (the parity ORACLE and the timed CPU baseline).

TEST INFRASTRUCTURE. Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / the CPU baseline. The
product package never imports it; the product path fails loudly without its HIP library.

Restates, op for op on CPU torch fp32, the reference's inference path:
  * detection        — ``src/Utils/Utils.py:15-20`` (NMS), ``src/graph_constructor/ConstructGraph.py:1161-1209``
  * graph + features — ``ConstructGraph.py:46-68,100-103,206-249,251-381``
  * MPN forward      — ``src/Models/MessagePassingNetwork/NodeClassificationMPNSimple.py:23-97``,
                       ``layers.py:8-86,157-274``, ``utils.py:6-19``
Pinned against the reference itself by ``tests/golden/*.npz`` (made by ``oracle/gen_golden.py``,
which runs the reference's own files under ``oracle/ref_shims.py``).

Defined where the reference is unpinned:
  * top-k ties: lower flat index wins (the CUDA radix-select order the reference ran on);
  * knn ties:   (squared integer distance, node index) — torch_cluster's order is unspecified;
  * feature_knn: fp32 fma-chain distance (torch_cluster's CUDA kernel as nvcc compiles it), then index;
  * score_based root ties: (score descending, node index) — torch.topk's tie order is unspecified.
"""
import math

import numpy as np

import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------------------
# Detection (Utils.py:15-20, ConstructGraph.py:1161-1209)
# ----------------------------------------------------------------------------------------


def nms_maxima(scoremap: torch.Tensor, pool_kernel: int) -> torch.Tensor:
    """Utils.py:15-20 — 1.0 where MaxPool2d(k,1,k//2) (implicit -inf padding) equals the input."""
    assert pool_kernel % 2 == 1
    pooled = F.max_pool2d(scoremap[None], pool_kernel, 1, pool_kernel // 2)[0]
    return torch.eq(pooled, scoremap).float()


def _topk_lowest_index(values: torch.Tensor, k: int):
    """Row-wise top-k, ties broken towards the lower index (stable descending sort)."""
    s, idx = torch.sort(values, dim=1, descending=True, stable=True)
    return s[:, :k], idx[:, :k]


def cat_unique(t1: torch.Tensor, t2: torch.Tensor) -> torch.Tensor:
    """ConstructGraph.py:1199-1209 — append rows of t2 not present in t1, order preserved."""
    if t1.shape[0] == 0 or t2.shape[0] == 0:
        return torch.cat([t1, t2], 0)
    same = (t1[:, None, :] == t2[None, :, :]).all(-1).any(0)
    return torch.cat([t1, t2[~same]], 0)


def joint_det_from_scoremap(scoremap, num_joints, threshold=0.007, pool_kernel=None, mask=None, hybrid_k=5):
    """ConstructGraph.py:1161-1196. Returns det [N,3] int64 (x, y, type) and scores [N] f32."""
    joint_map = nms_maxima(scoremap, pool_kernel)
    if mask is not None:
        joint_map = joint_map * mask[None]
    sm = scoremap * joint_map
    J, H, W = sm.shape
    flat = sm.reshape(J, -1)
    if threshold is not None:
        k = min(hybrid_k, flat.shape[1])
        vals, idx = _topk_lowest_index(flat, k)
        container = torch.zeros_like(flat)
        container.scatter_(1, idx, vals)
        t, pos = container.nonzero(as_tuple=True)
        top = torch.stack([pos % W, pos // W, t], 1)
        # where(s < thr, 0, s).nonzero(): kept iff not (s < thr) and s != 0 (NaN counts as kept)
        keep = ~(sm < threshold) & (sm != 0)
        t2, y2, x2 = keep.nonzero(as_tuple=True)
        thr = torch.stack([x2, y2, t2], 1)
        det = cat_unique(top, thr)
        scores = sm[det[:, 2], det[:, 1], det[:, 0]]
    else:
        k = 20
        vals, idx = _topk_lowest_index(flat, k)
        container = torch.zeros_like(flat)
        container.scatter_(1, idx, vals + 1e-10)
        t, pos = container.nonzero(as_tuple=True)
        scores = container[t, pos]
        assert t.shape[0] == k * num_joints
        det = torch.stack([pos % W, pos // W, t], 1)
    return det.long(), scores


# ----------------------------------------------------------------------------------------
# Graphs (ConstructGraph.py:363-381) and edge features (:289-359)
# ----------------------------------------------------------------------------------------


def fully_edge_index(n: int) -> torch.Tensor:
    """dense_to_sparse(ones) -> to_undirected -> remove_self_loops: all i!=j, sorted by (src,dst)."""
    src = torch.arange(n).repeat_interleave(n)
    dst = torch.arange(n).repeat(n)
    m = src != dst
    return torch.stack([src[m], dst[m]], 0)


def knn_edge_index(det: torch.Tensor, k: int = 50) -> torch.Tensor:
    """knn_graph(xy, k) (k+1 queried, self removed) -> to_undirected -> remove_self_loops."""
    n = det.shape[0]
    if n == 0:
        return torch.zeros(2, 0, dtype=torch.long)
    xy = det[:, :2]
    d2 = ((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1)            # exact integers
    order = torch.argsort(d2 * n + torch.arange(n)[None, :], dim=1)[:, :k + 1]
    adj = torch.zeros(n, n, dtype=torch.bool)
    adj.scatter_(1, order, True)                                      # adj[i, j]: j among i's nearest
    adj = adj | adj.t()
    adj.fill_diagonal_(False)
    src, dst = adj.nonzero(as_tuple=True)
    return torch.stack([src, dst], 0)


def feature_knn_edge_index(x: torch.Tensor, k: int = 50) -> torch.Tensor:
    """feature_knn_mpn_graph (ConstructGraph.py:370-374): knn_graph(x, k) over the node features
    (k+1 queried, self removed) -> to_undirected -> remove_self_loops. The distance is torch_cluster
    1.5.4's CUDA one (knn_cuda.cu: tmp += (x_j - x_i) * (x_j - x_i) over the channels in order, fp32,
    one fma per channel under nvcc's default contraction); each fma is evaluated as the exact f64
    t*t + acc rounded to fp32 (t*t of an fp32 t is exact in f64; the f64 sum's own rounding can
    double-round only on an fp32 midpoint). Ties: (distance, node index); NaN ranks last."""
    n = x.shape[0]
    if n == 0:
        return torch.zeros(2, 0, dtype=torch.long)
    xs = x.to(torch.float32).numpy()
    acc = np.zeros((n, n), np.float32)
    for c in range(xs.shape[1]):
        t = (xs[None, :, c] - xs[:, None, c]).astype(np.float64)     # [i, j] = x_j - x_i, fp32-rounded
        acc = (acc.astype(np.float64) + t * t).astype(np.float32)
    key = torch.from_numpy(acc.view(np.int32).astype(np.int64))
    key[torch.from_numpy(np.isnan(acc))] = 2 ** 32 - 1
    order = torch.argsort(key * n + torch.arange(n)[None, :], dim=1)[:, :k + 1]
    adj = torch.zeros(n, n, dtype=torch.bool)
    adj.scatter_(1, order, True)
    adj = adj | adj.t()
    adj.fill_diagonal_(False)
    src, dst = adj.nonzero(as_tuple=True)
    return torch.stack([src, dst], 0)


def score_based_edge_index(scores: torch.Tensor, k: int = 75) -> torch.Tensor:
    """score_based_graph (ConstructGraph.py:405-422): the k best-scoring nodes are roots; rows of
    roots in a dense adjacency -> to_undirected -> remove_self_loops. Edge (a, b), a != b, exists
    iff a or b is a root; sorted by (src, dst). Roots at tied scores: lower node index first (the
    reference's torch.topk leaves the tie order unspecified)."""
    n = scores.shape[0]
    if n < k:   # torch.topk raises for k > n (ConstructGraph.py:414)
        raise RuntimeError(f"score_based graph: selected index k={k} out of range for {n} detections")
    order = sorted(range(n), key=lambda i: (-float(scores[i]), i))
    root = torch.zeros(n, dtype=torch.bool)
    root[order[:k]] = True
    adj = root[:, None] | root[None, :]
    adj.fill_diagonal_(False)
    src, dst = adj.nonzero(as_tuple=True)
    return torch.stack([src, dst], 0)


def edge_features(det: torch.Tensor, edge_index: torch.Tensor, num_joints: int, norm_factor,
                  features_to_use, joint_tags=None, joint_scores=None) -> torch.Tensor:
    """ConstructGraph.py:305-359. joint_tags is the reference's ``tag_maps[type, y, x]`` of the
    squeezed tag maps: [N] for one tag dim, [N, F] otherwise."""
    jx, jy, jt = det[:, 0], det[:, 1], det[:, 2]
    s, d = edge_index[0], edge_index[1]
    E = edge_index.shape[1]
    onehot = torch.zeros(E, num_joints, dtype=torch.long)
    ar = torch.arange(E)
    onehot[ar, jt[s]] = 1
    onehot[ar, jt[d]] = 1
    dy = (jy[d] - jy[s]).float() / norm_factor
    dx = (jx[d] - jx[s]).float() / norm_factor
    mode = set(features_to_use)
    if mode == {"position", "connection_type"}:
        return torch.cat([dx[:, None], dy[:, None], onehot.float()], 1)
    if mode == {"connection_type"}:
        return onehot.float()
    if mode == {"nothing"}:
        return torch.zeros(E, 1)
    if mode == {"position"}:
        return torch.cat([dx[:, None], dy[:, None]], 1)
    if mode == {"position", "angle", "connection_type"}:
        ax, ay = (jx[s] - jx[d]).float(), (jy[s] - jy[d]).float()
        theta = torch.abs(torch.acos(ax * torch.rsqrt(ax ** 2 + ay ** 2)))
        theta[torch.isnan(theta)] = 0.0
        return torch.cat([dx[:, None], dy[:, None], theta[:, None], onehot.float()], 1)
    if mode == {"ae"}:                                                      # :337-339
        return torch.unsqueeze(joint_tags[d] - joint_tags[s], 1).norm(p=None, dim=1, keepdim=True)
    if mode == {"ae_normed"}:                                               # :340-343
        return ((joint_tags[d] - joint_tags[s]).norm(p=None, dim=1, keepdim=True).round() * 100
                - joint_scores[s, None])
    jt2 = joint_tags[:, None] if joint_tags is not None and joint_tags.dim() == 1 else joint_tags
    if mode == {"ae_tracking_1"}:                                           # :344-351
        t_a = 1.8425
        dist = (jt2[d] - jt2[s]).norm(p=None, dim=1, keepdim=True)
        return torch.div(t_a - dist, t_a)
    if mode == {"position", "connection_type", "ae_normed"}:                # :352-357
        dist = (jt2[d] - jt2[s]).norm(p=None, dim=1, keepdim=True)
        return torch.cat([dx[:, None], dy[:, None], onehot.float(), dist], 1)
    raise NotImplementedError(f"EDGE_FEATURES_TO_USE={features_to_use}")


def construct_graph(scoremaps, features, tagmaps, masks, gc, num_joints):
    """ConstructGraph.py:46-249, inference subset (joints_gt None). Returns the 15-tuple."""
    B, J, H, W = scoremaps.shape
    thr = gc.DETECT_THRESHOLD if gc.DETECT_THRESHOLD <= 1.5 else None
    norm = max(W, H) if gc.NORM_NODE_DISTANCE else 1
    xs, eas, eis, dets, scs, bis, tgs = [], [], [], [], [], [], []
    off = 0
    for b in range(B):
        det, sc = joint_det_from_scoremap(scoremaps[b], num_joints, threshold=thr,
                                          pool_kernel=gc.POOL_KERNEL_SIZE,
                                          mask=masks[b] if gc.MASK_CROWDS else None, hybrid_k=gc.HYBRID_K)
        x = features[b][:, det[:, 1], det[:, 0]].T
        if gc.GRAPH_TYPE == "fully":
            ei = fully_edge_index(det.shape[0])
        elif gc.GRAPH_TYPE == "knn":
            ei = knn_edge_index(det)
        elif gc.GRAPH_TYPE == "feature_knn":
            ei = feature_knn_edge_index(x)
        elif gc.GRAPH_TYPE == "score_based":
            ei = score_based_edge_index(sc, 75)
        else:
            raise NotImplementedError(gc.GRAPH_TYPE)
        tg = tagmaps[b, det[:, 2], det[:, 1], det[:, 0]]
        nf = math.prod(tg.shape[1:])                        # tag dims per node (1 for [B, J, H, W] maps)
        jt = tg.reshape(tg.shape[0], nf)
        jt = jt[:, 0] if nf == 1 else jt                    # tagmaps[batch].squeeze() (ConstructGraph.py:100)
        ea = edge_features(det, ei, num_joints, norm, gc.EDGE_FEATURES_TO_USE, jt, sc)
        xs.append(x); eas.append(ea); eis.append(ei + off); dets.append(det); scs.append(sc)
        bis.append(torch.full((det.shape[0],), b, dtype=torch.long)); tgs.append(tg)
        off += det.shape[0]
    return (torch.cat(xs, 0), torch.cat(eas, 0), torch.cat(eis, 1), None, None, None, None,
            torch.cat(dets, 0), None, None, None, torch.cat(scs, 0), torch.cat(bis, 0), None,
            torch.cat(tgs, 0))


# ----------------------------------------------------------------------------------------
# MPN (NodeClassificationMPNSimple.py, layers.py) on a state_dict
# ----------------------------------------------------------------------------------------


def _mlp(sd, prefix, x, sizes, bn, end_with_relu=False):
    """layers.py:8-29 (_make_mlp) in eval mode: Linear, then ReLU [+BN] between layers."""
    li = 0

    def lin(v):
        nonlocal li
        out = F.linear(v, sd[f"{prefix}.{li}.weight"], sd[f"{prefix}.{li}.bias"])
        li += 1
        return out

    def bnorm(v):
        nonlocal li
        out = F.batch_norm(v, sd[f"{prefix}.{li}.running_mean"], sd[f"{prefix}.{li}.running_var"],
                           sd[f"{prefix}.{li}.weight"], sd[f"{prefix}.{li}.bias"], False, 0.0, 1e-5)
        li += 1
        return out

    n = len(sizes)
    x = lin(x)
    if n != 1:
        x = F.relu(x); li += 1
        if bn:
            x = bnorm(x)
    for i in range(1, n):
        x = lin(x)
        if i != n - 1:
            x = F.relu(x); li += 1
            if bn:
                x = bnorm(x)
    if end_with_relu:
        x = F.relu(x); li += 1
        if bn:
            x = bnorm(x)
    return x


def _segment_softmax(a, index, n):
    """torch_scatter 2.0.4 scatter_softmax: exp(a - max_seg) / (sum_seg + 1e-12)."""
    mx = torch.full((n,), float("-inf"), dtype=a.dtype).scatter_reduce(0, index, a, "amax", include_self=True)
    mx = torch.where(torch.isneginf(mx), torch.zeros_like(mx), mx)
    ex = (a - mx[index]).exp()
    sm = torch.zeros(n, dtype=a.dtype).index_add_(0, index, ex)
    return ex / (sm + 1e-12)[index]


def _scatter(v, index, n, reduce):
    out = torch.zeros(n, v.shape[1], dtype=v.dtype)
    if reduce in ("add", "sum"):
        return out.index_add_(0, index, v)
    if reduce == "mean":
        s = out.index_add_(0, index, v)
        c = torch.zeros(n, dtype=v.dtype).index_add_(0, index, torch.ones(v.shape[0], dtype=v.dtype)).clamp(1)
        return s / c[:, None]
    if reduce == "max":
        m = torch.full((n, v.shape[1]), float("-inf"), dtype=v.dtype).scatter_reduce(
            0, index[:, None].expand_as(v), v, "amax", include_self=True)
        return torch.where(torch.isneginf(m), torch.zeros_like(m), m)
    raise ValueError(reduce)


def _type_map(summary, types):
    """utils.py:6-19 (sum_node_types)."""
    if summary == "not":
        return types
    lut = {"left_right": [0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8],
           "per_body_part": [0, 0, 0, 0, 0, 1, 1, 2, 3, 2, 3, 4, 5, 4, 5, 4, 5]}[summary]
    return torch.tensor(lut, dtype=torch.long)[types]


def mpn_layer(sd, cfg, x, e, edge_index, node_types):
    """TypeAwareMPNLayer.forward (layers.py:207-258) / MPLayer.forward (layers.py:63-86)."""
    p = "mpn_node_cls"
    j, i = edge_index[0], edge_index[1]                   # message flows j (source) -> i (target)
    n = x.shape[0]
    if getattr(cfg, "EDGE_MLP", "agnostic") == "per_type":
        e_new = _type_aware_edge_update(sd, f"{p}.mlp_edge", x[i], x[j], e, node_types[i], node_types[j],
                                        _num_types(cfg))
    else:
        h = F.relu(F.linear(torch.cat([x[i], x[j], e], 1), sd[f"{p}.mlp_edge.0.weight"], sd[f"{p}.mlp_edge.0.bias"]))
        e_new = F.relu(F.linear(h, sd[f"{p}.mlp_edge.2.weight"], sd[f"{p}.mlp_edge.2.bias"]))
    if cfg.AGGR_TYPE == "agnostic":
        m = F.relu(F.linear(torch.cat([x[i], e_new], 1), sd[f"{p}.mlp_node.0.weight"], sd[f"{p}.mlp_node.0.bias"]))
        agg = _scatter(m, i, n, cfg.AGGR)
        if getattr(cfg, "USE_NODE_UPDATE_MLP", False):
            agg = F.relu(F.linear(agg, sd[f"{p}.update_mlp.0.weight"], sd[f"{p}.update_mlp.0.bias"]))
        return agg, e_new
    src_type = node_types[j]
    num_types = _num_types(cfg)
    m = torch.zeros(e_new.shape[0], e_new.shape[1], dtype=e_new.dtype)
    xi_e = torch.cat([x[i], e_new], 1)
    for t in range(17):                                    # layers.py:271 hard-codes 17
        sel = src_type == t
        if sel.any():
            m[sel] = F.relu(F.linear(xi_e[sel], sd[f"{p}.mlp_node.mlp.{t}.0.weight"], sd[f"{p}.mlp_node.mlp.{t}.0.bias"]))
    upd = torch.zeros(n, num_types, m.shape[1], dtype=m.dtype)
    if cfg.AGGR_SUB in ("node_edge_attn", "node_edge_attn_per_type"):    # layers.py:240-251
        a = F.linear(e_new, sd[f"{p}.attn_net.0.weight"], sd[f"{p}.attn_net.0.bias"])
        for t in range(num_types):
            col = 0 if cfg.AGGR_SUB == "node_edge_attn" else t        # attn_index, layers.py:245
            sel = src_type == t
            if sel.any():
                alpha = _segment_softmax(a[sel, col], i[sel], n)
                upd[:, t] = _scatter(m[sel] * alpha[:, None], i[sel], n, "add")
    else:
        for t in range(num_types):
            sel = src_type == t
            if sel.any():
                upd[:, t] = _scatter(m[sel], i[sel], n, cfg.AGGR)
    utype = getattr(cfg, "UPDATE_TYPE", "mlp")
    if utype == "hierarch_mlp":
        x_new = _hierarch_mlp(sd, f"{p}.update_mlp", upd, num_types)
    elif utype == "hierarch_cnn":
        x_new = _hierarch_cnn(sd, f"{p}.update_mlp", upd)
    else:
        x_new = F.relu(F.linear(upd.reshape(n, -1), sd[f"{p}.update_mlp.0.weight"], sd[f"{p}.update_mlp.0.bias"]))
    return x_new, e_new


def _type_aware_edge_update(sd, p, nodes_1, nodes_2, edges, types_1, types_2, num_joints):
    """TypeAwareEdgeUpdate.forward (layers.py:288-303)."""
    rows = nodes_1.shape[0]
    out_dim = sd[f"{p}.edge_layer.bias"].shape[0]
    tmp_1 = torch.zeros(rows, out_dim, dtype=nodes_1.dtype)
    tmp_2 = torch.zeros(rows, out_dim, dtype=nodes_1.dtype)
    for t in range(num_joints):
        sel = types_1 == t
        tmp_1[sel] = F.linear(nodes_1[sel], sd[f"{p}.layer_1.{t}.weight"], sd[f"{p}.layer_1.{t}.bias"])
    for t in range(num_joints):
        sel = types_2 == t
        tmp_2[sel] = F.linear(nodes_2[sel], sd[f"{p}.layer_2.{t}.weight"], sd[f"{p}.layer_2.{t}.bias"])
    ed = F.linear(edges, sd[f"{p}.edge_layer.weight"], sd[f"{p}.edge_layer.bias"])
    cat = F.relu(torch.cat([tmp_1, tmp_2, ed], 1))
    return F.relu(F.linear(cat, sd[f"{p}.out.1.weight"], sd[f"{p}.out.1.bias"]))


def _hierarch_mlp(sd, p, update, num_joints):
    """HierarchUpdateMlp.forward (layers.py:109-128)."""
    n = update.shape[0]
    if num_joints == 17:
        order_1 = [(0, 1, 2, 3, 4), (5, 6), (7, 9), (8, 10), (11, 12), (13, 15), (14, 16)]
    else:
        order_1 = [(0, 1), (2, 3), (4, 6), (5, 7), (8, 9), (10, 12), (11, 13)]
    order_2 = [(0, 1), (1, 2), (1, 3), (1, 4), (4, 5), (4, 6)]
    d2 = update.shape[2] // 2
    out_1 = torch.zeros(n, 7, d2, dtype=update.dtype)
    out_2 = torch.zeros(n, 6, d2, dtype=update.dtype)
    for i, types in enumerate(order_1):
        out_1[:, i] = F.relu(F.linear(update[:, list(types)].reshape(n, -1), sd[f"{p}.first_layer.{i}.weight"],
                                      sd[f"{p}.first_layer.{i}.bias"]))
    for i, types in enumerate(order_2):
        out_2[:, i] = F.relu(F.linear(out_1[:, list(types)].reshape(n, -1), sd[f"{p}.second_layer.{i}.weight"],
                                      sd[f"{p}.second_layer.{i}.bias"]))
    return F.relu(F.linear(out_2.reshape(n, -1), sd[f"{p}.final.weight"], sd[f"{p}.final.bias"]))


def _hierarch_cnn(sd, p, update):
    """HierarchUpdateCnn.forward (layers.py:142-154)."""
    n = update.shape[0]
    update = update.permute(0, 2, 1)
    order_1 = [5, 6, 7, 9, 8, 10, 11, 12, 13, 15, 14, 16]
    order_2 = [0, 1, 0, 2, 0, 3, 3, 4, 3, 5]
    out_1 = F.relu(F.conv1d(update[:, :, order_1], sd[f"{p}.conv_1.weight"], sd[f"{p}.conv_1.bias"], stride=2))
    head = F.relu(F.linear(update[:, :, :4].reshape(n, -1), sd[f"{p}.head_layer.weight"], sd[f"{p}.head_layer.bias"]))
    update = torch.cat([head[:, :, None], out_1], dim=2)
    update = F.relu(F.conv1d(update[:, :, order_2], sd[f"{p}.conv_2.weight"], sd[f"{p}.conv_2.bias"], stride=2))
    return F.relu(F.linear(update.reshape(n, -1), sd[f"{p}.final.weight"], sd[f"{p}.final.bias"]))


def _num_types(cfg):
    return {"per_body_part": 6, "left_right": 9}.get(cfg.NODE_TYPE_SUMMARY, cfg.NUM_JOINTS)


def mpn_forward(sd, cfg, x, edge_attr, edge_index, node_types):
    """NodeClassificationMPNSimple.forward (NodeClassificationMPNSimple.py:62-97)."""
    types = _type_map(cfg.NODE_TYPE_SUMMARY, node_types)
    nf = _mlp(sd, "node_embedding", x, cfg.NODE_EMB.OUTPUT_SIZES, cfg.NODE_EMB.BN, cfg.NODE_EMB.END_WITH_RELU)
    if getattr(cfg, "LATE_FUSION_POS", False):   # LateFusionEdgeMLP.forward (NodeClassificationMPNSimple.py:18-21)
        single = [size // 2 for size in cfg.EDGE_EMB.OUTPUT_SIZES[:-1]]
        pos = _mlp(sd, "edge_embedding.pos_mlp", edge_attr[:, :2], single, cfg.EDGE_EMB.BN, cfg.EDGE_EMB.END_WITH_RELU)
        edg = _mlp(sd, "edge_embedding.edge_mlp", edge_attr[:, 2:], single, cfg.EDGE_EMB.BN, cfg.EDGE_EMB.END_WITH_RELU)
        ef = F.linear(F.relu(torch.cat([pos, edg], 1)), sd["edge_embedding.out.weight"], sd["edge_embedding.out.bias"])
    else:
        ef = _mlp(sd, "edge_embedding", edge_attr, cfg.EDGE_EMB.OUTPUT_SIZES, cfg.EDGE_EMB.BN, cfg.EDGE_EMB.END_WITH_RELU)
    nf0, ef0 = nf, ef
    pe, pn, pc = [], [], []

    def heads(v, ev):
        pn.append(_mlp(sd, "node_classification", v, cfg.NODE_CLASS.OUTPUT_SIZES, cfg.BN).squeeze())
        pc.append(_mlp(sd, "classification", v, cfg.CLASS.OUTPUT_SIZES, cfg.BN))
        if ev is not None:
            pe.append(_mlp(sd, "edge_classification", ev, cfg.EDGE_CLASS.OUTPUT_SIZES, cfg.BN).squeeze())

    aux = getattr(cfg, "AUX_LOSS_STEPS", 0)
    for it in range(cfg.STEPS):
        if cfg.SKIP:
            nf = torch.cat([nf0, nf], 1)
            ef = torch.cat([ef0, ef], 1)
        nf, ef = mpn_layer(sd, cfg, nf, ef, edge_index, types)
        if it >= cfg.STEPS - aux - 1:
            heads(nf, ef)
    for _ in range(getattr(cfg, "NODE_STEPS", 0)):
        raise NotImplementedError("NODE_STEPS > 0")
    pn.append(_mlp(sd, "node_classification", nf, cfg.NODE_CLASS.OUTPUT_SIZES, cfg.BN).squeeze())
    pc.append(_mlp(sd, "classification", nf, cfg.CLASS.OUTPUT_SIZES, cfg.BN))
    return pe, pn, pc, [None]


# ----------------------------------------------------------------------------------------
# Test-time front-end (PoseEstimation.py:329-452, multi_scales_testing.py:144-195)
# ----------------------------------------------------------------------------------------
def _taps(out_size, in_size):
    """torch's area_pixel_compute_source_index (align_corners=False) in fp32: i0, i1, l0, l1 per output."""
    f32 = np.float32
    scale = f32(in_size) / f32(out_size)
    src = (scale * (np.arange(out_size, dtype=f32) + f32(0.5))) - f32(0.5)
    src = np.maximum(src, f32(0))
    i0 = src.astype(np.int64)
    i1 = i0 + (i0 < in_size - 1)
    l1 = np.clip(src - i0.astype(f32), f32(0), f32(1))
    return i0, i1, (f32(1) - l1).astype(f32), l1.astype(f32)


def upsample_bilinear(m, size):
    """interpolate(m, size, bilinear, align_corners=False) on [..., h, w] float32, every product and sum
    rounded in fp32 in the order t0 = a lx0 + b lx1, t1 = c lx0 + d lx1, v = t0 ly0 + t1 ly1 (torch's
    CPU upsample evaluates the same expression, possibly contracting products into FMAs)."""
    m = np.asarray(m, dtype=np.float32)
    H, W = size
    y0, y1, ly0, ly1 = _taps(H, m.shape[-2])
    x0, x1, lx0, lx1 = _taps(W, m.shape[-1])
    r0, r1 = m[..., y0, :], m[..., y1, :]
    t0 = r0[..., x0] * lx0 + r0[..., x1] * lx1
    t1 = r1[..., x0] * lx0 + r1[..., x1] * lx1
    return (t0 * ly0[:, None] + t1 * ly1[:, None]).astype(np.float32)


def project_frontend(outputs, flip_outputs, size, num_joints, flip_index=None, divisor=None, tag_scale=0):
    """The front-end's image-size scoremaps [B, J, H, W] and tags [B, J, H, W, F] (F = 2 with a flipped
    pass) from per-scale network outputs [B, C, h, w]: heatmaps_avg = (up(out) + up(flip(flip_out))
    [:, flip_index]) / 2 per scale, summed in order and divided by `divisor`; tags of scale tag_scale
    (channels J..2J-1), flipped ones re-indexed by flip_index (TAG_PER_JOINT). fp32 numpy."""
    J = num_joints
    fi = np.arange(J) if flip_index is None else np.asarray(flip_index)
    outs = [np.asarray(o, dtype=np.float32) for o in outputs]
    flips = None if flip_outputs is None else [np.asarray(o, dtype=np.float32) for o in flip_outputs]
    acc = None
    for s, o in enumerate(outs):
        h = upsample_bilinear(o[:, :J], size)
        if flips is not None:
            hf = upsample_bilinear(flips[s][:, :J][:, fi][..., ::-1], size)
            h = ((h + hf) / np.float32(2.0)).astype(np.float32)
        acc = h if acc is None else (acc + h).astype(np.float32)
    scoremaps = (acc / np.float32(len(outs) if divisor is None else divisor)).astype(np.float32)
    tags = None
    if outs[tag_scale].shape[1] >= 2 * J:
        tl = [upsample_bilinear(outs[tag_scale][:, J:2 * J], size)[..., None]]
        if flips is not None:
            tl.append(upsample_bilinear(flips[tag_scale][:, J:2 * J][:, fi][..., ::-1], size)[..., None])
        tags = np.concatenate(tl, axis=4)
    return torch.from_numpy(scoremaps), None if tags is None else torch.from_numpy(tags)


def stage_merge(stage0, stage1, num_joints):
    """HigherHRNet's multi-stage merge of one pass at the last stage's resolution
    (PoseEstimation.py:343-364, and :387-412 before the flipped pass's flip; TEST.WITH_HEATMAPS [True, True],
    TEST.WITH_AE [True, False]): up = bilinear stage0 -> stage1's size (align_corners=False, fp32 in the
    projection's order); heatmaps (up[:, :J] + stage1[:, :J]) / 2, tags up[:, J:]. fp32 numpy -> torch."""
    J = num_joints
    s0 = np.asarray(stage0, dtype=np.float32)
    s1 = np.asarray(stage1, dtype=np.float32)
    up = upsample_bilinear(s0, (s1.shape[2], s1.shape[3]))
    heat = ((up[:, :J] + s1[:, :J]) / np.float32(2.0)).astype(np.float32)
    return torch.from_numpy(np.ascontiguousarray(np.concatenate([heat, up[:, J:]], 1)))
