"""CPU restatement of pose grouping — the parity ORACLE for ``pemp_pose_*``.

TEST INFRASTRUCTURE. Only ``tests/`` (and ``oracle/gen_golden_pose.py``) may import this module, as
the checker. The product path (``pemp_amd.pose``) never imports it.

Restates, in numpy / scipy / pure Python:
  * ``pred_to_ann`` prefix        — ``src/Utils/Utils.py:1445-1455`` (node threshold, PyG ``subgraph``)
  * ``pred_to_person``            — ``Utils.py:499-514`` (GAEC and ``threshold`` branches)
  * ``cluster_graph`` GAEC path   — ``src/Utils/correlation_clustering/correlation_clustering_utils.py:21-62``,
    ``extract_edge_matrix`` ``:99-136``, ``update_graph_with_edge_matrix`` ``:138-151``,
    ``cluster_andres_graph`` ``:187-245``
  * ``graph_cluster_to_persons``  — ``Utils.py:672-743``
Third party, not vendored (``andres_graph_wrapper`` is imported at ``correlation_clustering_utils.py:15``
but its native sources are absent): ``andres::graph::multicut::greedyAdditiveEdgeContraction`` is
restated from the published algorithm (``gaec`` below) with libstdc++'s binary-heap push/pop, so that
weight ties resolve exactly like ``std::priority_queue``. The GAEC core is therefore **parity unpinned**
against the original binary; everything around it is pinned by ``tests/golden/pose_*.npz``, made by
running the reference's own functions (``oracle/gen_golden_pose.py``).
"""
import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import connected_components


# ----------------------------------------------------------------------------------------
# libstdc++ heap (bits/stl_heap.h) — std::priority_queue<Edge> with operator< on w
# ----------------------------------------------------------------------------------------
def _push_heap_at(h, hole, top, value):
    parent = (hole - 1) // 2
    while hole > top and h[parent][0] < value[0]:
        h[hole] = h[parent]
        hole = parent
        parent = (hole - 1) // 2
    h[hole] = value


def heap_push(h, value):
    h.append(value)
    _push_heap_at(h, len(h) - 1, 0, value)


def heap_pop(h):
    top = h[0]
    last = h.pop()
    n = len(h)
    if n == 0:
        return top
    # __pop_heap(first, last-1, last-1): value = *result; *result = *first; __adjust_heap(first, 0, n, value)
    hole, second = 0, 0
    while second < (n - 1) // 2:
        second = 2 * (second + 1)
        if h[second][0] < h[second - 1][0]:
            second -= 1
        h[hole] = h[second]
        hole = second
    if (n & 1) == 0 and second == (n - 2) // 2:
        second = 2 * (second + 1)
        h[hole] = h[second - 1]
        hole = second - 1
    _push_heap_at(h, hole, 0, last)
    return top


def gaec(n, edges, weights):
    """andres greedyAdditiveEdgeContraction: edges [(a, b)], weights (double) -> cut labels (1 = cut)."""
    adj = [dict() for _ in range(n)]
    editions = [dict() for _ in range(n)]
    heap = []
    for (a, b), w in zip(edges, weights):
        w = float(w)
        adj[a][b] = adj[a].get(b, 0.0) + w
        adj[b][a] = adj[b].get(a, 0.0) + w
        lo, hi = min(a, b), max(a, b)
        editions[lo][hi] = editions[lo].get(hi, 0) + 1
        heap_push(heap, (w, lo, hi, editions[lo][hi]))
    parent = list(range(n))

    def find(v):
        while parent[v] != v:
            v = parent[v]
        return v

    while heap:
        w, a, b, ed = heap_pop(heap)
        if not adj[a] or b not in adj[a] or ed < editions[a][b]:
            continue
        if w < 0.0:
            break
        keep, merge = a, b
        if len(adj[keep]) < len(adj[merge]):
            keep, merge = merge, keep
        rk, rm = find(keep), find(merge)
        if rk != rm:
            parent[rm] = rk
        for p in sorted(adj[merge]):  # std::map iteration order
            if p == keep:
                continue
            pw = adj[merge][p]
            adj[keep][p] = adj[keep].get(p, 0.0) + pw
            adj[p][keep] = adj[p].get(keep, 0.0) + pw
            lo, hi = min(keep, p), max(keep, p)
            editions[lo][hi] = editions[lo].get(hi, 0) + 1
            heap_push(heap, (adj[keep][p], lo, hi, editions[lo][hi]))
        for p in list(adj[merge]):
            del adj[p][merge]
        adj[merge].clear()
    return np.array([0 if find(a) == find(b) else 1 for a, b in edges], dtype=np.int64)


# ----------------------------------------------------------------------------------------
# Reference path, restated
# ----------------------------------------------------------------------------------------
def subgraph(keep, edge_index, pred):
    """PyG 1.4.3 subgraph(subset=bool mask, relabel_nodes=False)."""
    m = keep[edge_index[0]] & keep[edge_index[1]]
    return edge_index[:, m], pred[m]


def cluster_gaec(num_nodes, edge_index, pred):
    """cluster_graph(graph, 'GAEC', complete=False) -> dense {0,1} matrix (1 = joined)."""
    m = int(edge_index.max()) + 1 if edge_index.shape[1] else 0
    dense = np.zeros((m, m), dtype=np.float32)
    np.add.at(dense, (edge_index[0], edge_index[1]), pred.astype(np.float32))
    if np.tril(dense).sum() == 0:
        dense = dense + dense.T
    else:
        dense = (dense + dense.T) / np.float32(2)
    np.fill_diagonal(dense, 1)
    attr = dense[edge_index[0], edge_index[1]]
    weights = attr - np.float32(0.5)
    up = edge_index[0] < edge_index[1]
    e = edge_index[:, up]
    cut = gaec(num_nodes, list(zip(e[0].tolist(), e[1].tolist())), weights[up].astype(np.float64))
    sol = np.zeros((num_nodes, num_nodes), dtype=np.int64)
    sol[e[0], e[1]] = 1 - cut
    sol += sol.T
    np.fill_diagonal(sol, 1)
    return sol


def graph_cluster_to_persons(joints, joint_scores, joint_connections, class_pred, num_joints,
                             scores_for_poses=None, allow_single_joint_persons=False):
    n = len(joints)
    adj = np.zeros([n, n])
    adj[joint_connections[0], joint_connections[1]] = 1
    n_comp, labels = connected_components(csr_matrix(adj), directed=False, return_labels=True)
    persons, mutant = [], False
    for i in range(n_comp):
        sel = labels == i
        pj = joints[sel].copy()
        ps = joint_scores[sel]
        pp = scores_for_poses[sel] if scores_for_poses is not None else None
        if class_pred is not None:
            pj[:, 2] = np.argmax(class_pred[sel], axis=1)
        if len(pj) > num_joints:
            mutant = True
        if len(pj) > 1:
            kp = np.zeros([num_joints, 3])
            for t in range(num_joints):
                s = pj[:, 2] == t
                if s.sum():
                    idx = np.argmax(ps[s])
                    kp[t] = pj[s][idx]
                    kp[t, 2] = np.max(ps[s])
                    if pp is not None:
                        kp[t, 2] = pp[s][idx]
            if (kp[:, 2] > 0).sum() > 0:
                persons.append(kp)
        elif len(pj) == 1 and allow_single_joint_persons:
            kp = np.zeros([num_joints, 3])
            if ps[0] < 0.1:
                continue
            kp[pj[:, 2], 2] = ps[0]
            kp[:, :2] = pj[0, :2]
            persons.append(kp)
    return np.array(persons), mutant, labels


def pred_to_person(joint_det, joint_scores, edge_index, pred, class_pred, cc_method, num_joints,
                   score_for_poses=None, allow_single_joint_persons=False):
    if cc_method == "GAEC":
        sol = cluster_gaec(len(joint_det), edge_index, pred)
        conn = np.stack(np.nonzero(sol))
    elif cc_method == "threshold":
        conn = edge_index[:, pred > np.float32(0.8)]
    else:
        raise NotImplementedError(cc_method)
    return graph_cluster_to_persons(joint_det, joint_scores, conn, class_pred, num_joints, score_for_poses,
                                    allow_single_joint_persons)


def pred_to_ann_persons(joint_det, joint_scores, edge_index, pred, th, class_pred, cc_method, num_joints,
                        score_map_scores=None):
    """pred_to_ann up to the grouped persons (Utils.py:1445-1459): None where the reference returns None."""
    if score_map_scores is not None and (score_map_scores > 0.1).sum() < 1:
        return None
    ei, p = subgraph(joint_scores > th, edge_index, pred)
    if ei.shape[1] == 0:
        return None
    persons, _, _ = pred_to_person(joint_det, joint_scores, ei, p, class_pred, cc_method, num_joints)
    if len(persons.shape) == 1:
        return None
    return persons


# ----------------------------------------------------------------------------------------
# Finishing: fill_mean (Utils.py:1468-1470), refine (:1026-1104), adjust (:917-936)
# ----------------------------------------------------------------------------------------
def fill_mean(persons):
    for i in range(len(persons)):
        persons[i, persons[i, :, 2] == 0, :2] = persons[i, persons[i, :, 2] != 0, :2].mean(axis=0)
    return persons


def refine(scoremaps, tag, keypoints):
    if len(tag.shape) == 3:
        tag = tag[:, :, :, None]
    tags = []
    for p in range(keypoints.shape[0]):
        pt = []
        for i in range(keypoints.shape[1]):
            if keypoints[p, i, 2] > 0:
                x, y = keypoints[p, i][:2].astype(np.int32)
                pt.append(tag[i, y, x])
        tags.append(np.array(pt))
    for p in range(keypoints.shape[0]):
        prev = np.mean(tags[p], axis=0)
        ans = []
        for i in range(keypoints.shape[1]):
            tmp = scoremaps[i]
            tt = (((tag[i] - prev[None, None, :]) ** 2).sum(axis=2) ** 0.5)
            y, x = np.unravel_index(np.argmax(tmp - np.round(tt)), tmp.shape)
            val = tmp[y, x]
            xx, yy = x, y
            x, y = x + 0.5, y + 0.5
            x += 0.25 if tmp[yy, min(xx + 1, tmp.shape[1] - 1)] > tmp[yy, max(xx - 1, 0)] else -0.25
            y += 0.25 if tmp[min(yy + 1, tmp.shape[0] - 1), xx] > tmp[max(0, yy - 1), xx] else -0.25
            ans.append((x, y, val))
        ans = np.array(ans)
        for i in range(scoremaps.shape[0]):
            if ans[i, 2] > 0 and keypoints[p, i, 2] == 0:
                keypoints[p, i, :2] = ans[i, :2]
                keypoints[p, i, 2] = 0.001
    return keypoints


def adjust(ans, det):
    for pid, person in enumerate(ans):
        for jid, joint in enumerate(person):
            if joint[2] > 0:
                y, x = joint[0], joint[1]
                xx, yy = int(x), int(y)
                tmp = det[jid]
                y += 0.25 if tmp[xx, min(yy + 1, tmp.shape[1] - 1)] > tmp[xx, max(yy - 1, 0)] else -0.25
                x += 0.25 if tmp[min(xx + 1, tmp.shape[0] - 1), yy] > tmp[max(0, xx - 1), yy] else -0.25
                ans[pid, jid, 1] = x + 0.5
                ans[pid, jid, 0] = y + 0.5
    return ans


def greedy_person_construction(joint_det, preds_nodes, preds_edges, preds_classes, edge_index, num_joints):
    """Utils.py:517-626 restated (numpy)."""
    joint_det = joint_det.copy()
    if preds_classes is not None:
        joint_det[:, 2] = preds_classes.argmax(axis=1)
    n = len(joint_det)
    adj = np.zeros((n, n), dtype=np.float64)
    adj[edge_index[0], edge_index[1]] = preds_edges
    adj = (adj.T + adj) / 2.0
    adj[np.diag_indices(n)] = 1.0
    taken = np.zeros_like(preds_nodes, dtype=np.int32) - 1
    for t in range(num_joints):
        tj = joint_det[:, 2] == t
        for i in range(n):
            if not tj[i] or taken[i] != -1:
                continue
            if preds_nodes[i] < 0.5:
                continue
            taken[i] = i
            for j in range(num_joints):
                if j == t:
                    continue
                row = adj[i].copy()
                row[joint_det[:, 2] != j] = 0.0
                score, idx = np.max(row), np.argmax(row)
                if score == 0.0 or idx == i:
                    continue
                if taken[idx] != -1 and adj[taken[idx], idx] > score:
                    continue
                taken[idx] = i
    persons = []
    for c in range(taken.max() + 1):
        sel = taken == c
        pj, ps = joint_det[sel], preds_nodes[sel]
        if len(pj) > 1:
            kp = np.zeros([num_joints, 3])
            for t in range(num_joints):
                s = pj[:, 2] == t
                if s.sum():
                    kp[t] = pj[s][np.argmax(ps[s])]
                    kp[t, 2] = np.max(ps[s])
            if (kp[:, 2] > 0).sum() > 0:
                persons.append(kp)
    return np.array(persons), taken
