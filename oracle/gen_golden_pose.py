"""Golden vectors for pose grouping, made by running the REFERENCE's own functions.

TEST INFRASTRUCTURE, run in the build container only (needs /root/reference):
    python oracle/gen_golden_pose.py        -> tests/golden/pose_*.npz

Executed from where they lie (ast-extracted, so the files' cv2 / matplotlib / tensorboard imports are
skipped): ``Utils.py`` ``pred_to_person`` (:499-514), ``graph_cluster_to_persons`` (:672-743),
``to_numpy`` (:36-40); ``correlation_clustering_utils.py`` ``cluster_graph`` (:21-64),
``extract_edge_matrix`` (:99-136), ``update_graph_with_edge_matrix`` (:138-151),
``cluster_andres_graph`` (:187-245). The ``pred_to_ann`` prefix (``Utils.py:1447-1453``: the
``score_map_scores`` check, ``subgraph`` on ``joint_scores > th``, the empty-graph and no-person
``None`` returns) is two lines and is restated here.
Stubs for absent third-party code: PyG ``to_dense_adj`` / ``dense_to_sparse`` / ``subgraph`` /
``Data``, and ``andres_graph_wrapper.Graph`` / ``cluster_GAEC`` = ``oracle.pose.gaec`` (the andres
library is not vendored: GAEC itself is parity unpinned). numpy>=1.24 dropped the ``np.int`` /
``np.float`` aliases the reference uses; the extracted functions see a numpy namespace with them
restored.
"""
import ast
import os
import sys
import types

import numpy as np
import torch
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import connected_components

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pose as opose  # noqa: E402
from oracle.ref_shims import REF_SRC, dense_to_sparse, subgraph  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def _np_compat():
    m = types.ModuleType("numpy_compat")
    m.__dict__.update(np.__dict__)
    m.int, m.float, m.bool = int, float, bool
    return m


def _extract(path, names, ns):
    with open(path) as f:
        tree = ast.parse(f.read(), filename=path)
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert {n.name for n in body} == set(names), names
    exec(compile(ast.Module(body=body, type_ignores=[]), path, "exec"), ns)
    return ns


class Graph:
    """PyG Data subset used by the extracted functions (x, edge_index, edge_attr, num_nodes, cpu)."""

    def __init__(self, x=None, edge_index=None, edge_attr=None):
        self.x, self.edge_index, self.edge_attr = x, edge_index, edge_attr

    @property
    def num_nodes(self):
        return self.x.shape[0]

    def cpu(self):
        return self


def to_dense_adj(edge_index, batch=None, edge_attr=None):
    n = int(edge_index.max()) + 1
    adj = torch.zeros(1, n, n, dtype=edge_attr.dtype)
    adj[0].index_put_((edge_index[0], edge_index[1]), edge_attr, accumulate=True)
    return adj


class AndresGraph:
    def __init__(self, edges, weights, n):
        self.edges, self.weights, self.n = edges, weights, n


def cluster_GAEC(g):
    return opose.gaec(g.n, list(zip(g.edges[0].tolist(), g.edges[1].tolist())), g.weights.astype(np.float64))


def load_reference_pose():
    npc = _np_compat()
    andres = types.SimpleNamespace(Graph=AndresGraph, cluster_GAEC=cluster_GAEC)
    ns_cc = {"np": npc, "torch": torch, "to_dense_adj": to_dense_adj, "andres_graph_wrapper": andres,
             "csr_matrix": csr_matrix, "connected_components": connected_components}
    _extract(os.path.join(REF_SRC, "Utils", "correlation_clustering", "correlation_clustering_utils.py"),
             ["cluster_graph", "extract_edge_matrix", "update_graph_with_edge_matrix", "cluster_andres_graph"], ns_cc)
    ns_u = {"np": npc, "torch": torch, "Graph": Graph, "cluster_graph": ns_cc["cluster_graph"],
            "dense_to_sparse": dense_to_sparse}
    _extract(os.path.join(REF_SRC, "Utils", "Utils.py"), ["pred_to_person", "graph_cluster_to_persons", "to_numpy",
                                                         "greedy_person_construction"], ns_u)
    return ns_u


def ref_pred_to_ann_persons(ref, joint_det, joint_scores, edge_index, pred, th, class_pred, cc_method, J,
                            score_map_scores):
    """Utils.py:1447-1459 restated around the reference's own pred_to_person (torch inputs, as valid.py
    passes them)."""
    T = torch.from_numpy
    joint_det, joint_scores, edge_index, pred = T(joint_det), T(joint_scores), T(edge_index), T(pred)
    class_pred = T(class_pred) if class_pred is not None else None
    if (score_map_scores > 0.1).sum() < 1:
        return None, None
    ei, p, = subgraph(joint_scores > th, edge_index, pred)[:2]
    if ei.shape[1] == 0:
        return None, None
    persons, _, labels = ref["pred_to_person"](joint_det, joint_scores, ei, p, class_pred, cc_method, num_joints=J)
    if len(persons.shape) == 1:
        return None, labels
    return persons, labels


# ----------------------------------------------------------------------------------------
# Synthetic MPN outputs: planted persons, probabilities from a noisy same-person score
# ----------------------------------------------------------------------------------------
def make_case(seed, J, persons, clutter, graph="fully", quant=0, lower_zero=False, class_probs=True):
    rng = np.random.default_rng(seed)
    rows, owner = [], []
    for p in range(persons):
        cx, cy = rng.integers(40, 600, size=2)
        for t in rng.choice(J, size=rng.integers(J // 2, J + 1), replace=False):
            rows.append((cx + rng.integers(-30, 31), cy + rng.integers(-30, 31), t))
            owner.append(p)
    for _ in range(clutter):
        rows.append((rng.integers(0, 640), rng.integers(0, 640), rng.integers(0, J)))
        owner.append(-1 - _)
    order = np.lexsort((np.array([r[0] for r in rows]), np.array([r[1] for r in rows]),
                        np.array([r[2] for r in rows])))
    det = np.array(rows, dtype=np.int64)[order]
    owner = np.array(owner)[order]
    n = len(det)
    src, dst = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    m = src != dst
    if graph == "sparse":
        keep_u = rng.random((n, n)) < 0.35
        keep_u = np.triu(keep_u, 1)
        m &= keep_u | keep_u.T
    ei = np.stack([src[m], dst[m]]).astype(np.int64)
    same = owner[ei[0]] == owner[ei[1]]
    logit = np.where(same, 2.0, -2.5) + rng.normal(0, 1.6, size=ei.shape[1])
    pred = (1.0 / (1.0 + np.exp(-logit))).astype(np.float32)
    if quant:
        pred = (np.round(pred * quant) / quant).astype(np.float32)
    if lower_zero:
        pred[ei[0] > ei[1]] = 0
    scores = rng.random(n).astype(np.float32)
    cls = None
    if class_probs:
        lg = rng.normal(0, 1, size=(n, J)).astype(np.float32)
        lg[np.arange(n), det[:, 2]] += 2.0
        cls = torch.softmax(torch.from_numpy(lg), dim=1).numpy()
    return det, scores, ei, pred, cls


CASES = {
    "pose_gaec_j17": dict(seed=1, J=17, persons=4, clutter=6),
    "pose_gaec_noclass": dict(seed=2, J=17, persons=3, clutter=3, class_probs=False),
    "pose_gaec_ties": dict(seed=3, J=17, persons=4, clutter=5, quant=8),
    "pose_gaec_lowerzero": dict(seed=4, J=17, persons=3, clutter=4, lower_zero=True),
    "pose_gaec_sparse_j14": dict(seed=5, J=14, persons=5, clutter=4, graph="sparse"),
    "pose_threshold": dict(seed=6, J=17, persons=3, clutter=4, method="threshold"),
    "pose_gaec_many": dict(seed=7, J=17, persons=9, clutter=12),
}
THRESHOLDS = {"pose_gaec_noclass": 0.5, "pose_gaec_many": 0.2}


def make_refine_case(seed, J, H, W, F, P, quant=0):
    """Scoremaps with person peaks over noise, tag maps that are piecewise per person plus noise, and
    keypoints [P, J, 3] with some joints detected (integer x, y inside the map, score > 0)."""
    rng = np.random.default_rng(seed)
    s = (rng.random((J, H, W)) * 0.2).astype(np.float32)
    tag = rng.normal(0, 0.3, size=(J, H, W, F)).astype(np.float32)
    kp = np.zeros((P, J, 3))
    for p in range(P):
        cx, cy = rng.integers(8, W - 8), rng.integers(8, H - 8)
        tv = rng.normal(p * 1.7, 0.2, size=F)
        nd = rng.integers(2, J + 1)
        for i in rng.choice(J, size=nd, replace=False):
            x, y = int(np.clip(cx + rng.integers(-6, 7), 0, W - 1)), int(np.clip(cy + rng.integers(-6, 7), 0, H - 1))
            s[i, y, x] = np.float32(0.5 + 0.5 * rng.random())
            tag[i, max(0, y - 3):y + 4, max(0, x - 3):x + 4] = (tv + rng.normal(0, 0.05, size=F)).astype(np.float32)
            kp[p, i] = (x, y, 0.2 + 0.8 * rng.random())
        for i in range(J):  # undetected joints: a peak somewhere in the person's tag region
            if kp[p, i, 2] == 0:
                x, y = int(np.clip(cx + rng.integers(-8, 9), 0, W - 1)), int(np.clip(cy + rng.integers(-8, 9), 0, H - 1))
                s[i, y, x] = np.float32(0.3 + 0.5 * rng.random())
                tag[i, max(0, y - 2):y + 3, max(0, x - 2):x + 3] = tv.astype(np.float32)
    if quant:
        s = (np.round(s * quant) / quant).astype(np.float32)
    return s, tag, kp


REFINE_CASES = {
    "pose_refine_f1": dict(seed=11, J=17, H=96, W=112, F=1, P=5),
    "pose_refine_f2": dict(seed=12, J=17, H=80, W=80, F=2, P=9),
    "pose_refine_ties_j14": dict(seed=13, J=14, H=64, W=72, F=1, P=12, quant=16),
}


def main_refine():
    npc = _np_compat()
    ns = _extract(os.path.join(REF_SRC, "Utils", "Utils.py"), ["refine", "adjust"], {"np": npc})
    for name, spec in REFINE_CASES.items():
        s, tag, kp = make_refine_case(**spec)
        tg = tag[..., 0] if spec["F"] == 1 and spec["seed"] % 2 else tag   # also the 3-D tag form
        filled = opose.fill_mean(kp.copy())
        refined = ns["refine"](s, tg, filled.copy())
        adjusted = ns["adjust"](refined.copy(), s)
        assert np.array_equal(refined, opose.refine(s, tg, filled.copy())), name
        assert np.array_equal(adjusted, opose.adjust(refined.copy(), s)), name
        np.savez_compressed(os.path.join(OUT, name + ".npz"), scoremaps=s, tag=tg, keypoints=kp, filled=filled,
                            refined=refined, adjusted=adjusted)
        print(f"{name}: P={len(kp)} added={(refined[:, :, 2] == 0.001).sum()}")


def main_greedy(ref):
    """greedy_ fixtures: the pred_to_ann prefix with cc_method "greedy" (Utils.py:505-507, 517-626)."""
    for name, spec in (("greedy_j17", dict(seed=21, J=17, persons=4, clutter=6)),
                       ("greedy_noclass", dict(seed=22, J=17, persons=3, clutter=3, class_probs=False)),
                       ("greedy_sparse_j14", dict(seed=23, J=14, persons=5, clutter=4, graph="sparse")),
                       ("greedy_many", dict(seed=24, J=17, persons=9, clutter=12))):
        J = spec["J"]
        det, scores, ei, pred, cls = make_case(**spec)
        th = 0.2
        persons, taken = ref_pred_to_ann_persons(ref, det, scores, ei, pred, th, cls, "greedy", J, scores)
        ei_s, p_s = subgraph(torch.from_numpy(scores > th), torch.from_numpy(ei), torch.from_numpy(pred))[:2]
        mine, mine_taken = opose.greedy_person_construction(det, scores, p_s.numpy(), cls, ei_s.numpy(), J)
        assert (persons is None) == (mine.ndim == 1), name
        if persons is not None:
            assert np.array_equal(persons, mine), name
        assert np.array_equal(np.asarray(taken), mine_taken), name
        np.savez_compressed(os.path.join(OUT, name + ".npz"), joint_det=det, joint_scores=scores, edge_index=ei,
                            pred=pred, th=np.float32(th), num_joints=np.int64(J), has_class=np.bool_(cls is not None),
                            class_probs=cls if cls is not None else np.zeros((0, J), np.float32),
                            none=np.bool_(persons is None),
                            persons=persons if persons is not None else np.zeros((0, J, 3)), taken=np.asarray(taken))
        print(f"{name}: N={len(det)} persons={None if persons is None else len(persons)}")


def main():
    main_refine()
    ref = load_reference_pose()
    for name, spec in CASES.items():
        spec = dict(spec)
        method = spec.pop("method", "GAEC")
        J = spec["J"]
        det, scores, ei, pred, cls = make_case(**spec)
        th = THRESHOLDS.get(name, 0.1)
        persons, labels = ref_pred_to_ann_persons(ref, det, scores, ei, pred, th, cls, method, J, scores)
        # the oracle restatement must agree with the reference's own functions
        mine = opose.pred_to_ann_persons(det, scores, ei, pred, th, cls, method, J, scores)
        assert (persons is None) == (mine is None), name
        if persons is not None:
            assert persons.shape == mine.shape and np.array_equal(persons, mine), name
        # direct graph_cluster_to_persons with single-joint persons and pose scores
        pose_sc = (scores * np.float32(0.5)).astype(np.float32)
        ei_s, p_s = subgraph(scores > th, ei, pred)[:2]
        sol = opose.cluster_gaec(len(det), ei_s, p_s) if ei_s.shape[1] else np.eye(len(det), dtype=np.int64)
        conn = np.stack(np.nonzero(sol))
        T = torch.from_numpy
        single, mutant, single_labels = ref["graph_cluster_to_persons"](
            T(det), T(scores), T(conn), T(cls) if cls is not None else None, J, T(pose_sc), True)
        out = dict(joint_det=det, joint_scores=scores, edge_index=ei, pred=pred, th=np.float32(th),
                   num_joints=np.int64(J), method=np.array(method), has_class=np.bool_(cls is not None),
                   class_probs=cls if cls is not None else np.zeros((0, J), np.float32),
                   none=np.bool_(persons is None),
                   persons=persons if persons is not None else np.zeros((0, J, 3)),
                   labels=labels if labels is not None else np.zeros(0, np.int64),
                   single_persons=single if single.ndim == 3 else np.zeros((0, J, 3)),
                   single_labels=single_labels, single_mutant=np.bool_(mutant), pose_scores=pose_sc)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
        print(f"{name}: N={len(det)} E={ei.shape[1]} persons={None if persons is None else len(persons)}")
    main_greedy(ref)


if __name__ == "__main__":
    main()
