"""Load the reference's own hot-path files on CPU torch, for golden-vector generation ONLY.

TEST INFRASTRUCTURE — never imported by the product package. Runs only in the build
container where ``/root/reference`` exists; the GPU box never sees this path.

The reference's hot-path files (``src/graph_constructor/ConstructGraph.py``,
``src/Models/MessagePassingNetwork/{layers,utils,NodeClassificationMPNSimple}.py``) import
third-party packages that are not installed here (torch_geometric 1.4.3, torch_scatter 2.0.4,
torch_cluster 1.5.4, torch_sparse 0.6.1 — pinned in ``requirements.txt:63-66``). This module
restates the *published semantics* of exactly the functions those files call and installs
them as ``sys.modules`` stubs, then loads the reference files by path. Nothing from the
reference is copied; its files are executed from where they lie.

Third-party restatements (call sites in the reference):
  * ``torch_geometric.utils.dense_to_sparse``  (ConstructGraph.py:378)
  * ``torch_geometric.utils.to_undirected``    (ConstructGraph.py:366,379) — PyG 1.4.3 concatenates
    both directions and coalesces via torch_sparse 0.6.1 ``coalesce`` = sorted-unique by (row, col).
  * ``torch_geometric.utils.remove_self_loops`` (ConstructGraph.py:367,380)
  * ``torch_geometric.utils.subgraph``          (ConstructGraph.py:157, training only)
  * ``torch_geometric.nn.knn_graph``            (ConstructGraph.py:365) — torch_cluster 1.5.4 knn with
    k+1 queried and self removed; its tie order is UNPINNED, restated with this build's rule
    (squared distance, then index).
  * ``torch_geometric.nn.MessagePassing``       (layers.py:4) — PyG 1.4.3 propagate: ``*_i`` args
    index ``edge_index[1]`` (target), ``*_j`` args ``edge_index[0]`` (source), aggregate gets
    ``index=edge_index[1]`` and ``dim_size=size[1]``.
  * ``torch_scatter.scatter/scatter_max/scatter_softmax`` (layers.py:5,239,249-250) —
    torch_scatter 2.0.4: empty segments give 0 for sum/mean/max; mean divides by count clamped
    to 1; ``scatter_softmax`` = exp(s - max_seg) / (sum_seg + 1e-12).
"""
import ast
import importlib.util
import inspect
import os
import sys
import types

import torch

REF_ROOT = os.environ.get("PEMP_REFERENCE_ROOT", "/root/reference")
REF_SRC = os.path.join(REF_ROOT, "src")


def reference_available() -> bool:
    return os.path.isfile(os.path.join(REF_SRC, "graph_constructor", "ConstructGraph.py"))


# ----------------------------------------------------------------------------------------
# torch_scatter 2.0.4 restatement
# ----------------------------------------------------------------------------------------
def _broadcast(index, src, dim):
    if dim < 0:
        dim = src.dim() + dim
    if index.dim() == 1:
        for _ in range(0, dim):
            index = index.unsqueeze(0)
    for _ in range(index.dim(), src.dim()):
        index = index.unsqueeze(-1)
    return index.expand_as(src)


def _out_size(src, index, dim, dim_size):
    size = list(src.size())
    if dim < 0:
        dim = src.dim() + dim
    if dim_size is not None:
        size[dim] = dim_size
    elif index.numel() == 0:
        size[dim] = 0
    else:
        size[dim] = int(index.max()) + 1
    return size, dim


def scatter_sum(src, index, dim=-1, out=None, dim_size=None):
    index = _broadcast(index, src, dim)
    size, dim = _out_size(src, index, dim, dim_size)
    res = torch.zeros(size, dtype=src.dtype, device=src.device)
    return res.scatter_add_(dim, index, src)


def scatter_mean(src, index, dim=-1, out=None, dim_size=None):
    s = scatter_sum(src, index, dim, dim_size=dim_size)
    ones = torch.ones(index.size(), dtype=src.dtype, device=src.device)
    cnt = scatter_sum(ones, index, dim if dim >= 0 else src.dim() + dim, dim_size=s.size(dim))
    cnt.clamp_(1)
    cnt = _broadcast(cnt, s, dim)
    return s / cnt


def scatter_max(src, index, dim=-1, out=None, dim_size=None):
    index_b = _broadcast(index, src, dim)
    size, dim = _out_size(src, index_b, dim, dim_size)
    res = torch.full(size, float("-inf"), dtype=src.dtype, device=src.device)
    res = res.scatter_reduce(dim, index_b, src, reduce="amax", include_self=True)
    res = torch.where(torch.isneginf(res), torch.zeros_like(res), res)
    return res, None


def scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum"):
    if reduce in ("sum", "add"):
        return scatter_sum(src, index, dim, dim_size=dim_size)
    if reduce == "mean":
        return scatter_mean(src, index, dim, dim_size=dim_size)
    if reduce == "max":
        return scatter_max(src, index, dim, dim_size=dim_size)[0]
    raise ValueError(reduce)


def scatter_softmax(src, index, dim=-1, eps=1e-12):
    index_b = _broadcast(index, src, dim)
    max_value_per_index = scatter_max(src, index_b, dim=dim)[0]
    max_per_src_element = max_value_per_index.gather(dim, index_b)
    recentered = src - max_per_src_element
    recentered_exp = recentered.exp()
    sum_per_index = scatter_sum(recentered_exp, index_b, dim)
    normalizing = (sum_per_index + eps).gather(dim, index_b)
    return recentered_exp.div(normalizing)


# ----------------------------------------------------------------------------------------
# torch_geometric 1.4.3 (+ torch_sparse 0.6.1 coalesce) restatement
# ----------------------------------------------------------------------------------------
def _coalesce(edge_index, n):
    key = edge_index[0] * n + edge_index[1]
    key = torch.unique(key, sorted=True)
    return torch.stack([key // n, key % n], 0)


def dense_to_sparse(adj):
    index = adj.nonzero(as_tuple=False).t()
    value = adj[index[0], index[1]]
    return index, value


def to_undirected(edge_index, num_nodes=None):
    n = int(edge_index.max()) + 1 if num_nodes is None else num_nodes
    row, col = edge_index
    both = torch.stack([torch.cat([row, col]), torch.cat([col, row])], 0)
    return _coalesce(both, n)


def remove_self_loops(edge_index, edge_attr=None):
    mask = edge_index[0] != edge_index[1]
    return edge_index[:, mask], (None if edge_attr is None else edge_attr[mask])


def subgraph(subset, edge_index, edge_attr=None, relabel_nodes=False, num_nodes=None):
    mask = subset[edge_index[0]] & subset[edge_index[1]]
    edge_index = edge_index[:, mask]
    edge_attr = edge_attr[mask] if edge_attr is not None else None
    if relabel_nodes:
        n_idx = torch.zeros(subset.numel(), dtype=torch.long)
        n_idx[subset] = torch.arange(int(subset.sum()))
        edge_index = n_idx[edge_index]
    return edge_index, edge_attr


def knn_graph(x, k, batch=None, loop=False, flow="source_to_target", cosine=False):
    """torch_cluster 1.5.4 knn_graph; tie order restated as (squared distance, index)."""
    n = x.shape[0]
    kk = k if loop else k + 1
    d2 = ((x[:, None, :].double() - x[None, :, :].double()) ** 2).sum(-1)
    order = torch.argsort(d2, dim=1, stable=True)[:, :kk]          # [n, kk] nearest per query
    y_idx = torch.arange(n)[:, None].expand_as(order).reshape(-1)   # query (target)
    x_idx = order.reshape(-1)                                        # neighbour (source)
    row, col = (x_idx, y_idx) if flow == "source_to_target" else (y_idx, x_idx)
    if not loop:
        m = row != col
        row, col = row[m], col[m]
    return torch.stack([row, col], 0)


class MessagePassing(torch.nn.Module):
    """PyG 1.4.3 MessagePassing.propagate restated (flow source_to_target, node_dim 0)."""
    _special = {"edge_index", "edge_index_i", "edge_index_j", "size", "size_i", "size_j",
                "index", "dim_size"}

    def __init__(self, aggr="add", flow="source_to_target", node_dim=0):
        super().__init__()
        self.aggr = aggr
        self.flow = flow
        self.node_dim = node_dim
        self.__msg_params__ = list(inspect.signature(self.message).parameters.items())
        self.__aggr_params__ = list(inspect.signature(self.aggregate).parameters.items())[1:]
        self.__update_params__ = list(inspect.signature(self.update).parameters.items())[1:]
        names = set(k for k, _ in self.__msg_params__ + self.__aggr_params__ + self.__update_params__)
        self.__user_args__ = names - self._special

    def _collect(self, edge_index, size, kwargs):
        i, j = (1, 0) if self.flow == "source_to_target" else (0, 1)
        out = {}
        for arg in self.__user_args__:
            if arg[-2:] in ("_i", "_j"):
                idx = i if arg[-2:] == "_i" else j
                data = kwargs.get(arg[:-2], inspect.Parameter.empty)
                if torch.is_tensor(data):
                    if size[idx] is None:
                        size[idx] = data.size(self.node_dim)
                    data = data.index_select(self.node_dim, edge_index[idx])
                out[arg] = data
            else:
                out[arg] = kwargs.get(arg, inspect.Parameter.empty)
        size[0] = size[1] if size[0] is None else size[0]
        size[1] = size[0] if size[1] is None else size[1]
        out.update(edge_index=edge_index, edge_index_i=edge_index[i], edge_index_j=edge_index[j],
                   size=size, size_i=size[i], size_j=size[j], index=edge_index[i], dim_size=size[i])
        return out

    @staticmethod
    def _distribute(params, kwargs):
        res = {}
        for key, p in params:
            data = kwargs.get(key, inspect.Parameter.empty)
            if data is inspect.Parameter.empty:
                if p.default is inspect.Parameter.empty:
                    raise TypeError(f"Required parameter {key} is empty.")
                data = p.default
            res[key] = data
        return res

    def propagate(self, edge_index, size=None, **kwargs):
        size = [None, None] if size is None else list(size)
        kw = self._collect(edge_index, size, kwargs)
        out = self.message(**self._distribute(self.__msg_params__, kw))
        out = self.aggregate(out, **self._distribute(self.__aggr_params__, kw))
        out = self.update(out, **self._distribute(self.__update_params__, kw))
        return out

    def message(self, x_j):
        return x_j

    def aggregate(self, inputs, index, dim_size=None):
        return scatter(inputs, index, dim=self.node_dim, dim_size=dim_size, reduce=self.aggr)

    def update(self, inputs):
        return inputs


# ----------------------------------------------------------------------------------------
# Loader
# ----------------------------------------------------------------------------------------
def _extract_functions(path, names):
    """Execute only the named top-level functions of a reference file (avoids its cv2 imports)."""
    with open(path) as f:
        tree = ast.parse(f.read(), filename=path)
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    mod = ast.Module(body=body, type_ignores=[])
    ns = {"torch": torch, "nn": torch.nn}
    exec(compile(mod, path, "exec"), ns)
    return {n: ns[n] for n in names}


def install_stubs():
    tg = types.ModuleType("torch_geometric")
    tgu = types.ModuleType("torch_geometric.utils")
    tgn = types.ModuleType("torch_geometric.nn")
    for f in (dense_to_sparse, to_undirected, remove_self_loops, subgraph):
        setattr(tgu, f.__name__, f)
    tgn.knn_graph = knn_graph
    tgn.MessagePassing = MessagePassing
    tg.utils, tg.nn = tgu, tgn
    ts = types.ModuleType("torch_scatter")
    ts.scatter, ts.scatter_max, ts.scatter_softmax = scatter, scatter_max, scatter_softmax
    ts.scatter_add = scatter_sum
    utils_pkg = types.ModuleType("Utils")
    utils_pkg.__path__ = []
    utils_utils = types.ModuleType("Utils.Utils")
    fns = _extract_functions(os.path.join(REF_SRC, "Utils", "Utils.py"),
                             ["non_maximum_suppression", "subgraph_mask"])
    for k, v in fns.items():
        setattr(utils_utils, k, v)
    utils_pkg.Utils = utils_utils
    sys.modules.update({
        "torch_geometric": tg, "torch_geometric.utils": tgu, "torch_geometric.nn": tgn,
        "torch_scatter": ts, "Utils": utils_pkg, "Utils.Utils": utils_utils,
    })


def _load(name, path, package=None):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    if package is not None:
        mod.__package__ = package
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    """Returns (ConstructGraph module, NodeClassificationMPNSimple class, layers module)."""
    if not reference_available():
        raise RuntimeError("reference tree not present")
    sys.dont_write_bytecode = True
    install_stubs()
    cg = _load("ref_ConstructGraph", os.path.join(REF_SRC, "graph_constructor", "ConstructGraph.py"))
    pkg = types.ModuleType("ref_mpn")
    pkg.__path__ = [os.path.join(REF_SRC, "Models", "MessagePassingNetwork")]
    sys.modules["ref_mpn"] = pkg
    mpn_dir = pkg.__path__[0]
    layers = _load("ref_mpn.layers", os.path.join(mpn_dir, "layers.py"), "ref_mpn")
    _load("ref_mpn.utils", os.path.join(mpn_dir, "utils.py"), "ref_mpn")
    simple = _load("ref_mpn.NodeClassificationMPNSimple",
                   os.path.join(mpn_dir, "NodeClassificationMPNSimple.py"), "ref_mpn")
    return cg, simple.NodeClassificationMPNSimple, layers
