"""Configuration surface of the hot path: the reference's ``MODEL.GC.*`` / ``MODEL.MPN.*`` keys.

Restates the defaults of ``src/config/default_config.py:112-165`` (yacs is not a dependency here)
with a small attribute-dict ``CfgNode`` that reads the reference's experiment YAMLs
(``experiments/**.yaml``) and ``KEY VALUE`` command-line overrides, as ``update_config`` /
``update_config_command`` do (``default_config.py:246-260``).
"""
import ast
import copy

import yaml


class CfgNode(dict):
    def __init__(self, init=None, new_allowed=False):
        super().__init__()
        object.__setattr__(self, "_new_allowed", new_allowed)
        for k, v in (init or {}).items():
            self[k] = CfgNode(v, new_allowed) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def clone(self):
        return copy.deepcopy(self)

    def merge(self, other: dict, path=""):
        for k, v in other.items():
            if k not in self and not self._new_allowed:
                raise KeyError(f"Non-existent config key: {path}{k}")
            cur = self.get(k)
            if isinstance(v, dict):
                if not isinstance(cur, CfgNode):
                    cur = CfgNode({}, new_allowed=True)
                    self[k] = cur
                cur.merge(v, path + k + ".")
            else:
                self[k] = _coerce(v, cur)
        return self


def _coerce(v, cur):
    """yacs-like: literal strings are evaluated; '17 + 2' style sums become ints."""
    if isinstance(v, str):
        try:
            v = ast.literal_eval(v)
        except (ValueError, SyntaxError):
            parts = v.split("+")
            if len(parts) > 1 and all(p.strip().lstrip("-").isdigit() for p in parts):
                v = sum(int(p) for p in parts)
    if isinstance(cur, float) and isinstance(v, int) and not isinstance(v, bool):
        v = float(v)
    if isinstance(cur, tuple) and isinstance(v, list):
        v = tuple(v)
    return v


def _defaults():
    return {
        "MODEL": {
            "MPN": CfgNode({
                "NODE_TYPE_SUMMARY": "not", "NAME": "VanillaMPN", "STEPS": 10, "EDGE_MLP": "agnostic",
                "NODE_INPUT_DIM": 128, "AGGR_TYPE": "agnostic", "EDGE_INPUT_DIM": 19,
                "EDGE_FEATURE_DIM": 64, "EDGE_FEATURE_HIDDEN": 64, "NODE_FEATURE_DIM": 64,
                "USE_NODE_UPDATE_MLP": False,
                "NODE_EMB": CfgNode({}, True), "EDGE_EMB": CfgNode({}, True), "CLASS": CfgNode({}, True),
                "BN": True, "AGGR": "max", "AGGR_SUB": "None", "UPDATE_TYPE": "mlp", "SKIP": False,
                "AUX_LOSS_STEPS": 0, "DROP_FEATURE": "", "EDGE_STEPS": 0, "LATE_FUSION_POS": False,
                "NUM_JOINTS": 17, "NODE_STEPS": 0,
            }, new_allowed=True),
            "GC": {
                "NAME": "NaiveGraphConstructor", "POOL_KERNEL_SIZE": 3, "CHEAT": False, "USE_GT": False,
                "USE_NEIGHBOURS": False, "EDGE_LABEL_METHOD": 4, "MASK_CROWDS": True,
                "DETECT_THRESHOLD": 0.005, "WITH_BACKGROUND": False, "HYBRID_K": 5,
                "MATCHING_RADIUS": 0.1, "INCLUSION_RADIUS": 0.75, "GRAPH_TYPE": "knn", "CC_METHOD": "GAEC",
                "NORM_NODE_DISTANCE": False, "IMAGE_CENTRIC_SAMPLING": False, "NODE_MATCHING_RADIUS": 0.5,
                "NODE_INCLUSION_RADIUS": 0.7, "WEIGHT_CLASS_LOSS": False,
                "EDGE_FEATURES_TO_USE": ["position", "connection_type"], "NODE_DROPOUT": 0.0,
            },
        },
        "DATASET": {"NUM_JOINTS": 17, "MAX_NUM_PEOPLE": 30, "SIGMA": 2, "INPUT_SIZE": 512},
        "TEST": {"SCALE_FACTOR": [1.0]},
    }


def get_config() -> CfgNode:
    return CfgNode(_defaults(), new_allowed=True)


def update_config(cfg: CfgNode, yaml_path: str) -> CfgNode:
    with open(yaml_path) as f:
        data = yaml.safe_load(f) or {}
    cfg.merge(data)
    return cfg


def update_config_command(cfg: CfgNode, opts) -> CfgNode:
    opts = list(opts or [])
    if len(opts) % 2:
        raise ValueError("overrides must be KEY VALUE pairs")
    for key, val in zip(opts[0::2], opts[1::2]):
        node = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            node = node[p]
        node[parts[-1]] = _coerce(val, node.get(parts[-1]))
    return cfg


def published_mpn_config(num_joints: int = 17, steps: int = 10, variant: str = "attn") -> CfgNode:
    """``MODEL.MPN`` of ``experiments/hybrid_class_agnostic_end2end/model_58_4.yaml:91-139`` (variant
    "attn"; "attn_per_type" swaps in AGGR_SUB node_edge_attn_per_type) or ``experiments/connectivity/fully_54_3.yaml:91-134`` (variant "max")."""
    mlp = lambda sizes, bn=True: CfgNode({"BN": bn, "END_WITH_RELU": False, "OUTPUT_SIZES": sizes}, True)
    c = get_config().MODEL.MPN
    c.merge({
        "NAME": "NodeClassificationMPN", "STEPS": steps, "NODE_STEPS": 0, "NODE_INPUT_DIM": 128,
        "EDGE_INPUT_DIM": num_joints + 2, "NODE_FEATURE_DIM": 64, "EDGE_FEATURE_DIM": 64,
        "EDGE_FEATURE_HIDDEN": 64, "BN": False, "SKIP": True, "NUM_JOINTS": num_joints,
        "NODE_THRESHOLD": 1.0,
    })
    c.NODE_EMB = mlp([128, 64, 64])
    c.EDGE_EMB = mlp([32, 64, 64, 64])
    c.EDGE_CLASS = CfgNode({"BN": True, "OUTPUT_SIZES": [64, 32, 1]}, True)
    c.NODE_CLASS = CfgNode({"BN": True, "OUTPUT_SIZES": [64, 32, 1]}, True)
    c.CLASS = CfgNode({"BN": True, "OUTPUT_SIZES": [64, 32, num_joints]}, True)
    if variant in ("attn", "attn_per_type"):
        sub = "node_edge_attn" if variant == "attn" else "node_edge_attn_per_type"
        c.merge({"AGGR_TYPE": "per_type", "AGGR": "add", "AGGR_SUB": sub, "UPDATE_TYPE": "mlp"})
    else:
        c.merge({"AGGR_TYPE": "agnostic", "AGGR": variant})
    return c


def inference_gc_config(graph_type: str = "fully", pool_kernel: int = 5, mask_crowds: bool = False) -> CfgNode:
    """``MODEL.GC`` as run by valid.py (``README.md:153-167``: POOL_KERNEL_SIZE 5, MASK_CROWDS False)."""
    g = get_config().MODEL.GC
    g.merge({"POOL_KERNEL_SIZE": pool_kernel, "MASK_CROWDS": mask_crowds, "DETECT_THRESHOLD": 0.1,
             "HYBRID_K": 5, "GRAPH_TYPE": graph_type, "NORM_NODE_DISTANCE": True,
             "EDGE_FEATURES_TO_USE": ["position", "connection_type"], "EDGE_LABEL_METHOD": 6})
    return g
