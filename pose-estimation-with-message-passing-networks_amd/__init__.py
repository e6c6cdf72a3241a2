"""MI355X-native keypoint-graph hot path of nibox/Pose-Estimation-with-Message-Passing-Networks.

Drop-in for the reference's ``get_graph_constructor(config, **kw).construct_graph()``
(``src/graph_constructor/__init__.py:4-5``) and ``get_mpn_model(config.MODEL.MPN)``
(``src/Models/MessagePassingNetwork/__init__.py:27-73``), computed by hand-written gfx950 HIP
kernels behind the C-ABI library ``csrc/libpemp.so`` (``include/pemp.h``).

Importing the package does not load the HIP library; the first compute call does, and fails
loudly if it is missing or no HIP device is present.
"""
__version__ = "0.1.0"


def get_graph_constructor(config, **kwargs):
    from .graph_constructor import get_graph_constructor as _g
    return _g(config, **kwargs)


def get_mpn_model(config, **kwargs):
    from .mpn import get_mpn_model as _m
    return _m(config, **kwargs)


def bind_mpn(model):
    """Capacity mode: construct_graph queues ``model``'s forward behind its capacity graph build, before the
    detection counts reach the host (graph_constructor.NaiveGraphConstructor.bind_mpn); ``None`` unbinds."""
    from .graph_constructor import NaiveGraphConstructor as _n
    _n.bind_mpn(model)


def ProjectedMaps(maps, size, divisor=None, gather=None):
    """Lazy image-size projection of per-scale feature maps for ``features=`` (frontend.py); ``gather``: the
    model's feature_gather Conv2d, evaluated at the detections only."""
    from .frontend import ProjectedMaps as _p
    return _p(maps, size, divisor, gather)


def ProjectedHeatmaps(outputs, size, num_joints, flip_outputs=None, flip_index=None, divisor=None, tag_scale=0,
                      tag_per_joint=True):
    """The test front-end's image-size heatmaps / tags evaluated on demand, for ``scoremaps=`` and
    ``tagmaps=`` (frontend.py)."""
    from .frontend import ProjectedHeatmaps as _p
    return _p(outputs, size, num_joints, flip_outputs, flip_index, divisor, tag_scale, tag_per_joint)
