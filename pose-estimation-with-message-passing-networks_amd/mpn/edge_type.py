"""EDGE_MLP per_type of ``TypeAwareMPNLayer`` (``layers.py:275-303``): the reference's parameter
container (identical ``state_dict`` keys); ``mpn/fold.py`` maps it onto the edge pass and
``node_ept_kernel``."""
import torch.nn as nn


class TypeAwareEdgeUpdate(nn.Module):
    """``layers.py:275-303`` (EDGE_MLP per_type): per-type target / source Linears, a shared edge
    Linear, then ReLU -> Linear(3 h, h) -> ReLU. Parameters only; folded by mpn/fold.py."""

    def __init__(self, node_feature_dim, edge_feature_dim, output_dim, num_joints):
        super().__init__()
        self.layer_1 = nn.ModuleList([nn.Linear(node_feature_dim, output_dim) for _ in range(num_joints)])
        self.layer_2 = nn.ModuleList([nn.Linear(node_feature_dim, output_dim) for _ in range(num_joints)])
        self.edge_layer = nn.Linear(edge_feature_dim, output_dim)
        self.out = nn.Sequential(nn.ReLU(inplace=True), nn.Linear(3 * output_dim, output_dim), nn.ReLU(inplace=True))
        self.output_dim, self.num_joints = output_dim, num_joints
