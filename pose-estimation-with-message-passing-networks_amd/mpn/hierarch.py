"""Hierarchical node updates of ``TypeAwareMPNLayer`` (UPDATE_TYPE hierarch_mlp / hierarch_cnn,
``layers.py:89-154``): the reference's parameter containers (identical ``state_dict`` keys) and
type orders. ``mpn/fold.py`` folds them into dense layers for ``node_mlp_kernel``."""
import torch.nn as nn

# layers.py:115-119 (17 types) / :117-119 (14 types): first- and second-level type groups
HIERARCH_ORDER_1 = {17: [(0, 1, 2, 3, 4), (5, 6), (7, 9), (8, 10), (11, 12), (13, 15), (14, 16)],
                    14: [(0, 1), (2, 3), (4, 6), (5, 7), (8, 9), (10, 12), (11, 13)]}
HIERARCH_ORDER_2 = [(0, 1), (1, 2), (1, 3), (1, 4), (4, 5), (4, 6)]
# layers.py:148-149
HIERARCH_CNN_ORDER_1 = [5, 6, 7, 9, 8, 10, 11, 12, 13, 15, 14, 16]
HIERARCH_CNN_ORDER_2 = [0, 1, 0, 2, 0, 3, 3, 4, 3, 5]


class HierarchUpdateMlp(nn.Module):
    """``layers.py:89-128`` (parameters only; folded into dense layers by mpn/fold.py)."""

    def __init__(self, node_dim, num_joints):
        super().__init__()
        if num_joints not in (17, 14):
            raise ValueError(f"HierarchUpdateMlp needs 17 or 14 types (got {num_joints})")   # :96 assert
        self.node_dim, self.num_joints = node_dim, num_joints
        first_in = 5 if num_joints == 17 else 2
        self.first_layer = nn.ModuleList([nn.Linear(node_dim * first_in, node_dim // 2)] +
                                         [nn.Linear(node_dim * 2, node_dim // 2) for _ in range(6)])
        self.second_layer = nn.ModuleList([nn.Linear(2 * node_dim // 2, node_dim // 2) for _ in range(6)])
        self.final = nn.Linear(6 * node_dim // 2, node_dim)
        self.relu = nn.ReLU(inplace=True)


class HierarchUpdateCnn(nn.Module):
    """``layers.py:131-154`` (parameters only; folded into dense layers by mpn/fold.py)."""

    def __init__(self, node_dim):
        super().__init__()
        self.head_layer = nn.Linear(node_dim * 4, node_dim // 2)
        self.conv_1 = nn.Conv1d(node_dim, node_dim // 2, 2, 2)
        self.conv_2 = nn.Conv1d(node_dim // 2, node_dim // 2, 2, 2)
        self.final = nn.Linear(5 * node_dim // 2, node_dim)
        self.relu = nn.ReLU(inplace=True)
