"""Test-time front-end pieces adjacent to the graph path.

``ProjectedMaps`` stands in for the image-size feature map the reference materialises at test time
-- ``interpolate(feature_gather(feat), size=(H, W), mode='bilinear', align_corners=False)`` per
scale (``PoseEstimation.py:426-452``), summed over scales and divided by their count
(``multi_scales_testing.py:182-190``, ``PoseEstimation.py:244``) -- and is accepted by
``get_graph_constructor(features=...)``. The graph constructor then interpolates the N detections
only (``pemp_gather_projected``): at 640x640 that skips writing and re-reading a [128, H, W] fp32
map (210 MB) per scale.
"""
import torch


class ProjectedMaps:
    def __init__(self, maps, size, divisor=None):
        """maps: list of [B, C, h_s, w_s] tensors (one per scale); size: (H, W) of the projection;
        divisor: the reference's float(len(TEST.SCALE_FACTOR)) (default: number of maps)."""
        if isinstance(maps, torch.Tensor):
            maps = [maps]
        maps = list(maps)
        if not maps or len(maps) > 8:
            raise ValueError("ProjectedMaps: 1 to 8 maps")
        B, C = maps[0].shape[:2]
        for m in maps:
            if m.dim() != 4 or m.shape[0] != B or m.shape[1] != C:
                raise ValueError("ProjectedMaps: every map is [B, C, h, w] with the same B and C")
        self.maps = maps
        self.size = (int(size[0]), int(size[1]))
        self.divisor = float(len(maps) if divisor is None else divisor)
        self.shape = torch.Size([B, C, self.size[0], self.size[1]])
        self.dtype = torch.float32
        self.device = maps[0].device

    def to(self, device):
        return ProjectedMaps([m.to(device) for m in self.maps], self.size, self.divisor)

    def materialize(self):
        """The reference's dense map (for checks): sum of the projections / divisor."""
        acc = None
        for m in self.maps:
            p = torch.nn.functional.interpolate(m.float(), size=self.size, mode="bilinear", align_corners=False)
            acc = p if acc is None else acc + p
        return acc / self.divisor
