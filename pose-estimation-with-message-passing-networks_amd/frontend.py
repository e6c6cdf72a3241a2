"""Test-time front-end pieces adjacent to the graph path.

``ProjectedMaps`` stands in for the image-size feature map the reference materialises at test time
-- ``interpolate(feature_gather(feat), size=(H, W), mode='bilinear', align_corners=False)`` per
scale (``PoseEstimation.py:426-452``), summed over scales and divided by their count
(``multi_scales_testing.py:182-190``, ``PoseEstimation.py:244``) -- and is accepted by
``get_graph_constructor(features=...)``. The graph constructor then interpolates the N detections
only (``pemp_gather_projected``): at 640x640 that skips writing and re-reading a [128, H, W] fp32
map (210 MB) per scale. With ``gather=`` (the model's ``feature_gather`` Conv2d, ``PoseEstimation.py:64-66``,
applied per scale at ``:341``) the maps are the raw backbone features and the conv is evaluated at the four
bilinear taps of each detection only (``pemp_gather_projected_conv``) instead of over the whole map.
"""
import torch


class ProjectedMaps:
    def __init__(self, maps, size, divisor=None, gather=None):
        """maps: list of [B, C, h_s, w_s] tensors (one per scale); size: (H, W) of the projection;
        divisor: the reference's float(len(TEST.SCALE_FACTOR)) (default: number of maps);
        gather: optional nn.Conv2d applied to each map before the projection (the model's feature_gather:
        stride 1, dilation 1, groups 1, square kernel <= 7, symmetric zero padding < kernel)."""
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
        self.gather = gather
        if gather is not None:
            if not isinstance(gather, torch.nn.Conv2d):
                raise TypeError("ProjectedMaps: gather must be an nn.Conv2d (the model's feature_gather)")
            k = gather.kernel_size
            pad = gather.padding
            if (isinstance(pad, str) or k[0] != k[1] or pad[0] != pad[1] or tuple(gather.stride) != (1, 1)
                    or tuple(gather.dilation) != (1, 1) or gather.groups != 1 or gather.padding_mode != "zeros"
                    or not 1 <= k[0] <= 7 or not 0 <= pad[0] < k[0]):
                raise NotImplementedError("ProjectedMaps: gather conv must be stride 1, dilation 1, groups 1, square "
                                          "kernel <= 7 with symmetric zero padding < kernel")
            if gather.in_channels != C:
                raise ValueError(f"ProjectedMaps: gather expects {gather.in_channels} channels, maps have {C}")
            if gather.out_channels > 512:
                raise NotImplementedError("ProjectedMaps: gather conv with more than 512 output channels")
            C = gather.out_channels
        self.shape = torch.Size([B, C, self.size[0], self.size[1]])
        self.dtype = torch.float32
        self.device = maps[0].device

    def to(self, device):
        return ProjectedMaps([m.to(device) for m in self.maps], self.size, self.divisor,
                             None if self.gather is None else self.gather.to(device))

    def conv_params(self):
        """(weight transposed to [Cin, k, k, Cout] fp32 contiguous, bias fp32 or None, k, pad) for the C-ABI;
        the transpose is cached against the weight's version counter."""
        g = self.gather
        w = g.weight
        key = (w.data_ptr(), w._version, w.device)
        cache = getattr(self, "_wt_cache", None)
        if cache is None or cache[0] != key:
            with torch.no_grad():
                wt = w.detach().float().permute(1, 2, 3, 0).contiguous()
                b = None if g.bias is None else g.bias.detach().float().contiguous()
            self._wt_cache = cache = (key, wt, b)
        return cache[1], cache[2], g.kernel_size[0], g.padding[0]

    def materialize(self):
        """The reference's dense map (for checks): sum of the projections / divisor, computed with the
        reference's own torch ops (feature_gather conv first when given)."""
        acc = None
        for m in self.maps:
            m = m.float()
            if self.gather is not None:
                with torch.no_grad():
                    m = self.gather(m)
            p = torch.nn.functional.interpolate(m, size=self.size, mode="bilinear", align_corners=False)
            acc = p if acc is None else acc + p
        return acc / self.divisor


class ProjectedHeatmaps:
    """The test front-end's heatmaps and tag maps at the image size, never materialised
    (``PoseEstimation.py:329-452`` ``_get_multi_stage_outputs`` with ``FLIP_TEST`` and ``PROJECT2IMAGE``,
    ``multi_scales_testing.py:144-195`` ``aggregate_results_mpn``, ``PoseEstimation.py:227-229``).

    Pass it as BOTH ``scoremaps=`` and ``tagmaps=`` of ``get_graph_constructor``: detection then evaluates
    ``s = (sum_s (up(out_s) + up(flip(flip_out_s))[flip_index]) / 2) / divisor`` inside its NMS loads
    (``pemp_detect_projected``) and the joint tags are sampled at the detections
    (``pemp_gather_projected_tags``): nothing of size [B, J, H, W] is written.

    outputs: list over scales of [B, C, h_s, w_s] network outputs of the forward pass (heatmaps in channels
    0..J-1, per-joint tags in J..2J-1 when tags are used); flip_outputs: the flipped-image pass as the
    network produced it (same shapes, not un-flipped) or None; flip_index: the FLIP_CONFIG permutation;
    size: (H, W); tag_scale: index of the scale whose tags are kept (the reference keeps scale 1.0);
    tag_per_joint: MODEL.HRNET.TAG_PER_JOINT. Scales in the reference's order (descending scale factor).

    Tags: the reference keeps ``output[:, J:]`` and re-indexes the flipped pass by flip_index only when
    TAG_PER_JOINT is set (``PoseEstimation.py:406-410``); ``construct_graph`` then reads channel ``type`` of
    that map (``ConstructGraph.py:103``), which exists only with one tag channel per joint. So tags need
    exactly J tag channels (C == 2J) and TAG_PER_JOINT; a shared tag channel is refused (with it the
    reference's own joint-tag gather indexes past the map)."""

    def __init__(self, outputs, size, num_joints, flip_outputs=None, flip_index=None, divisor=None, tag_scale=0,
                 tag_per_joint=True):
        if isinstance(outputs, torch.Tensor):
            outputs = [outputs]
        outputs = [o.float().contiguous() for o in outputs]
        if not outputs or len(outputs) > 4:
            raise ValueError("ProjectedHeatmaps: 1 to 4 scales")
        if flip_outputs is not None:
            if isinstance(flip_outputs, torch.Tensor):
                flip_outputs = [flip_outputs]
            flip_outputs = [o.float().contiguous() for o in flip_outputs]
            if len(flip_outputs) != len(outputs) or any(a.shape != b.shape for a, b in zip(outputs, flip_outputs)):
                raise ValueError("ProjectedHeatmaps: flip_outputs must match outputs scale by scale")
        B, C = outputs[0].shape[:2]
        J = int(num_joints)
        for o in outputs:
            if o.dim() != 4 or o.shape[0] != B or o.shape[1] != C:
                raise ValueError("ProjectedHeatmaps: every output is [B, C, h, w] with the same B and C")
        if C < J:
            raise ValueError(f"ProjectedHeatmaps: {C} channels < {J} joints")
        if C != J and C != 2 * J:
            raise ValueError(f"ProjectedHeatmaps: {C} channels: expected J = {J} (heatmaps only) or 2J (heatmaps + "
                             "one tag channel per joint)")
        if C == 2 * J and not tag_per_joint:
            raise NotImplementedError("ProjectedHeatmaps: TAG_PER_JOINT False (a shared tag channel; the reference's "
                                      "joint-tag gather, ConstructGraph.py:103, indexes it by joint type)")
        self.outputs, self.flip_outputs = outputs, flip_outputs
        self.num_joints = J
        self.size = (int(size[0]), int(size[1]))
        self.divisor = float(len(outputs) if divisor is None else divisor)
        self.tag_scale = int(tag_scale)
        self.tag_per_joint = bool(tag_per_joint)
        self.device = outputs[0].device
        fi = list(range(J)) if flip_index is None else [int(v) for v in flip_index]
        if sorted(fi) != list(range(J)):
            raise ValueError("ProjectedHeatmaps: flip_index must be a permutation of the joints")
        self.flip_index = torch.tensor(fi, dtype=torch.int32, device=self.device)
        self.shape = torch.Size([B, J, self.size[0], self.size[1]])
        self.dtype = torch.float32
        self.has_tags = C == 2 * J
        self.tag_dims = 2 if flip_outputs is not None else 1

    @classmethod
    def from_stages(cls, stage_outputs, size, num_joints, flip_stage_outputs=None, flip_index=None, divisor=None,
                    tag_scale=0, tag_per_joint=True):
        """The same from HigherHRNet's per-stage outputs (``_get_multi_stage_outputs``, ``PoseEstimation.py:338-412``,
        with the published TEST.WITH_HEATMAPS [True, True] / TEST.WITH_AE [True, False]): stage_outputs is a list
        over scales of (stage0 [B, C0, h/4-res], stage1 [B, C1, h/2-res]) pairs as the backbone returns them,
        flip_stage_outputs the same for the flipped image (as the network produced it, not un-flipped). Each pair
        is merged at the last stage's resolution -- (up(stage0) + stage1) / 2 for the heatmaps, up(stage0) for the
        tags -- by ``pemp_stage_merge`` (one HBM pass, on the current stream); the image-size projection, the flip
        average and the scale sum stay on demand in the detection's loads."""
        from . import _lib
        L = _lib.lib()
        J = int(num_joints)

        def merge(pair):
            s0, s1 = (t.float().contiguous() for t in pair)
            if s0.dim() != 4 or s1.dim() != 4 or s0.shape[0] != s1.shape[0]:
                raise ValueError("ProjectedHeatmaps.from_stages: stages are [B, C, h, w] with the same B")
            B, C0, h0, w0 = s0.shape
            C1, h1, w1 = s1.shape[1:]
            out = torch.empty(B, C0, h1, w1, dtype=torch.float32, device=s0.device)
            _lib.check(L.pemp_stage_merge(s0.data_ptr(), C0, h0, w0, s1.data_ptr(), C1, h1, w1, B, J, out.data_ptr(),
                                          _lib.stream(s0.device)))
            return out

        outs = [merge(p) for p in stage_outputs]
        flips = None if flip_stage_outputs is None else [merge(p) for p in flip_stage_outputs]
        return cls(outs, size, num_joints, flips, flip_index, divisor, tag_scale, tag_per_joint)

    @staticmethod
    def merge_stages_reference(stage0, stage1, num_joints):
        """The reference's own torch ops for one pass of one scale (``PoseEstimation.py:343-364``): heatmaps
        ``(0 + up(stage0)[:, :J] + stage1[:, :J]) / 2`` and tags ``up(stage0)[:, J:]``, concatenated (for checks)."""
        J = int(num_joints)
        up = torch.nn.functional.interpolate(stage0.float(), size=(stage1.size(2), stage1.size(3)), mode="bilinear",
                                             align_corners=False)
        heat = 0
        heat += up[:, :J]
        heat += stage1.float()[:, :J]
        return torch.cat([heat / 2, up[:, J:]], 1)

    def to(self, device):
        return ProjectedHeatmaps([o.to(device) for o in self.outputs], self.size, self.num_joints,
                                 None if self.flip_outputs is None else [o.to(device) for o in self.flip_outputs],
                                 self.flip_index.tolist(), self.divisor, self.tag_scale, self.tag_per_joint)

    def _interp(self, m):
        return torch.nn.functional.interpolate(m, size=self.size, mode="bilinear", align_corners=False)

    def materialize(self):
        """The reference's dense tensors, computed by its own torch ops (for refine / adjust and checks):
        (scoremaps [B, J, H, W], tags [B, J, H, W, F] or None)."""
        J, fi = self.num_joints, self.flip_index.long()
        acc = None
        for s, o in enumerate(self.outputs):
            h = self._interp(o[:, :J])
            if self.flip_outputs is not None:
                hf = self._interp(torch.flip(self.flip_outputs[s], [3])[:, :J][:, fi])
                h = (h + hf) / 2.0
            acc = h if acc is None else acc + h
        scoremaps = acc / self.divisor
        tags = None
        if self.has_tags:
            o = self.outputs[self.tag_scale]
            tl = [self._interp(o[:, J:2 * J]).unsqueeze(4)]
            if self.flip_outputs is not None:
                f = torch.flip(self.flip_outputs[self.tag_scale], [3])[:, J:2 * J][:, fi]
                tl.append(self._interp(f).unsqueeze(4))
            tags = torch.cat(tl, dim=4)
        return scoremaps, tags

    def project(self):
        """The image-size maps materialised on the device by the library (pemp_project_maps), with the
        values the detection samples: (scoremaps [B, J, H, W], tags [B, J, H, W, F] or None)."""
        from . import _lib
        L = _lib.lib()
        B, J, (H, W) = self.outputs[0].shape[0], self.num_joints, self.size
        s = torch.empty(B, J, H, W, dtype=torch.float32, device=self.device)
        t = torch.empty(self.tag_dims, B, J, H, W, dtype=torch.float32, device=self.device) if self.has_tags else None
        c = self.c_struct()
        import ctypes
        _lib.check(L.pemp_project_maps(ctypes.addressof(c), B, J, H, W, self.tag_scale, s.data_ptr(),
                                       None if t is None else t.data_ptr(), _lib.stream(self.device)))
        return s, None if t is None else t.permute(1, 2, 3, 4, 0).contiguous()

    def c_struct(self):
        """pemp_proj_maps for the C-ABI (keeps the tensors alive through self)."""
        from . import _lib
        s = _lib.PempProjMaps()
        s.num_scales = len(self.outputs)
        s.channels = self.outputs[0].shape[1]
        for i, o in enumerate(self.outputs):
            s.maps[i] = o.data_ptr()
            s.flip_maps[i] = self.flip_outputs[i].data_ptr() if self.flip_outputs is not None else None
            s.h[i], s.w[i] = o.shape[2], o.shape[3]
        s.flip_index = self.flip_index.data_ptr()
        s.divisor = self.divisor
        return s
