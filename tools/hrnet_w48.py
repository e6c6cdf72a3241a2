"""HigherHRNet-w48 compute graph with random weights, for the backbone timing leg of bench.py (`--backbone`).

SURVEY §8(d) C3: "e2e adds the HRNet-w48 640 backbone (random weights) + front-end" — the backbone is out of
scope for acceleration (north_star keeps it frozen on PyTorch-ROCm), so this is plain torch on MIOpen, written
from the architecture the reference configures (experiments/hybrid_class_agnostic_end2end/model_58_4_4.yaml:38-94:
STEM 64, stage 2/3/4 with 1/4/3 modules of 4 BasicBlocks per branch at widths 48/96/192/384, SUM fusion, a 1x1
final layer for 2 x 17 heatmap + tag channels at 1/4 resolution, one 4x4 deconvolution on the concatenation of the
features and that output, 4 BasicBlocks, 17 heatmaps at 1/2 resolution; the forward of
src/Models/HigherHRNet/hrnet.py:480-545 with FEATURE_FUSION small). Not a parity component: no weights are loaded
and nothing downstream reads its numbers; it measures the time a batch of 640 px images spends in the backbone."""
import torch
import torch.nn as nn
import torch.nn.functional as F


def conv_bn(cin, cout, k=3, stride=1, relu=True):
    layers = [nn.Conv2d(cin, cout, k, stride, k // 2, bias=False), nn.BatchNorm2d(cout)]
    if relu:
        layers.append(nn.ReLU(inplace=True))
    return nn.Sequential(*layers)


class Basic(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.a = conv_bn(c, c)
        self.b = conv_bn(c, c, relu=False)

    def forward(self, x):
        return F.relu(x + self.b(self.a(x)))


class Bottleneck(nn.Module):
    def __init__(self, cin, mid):
        super().__init__()
        self.body = nn.Sequential(conv_bn(cin, mid, 1), conv_bn(mid, mid), conv_bn(mid, 4 * mid, 1, relu=False))
        self.skip = conv_bn(cin, 4 * mid, 1, relu=False) if cin != 4 * mid else nn.Identity()

    def forward(self, x):
        return F.relu(self.skip(x) + self.body(x))


class Module(nn.Module):
    """One multi-resolution module: 4 BasicBlocks per branch, then every output branch sums every input branch
    (1x1 conv + nearest upsampling from coarser ones, chains of strided 3x3 convs from finer ones)."""

    def __init__(self, widths, outputs):
        super().__init__()
        self.branches = nn.ModuleList([nn.Sequential(*[Basic(c) for _ in range(4)]) for c in widths])
        self.fuse = nn.ModuleList()
        for i in range(outputs):
            row = nn.ModuleList()
            for j, cj in enumerate(widths):
                if j == i:
                    row.append(nn.Identity())
                elif j > i:
                    row.append(conv_bn(cj, widths[i], 1, relu=False))
                else:
                    steps = [conv_bn(cj, cj, 3, 2) for _ in range(i - j - 1)]
                    steps.append(conv_bn(cj, widths[i], 3, 2, relu=False))
                    row.append(nn.Sequential(*steps))
            self.fuse.append(row)

    def forward(self, xs):
        xs = [b(x) for b, x in zip(self.branches, xs)]
        out = []
        for i, row in enumerate(self.fuse):
            acc = None
            for j, f in enumerate(row):
                y = f(xs[j])
                if j > i:
                    y = F.interpolate(y, scale_factor=2 ** (j - i), mode="nearest")
                acc = y if acc is None else acc + y
            out.append(F.relu(acc))
        return out


class HigherHRNetW48(nn.Module):
    def __init__(self, joints=17):
        super().__init__()
        w = [48, 96, 192, 384]
        self.stem = nn.Sequential(conv_bn(3, 64, 3, 2), conv_bn(64, 64, 3, 2))
        self.layer1 = nn.Sequential(Bottleneck(64, 64), *[Bottleneck(256, 64) for _ in range(3)])
        self.t1 = nn.ModuleList([conv_bn(256, w[0]), conv_bn(256, w[1], 3, 2)])
        self.s2 = nn.ModuleList([Module(w[:2], 2)])
        self.t2 = conv_bn(w[1], w[2], 3, 2)
        self.s3 = nn.ModuleList([Module(w[:3], 3) for _ in range(4)])
        self.t3 = conv_bn(w[2], w[3], 3, 2)
        self.s4 = nn.ModuleList([Module(w, 4) for _ in range(2)] + [Module(w, 1)])
        self.final0 = nn.Conv2d(w[0], 2 * joints, 1)
        self.deconv = nn.Sequential(nn.ConvTranspose2d(w[0] + 2 * joints, w[0], 4, 2, 1, bias=False),
                                    nn.BatchNorm2d(w[0]), nn.ReLU(inplace=True), *[Basic(w[0]) for _ in range(4)])
        self.final1 = nn.Conv2d(w[0], joints, 1)

    def forward(self, img):
        x = self.layer1(self.stem(img))
        xs = [self.t1[0](x), self.t1[1](x)]
        for m in self.s2:
            xs = m(xs)
        xs = xs + [self.t2(xs[-1])]
        for m in self.s3:
            xs = m(xs)
        xs = xs + [self.t3(xs[-1])]
        for m in self.s4:
            xs = m(xs)
        x = xs[0]
        y0 = self.final0(x)                                   # heatmaps + tags, 1/4 resolution
        big = self.deconv(torch.cat([x, y0], 1))
        y1 = self.final1(big)                                 # heatmaps, 1/2 resolution
        feats = F.interpolate(x, size=big.shape[2:], mode="bilinear", align_corners=False)   # FEATURE_FUSION small
        return [y0, y1], feats
