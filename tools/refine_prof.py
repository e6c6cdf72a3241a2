"""Refine kernel timing at the bench size (17 x 640 x 640; args: persons (9), F (1)): run under
rocprofv3 --kernel-trace --stats."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pemp_amd import pose as ppose  # noqa: E402

rng = np.random.default_rng(0)
J, H, W, P = 17, 640, 640, int(sys.argv[1]) if len(sys.argv) > 1 else 9
F = int(sys.argv[2]) if len(sys.argv) > 2 else 1
s = torch.rand(J, H, W, device="cuda")
tag = torch.rand(J, H, W, F, device="cuda")
kp = np.zeros((P, J, 3))
for p in range(P):
    for i in rng.choice(J, 10, replace=False):
        kp[p, i] = (rng.integers(0, W), rng.integers(0, H), 0.5)
for _ in range(20):
    ppose.refine(s, tag, kp.copy())
torch.cuda.synchronize()
print("ok")
