"""KernelSHAP weights: the reference's `Kernel` class (kernels.py:6-174) on the HIP engine.

`Kernel(mask).compute()` bit-packs the bool mask on the device, popcounts every row and
evaluates the reference formula in fp64 (exact binomial for S-1 <= 1000, the ref-1000
approximation with its 0.9 back-off above) in the `xpg_shap_kernel` HIP kernel.  The two
static helpers keep the reference signatures for callers that use them directly.
"""
import math

import torch

from . import engine


def _binom(n, k):
    n, k = int(n), int(k)
    return float(math.comb(n, k)) if 0 <= k <= n else 0.0


class Kernel:
    def __init__(self, mask):
        self.mask = mask

    @staticmethod
    def approximate_shap_kernel(num_active, num_total, device, ref=1000):
        """kernels.py:23-80 (host helper, float64 tensor on `device`)."""
        choose = torch.tensor([_binom(ref, i) for i in range(ref)], dtype=torch.float64)
        choose = ((choose + 1e-10) * num_total / 1000).to(device)
        index = (num_active * 1000 / num_total).long()
        index = torch.clip(index, min=0, max=len(choose) - 1)
        return float(num_total) / (choose[index] * num_active.double() *
                                   (num_total - num_active).double())

    @staticmethod
    def original_shap_kernel(num_active, num_total, device):
        """kernels.py:83-113 (host helper)."""
        choose = torch.tensor([_binom(num_total + 1, k) for k in num_active.reshape(-1).tolist()],
                              dtype=torch.float64).reshape(num_active.shape).to(device)
        return num_total / (choose * (num_total + 1 - num_active) * num_active)

    def compute(self):
        """kernels.py:115-174 on the device: fp64 [rows]."""
        mask = self.mask
        bits = engine.pack_masks(mask)
        return engine.shap_kernel(bits, mask.shape[1])
