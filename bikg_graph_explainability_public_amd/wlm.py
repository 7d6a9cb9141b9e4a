"""Weighted linear surrogate: the reference's wlm.py API (wlm.py:17-520), same names/outputs.

`train_model` keeps its signature and return value (weights list, losses list, best epoch)
but runs the whole epoch loop on the device: all mask batches are bit-packed once, every
row's GNN output comes from one ForwardPlan launch chain, the KernelSHAP weights from one
kernel, and all Adam steps from `xpg_wlm_fit` (one persistent workgroup).  The returned
weights are the final-epoch weights, as in the reference (quirk Q2, wlm.py:94,264-266).
"""
import math

import numpy as np
import torch
from torch import nn

from . import engine, pipeline
from .data import Data
from .kernels import Kernel
from .model import Model


class LinearRegression(nn.Module):
    """wlm.py:17-61 — bias-free linear surrogate `mask @ w`."""

    def __init__(self, num_elements):
        assert isinstance(num_elements, int)
        super().__init__()
        self.layer = nn.Linear(int(num_elements), 1, bias=False)

    def forward(self, X):
        return self.layer(X)

    @staticmethod
    def initial_weights(num_elements):
        """The weight row LinearRegression(num_elements) draws, [num_elements]: nn.Linear's
        reset_parameters (one kaiming_uniform_(a=sqrt(5)) on the [1, S] weight, no bias) on the
        same torch CPU generator -- bit-identical values and generator state, without building
        a module per repeat (~35 us each)."""
        assert isinstance(num_elements, int)
        n = int(num_elements)
        if n == 0:
            return torch.empty(0)
        bound = LinearRegression.init_bound(n)
        with torch.no_grad():
            return torch.empty(n).uniform_(-bound, bound)

    @staticmethod
    def init_bound(n):
        """kaiming_uniform_(a=sqrt(5)) on a [1, n] weight: fan_in n, leaky_relu gain, bound
        sqrt(3) * std (the same float operations as torch.nn.init, so the same bound)."""
        gain = math.sqrt(2.0 / (1 + math.sqrt(5) ** 2))
        return math.sqrt(3.0) * (gain / math.sqrt(n))


def model_updates(linear_model, loss, best_loss):
    """wlm.py:64-98 (returns the live parameter generator, as the reference does)."""
    return linear_model.parameters(), loss.item()


def regularizer(net, factor):
    """wlm.py:101-129 — factor * mean |params|."""
    flat = torch.abs(torch.cat([p.view(-1) for p in net.parameters()]))
    return factor * (flat.sum() / flat.shape[0])


def weighted_mse_loss(input, target, weight):
    """wlm.py:491-520."""
    diff = (input.flatten() - target) ** 2
    return torch.mean(weight * diff) / (weight.sum())


class _ReduceLROnPlateau(torch.optim.lr_scheduler.ReduceLROnPlateau):
    def __init__(self, *a, **kw):
        kw.pop("verbose", None)
        super().__init__(*a, **kw)


def optimizer_scheduler(params, arch):
    """wlm.py:441-488 — Adam(lr, weight_decay=1e-2) + ReduceLROnPlateau (never stepped)."""
    opt, lr, patience = params["optimizer"], params["lr"], params["lr_patience"]
    assert isinstance(opt, str), "Optimizer is not string"
    assert isinstance(lr, (float, int)), "Learning rate given is not numeric"
    assert isinstance(patience, (float, int)), "Patience for scheduler is not string"
    optimizer = None
    if opt.strip().lower() == "adam":
        optimizer = torch.optim.Adam(arch.parameters(), lr=abs(lr), weight_decay=1e-2)
    else:
        print("Optimizer choice not available. Please choose between 'adam'")
    sch = _ReduceLROnPlateau(optimizer, "min", patience=abs(int(patience)))
    return optimizer, sch


def kernel_output(mask, data_class, model_class, problem, element_index=None, node_type=None,
                  edge_type=None, node_type_names=None, edge_type_names=None, padded_dims=None):
    """wlm.py:284-438 — (KernelSHAP weights fp64 [B], model outputs [B, 1]) for one batch."""
    plan = pipeline.build_plan(model_class.arch, data_class.feat, data_class.edge_index,
                               [element_index], node_type, edge_type, node_type_names,
                               edge_type_names, padded_dims)
    if plan is not None:
        y = plan.forward(engine.pack_masks(mask))
    else:
        y = pipeline.generic_outputs(model_class.arch, data_class.feat, data_class.edge_index,
                                     mask, element_index, problem, node_type, edge_type,
                                     node_type_names, edge_type_names, padded_dims).view(-1, 1)
    return Kernel(mask).compute(), y


def train_model(mask_loader, params, feat, edge_index, linear_model, arch, problem,
                element_index=None, node_type=None, edge_type=None, node_type_names=None,
                edge_type_names=None, padded_dims=None):
    """wlm.py:132-278 on the device.  Returns ([final weights [S]], losses, best_epoch)."""
    arch.eval()
    mask = torch.cat([m for m in mask_loader], dim=0)
    dev = feat.device
    mask = mask.to(dev)
    S = mask.shape[1]
    batch = mask_loader.batch_size
    bits = engine.pack_masks(mask)
    plan = pipeline.build_plan(arch, feat, edge_index, [element_index], node_type, edge_type,
                               node_type_names, edge_type_names, padded_dims)
    if plan is not None:
        y = plan.forward(bits)[:, 0]
    else:
        y = pipeline.generic_outputs(arch, feat, edge_index, mask, element_index, problem,
                                     node_type, edge_type, node_type_names, edge_type_names,
                                     padded_dims, batch)
    w0 = linear_model.layer.weight.detach()
    w, losses, best, _ = pipeline.fit_repeat(bits, S, batch, y, w0, params)
    with torch.no_grad():
        linear_model.layer.weight.copy_(w.view_as(linear_model.layer.weight))
    return [linear_model.layer.weight[0]], losses.cpu().tolist(), int(best.item())


__all__ = ["LinearRegression", "model_updates", "regularizer", "train_model", "kernel_output",
           "optimizer_scheduler", "weighted_mse_loss", "Data", "Model"]
