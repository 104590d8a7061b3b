"""Masked L2 loss (reference graphphysics/utils/loss.py:10-65)."""
import torch
from torch.nn.modules.loss import _Loss

from graphphysics.utils.nodetype import NodeType


def _prepare_mask_for_loss(network_output, node_type, masks, selected_indexes=None):
    mask = node_type == masks[0]
    for m in masks[1:]:
        mask = torch.logical_or(mask, node_type == m)
    if selected_indexes is not None:
        n = network_output.shape[0]
        keep = ~torch.isin(torch.arange(n, device=network_output.device),
                           selected_indexes.to(network_output.device))
        mask = torch.logical_and(keep, mask)
    return mask


class L2Loss(_Loss):
    @property
    def __name__(self):
        return "MSE"

    def forward(self, target, network_output, node_type, masks: list, selected_indexes=None):
        mask = _prepare_mask_for_loss(network_output, node_type, masks, selected_indexes)
        return torch.mean(((network_output - target) ** 2)[mask])


def masked_mse(target, network_output, node_type, masks, count=None):
    """Same value as L2Loss without boolean indexing (no data-dependent shapes, no host sync, so it
    can live inside a captured hipGraph): Σ mask·err² / (Σ mask · n_out). `count` overrides the
    denominator's mask count (data-parallel global count)."""
    m = _prepare_mask_for_loss(network_output, node_type, masks).to(network_output.dtype)
    err = ((network_output - target) ** 2).sum(dim=1)
    cnt = m.sum() if count is None else count
    return (err * m).sum() / (cnt * network_output.shape[1])


__all__ = ["L2Loss", "NodeType", "_prepare_mask_for_loss", "masked_mse"]
