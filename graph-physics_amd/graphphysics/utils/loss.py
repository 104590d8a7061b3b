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


class _NativeMaskedMSE(torch.autograd.Function):
    """masked_mse on libmgn (mgn_masked_mse / mgn_masked_mse_backward): one launch each way."""

    @staticmethod
    def forward(ctx, out, target, node_type, type_mask, count):
        from graphphysics import _native as nat

        out_c, tgt_c = out.detach().contiguous(), target.detach().float().contiguous()
        rows, cols = out_c.shape
        loss = torch.empty((), dtype=torch.float32, device=out.device)
        cnt = torch.empty((), dtype=torch.float32, device=out.device)
        ws = torch.empty(int(nat.lib().mgn_masked_mse_workspace_bytes(rows)), dtype=torch.uint8, device=out.device)
        nat.check(nat.lib().mgn_masked_mse(nat.ptr(out_c), nat.ptr(tgt_c), rows, cols, nat.ptr(node_type),
                                           node_type.stride(0), type_mask, nat.ptr(count), nat.ptr(loss),
                                           nat.ptr(cnt), nat.ptr(ws), ws.numel(), nat.stream_ptr(out.device)))
        ctx.save_for_backward(out_c, tgt_c, node_type, cnt)
        ctx.type_mask = type_mask
        return loss

    @staticmethod
    def backward(ctx, gloss):
        from graphphysics import _native as nat

        out_c, tgt_c, node_type, cnt = ctx.saved_tensors
        rows, cols = out_c.shape
        g = torch.empty_like(out_c)
        gl = gloss.detach().float().contiguous()
        nat.check(nat.lib().mgn_masked_mse_backward(nat.ptr(out_c), nat.ptr(tgt_c), rows, cols, nat.ptr(node_type),
                                                    node_type.stride(0), ctx.type_mask, nat.ptr(cnt), nat.ptr(gl),
                                                    nat.ptr(g), nat.stream_ptr(out_c.device)))
        return g, None, None, None, None


def _native_loss_ok(target, network_output, node_type, masks, count):
    return (network_output.is_cuda and network_output.dim() == 2 and network_output.dtype == torch.float32
            and target.shape == network_output.shape and node_type.dim() == 1
            and node_type.dtype == torch.float32 and node_type.device == network_output.device
            and all(0 <= int(m) < 32 for m in masks) and not target.requires_grad
            and (count is None or (count.dtype == torch.float32 and count.numel() == 1)))


def masked_mse(target, network_output, node_type, masks, count=None):
    """Same value as L2Loss without boolean indexing (no data-dependent shapes, no host sync, so it
    can live inside a captured hipGraph): Σ mask·err² / (Σ mask · n_out). `count` overrides the
    denominator's mask count (data-parallel global count). CUDA fp32: one native launch each way."""
    if _native_loss_ok(target, network_output, node_type, masks, count):
        tmask = 0
        for m in masks:
            tmask |= 1 << int(m)
        return _NativeMaskedMSE.apply(network_output, target, node_type, tmask,
                                      count.reshape(()) if count is not None else None)
    m = _prepare_mask_for_loss(network_output, node_type, masks).to(network_output.dtype)
    err = ((network_output - target) ** 2).sum(dim=1)
    cnt = m.sum() if count is None else count
    return (err * m).sum() / (cnt * network_output.shape[1])


__all__ = ["L2Loss", "NodeType", "_prepare_mask_for_loss", "masked_mse"]
