"""Depth-relation helpers (mirrors pldepth/data/depth_utils.py).

``get_depth_relation`` is the scalar host helper the reference's samplers and eval code call
(depth_utils.py:5-21); the samplers' hot use of it lives inside pld_sampler_rank.
``prepare_fully_fledged_loss_input`` (depth_utils.py:39-61) is fused into pld_listmle_fwd_bwd;
the standalone form here serves callers that want the gathered depths themselves.
"""
import numpy as np
import torch


def get_depth_relation(depth1, depth2, threshold=None):
    if threshold is None:
        if depth1 > depth2:
            return 1
        elif depth1 < depth2:
            return -1
        return 0
    epsilon = 1e-10
    ratio = (depth1 + epsilon) / (depth2 + epsilon)
    if ratio >= 1 + threshold:
        return 1
    elif ratio <= 1 / (1 + threshold):
        return -1
    return 0


def prepare_fully_fledged_loss_input(labels, logits, batch_size, ranking_size, debug=False):
    """(selected_depths [B*R, L], labels [B*R, L]) as device tensors (gather on the GPU)."""
    lab = torch.as_tensor(labels, dtype=torch.float32)
    pred = torch.as_tensor(logits, dtype=torch.float32)
    if pred.device != lab.device:
        lab = lab.to(pred.device)
    rankings = lab.reshape(batch_size, -1, ranking_size, 2)
    pred_maps = pred.reshape(batch_size, -1)
    idx = rankings[..., 0].reshape(batch_size, -1).to(torch.int64)
    sel = torch.gather(pred_maps, 1, idx).reshape(-1, ranking_size)
    return sel, rankings[..., 1].reshape(-1, ranking_size)
