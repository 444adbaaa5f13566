"""Plackett-Luce (ListMLE) losses on the GPU (mirrors pldepth/losses/nll_loss.py).

``HourglassNegativeLogLikelihood(ranking_size, batch_size)`` keeps the reference's constructor and
call signature (``loss(y_true[B,R,L,2], y_pred[B,H,W,1]) -> scalar``, nll_loss.py:32-40); the
gather of predicted depths at the sampled pixels (depth_utils.py:39-61), tfr ListMLE and the
SUM_OVER_BATCH_SIZE reduction run as one HIP kernel that also produces d loss / d y_pred
(``loss_and_grad``), which the model's backward pass consumes. ``NegativeLogLikelihoodLoss`` is the
per-list variant (nll_loss.py:10-29: logits already [*, L]).
"""
import numpy as np
import torch

from .. import kernels as K


def _dev(t, device="cuda"):
    if isinstance(t, torch.Tensor):
        return t.to(device=device, dtype=torch.float32).contiguous()
    return torch.as_tensor(np.ascontiguousarray(t, dtype=np.float32), device=device)


class HourglassNegativeLogLikelihood(object):
    def __init__(self, ranking_size, batch_size, reduction="auto", name=None,
                 lambda_weight=None, debug=False):
        if lambda_weight is not None:
            raise NotImplementedError("ListMLE lambda weights are not used by any PLDepth driver")
        self.ranking_size = int(ranking_size)
        self.batch_size = int(batch_size)
        self.name = name
        self._buf = {}

    def _buffers(self, pred, n_lists):
        key = (pred.shape, n_lists, pred.device)
        if key not in self._buf:
            self._buf[key] = (torch.empty_like(pred),
                              torch.empty(n_lists, device=pred.device),
                              torch.empty(1, device=pred.device))
        return self._buf[key]

    def loss_and_grad(self, y_true, y_pred, dpred=None):
        """(loss [1] device tensor, d loss / d y_pred with y_pred's shape)."""
        B, L = self.batch_size, self.ranking_size
        y_pred = _dev(y_pred)
        y_true = _dev(y_true, y_pred.device)
        n_lists = y_true.numel() // (2 * L)
        if n_lists % B:
            raise ValueError(f"y_true holds {n_lists} rankings, not a multiple of batch {B}")
        R = n_lists // B
        g, nll, loss = self._buffers(y_pred, n_lists)
        if dpred is not None:
            g = dpred
        K.listmle_fwd_bwd(y_pred, y_true, B, R, L, dpred=g, nll=nll, loss=loss)
        return loss, g

    def __call__(self, y_true, y_pred, sample_weight=None):
        if sample_weight is not None:
            raise NotImplementedError("sample weights are not used by any PLDepth driver")
        loss, _ = self.loss_and_grad(y_true, y_pred)
        return loss


class NegativeLogLikelihoodLoss(object):
    """Per-list ListMLE: y_true (labels) and y_pred (logits) both [..., L]."""

    def __init__(self, ranking_size, reduction="auto", name=None, lambda_weight=None):
        if lambda_weight is not None:
            raise NotImplementedError
        self.ranking_size = int(ranking_size)

    def loss_and_grad(self, y_true, y_pred):
        L = self.ranking_size
        y_pred = _dev(y_pred)
        labels = _dev(y_true, y_pred.device).reshape(-1, L)
        N = labels.shape[0]
        # each list is its own "image" of L pixels, ranked in place (index column = position)
        idx = torch.arange(L, device=y_pred.device, dtype=torch.float32).expand(N, L)
        yt = torch.stack([idx, labels], -1).contiguous()
        pred = y_pred.reshape(N, L).contiguous()
        loss, g, _ = K.listmle_fwd_bwd(pred, yt, N, 1, L)
        return loss, g.reshape(y_pred.shape)

    def __call__(self, y_true, y_pred, sample_weight=None):
        return self.loss_and_grad(y_true, y_pred)[0]


MetaBatchListMLELoss = NegativeLogLikelihoodLoss
