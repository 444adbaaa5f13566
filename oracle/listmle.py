"""fp64 numpy restatement of the PLDepth loss — TEST INFRASTRUCTURE (see oracle/__init__).

Restates:
  * ``prepare_fully_fledged_loss_input``  pldepth/data/depth_utils.py:39-61
      rankings = reshape(labels, [B, -1, L, 2]); pred = reshape(logits, [B, H*W]);
      idx = int32(rankings[..., 0]); s = gather(pred, idx, batch_dims=1) -> [B*R, L];
      labels = rankings[..., 1] -> [B*R, L]
  * ``FullyFledgedMetaBatchListMLELoss.compute_unreduced_loss``  pldepth/losses/nll_loss.py:51-62
  * tensorflow_ranking==0.3.1 ``ListMLELoss.compute_unreduced_loss`` (third party, not vendored —
    restated from its published source; PARITY UNPINNED: neither TF nor tfr is installable here):
      valid = label >= 0; label' = valid ? label : 0; s' = valid ? s : log(1e-10)
      score = valid ? label' : min_j(label') - 1e-6
      sort (score desc; tfr shuffles ties with seed 37 — here ties keep a fixed order, see below)
      m = max s';  C_i = sum_{j>=i} exp(s'_j - m);  nll = sum_i (log C_i - (s'_i - m))
  * Keras ``Loss`` reduction AUTO -> SUM_OVER_BATCH_SIZE: mean over the N = B*R lists.

Backward (closed form): d nll / d s'_k = exp(s'_k - m) * sum_{i<=k} 1/C_i - 1 (sorted order);
invalid elements receive zero gradient (the ``where`` selects a constant); the gather's gradient
scatters-adds into the dense [B, H*W] map (duplicates accumulate).

Tie order. tfr breaks label ties with a random shuffle, so the reference loss itself is random on
tied lists. Here (and in the HIP kernel) ties keep a deterministic order: stable descending sort
in which, among equal scores, the element that came LATER in the list goes first (the same rule
the sampler uses). Tests use tie-free labels for exact parity and check tied lists against the
set of losses over all tie permutations.
"""
import numpy as np

LOG_EPS = np.log(1e-10)


def sort_order(scores):
    """Descending order; ties: later position first (stable ascending argsort, reversed)."""
    return np.argsort(scores, axis=-1, kind="stable")[..., ::-1]


def listmle_fwd_bwd(s, labels):
    """Per-list ListMLE. s, labels: [N, L]. Returns (nll [N] fp64, dnll/ds [N, L] fp64)."""
    s = np.asarray(s, np.float64)
    lab = np.asarray(labels, np.float64)
    valid = lab >= 0
    lab0 = np.where(valid, lab, 0.0)
    sv = np.where(valid, s, LOG_EPS)
    score = np.where(valid, lab0, lab0.min(axis=1, keepdims=True) - 1e-6)
    order = sort_order(score)
    t = np.take_along_axis(sv, order, axis=1)
    m = t.max(axis=1, keepdims=True)
    e = np.exp(t - m)
    C = np.cumsum(e[:, ::-1], axis=1)[:, ::-1]
    nll = (np.log(C) - (t - m)).sum(axis=1)
    g_sorted = e * np.cumsum(1.0 / C, axis=1) - 1.0
    g = np.empty_like(g_sorted)
    np.put_along_axis(g, order, g_sorted, axis=1)
    g = np.where(valid, g, 0.0)
    return nll, g


def hourglass_nll(y_true, y_pred, batch_size, ranking_size):
    """``HourglassNegativeLogLikelihood(ranking_size, batch_size)(y_true, y_pred)``.

    y_true: [B, R, L, 2] (float32 flat index, gt); y_pred: [B, H, W(, 1)].
    Returns (loss fp64 scalar, dloss/dy_pred fp64 with y_pred's shape).
    """
    B, L = batch_size, ranking_size
    rk = np.asarray(y_true, np.float32).reshape(B, -1, L, 2)
    pred = np.asarray(y_pred, np.float64).reshape(B, -1)
    idx = rk[..., 0].reshape(B, -1).astype(np.int32)  # tf.cast(float32 -> int32) truncates
    s = np.take_along_axis(pred, idx, axis=1).reshape(-1, L)
    lab = rk[..., 1].reshape(-1, L)
    nll, g = listmle_fwd_bwd(s, lab)
    N = nll.shape[0]
    loss = nll.mean()
    dpred = np.zeros_like(pred)
    gb = (g / N).reshape(B, -1)
    for b in range(B):
        np.add.at(dpred[b], idx[b], gb[b])
    return loss, dpred.reshape(np.shape(y_pred))
