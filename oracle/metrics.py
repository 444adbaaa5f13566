"""CPU restatement of the test-pass metrics (TEST INFRASTRUCTURE ONLY — imported by tests/ as
the checker; the product path is pldepth_amd/csrc/metrics.hip).

  ordinal_error  pldepth/active_learning/metrics.py:60-70
  calc_d         metrics.py:92-109 (+ calcDCG :83-89)

Index draws are taken as arguments (the reference's np.random.seed + choice calls are
reproduced by pldepth_amd.active_learning.metrics and by the golden-vector script).
cv2.normalize(op, None, 0, 1, cv2.NORM_MINMAX) is restated from OpenCV's documented formula
(scale = 1/(max - min), 0 when max - min <= DBL_EPSILON; shift = -min*scale; fp32 result):
OpenCV is not installed here, so that one step is unpinned.
Pinned by tests/golden/metrics_golden.npz (tests/golden/make_metrics_golden.py: the reference's
metrics functions run in this container on seeded inputs).
"""
import numpy as np


def ordinal_error(op, gt, idx0, idx1):
    """metrics.py:64-70 with the pair indices given."""
    op_flat = np.asarray(op).flatten()
    gt_flat = np.asarray(gt).flatten()
    out_order = np.greater(op_flat[idx0], op_flat[idx1])
    gt_order = np.greater(gt_flat[idx0], gt_flat[idx1])
    return 1 - np.equal(out_order, gt_order).sum() / len(idx0)


def minmax_normalize(op):
    """cv2.normalize(op, None, 0, 1, cv2.NORM_MINMAX) on float32 (metrics.py:93)."""
    op = np.asarray(op, np.float32)
    smin, smax = float(op.min()), float(op.max())
    scale = 1.0 / (smax - smin) if (smax - smin) > np.finfo(np.float64).eps else 0.0
    shift = -smin * scale
    return (op.astype(np.float64) * scale + shift).astype(np.float32)


def calc_dcg(rel_list):
    """metrics.py:83-89."""
    log_i_1 = np.log2(np.arange(np.shape(rel_list)[0]) + 2)
    return (rel_list / log_i_1).sum()


def calc_d(op, gt, ids):
    """metrics.py:92-109 with the list indices given."""
    op_flat = minmax_normalize(op).flatten()
    gt_flat = np.asarray(gt).flatten()
    sorted_dist_list = np.sort(op_flat[ids])
    sorted_gt_list = np.sort(gt_flat[ids])
    rel_dist_list = 1 / (sorted_dist_list + 1)
    rel_gt = 1 / (sorted_gt_list + 1)
    return calc_dcg(rel_dist_list) / calc_dcg(rel_gt)
