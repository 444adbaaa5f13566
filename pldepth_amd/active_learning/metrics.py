"""Drop-in for ``pldepth/active_learning/metrics.py`` (the metrics ``PLDepth.py:189-192`` reports
after training), computed on the GPU for whole batches of images.

Same names, arguments and results as the reference:
  * ``ordinal_error(op, gt, imsize=(448, 448), num=5000)``   metrics.py:60-70
  * ``calc_err(model, test_im, test_gt, img_size=(448, 448))`` metrics.py:73-80
  * ``calcDCG(rel_list)``                                      metrics.py:83-89
  * ``calc_d(op, gt, imsize=(224, 224), list_size=200)``      metrics.py:92-109
  * ``dcg_metric(model, test_im, test_gt, list_size=200)``    metrics.py:112-120
The random pixel pairs / lists are drawn on the host with the reference's exact numpy calls
(``np.random.seed(10)`` / ``np.random.seed(69)`` + ``np.random.choice(..., replace=False)``, which
also leave the global numpy RNG in the same state); the comparisons, min-max normalisation,
sorting and DCG sums run in ``pld_ordinal_error`` / ``pld_dcg_ratio``. Reference quirks kept:
``dcg_metric`` calls ``calc_d`` without ``imsize``, so lists are drawn from the first 224*224
pixels whatever the image size.

The edge metrics (``depth_edge_metric``, ``calc_depth_metrics``, Hausdorff helpers) need OpenCV's
Canny / distance transform and are not part of this build.
"""
import numpy as np
import torch

from .. import kernels as K


def _pairs(imsize, num):
    np.random.seed(10)
    idx = np.random.choice(list(range(imsize[0] * imsize[1])), num * 2, replace=False)
    idx0, idx1 = np.split(idx, 2)
    return idx0, idx1


def _list_ids(imsize, list_size):
    np.random.seed(69)
    return np.random.choice(np.arange(imsize[0] * imsize[1]), size=list_size, replace=False)


def _dev(a, dtype=torch.float32):
    if isinstance(a, torch.Tensor):
        return a.to(device="cuda", dtype=dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a), dtype=np.float32 if dtype ==
                                                 torch.float32 else np.int32)).cuda()


def _flat(a):
    t = _dev(a)
    return t.reshape(1, -1) if t.dim() <= 3 else t.reshape(t.shape[0], -1)


def _check_ids(ids, hw, who):
    if ids.size and (ids.max() >= hw or ids.min() < 0):
        raise ValueError(f"{who}: sampled index {int(ids.max())} outside an image of {hw} pixels")


def ordinal_error(op, gt, imsize=(448, 448), num=5000):
    """1 - fraction of `num` random pixel pairs whose predicted depth order (op[a] > op[b])
    matches the ground-truth order."""
    idx0, idx1 = _pairs(imsize, num)
    p, g = _flat(op), _flat(gt)
    _check_ids(np.concatenate([idx0, idx1]), p.shape[1], "ordinal_error")
    e = K.ordinal_error(p, g, _dev(idx0, torch.int32), _dev(idx1, torch.int32))
    return float(e[0].item())


def _predict_batches(model, test_im):
    """Inference-mode predictions, device-resident, one engine batch at a time."""
    x = test_im if isinstance(test_im, torch.Tensor) else np.asarray(test_im, np.float32)
    B = model.engine.B
    for i in range(0, x.shape[0], B):
        xb = x[i:i + B]
        k = xb.shape[0]
        if k < B:  # pad the tail batch
            if isinstance(xb, torch.Tensor):
                xb = torch.cat([xb, torch.zeros((B - k,) + tuple(xb.shape[1:]), device=xb.device)])
            else:
                xb = np.concatenate([xb, np.zeros((B - k,) + tuple(xb.shape[1:]), np.float32)])
        yield i, k, model(xb, training=False)[:k]


def calc_err(model, test_im, test_gt, img_size=(448, 448)):
    """Mean ordinal error of the model's predictions over a test set."""
    idx0, idx1 = _pairs(img_size, 5000)
    i0, i1 = _dev(idx0, torch.int32), _dev(idx1, torch.int32)
    errs = []
    for i, k, pred in _predict_batches(model, test_im):
        p = pred.reshape(k, -1).contiguous()
        _check_ids(np.concatenate([idx0, idx1]), p.shape[1], "calc_err")
        g = _dev(np.asarray(test_gt[i:i + k]) if not isinstance(test_gt, torch.Tensor)
                 else test_gt[i:i + k]).reshape(k, -1)
        errs.append(K.ordinal_error(p, g, i0, i1).cpu().numpy())
    return float(np.mean(np.concatenate(errs))) if errs else float("nan")


def calcDCG(rel_list):
    log_i_1 = np.log2(np.arange(np.shape(rel_list)[0]) + 2)
    return (rel_list / log_i_1).sum()


def calc_d(op, gt, imsize=(224, 224), list_size=200):
    """nDCG-style ratio of the sorted (min-max normalised) predicted depths of `list_size` random
    pixels against the sorted ground truth of the same pixels."""
    ids = _list_ids(imsize, list_size)
    p, g = _flat(op), _flat(gt)
    _check_ids(ids, p.shape[1], "calc_d")
    return float(K.dcg_ratio(p, g, _dev(ids, torch.int32))[0].item())


def dcg_metric(model, test_im, test_gt, list_size=200):
    """Mean calc_d over a test set (lists drawn from the first 224*224 pixels, as the reference's
    call without imsize does)."""
    ids = _list_ids((224, 224), list_size)
    idd = _dev(ids, torch.int32)
    out = []
    for i, k, pred in _predict_batches(model, test_im):
        p = pred.reshape(k, -1).contiguous()
        _check_ids(ids, p.shape[1], "dcg_metric")
        g = _dev(np.asarray(test_gt[i:i + k]) if not isinstance(test_gt, torch.Tensor)
                 else test_gt[i:i + k]).reshape(k, -1)
        out.append(K.dcg_ratio(p, g, idd).cpu().numpy())
    return float(np.mean(np.concatenate(out))) if out else float("nan")


def depth_edge_metric(op, gt, imsize=(224, 224)):
    raise NotImplementedError("depth_edge_metric needs OpenCV Canny/distanceTransform "
                              "(not part of this build; SURVEY §2 eval metrics)")


def calc_depth_metrics(model, test_im, test_gt):
    raise NotImplementedError("calc_depth_metrics needs OpenCV Canny/distanceTransform "
                              "(not part of this build; SURVEY §2 eval metrics)")
