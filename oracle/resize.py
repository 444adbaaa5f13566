"""CPU restatement of tf.image.resize as the HR-WSI data-access object uses it (TEST
INFRASTRUCTURE ONLY — the product path is pldepth_amd/csrc/resize.hip).

pldepth/data/dao/hr_wsi.py:65-74: images and depth maps BILINEAR, masks NEAREST_NEIGHBOR, TF2
defaults (antialias=False, half_pixel_centers=True), restated from TF's resize kernels
(resize_bilinear_op.cc compute_interpolation_weights / compute_lerp with HalfPixelScaler;
resize_nearest_neighbor_op.cc with HalfPixelScalerForNN), fp32 arithmetic, un-fused.
**Parity unpinned**: TensorFlow is not installed here and the reference ships no resize fixtures;
the restatement is checked against hand-derived known answers (tests/test_hrwsi.py).
"""
import numpy as np


def _f(x):
    return np.float32(x)


def _weights(in_size, out_size):
    scale = _f(in_size) / _f(out_size)
    src = (np.arange(out_size, dtype=np.float32) + _f(0.5)) * scale - _f(0.5)
    fl = np.floor(src)
    lower = np.maximum(fl.astype(np.int64), 0)
    upper = np.minimum(np.ceil(src).astype(np.int64), in_size - 1)
    return lower, upper, (src - fl).astype(np.float32)


def resize_bilinear(x, oh, ow):
    """x: [n, h, w, c] float32 -> [n, oh, ow, c]."""
    x = np.asarray(x, np.float32)
    y0, y1, ly = _weights(x.shape[1], oh)
    x0, x1, lx = _weights(x.shape[2], ow)
    lx = lx[None, None, :, None]
    ly = ly[None, :, None, None]
    tl, tr = x[:, y0][:, :, x0], x[:, y0][:, :, x1]
    bl, br = x[:, y1][:, :, x0], x[:, y1][:, :, x1]
    top = tl + (tr - tl) * lx
    bot = bl + (br - bl) * lx
    return (top + (bot - top) * ly).astype(np.float32)


def resize_nearest(x, oh, ow):
    x = np.asarray(x)
    sy = _f(x.shape[1]) / _f(oh)
    sx = _f(x.shape[2]) / _f(ow)
    iy = np.minimum(np.floor((np.arange(oh, dtype=np.float32) + _f(0.5)) * sy).astype(np.int64),
                    x.shape[1] - 1)
    ix = np.minimum(np.floor((np.arange(ow, dtype=np.float32) + _f(0.5)) * sx).astype(np.int64),
                    x.shape[2] - 1)
    return x[:, iy][:, :, ix]
