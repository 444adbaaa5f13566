"""HR-WSI data access: the tf.image.resize restatement (known answers, CPU),
the HIP resize kernels against it bit for bit, and the data-access object end to end on a
synthetic on-disk HR-WSI tree (GPU)."""
import os

import numpy as np
import pytest

from oracle import resize as OR


def test_oracle_bilinear_known_answers():
    # TF2 half-pixel centres: [a, b] -> [a, .75a + .25b, .25a + .75b, b]; 4 -> 2 averages pairs
    x = np.array([1.0, 5.0], np.float32).reshape(1, 1, 2, 1)
    y = OR.resize_bilinear(x, 1, 4).ravel()
    assert np.array_equal(y, np.array([1.0, 2.0, 4.0, 5.0], np.float32))
    x = np.array([1.0, 3.0, 10.0, 20.0], np.float32).reshape(1, 4, 1, 1)
    assert np.array_equal(OR.resize_bilinear(x, 2, 1).ravel(), np.array([2.0, 15.0], np.float32))
    z = np.random.default_rng(0).random((2, 7, 5, 3), dtype=np.float32)
    assert np.array_equal(OR.resize_bilinear(z, 7, 5), z)  # identity


def test_oracle_nearest_known_answers():
    x = np.arange(4, dtype=np.float32).reshape(1, 1, 4, 1)
    assert np.array_equal(OR.resize_nearest(x, 1, 2).ravel(), np.array([1.0, 3.0], np.float32))
    x = np.arange(2, dtype=np.float32).reshape(1, 1, 2, 1)
    assert np.array_equal(OR.resize_nearest(x, 1, 4).ravel(), np.array([0, 0, 1, 1], np.float32))


def _write_tree(root, sizes, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    for split in ("train", "val"):
        for d in ("imgs", "gts", "valid_masks"):
            os.makedirs(os.path.join(root, split, d), exist_ok=True)
        for i, (h, w) in enumerate(sizes):
            name = f"{split}_{i:03d}"
            Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(
                os.path.join(root, split, "imgs", name + ".jpg"), quality=90)
            Image.fromarray(rng.integers(0, 256, (h, w), dtype=np.uint8)).save(
                os.path.join(root, split, "gts", name + ".png"))
            Image.fromarray((rng.random((h, w)) < 0.9).astype(np.uint8) * 255).save(
                os.path.join(root, split, "valid_masks", name + ".png"))


@pytest.mark.gpu
@pytest.mark.parametrize("h,w,oh,ow,c", [(37, 53, 448, 448, 3), (600, 800, 224, 224, 1),
                                         (448, 448, 448, 448, 3), (31, 17, 64, 80, 2),
                                         (300, 200, 448, 224, 1)])
def test_resize_kernels_match_oracle(cuda, h, w, oh, ow, c):
    import torch
    from pldepth_amd import kernels as K
    x = np.random.default_rng(h).random((2, h, w, c), dtype=np.float32)
    t = torch.from_numpy(x).cuda()
    assert np.array_equal(K.resize(t, oh, ow, "bilinear").cpu().numpy(),
                          OR.resize_bilinear(x, oh, ow))
    assert np.array_equal(K.resize(t, oh, ow, "nearest").cpu().numpy(),
                          OR.resize_nearest(x, oh, ow))


@pytest.mark.gpu
def test_hrwsi_dao_end_to_end(cuda, tmp_path):
    from PIL import Image
    from pldepth_amd.data.dao.hr_wsi import HRWSITFDataAccessObject
    sizes = [(60, 90), (60, 90), (45, 33), (120, 100)]
    _write_tree(str(tmp_path), sizes)
    dao = HRWSITFDataAccessObject(str(tmp_path), (64, 80, 3), seed=3)
    imgs, gts, masks = dao.get_validation_dataset()
    assert imgs.shape == (4, 64, 80, 3) and gts.shape == (4, 64, 80, 1)
    assert masks.shape == (4, 64, 80)
    for i, (h, w) in enumerate(sizes):  # val order = sorted file names
        name = os.path.join(str(tmp_path), "val", "{}", f"val_{i:03d}")
        im = np.asarray(Image.open(name.format("imgs") + ".jpg").convert("RGB"),
                        np.float32)[None] / np.float32(255)
        gt = np.asarray(Image.open(name.format("gts") + ".png").convert("L"),
                        np.float32)[None, ..., None] / np.float32(255)
        mk = np.asarray(Image.open(name.format("valid_masks") + ".png").convert("L"),
                        np.float32)[None, ..., None] / np.float32(255)
        assert np.array_equal(imgs[i], OR.resize_bilinear(im, 64, 80)[0])
        assert np.array_equal(gts[i], OR.resize_bilinear(gt, 64, 80)[0])
        assert np.array_equal(masks[i], OR.resize_nearest(mk, 64, 80)[0, ..., 0])
    tr = dao.get_training_dataset(size=3)
    assert tr[0].shape == (3, 64, 80, 3)  # seeded shuffle of the train split, first 3
    test = dao.get_test_dataset()
    assert len(test) == 4 and test[0][0].shape == (64, 80, 3) and test[0][1].shape == (64, 80, 1)
