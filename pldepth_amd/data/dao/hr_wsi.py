"""Drop-in for ``pldepth/data/dao/hr_wsi.py``: the HR-WSI on-disk layout
``<root>/{train,val}/imgs/*.jpg`` + ``gts/*.png`` + ``valid_masks/*.png``.

Same class, constructor and methods as the reference (hr_wsi.py:8-83). Files are decoded on the
host (Pillow, a thread pool) and resized on the GPU (``pld_resize_bilinear`` for images and depth
maps, ``pld_resize_nearest`` for masks — tf.image.resize's TF2 semantics); the datasets come back
as stacked arrays (images [N,H,W,3], depths [N,H,W,1], masks [N,H,W]) — the element shapes of
the reference's tf.data pipelines — ready for ``HourglassLargeScaleDataProvider``.
Differences: file order for ``shuffle=True`` is a seeded numpy permutation of the sorted file list
(TF's list_files shuffle is not reproducible without TF); ``size`` takes the first ``size`` files.
"""
import glob
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from ... import kernels as K
from ..data_meta import TFDataAccessObject


class HRWSITFDataAccessObject(TFDataAccessObject):
    def __init__(self, root_path, target_shape, seed):
        self.root_path = root_path
        self.target_shape = tuple(target_shape[:2])
        self.seed = seed

    def get_training_dataset(self, size=None):
        return self.construct_raw_file_dataset('train', zip_ds=False, shuffle=True, size=size)

    def get_validation_dataset(self, size=None):
        return self.construct_raw_file_dataset('val', zip_ds=False, shuffle=False, size=size)

    def get_test_dataset(self, zip_ds=True, exclude_mask=True):
        imgs, gts, masks = self.construct_raw_file_dataset('val', zip_ds=False, shuffle=False)
        if exclude_mask:
            return list(zip(imgs, gts)) if zip_ds else (imgs, gts)
        return list(zip(imgs, gts, masks)) if zip_ds else (imgs, gts, masks)

    def get_combined_dataset(self):
        return self.construct_raw_file_dataset('*', zip_ds=False, shuffle=True)

    def get_file_dataset(self, file_names, file_extension=".jpg"):
        if file_extension == ".jpg":
            fn = self.read_file_jpg
        elif file_extension == ".png":
            def fn(f):
                return self.read_file_png(f, num_channels=1)
        else:
            raise NotImplementedError("Unsupported file extension '{}'.".format(file_extension))
        with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
            return list(ex.map(fn, file_names))

    def _resize(self, arrays, method):
        """Resize a list of [h, w, c] arrays (equal shapes batched per launch) on the GPU."""
        H, W = self.target_shape
        out = np.empty((len(arrays), H, W, arrays[0].shape[-1]) if arrays else (0, H, W, 1),
                       np.float32)
        i = 0
        while i < len(arrays):
            j = i
            while j < len(arrays) and arrays[j].shape == arrays[i].shape and j - i < 64:
                j += 1
            x = torch.from_numpy(np.stack(arrays[i:j])).cuda()
            out[i:j] = K.resize(x, H, W, method).cpu().numpy()
            i = j
        return out

    def construct_raw_file_dataset(self, set_indicator, zip_ds=True, shuffle=False, size=None):
        file_names_imgs = sorted(glob.glob(os.path.join(self.root_path, set_indicator, "imgs",
                                                        "*.jpg")))
        if shuffle:
            file_names_imgs = [file_names_imgs[i] for i in
                               np.random.RandomState(self.seed).permutation(len(file_names_imgs))]
        if size:
            file_names_imgs = file_names_imgs[:size]
        file_names_gts = [s.replace('imgs', 'gts').replace('.jpg', '.png') for s in file_names_imgs]
        file_names_masks = [s.replace('imgs', 'valid_masks').replace('.jpg', '.png')
                            for s in file_names_imgs]
        imgs = self._resize(self.get_file_dataset(file_names_imgs, ".jpg"), "bilinear")
        gts = self._resize(self.get_file_dataset(file_names_gts, ".png"), "bilinear")
        masks = self._resize(self.get_file_dataset(file_names_masks, ".png"), "nearest")[..., 0]
        if zip_ds:
            return list(zip(imgs, gts, masks))
        return imgs, gts, masks
