"""Mirror of ``pldepth/data/data_meta.py``: the data-access-object base and the file readers.

``read_file_png`` / ``read_file_jpg`` decode with Pillow on the host (the reference decodes with
tf.image.decode_png / decode_jpeg, data_meta.py:38-43) and scale to [0, 1] float32. PNG decoding
is lossless (identical pixels); JPEG decoders may differ from libjpeg-as-built-in-TF in the last
bit of some pixels (unpinned: TF is not installed here).
"""
import abc

import numpy as np
from PIL import Image


class TFDataAccessObject(abc.ABC):
    @abc.abstractmethod
    def get_training_dataset(self):
        pass

    @abc.abstractmethod
    def get_validation_dataset(self):
        pass

    @abc.abstractmethod
    def get_test_dataset(self):
        pass

    @staticmethod
    def _decode(file_path, num_channels):
        if isinstance(file_path, bytes):
            file_path = file_path.decode()
        with Image.open(file_path) as im:
            im = im.convert("L" if num_channels == 1 else "RGB")
            a = np.asarray(im, dtype=np.uint8)
        if num_channels == 1:
            a = a[..., None]
        return a.astype(np.float32) / np.float32(255.0)

    @staticmethod
    def read_file_png(file_path, num_channels=3):
        return TFDataAccessObject._decode(file_path, num_channels)

    @staticmethod
    def read_file_jpg(file_path, num_channels=3):
        return TFDataAccessObject._decode(file_path, num_channels)
