"""Keras HDF5 weight files (reference PLDepth.py:136-137,180-181,
tracking_utils.py:21-30). h5py / libhdf5 are not installed anywhere in this image, so parity
with files written by the reference's Keras is UNPINNED: these tests pin the in-tree HDF5 codec
by round trips and by the byte-level structures the format specification fixes, and the Keras
layout (names, order, shapes) against the reference's graph."""
import struct

import numpy as np
import pytest
import torch

from pldepth_amd.util import hdf5
from pldepth_amd.util import keras_h5


def _cpu_engine(H=64, seed=0):
    from pldepth_amd.models import effnet_ff as E

    class _CPU(E.EffNetFF):
        def __init__(self):
            self.H, self.W, self.B = H, H, 1
            self.device = torch.device("cpu")
            self.params, self.frozen, self.stats = E.FlatStore(), E.FlatStore(), E.FlatStore()
            self.bns, self.convs = [], []
            self._build_spec()
            for s in (self.params, self.frozen, self.stats):
                s.materialize("cpu")

        def set_weights(self, w):
            for store in (self.params, self.frozen, self.stats):
                for name, shape, _ in store.specs:
                    if name in w:
                        store[name].copy_(torch.as_tensor(np.asarray(w[name], np.float32)
                                                          .reshape(shape)))

    e = _CPU()
    e.init_weights(seed)
    return e


def test_hdf5_round_trip_groups_datasets_attrs(tmp_path):
    root = hdf5.Group({"names": np.array([b"a", b"bcd"]), "s": "tensorflow",
                       "i": np.int64(-3), "f": np.array([1.5, 2.5], np.float32)})
    rng = np.random.default_rng(0)
    arrays = {}
    for i in range(70):  # > one symbol-table node per group
        p = f"g{i % 7}/layer{i}/kernel:0"
        arrays[p] = rng.standard_normal((i % 4 + 1, 3)).astype(np.float32 if i % 2 else
                                                                 np.float64)
        root.create_dataset(p, arrays[p])
    root.create_dataset("scalar", np.array(7, np.int64))
    root.create_dataset("u8", np.arange(5, dtype=np.uint8))
    root.create_dataset("empty", np.zeros((0, 3), np.float32))
    path = tmp_path / "t.h5"
    hdf5.save(str(path), root)
    assert hdf5.is_hdf5(str(path))
    r = hdf5.load(str(path))
    for p, a in arrays.items():
        b = r[p].data
        assert b.dtype == a.dtype and np.array_equal(a, b), p
    assert int(r["scalar"].data) == 7 and r["scalar"].data.shape == ()
    assert np.array_equal(r["u8"].data, np.arange(5))
    assert r["empty"].data.shape == (0, 3)
    assert list(r.attrs["names"]) == [b"a", b"bcd"]
    assert bytes(r.attrs["s"]) == b"tensorflow" and int(r.attrs["i"]) == -3
    assert np.array_equal(r.attrs["f"], [1.5, 2.5])


def test_hdf5_superblock_and_group_structures(tmp_path):
    """Superblock v0 fields, symbol-table entry of the root, local heap and B-tree signatures at
    the addresses the file records (HDF5 format spec, 'Disk Format: Level 0/1')."""
    root = hdf5.Group()
    root.create_dataset("x", np.ones(3, np.float32))
    path = tmp_path / "s.h5"
    hdf5.save(str(path), root)
    raw = path.read_bytes()
    assert raw[:8] == b"\x89HDF\r\n\x1a\n"
    assert raw[8:16] == bytes([0, 0, 0, 0, 0, 8, 8, 0])
    leaf_k, int_k = struct.unpack_from("<HH", raw, 16)
    assert leaf_k >= 4 and int_k == 16
    base, free, eof, drv = struct.unpack_from("<QQQQ", raw, 24)
    assert base == 0 and free == drv == hdf5.UNDEF and eof == len(raw)
    _, oh, cache, _, bt, hp = struct.unpack_from("<QQIIQQ", raw, 56)
    assert cache == 1 and raw[oh] == 1  # object header version 1
    assert raw[bt:bt + 4] == b"TREE" and raw[hp:hp + 4] == b"HEAP"


def test_keras_layout_names_order_and_shapes():
    eng = _cpu_engine()
    layout = keras_h5.keras_layout(eng)
    names = [n for n, _ in layout]
    # graph order of the weighted layers: Normalization, stem, block1a, ..., top, decoder
    assert names[:9] == ["normalization", "stem_conv", "stem_bn", "block1a_dwconv", "block1a_bn",
                         "block1a_se_reduce", "block1a_se_expand", "block1a_project_conv",
                         "block1a_project_bn"]
    assert names[9:11] == ["block2a_expand_conv", "block2a_expand_bn"]
    assert names[-13:] == ["top_conv", "top_bn", "conv2d", "batch_normalization", "conv2d_1",
                           "batch_normalization_1", "conv2d_2", "batch_normalization_2",
                           "conv2d_3", "batch_normalization_3", "conv2d_4",
                           "batch_normalization_4", "conv2d_5"]
    d = dict(layout)
    assert [w[0] for w in d["stem_bn"]] == ["stem_bn/gamma:0", "stem_bn/beta:0",
                                            "stem_bn/moving_mean:0", "stem_bn/moving_variance:0"]
    assert [w[0] for w in d["conv2d_5"]] == ["conv2d_5/kernel:0", "conv2d_5/bias:0"]
    assert d["conv2d"][0][3] == (3, 3, 1280, 672)
    assert d["block2a_dwconv"][0][3] == (3, 3, 96, 1)  # DepthwiseConv2D kernel [k,k,c,1]
    assert [w[0] for w in d["normalization"]] == ["normalization/mean:0",
                                                  "normalization/variance:0",
                                                  "normalization/count:0"]
    # 49 encoder BNs + 5 decoder BNs, 16 depthwise, 6 decoder convs
    assert sum(n.endswith("bn") or n.startswith("batch_normalization") for n in names) == 54
    assert len(layout) == 3 + 16 * 6 + 15 * 2 + 2 + 11


def test_keras_weights_round_trip_by_name_and_by_order(tmp_path):
    src, dst = _cpu_engine(seed=1), _cpu_engine(seed=2)
    path = str(tmp_path / "w.h5")
    keras_h5.save_weights(src, path)
    assert keras_h5.load_weights(dst, path) == "name"
    a, b = src.get_weights(), dst.get_weights()
    assert set(a) == set(b) and all(np.array_equal(a[k], b[k]) for k in a)
    # a file from a session whose automatic decoder names were numbered differently
    # (conv2d_6 ...): Keras' load_weights maps by graph order
    root = hdf5.load(path)
    ren = hdf5.Group(dict(root.attrs))
    names = keras_h5._load_attr(root, "layer_names")
    new_names = []
    for n in names:
        m = {"conv2d": "conv2d_6", "batch_normalization": "batch_normalization_5"}.get(n, n)
        if m.startswith("conv2d_") and n != "conv2d":
            m = f"conv2d_{int(n.split('_')[1]) + 6}"
        new_names.append(m)
        g = ren.create_group(m)
        wn = keras_h5._load_attr(root[n], "weight_names")
        g.attrs["weight_names"] = np.array([(m + w[len(n):]).encode() for w in wn])
        for w in wn:
            g.create_dataset(m + w[len(n):], root[n][w].data)
    ren.attrs["layer_names"] = np.array([n.encode() for n in new_names])
    p2 = str(tmp_path / "w2.h5")
    hdf5.save(p2, ren)
    dst2 = _cpu_engine(seed=3)
    assert keras_h5.load_weights(dst2, p2) == "order"
    c = dst2.get_weights()
    assert all(np.array_equal(a[k], c[k]) for k in a)


def test_keras_weights_mismatch_raises(tmp_path):
    src = _cpu_engine()
    path = str(tmp_path / "w.h5")
    keras_h5.save_weights(src, path)
    root = hdf5.load(path)
    names = keras_h5._load_attr(root, "layer_names")
    root.attrs["layer_names"] = np.array([n.encode() for n in names[:-1]])
    p2 = str(tmp_path / "short.h5")
    hdf5.save(p2, root)
    with pytest.raises(ValueError, match="containing"):
        keras_h5.load_weights(_cpu_engine(), p2)
    bad = hdf5.load(path)
    k = "conv2d_5/conv2d_5/kernel:0"
    bad["conv2d_5"].members["conv2d_5"].members["kernel:0"] = hdf5.Dataset(
        np.zeros((3, 3, 32, 2), np.float32))
    p3 = str(tmp_path / "shape.h5")
    hdf5.save(p3, bad)
    with pytest.raises(ValueError, match="shape"):
        keras_h5.load_weights(_cpu_engine(), p3)
    assert k


def test_model_checkpoint_saves_only_on_improvement(tmp_path):
    from pldepth_amd.util.training_utils import ModelCheckpoint

    class _M:
        saved = []

        def save(self, p):
            self.saved.append(p)

    cb = ModelCheckpoint(str(tmp_path / "m{epoch:02d}.h5"), monitor="val_loss",
                         save_best_only=True)
    cb.set_model(_M())
    for e, v in enumerate([3.0, 2.0, 2.5, 1.0]):
        cb.on_epoch_end(e, {"val_loss": v, "loss": 0.0})
    assert [p.split("/")[-1] for p in _M.saved] == ["m01.h5", "m02.h5", "m04.h5"]


def _attr_message(raw, oh_addr, name):
    """The body of attribute `name` in the version-1 object header at oh_addr."""
    nmsg, _, size = struct.unpack_from("<HII", raw, oh_addr + 2)
    q = oh_addr + 16
    for _ in range(nmsg):
        mt, ms = struct.unpack_from("<HH", raw, q)
        body = raw[q + 8:q + 8 + ms]
        q += 8 + ms
        if mt == 0x000C:
            nsz = struct.unpack_from("<H", body, 2)[0]
            if body[8:8 + nsz].rstrip(b"\0") == name.encode():
                return body
    raise KeyError(name)


def test_vlen_string_root_attributes_as_h5py_writes_them(tmp_path):
    """h5py stores a Python str attribute as a variable-length UTF-8 string (class 9,
    elements in a global-heap collection). A weights file whose root `backend` /
    `keras_version` and a model file whose `model_config` are vlen strings load through
    keras_h5 (load_weights, read_model_config). The byte layout checked below is the format
    specification's (datatype class 9 v1, 'GCOL' v1 collection >= 4 KiB, 16-byte heap ids);
    no h5py exists here to write a reference file, so parity with h5py output stays unpinned."""
    src, dst = _cpu_engine(seed=4), _cpu_engine(seed=5)
    root = hdf5.Group()
    keras_h5._write_weights(src, root)
    root.attrs["backend"] = hdf5.VLenStr("tensorflow")
    root.attrs["keras_version"] = hdf5.VLenStr("2.4.0")
    path = tmp_path / "vlen.h5"
    hdf5.save(str(path), root)
    raw = path.read_bytes()
    oh = struct.unpack_from("<Q", raw, 64)[0]
    body = _attr_message(raw, oh, "keras_version")
    nsz, tsz, ssz = struct.unpack_from("<HHH", body, 2)
    p = 8 + nsz + (-nsz % 8)
    dt = body[p:p + tsz]
    # class 9 v1, string / null-terminated / UTF-8, size 16, base: 1-byte unsigned int
    assert dt[:8] == bytes([0x19, 0x01, 0x01, 0x00, 16, 0, 0, 0])
    assert dt[8:20] == bytes([0x10, 0, 0, 0, 1, 0, 0, 0, 0, 0, 8, 0])
    p += tsz + (-tsz % 8) + ssz + (-ssz % 8)
    ln, coll, idx = struct.unpack_from("<IQI", body, p)
    assert (ln, idx) == (5, 1) and raw[coll:coll + 4] == b"GCOL" and raw[coll + 4] == 1
    assert struct.unpack_from("<Q", raw, coll + 8)[0] >= 4096
    assert raw[coll + 32:coll + 37] == b"2.4.0"
    r = hdf5.load(str(path))
    assert r.attrs["keras_version"] == "2.4.0" and r.attrs["backend"] == "tensorflow"
    assert keras_h5.load_weights(dst, str(path)) == "name"
    a, b = src.get_weights(), dst.get_weights()
    assert all(np.array_equal(a[k], b[k]) for k in a)
    # model file: model_config as a vlen str
    root.attrs["model_config"] = hdf5.VLenStr('{"class_name": "FullyFledgedModel"}')
    hdf5.save(str(path), root)
    assert keras_h5.read_model_config(str(path)) == {"class_name": "FullyFledgedModel"}


def test_unsupported_attribute_type_is_skipped(tmp_path):
    """An attribute of a datatype the reader does not decode (here: class 6, compound) is
    skipped with a warning; the rest of the file still loads."""
    root = hdf5.Group({"keep": np.int64(3), "odd": np.int64(5)})
    root.create_dataset("x", np.ones(2, np.float32))
    path = tmp_path / "u.h5"
    hdf5.save(str(path), root)
    raw = bytearray(path.read_bytes())
    oh = struct.unpack_from("<Q", raw, 64)[0]
    body = _attr_message(bytes(raw), oh, "odd")
    at = bytes(raw).index(body)
    nsz = struct.unpack_from("<H", body, 2)[0]
    dpos = at + 8 + nsz + (-nsz % 8)
    raw[dpos] = (1 << 4) | 6  # datatype class -> compound
    path.write_bytes(bytes(raw))
    with pytest.warns(UserWarning, match="attribute skipped"):
        r = hdf5.load(str(path))
    assert "odd" not in r.attrs and int(r.attrs["keep"]) == 3
    assert np.array_equal(r["x"].data, [1, 1])
