"""Keras HDF5 weight / model files for the HIP engines.

The reference reads and writes Keras' HDF5 formats through h5py: ``model.load_weights(path)``
(pldepth/PLDepth.py:136-137), ``model.save('....h5')`` (:181), ``ModelCheckpoint('...h5',
monitor='val_loss', save_best_only=True)`` (pldepth/util/tracking_utils.py:21-30) and
``tf.keras.models.load_model`` (run_scripts/rnd_on_info_pretrain.py:98). This module writes the
same layout Keras 2.4's ``hdf5_format`` does (via pldepth_amd.util.hdf5):

  weights file   root attrs ``backend``, ``keras_version``, ``layer_names`` (every layer with
                 weights, in graph order); one group per layer with attr ``weight_names``
                 (``<layer>/<weight>:0``) and the datasets at those (nested) paths;
  model file     root attrs ``model_config`` (JSON), ``training_config``, ``keras_version``,
                 ``backend``; the weights file layout under ``model_weights``; Adam's slots under
                 ``optimizer_weights`` (``Adam/iter:0``, then every ``Adam/<var>/m:0``, ``v:0``,
                 ``vhat:0`` — the amsgrad slot order).

Layer naming follows the Keras graph: EfficientNetB0's own layer names, and for the decoder
layers that pl_hourglass.py:59-96 leaves unnamed, Keras' automatic ``conv2d``, ``conv2d_1``, ...,
``batch_normalization``, ... (a fresh session's names). Loading follows ``load_weights``: by
layer name when every layer of the file is a layer of the model, else by graph order (how Keras
loads a file whose automatic names were numbered in another session), with a shape check per
weight. DepthwiseConv2D kernels are stored [k, k, c, 1] as Keras does.
"""
import json

import numpy as np
import torch

from . import hdf5

KERAS_VERSION = b"2.4.0"
BACKEND = b"tensorflow"
HDF5_OBJECT_HEADER_LIMIT = 64512  # Keras splits larger attributes (hdf5_format.py)


def keras_layout(eng):
    """[(keras_layer, [(keras_weight_name, store, store_name, keras_shape)])] in graph order.

    store: 'params' | 'frozen' | 'stats' | None (a constant the file carries that the engine
    does not train, e.g. the Normalization layer's ``count``)."""
    rename = getattr(eng, "KERAS_RENAME", {})
    items = []
    for sname in ("params", "frozen", "stats"):
        store = getattr(eng, sname)
        for name, shape, _ in store.specs:
            items.append((store.order.get(name, 0), sname, name, shape))
    items.sort(key=lambda t: t[0])
    layers = {}
    for _, sname, name, shape in items:
        layer, rest = name.split("/", 1)
        klayer = rename.get(layer, layer)
        kshape = tuple(shape)
        if rest.endswith("depthwise_kernel") and len(kshape) == 3:
            kshape = kshape + (1,)
        layers.setdefault(klayer, []).append((f"{klayer}/{rest}:0", sname, name, kshape))
    for klayer, extra in getattr(eng, "KERAS_EXTRA_WEIGHTS", {}).items():
        for wname, value in extra:
            layers[klayer].append((f"{klayer}/{wname}:0", None, np.asarray(value), ()))
    return list(layers.items())


def _weight_key(kname):
    """'conv2d_7/kernel:0' -> 'kernel'; 'ffl0/conv0/kernel:0' -> 'conv0/kernel'."""
    return kname.split("/", 1)[1].rsplit(":", 1)[0]


def _save_attr(group, name, values):
    """Keras save_attributes_to_hdf5_group: split attributes above the header limit."""
    data = np.array(values, dtype=f"S{max([len(v) for v in values] + [1])}")
    n_chunks = 1
    while data.nbytes / n_chunks > HDF5_OBJECT_HEADER_LIMIT:
        n_chunks += 1
    if n_chunks == 1:
        group.attrs[name] = data
    else:
        for i, chunk in enumerate(np.array_split(data, n_chunks)):
            group.attrs[f"{name}{i}"] = chunk


def _load_attr(group, name):
    """Keras load_attributes_from_hdf5_group."""
    if name in group.attrs:
        vals = group.attrs[name]
    else:
        vals, i = [], 0
        while f"{name}{i}" in group.attrs:
            vals.extend(list(group.attrs[f"{name}{i}"]))
            i += 1
    return [v.decode("utf8") if isinstance(v, bytes) else str(v) for v in np.atleast_1d(vals)]


def _store_value(eng, sname, name):
    return getattr(eng, sname)[name].detach().cpu().numpy()


def _write_weights(eng, group):
    group.attrs["backend"] = BACKEND
    group.attrs["keras_version"] = KERAS_VERSION
    layout = keras_layout(eng)
    _save_attr(group, "layer_names", [k.encode("utf8") for k, _ in layout])
    for klayer, ws in layout:
        g = group.create_group(klayer)
        _save_attr(g, "weight_names", [w[0].encode("utf8") for w in ws])
        for kname, sname, name, kshape in ws:
            val = name if sname is None else _store_value(eng, sname, name).reshape(kshape)
            g.create_dataset(kname, val)
    return layout


def save_weights(eng, path):
    """model.save_weights('... .h5') (Keras HDF5 weights format)."""
    root = hdf5.Group()
    _write_weights(eng, root)
    hdf5.save(path, root)


def _read_layers(path):
    root = hdf5.load(path)
    wroot = root["model_weights"] if "model_weights" in root else root
    names = _load_attr(wroot, "layer_names")
    layers = []
    for ln in names:
        g = wroot[ln]
        wn = _load_attr(g, "weight_names")
        if wn:
            layers.append((ln, [(w, np.asarray(g[w].data)) for w in wn]))
    return root, layers


def load_weights(eng, path):
    """model.load_weights(path) for a Keras HDF5 weights or model file. Returns the mapping
    mode used ('name' or 'order')."""
    _, flayers = _read_layers(path)
    ours = keras_layout(eng)
    by_name = dict(ours)
    if all(ln in by_name for ln, _ in flayers) and len(flayers) == len(ours):
        pairs, mode = [(by_name[ln], ln, ws) for ln, ws in flayers], "name"
    else:
        if len(flayers) != len(ours):
            raise ValueError(f"You are trying to load a weight file containing {len(flayers)} "
                             f"layers into a model with {len(ours)} layers.")
        pairs, mode = [(o[1], ln, ws) for o, (ln, ws) in zip(ours, flayers)], "order"
    updates = {}
    for mine, fname, fws in pairs:
        fmap = {_weight_key(k): v for k, v in fws}
        for kname, sname, name, kshape in mine:
            key = _weight_key(kname)
            if sname is None:  # a constant the engine does not use (Normalization count)
                continue
            if key not in fmap:
                raise ValueError(f"layer {fname}: weight {key} missing from the file")
            v = fmap[key]
            if tuple(v.shape) != tuple(kshape):
                raise ValueError(f"layer {fname}: weight {key} has shape {v.shape}, the model "
                                 f"expects {kshape}")
            updates[name] = v.astype(np.float32)
    eng.set_weights(updates)
    return mode


def save_model(model, path):
    """model.save('... .h5'): config + weights + Adam(amsgrad) slots (Keras save_model_to_hdf5)."""
    eng = model.engine
    root = hdf5.Group()
    root.attrs["backend"] = BACKEND
    root.attrs["keras_version"] = KERAS_VERSION
    root.attrs["model_config"] = json.dumps({
        "class_name": type(model).__name__,
        "config": {"name": getattr(model, "name", "model"),
                   "input_shape": [eng.H, eng.W, 3], "batch_size": eng.B,
                   "asc_depth_order": bool(model.asc_depth_order)}}).encode("utf8")
    opt = model.optimizer
    if opt is not None:
        root.attrs["training_config"] = json.dumps({
            "loss": type(model.loss).__name__ if model.loss is not None else None,
            "optimizer_config": {"class_name": "Adam", "config": {
                "name": "Adam", "learning_rate": float(opt.lr), "beta_1": opt.beta_1,
                "beta_2": opt.beta_2, "epsilon": opt.epsilon, "amsgrad": True}}}).encode("utf8")
    layout = _write_weights(eng, root.create_group("model_weights"))
    if opt is not None and model.trainer is not None:
        tr = model.trainer
        og = root.create_group("optimizer_weights")
        names, vals = ["Adam/iter:0"], [np.array(int(tr.step_dev.item()) - 1, np.int64)]
        m, v, vh = eng.adam_state()
        trainable = [(kn, name) for _, ws in layout for kn, sn, name, _ in ws
                     if sn == "params"]
        for slot, buf in (("m", m), ("v", v), ("vhat", vh)):
            for kn, name in trainable:
                _, shape, off = next(s for s in eng.params.specs if s[0] == name)
                n = int(np.prod(shape))
                names.append(f"Adam/{kn.rsplit(':', 1)[0]}/{slot}:0")
                vals.append(buf[off:off + n].detach().cpu().numpy().reshape(
                    _keras_shape(eng, name)))
        _save_attr(og, "weight_names", [n.encode("utf8") for n in names])
        for n, val in zip(names, vals):
            og.create_dataset(n, val)
    hdf5.save(path, root)


def _keras_shape(eng, name):
    for _, ws in keras_layout(eng):
        for kn, sn, nm, ks in ws:
            if nm == name:
                return ks
    raise KeyError(name)


def read_model_config(path):
    root = hdf5.load(path)
    cfg = root.attrs.get("model_config")
    if cfg is None:
        raise ValueError(f"{path}: no model_config (a weights-only file; use load_weights)")
    if not isinstance(cfg, str):  # fixed-length bytes (Keras' .encode) or a vlen str (h5py str)
        cfg = bytes(np.asarray(cfg)).decode("utf8")
    return json.loads(cfg)


def load_optimizer_state(model, path):
    """Restore Adam(amsgrad) slots + iteration count saved by save_model (if present)."""
    root = hdf5.load(path)
    if "optimizer_weights" not in root or model.trainer is None:
        return False
    og = root["optimizer_weights"]
    eng = model.engine
    m, v, vh = eng.adam_state()
    by_kname = {}
    for _, ws in keras_layout(eng):
        for kn, sn, name, _ in ws:
            if sn == "params":
                by_kname[kn.rsplit(":", 1)[0]] = name
    for wn in _load_attr(og, "weight_names"):
        val = np.asarray(og[wn].data)
        if wn == "Adam/iter:0":
            model.trainer.step_dev.fill_(int(val) + 1)
            continue
        var, slot = wn[len("Adam/"):].rsplit(":", 1)[0].rsplit("/", 1)
        _, shape, off = next(s for s in eng.params.specs if s[0] == by_kname[var])
        buf = {"m": m, "v": v, "vhat": vh}[slot]
        n = int(np.prod(shape))
        buf[off:off + n].copy_(torch.from_numpy(val.reshape(-1).astype(np.float32)))
    return True
