"""Models: the reference's factories (PLDepthNet, pl_hourglass, redweb) over the HIP engines."""


def load_model(filepath, custom_objects=None, compile=True):
    """tf.keras.models.load_model for a file written by ``model.save('... .h5')``
    (run_scripts/rnd_on_info_pretrain.py:98): rebuilds the model from its ``model_config``,
    loads the weights, and — once the caller compiles it (the loss is a custom object Keras too
    would need ``custom_objects`` for) — the saved Adam slots and iteration count.
    ``custom_objects`` is accepted for signature compatibility and unused."""
    from ..util import keras_h5
    from .pl_hourglass import EffNetFullyFledged
    from .redweb import ReDWebNetTFVersion
    cfg = keras_h5.read_model_config(filepath)
    classes = {"EffNetFullyFledged": EffNetFullyFledged, "ReDWebNetTFVersion": ReDWebNetTFVersion}
    cls = classes.get(cfg["class_name"])
    if cls is None:
        raise ValueError(f"unknown model class {cfg['class_name']!r} in {filepath}")
    c = cfg["config"]
    model, _ = cls.get_model_and_normalization(c["input_shape"], None,
                                               batch_size=c["batch_size"])
    model.asc_depth_order = c.get("asc_depth_order", False)
    model.load_weights(filepath)
    model._pending_optimizer_state = filepath
    return model
