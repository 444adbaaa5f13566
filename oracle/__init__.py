"""CPU oracle for the PLDepth training hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker (or the timed CPU baseline). The product path
(``pldepth_amd``) never imports it and has no CPU fallback: it fails loudly when the HIP library
is missing.

Contents (each function cites the reference file:line it restates):
  * ``oracle.sampler``  — numpy restatement of the ranking samplers
                          (``pldepth/data/sampling.py``), pinned bit-for-bit against golden
                          vectors captured from the reference itself (``tests/golden``).
  * ``oracle.listmle``  — numpy fp64 restatement of ``prepare_fully_fledged_loss_input``
                          (``pldepth/data/depth_utils.py:39-61``) + tensorflow_ranking 0.3.1
                          ``ListMLELoss`` (third-party, not vendored: parity unpinned — no TF here).
  * ``oracle.effnet``   — torch-CPU (fp64) restatement of the ``ff_effnet`` graph
                          (``pldepth/models/pl_hourglass.py:45-100`` + Keras EfficientNetB0
                          semantics; third-party, parity unpinned).
  * ``oracle.adam``     — Keras/TF Adam(amsgrad=True) update (``pldepth/PLDepth.py:133``).
  * ``oracle.sgdr``     — ``SGDRScheduler`` (``pldepth/util/training_utils.py:20-97``).
"""
