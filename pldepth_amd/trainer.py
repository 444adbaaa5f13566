"""One data-parallel replica of the PLDepth training step, end to end on the GPU.

Replaces, per step, what ``model.fit`` (pldepth/PLDepth.py:176) drives: the ranking sampler the
reference runs on the host under tf.numpy_function (hourglass_provider.py:55-58 ->
sampling.py), the ff_effnet forward/backward (pl_hourglass.py:45-100), the ListMLE loss
(nll_loss.py:32-62) and Adam(amsgrad) (PLDepth.py:133) — plus, for N > 1 GPUs, the gradient
all-reduce the reference never had: one process per GPU, torch.distributed with the
"nccl" backend (= RCCL over xGMI), per-rank batch B, BN statistics per replica (MirroredStrategy
semantics), one fp32 all-reduce of the flat gradient buffer, 1/world folded into Adam.

Stepping: the whole step is stream-ordered HIP work with no host synchronisation, replayed from
hipGraphs captured after a first eager step. Inside the backward the decoder's weight gradients
run on a side stream concurrently with the rest of the chain (engine.overlap_wgrad). N = 1: one
graph per step. N > 1: the compute (sampler -> forward -> ListMLE -> backward) is one graph;
then the gradient is all-reduced in ~8 MB tensor-aligned buckets in reverse layer order (RCCL on
its own stream, issued through torch.distributed between graph launches), and a side stream runs
each bucket's Adam-AMSGrad + filter refresh (one captured graph per bucket) as soon as it lands —
the exchange overlaps the optimizer step. Per-step scalars (learning rate, step counter) live in
device memory.
"""
import os

import numpy as np
import torch

from . import dp
from . import kernels as K
from .models.effnet_ff import EffNetFF
from .models.redweb_ff import RedWebFF

ENGINES = {"ff_effnet": EffNetFF, "ff_redweb": RedWebFF, "ff_resnet": RedWebFF}

SAMPLING_TYPES = {0: "thresh", 1: "info", 3: "pure"}  # PLDepth.py:97-108 --sampling_type


class ReplicaTrainer:
    def __init__(self, input_shape=(448, 448, 3), batch_size=32, ranking_size=5,
                 rankings_per_image=100, sampling_type=1, seed=0, rank=0, world_size=1,
                 process_group=None, model="ff_effnet", drop_connect=True, engine=None,
                 gpu_sampler=True, beta_1=0.9, beta_2=0.999, epsilon=1e-7, dp_overlap=None):
        """gpu_sampler=False: rankings come from the caller (set_rankings), as model.fit feeds
        y_true batches; otherwise the GPU sampler draws them from (gt, mask) each step.
        dp_overlap (N > 1; default from PLD_DP_OVERLAP, on): all-reduce the decoder's gradient
        buckets while the encoder's backward runs (engines with backward_decoder /
        backward_encoder and deferred weight gradients; others take the post-backward
        exchange)."""
        if engine is None and model not in ENGINES:
            raise ValueError(f"unknown model {model!r} (expected one of {sorted(ENGINES)})")
        self.gpu_sampler = gpu_sampler
        self.betas = (beta_1, beta_2, epsilon)
        self.B, self.L, self.R = batch_size, ranking_size, rankings_per_image
        self.H, self.W = input_shape[:2]
        self.strategy = SAMPLING_TYPES[sampling_type] if isinstance(sampling_type, int) \
            else sampling_type
        self.rank, self.world = rank, world_size
        self.pg = process_group
        self.seed = seed
        dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.engine = engine if engine is not None else ENGINES[model](input_shape, batch_size,
                                                                       device=dev, seed=seed)
        self.engine.drop_connect = drop_connect
        B, H, W, L, R = self.B, self.H, self.W, self.L, self.R
        self.n_cand = K.sampler_candidates(R, self.strategy)
        self.R_out = self.n_cand if self.strategy == "pure" else R
        # data (resident in HBM): image batch lives in the engine's input buffer
        self.x = self.engine.act["input"]
        self.gt = torch.zeros(B, H, W, device=dev)
        self.mask = torch.ones(B, H, W, device=dev)
        # sampler state
        self.valid_idx = torch.empty(B, H * W, dtype=torch.int32, device=dev)
        self.nvalid = torch.empty(B, dtype=torch.int32, device=dev)
        self.minmax = torch.empty(B, 2, device=dev)
        self.draws = torch.empty(B, self.n_cand, L, dtype=torch.int32, device=dev)
        self.y_true = torch.empty(B, self.R_out, L, 2, device=dev)
        # loss state
        self.nll = torch.empty(B * self.R_out, device=dev)
        self.loss = torch.zeros(1, device=dev)
        self.dpred = torch.empty(B, H, W, 1, device=dev)
        # per-step scalars on the device
        self.step_dev = torch.ones(1, dtype=torch.int64, device=dev)
        self.lr_dev = torch.full((1,), 0.01, device=dev)
        self.m, self.v, self.vhat = self.engine.adam_state()
        self.graphs = None
        self.stream = torch.cuda.Stream(device=dev)
        self.side = torch.cuda.Stream(device=dev)  # per-bucket optimizer updates (N > 1)
        if dp_overlap is None:  # (an explicit True also serves a single-rank group: tests)
            dp_overlap = world_size > 1 and os.environ.get("PLD_DP_OVERLAP", "1") == "1"
        eng = self.engine
        self.dp_overlap = bool(dp_overlap and hasattr(eng, "backward_decoder")
                               and getattr(eng, "overlap_wgrad", 0) == 2)
        if self.dp_overlap:
            # the decoder's weight gradients and, after them, the decoder buckets' all-reduces
            self.wside = torch.cuda.Stream(device=dev)
            self._ev_dec = torch.cuda.Event()
            # timing marks of the last overlapped step (tests): the first all-reduce issued on
            # wside, the end of the encoder backward on the trainer stream
            self._ev_ar = torch.cuda.Event(enable_timing=True)
            self._ev_bwd = torch.cuda.Event(enable_timing=True)

    # ------------------------------------------------------------------ data
    def set_batch(self, images, gt, mask):
        """images [B,H,W,3] model input (the [0,1] images after the model's preprocess_fn:
        identity for ff_effnet, caffe mean subtraction for ff_redweb), gt [B,H,W], mask [B,H,W]
        (>0 valid) — host or device.
        The copies are ordered on the trainer's stream (before the next step's kernels), after
        whatever the caller's current stream has queued (e.g. the sampler or a producer kernel
        that wrote a device source)."""
        self._order_after_caller()
        with torch.cuda.stream(self.stream):
            for src, dst in ((images, self.x), (gt, self.gt), (mask, self.mask)):
                if src is not None:
                    t = torch.as_tensor(src, dtype=torch.float32)
                    dst.copy_(t.reshape(dst.shape))
                    self._keep_alive(t)

    def _order_after_caller(self):
        """The trainer's stream waits for the caller's current stream: device tensors handed
        to set_batch / set_rankings may still be in flight there."""
        cur = torch.cuda.current_stream(self.device)
        if cur != self.stream:
            self.stream.wait_stream(cur)

    def _keep_alive(self, t):
        """A device source freed by the caller must not be recycled before the trainer stream's
        copy has read it (caching-allocator reuse across streams)."""
        if t.is_cuda:
            t.record_stream(self.stream)

    def set_rankings(self, y_true):
        """External rankings [B, R, L, 2] (float32 flat index, depth) for the next step."""
        y = torch.as_tensor(y_true, dtype=torch.float32)
        R = y.numel() // (2 * self.B * self.L)
        if R != self.R_out or self.y_true.numel() != y.numel():
            if self.graphs is not None:
                raise ValueError("ranking count changed after graph capture")
            self.R_out = R
            self.y_true = torch.empty(self.B, R, self.L, 2, device=self.device)
            self.nll = torch.empty(self.B * R, device=self.device)
        self._order_after_caller()
        with torch.cuda.stream(self.stream):
            self.y_true.copy_(y.reshape(self.y_true.shape))
            self._keep_alive(y)

    # ------------------------------------------------------------------ phases
    def _sample(self):
        if not self.gpu_sampler:
            return
        K.sampler_compact(self.mask, self.gt, self.valid_idx, self.nvalid, self.minmax)
        K.sampler_draw(self.nvalid, self.n_cand, self.L, self.seed, self.step_dev,
                       self.rank * self.B, self.draws)
        K.sampler_rank(self.gt, self.valid_idx, self.nvalid, self.minmax, self.draws, self.R,
                       self.L, self.strategy, self.y_true)

    def _fwd_loss(self):
        eng = self.engine
        eng.forward(training=True, step=self.step_dev, image_offset=self.rank * self.B)
        K.listmle_fwd_bwd(eng.act["pred"], self.y_true, self.B, self.R_out, self.L,
                          dpred=self.dpred, nll=self.nll, loss=self.loss, zero_dpred=True)

    def _fwd_bwd(self):
        self._fwd_loss()
        self.engine.backward(self.dpred)

    def _update(self):
        eng = self.engine
        b1, b2, eps = self.betas
        K.adam_amsgrad_dev(eng.params.buf, eng.grads.buf, self.m, self.v, self.vhat, self.lr_dev,
                           self.step_dev, b1, b2, eps, grad_scale=1.0 / self.world)
        eng.refresh_trainable()
        K.step_increment(self.step_dev)

    # ------------------------------------------------------------------ data parallel
    BUCKET_BYTES = 8 << 20

    def _dp_buckets(self):
        """Reverse-order, tensor-aligned gradient buckets (dp.tensor_buckets), built once."""
        if not hasattr(self, "_buckets"):
            eng = self.engine
            self._buckets = dp.tensor_buckets([off for _, _, off in eng.params.specs],
                                              eng.grads.buf.numel(), self.BUCKET_BYTES)
        return self._buckets

    def _dp_refresh_convs(self, lo, hi):
        """Trainable convs whose kernel lies in flat range [lo, hi)."""
        eng = self.engine
        return [c for c in eng.convs if c.trainable and lo <= eng.param_offset(c.wk) < hi]

    def _dp_update(self, lo, hi):
        """Adam-AMSGrad of flat range [lo, hi) (grad_scale 1/world) and the refresh of the
        native filter copies of the convs in it, on the current (side) stream."""
        eng = self.engine
        b1, b2, eps = self.betas
        K.adam_amsgrad_dev(eng.params.buf[lo:hi], eng.grads.buf[lo:hi], self.m[lo:hi],
                           self.v[lo:hi], self.vhat[lo:hi], self.lr_dev, self.step_dev, b1, b2,
                           eps, grad_scale=1.0 / self.world)
        for c in self._dp_refresh_convs(lo, hi):
            c.refresh()

    def _dp_exchange(self, updates=None):
        """After the backward (on self.stream): each bucket's all-reduce (RCCL, ordered after
        the backward by c10d) and, on the side stream as soon as it lands, that bucket's update
        — eager (_dp_update) or its captured graph (updates[i]); the updates of the first
        buckets overlap the all-reduces of the later ones. Then the step counter advances (Adam's
        bias correction and the next step's Philox keys read it)."""
        grads = self.engine.grads.buf
        self.side.wait_stream(self.stream)
        works = []
        for i, (lo, hi) in enumerate(self._dp_buckets()):
            work = dp.allreduce_bucket(grads, lo, hi, self.pg)
            with torch.cuda.stream(self.side):
                work.wait()
                if updates is None:
                    self._dp_update(lo, hi)
                else:
                    updates[i].launch()
            works.append(work)
        self._dp_works = works
        self.stream.wait_stream(self.side)
        K.step_increment(self.step_dev)

    def _dp_decoder_split(self):
        """Index of the first bucket holding an encoder tensor: buckets [0, split) hold only
        decoder tensors (final once the decoder backward and its weight gradients are)."""
        if not hasattr(self, "_dp_split"):
            eng = self.engine
            enc_hi = max((off + int(np.prod(shape)) for name, shape, off in eng.params.specs
                          if not name.startswith(("dec_", "final"))), default=0)
            bs = self._dp_buckets()
            self._dp_split = next((i for i, (lo, hi) in enumerate(bs) if lo < enc_hi), len(bs))
        return self._dp_split

    def _dp_exchange_overlap(self, updates=None):
        """dp_overlap: the decoder buckets' all-reduces issued on wside right behind the
        decoder's weight gradients (the trainer stream meanwhile runs the encoder backward),
        the encoder buckets' after the encoder backward on the trainer stream; each bucket's
        update on the side stream as it lands (as _dp_exchange)."""
        grads = self.engine.grads.buf
        split = self._dp_decoder_split()
        works = []
        for i, (lo, hi) in enumerate(self._dp_buckets()):
            if i < split:
                with torch.cuda.stream(self.wside):
                    if i == 0:
                        self._ev_ar.record(self.wside)
                    work = dp.allreduce_bucket(grads, lo, hi, self.pg)
            else:
                if i == split:
                    self._ev_bwd.record(self.stream)
                    self.side.wait_stream(self.stream)
                work = dp.allreduce_bucket(grads, lo, hi, self.pg)
            with torch.cuda.stream(self.side):
                work.wait()
                if updates is None:
                    self._dp_update(lo, hi)
                else:
                    updates[i].launch()
            works.append(work)
        if split == len(works):
            self._ev_bwd.record(self.stream)
        self._dp_works = works
        self.stream.wait_stream(self.side)
        self.stream.wait_stream(self.wside)
        K.step_increment(self.step_dev)

    def _launch_deferred(self, deferred=None, graph=None):
        """The decoder's deferred weight gradients on wside, after the decoder chain."""
        self._ev_dec.record(self.stream)
        self.wside.wait_event(self._ev_dec)
        with torch.cuda.stream(self.wside):
            if graph is not None:
                graph.launch()
            else:
                for wg in deferred:
                    wg()

    def _step_dp(self):
        """One data-parallel step (N > 1), eager, on self.stream (+ RCCL and the side stream)."""
        self._sample()
        if self.dp_overlap:
            self._fwd_loss()
            deferred = self.engine.backward_decoder(self.dpred)
            self._launch_deferred(deferred)
            self.engine.backward_encoder()
            self._dp_exchange_overlap()
            return
        self._fwd_bwd()
        self._dp_exchange()

    def _capture_dp(self):
        """N > 1 capture: the compute (sampler, forward, ListMLE, backward with its weight-
        gradient side stream) is one graph; each bucket's update another, on the side stream.
        A replay launches the compute graph, then issues the bucket all-reduces through
        torch.distributed between the update graphs (the collectives stay outside the graphs:
        RCCL's own stream, c10d's stream dependencies and work objects run as they do eagerly).
        Per step the host issues 1 + 2 x buckets launches and the collectives."""
        torch.cuda.synchronize()
        if self.dp_overlap:
            # three compute graphs: sampler -> forward -> ListMLE -> decoder backward; the
            # decoder's weight gradients (captured on wside); the encoder backward
            dec = []
            with torch.cuda.stream(self.stream):
                g1 = K.Graph().capture(lambda: (self._sample(), self._fwd_loss(),
                                                dec.extend(self.engine.backward_decoder(self.dpred))))
            with torch.cuda.stream(self.wside):
                gw = K.Graph().capture(lambda: [wg() for wg in dec])
            with torch.cuda.stream(self.stream):
                g2 = K.Graph().capture(self.engine.backward_encoder)
            graphs = [g1, gw, g2]
        else:
            with torch.cuda.stream(self.stream):
                graphs = [K.Graph().capture(lambda: (self._sample(), self._fwd_bwd()))]
        with torch.cuda.stream(self.side):
            upd = [K.Graph().capture(lambda lo=lo, hi=hi: self._dp_update(lo, hi))
                   for lo, hi in self._dp_buckets()]
        torch.cuda.synchronize()
        self.graphs = graphs
        self.bucket_graphs = upd

    def _replay_dp(self):
        """One captured N > 1 step on self.stream (the caller's current stream)."""
        self.graphs[0].launch()
        if self.dp_overlap:
            self._launch_deferred(graph=self.graphs[1])
            self.graphs[2].launch()
            self._dp_exchange_overlap(self.bucket_graphs)
            return
        self._dp_exchange(self.bucket_graphs)

    # ------------------------------------------------------------------ driving
    def step_eager(self, lr):
        with torch.cuda.stream(self.stream):
            K.set_scalar(self.lr_dev, lr)
            if self.world > 1:
                self._step_dp()
                return
            self._sample()
            self._fwd_bwd()
            self._update()

    def capture(self):
        """Capture the step into hipGraph(s). Call after one eager step (workspaces sized)."""
        if self.world > 1:
            self._capture_dp()
            return
        torch.cuda.synchronize()
        with torch.cuda.stream(self.stream):
            g = K.Graph().capture(lambda: (self._sample(), self._fwd_bwd(), self._update()))
            self.graphs = [g]
        torch.cuda.synchronize()

    def step(self, lr):
        if self.graphs is None:
            return self.step_eager(lr)
        with torch.cuda.stream(self.stream):
            K.set_scalar(self.lr_dev, lr)
            if self.world > 1:
                self._replay_dp()
                return
            self.graphs[0].launch()

    def loss_value(self):
        torch.cuda.current_stream().wait_stream(self.stream)
        return float(self.loss.item())

    def synchronize(self):
        self.stream.synchronize()
