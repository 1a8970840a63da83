"""Train/eval step engine (mirrors engine/flax_engine.py:13-134).

Same public names and call shapes as the reference:

    state = create_train_state(rng, model_def, learning_rate, image_shape, num_classes, cfg, curvature_batch)
    train_step = make_train_step(return_updates=False)
    state, metrics = train_step(state, (images, labels), rng)        # metrics: {'loss', 'accuracy'}
    eval_step = make_eval_step();  metrics = eval_step(state, (images, labels))

Differences that are MI355X design, not semantics: ``state`` is mutated in
place (and returned) instead of rebuilt; the reference's redundant second
forward (flax_engine.py:107-109, same rng -> same metrics) is skipped; the
whole step (forward, backward, optimizer) can be captured into one hipGraph
(``GraphedTrainStep``) because every kernel runs on the current stream with
device-resident seeds/counters.
"""
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import torch

from .. import kernels as K
from ..optim.adamw import AdamW
from ..optim.base import apply_updates
from ..optim.factory import get_optimizer
from ..models.vit_small import BatchStats
from ..params import ParamStore
from . import data_parallel as dp


def _seed_of(rng, step):
    if rng is None:
        return None
    if isinstance(rng, torch.Generator):
        return int(torch.randint(0, 2 ** 31 - 1, (1,), generator=rng).item())
    if isinstance(rng, torch.Tensor):
        return int(rng.reshape(-1)[-1].item()) & 0x7FFFFFFF
    try:
        return int(rng) & 0x7FFFFFFF
    except TypeError:
        return (hash(rng) + step) & 0x7FFFFFFF


def cross_entropy_loss(logits, labels):
    """flax_engine.py:13-16 on the GPU kernel (mean softmax CE)."""
    return compute_metrics(logits, labels)["loss"]


def compute_metrics(logits, labels) -> Dict[str, torch.Tensor]:
    """flax_engine.py:19-22: {'loss': mean CE, 'accuracy': mean(argmax == label)}."""
    R = logits.shape[0]
    lg = logits if logits.stride(-1) == 1 else logits.contiguous()
    rl = torch.empty(R, dtype=torch.float32, device=lg.device)
    rc = torch.empty(R, dtype=torch.float32, device=lg.device)
    out = torch.empty(2, dtype=torch.float32, device=lg.device)
    K.xent(lg, labels.to(torch.int32), rl, rc)
    K.mean2(rl, rc, R, 1.0 / R, out)
    return {"loss": out[0], "accuracy": out[1]}


@dataclass
class TrainState:
    """flax TrainState (+ batch_stats) with the MI355X runtime attached."""
    step: int
    params: ParamStore
    opt_state: Any
    tx: Any
    apply_fn: Any                       # the model definition (bind() -> runner)
    batch_stats: Any = None
    runners: Dict[tuple, Any] = field(default_factory=dict)
    gscale: Optional[torch.Tensor] = None

    def runner_for(self, image_shape):
        key = tuple(int(s) for s in image_shape)
        r = self.runners.get(key)
        if r is None:
            kw = {} if self.batch_stats is None else {"batch_stats": self.batch_stats}
            r = self.apply_fn.bind(self.params, key, self.params.device, **kw)
            self.runners[key] = r
        return r

    def replace(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)
        return self


def create_train_state(rng, model_def, learning_rate: float, image_shape, num_classes: int, cfg=None,
                       curvature_batch=None, device="cuda", init_params=None, init_batch_stats=None):
    """flax_engine.py:30-66.  ``init_params`` ({name: tensor}) overrides the
    initialiser (parity tests inject the oracle's params); ``init_batch_stats`` likewise for the
    BatchNorm variant's running averages (default: flax's zeros / ones)."""
    seed = _seed_of(rng, 0) or 0
    layout = model_def.layout(image_shape)
    store = ParamStore(layout, device)
    store.load(init_params if init_params is not None else model_def.init(seed, image_shape))
    batch_stats = None
    shapes = getattr(model_def, "batch_stats_shapes", lambda: {})()
    if shapes:   # variables.get("batch_stats") (flax_engine.py:46-47)
        batch_stats = BatchStats(shapes, store.device)
        batch_stats.load(init_batch_stats if init_batch_stats is not None else model_def.init_batch_stats())
    if cfg is None:
        tx = AdamW(learning_rate, weight_decay=1e-4)   # optax.adamw default weight_decay
    else:
        tx = get_optimizer(cfg, model_def=model_def, curvature_batch=curvature_batch, batch_stats=batch_stats)
    opt_state = tx.init(store)
    st = TrainState(step=0, params=store, opt_state=opt_state, tx=tx, apply_fn=model_def, batch_stats=batch_stats)
    st.runner_for(image_shape)
    return st


def _prepare(runner, images, labels):
    if images.device != runner.labels.device:
        images = images.to(runner.labels.device, non_blocking=True)
    if labels is not None and (labels.device != runner.labels.device or labels.dtype != torch.int32):
        labels = labels.to(device=runner.labels.device, dtype=torch.int32, non_blocking=True)
    return images.contiguous(), labels


def _reduce_batch_stats(state):
    """Under data parallelism every rank's BatchNorm sees its own micro-batch; the running averages
    (linear EMAs) are averaged over ranks once per step so the replicas stay identical."""
    if state.batch_stats is not None and dp.world_size() > 1:
        dp.all_reduce_mean_(state.batch_stats.flat)


def make_train_step(return_updates: bool = False):
    """flax_engine.py:95-123."""

    def train_step(state: TrainState, batch, rng=None):
        images, labels = batch
        runner = state.runner_for(images.shape)
        images, labels = _prepare(runner, images, labels)
        seed = _seed_of(rng, state.step)
        if seed is None:
            K.seed_next(runner.seed)
        else:
            runner.seed.fill_(seed)
        store = state.params
        store.settle()   # a GraphedTrainStep's deferred matrix phase, if any, first
        store.zero_grad()
        metrics = runner.forward(images, labels, train=True, need_grad=True)
        runner.backward(train=True)
        dp.all_reduce_grads(store)
        _reduce_batch_stats(state)
        if return_updates:
            grads = {k: v.clone() for k, v in store.grads.items()}
            updates, state.opt_state = state.tx.update(store.grads, state.opt_state, store)
            updates = {k: v.clone() for k, v in updates.items()}
            apply_updates(store, updates)
            state.step += 1
            return state, {"loss": metrics[0], "accuracy": metrics[1]}, grads, updates
        state.tx.step_(store, state.opt_state)
        state.step += 1
        return state, {"loss": metrics[0], "accuracy": metrics[1]}

    return train_step


def make_eval_step():
    """flax_engine.py:126-134 (deterministic forward, no dropout)."""

    def eval_step(state: TrainState, batch):
        images, labels = batch
        runner = state.runner_for(images.shape)
        images, labels = _prepare(runner, images, labels)
        state.params.settle()
        m = runner.forward(images, labels, train=False, need_grad=False)
        return {"loss": m[0].clone(), "accuracy": m[1].clone()}

    return eval_step


def _device_storages(objs, depth=6):
    """Every device storage reachable from objs (tensors, dicts, lists, plain objects)."""
    found, seen = {}, set()

    def walk(o, d):
        if isinstance(o, torch.Tensor):
            if o.is_cuda:
                st = o.untyped_storage()
                found.setdefault(st.data_ptr(), st)
            return
        if d <= 0 or id(o) in seen or isinstance(o, (str, bytes, int, float, bool, type(None))):
            return
        seen.add(id(o))
        if isinstance(o, dict):
            vals = o.values()
        elif isinstance(o, (list, tuple)):
            vals = o
        elif hasattr(o, "__dict__"):
            vals = vars(o).values()
        else:
            return
        for v in vals:
            walk(v, d - 1)

    for o in objs:
        walk(o, depth)
    return list(found.values())


def _host_scalars(obj, depth=6):
    """(owner, key, value) for every host int/float/bool reachable from obj through plain objects,
    dicts and lists -- e.g. Soap's ``host_step`` inside a ScheduleFree state's ``base``."""
    found, seen = [], set()

    def walk(o, d):
        if d <= 0 or id(o) in seen or isinstance(o, (torch.Tensor, str, bytes, type(None))):
            return
        seen.add(id(o))
        if isinstance(o, dict):
            items = list(o.items())
        elif isinstance(o, list):
            items = list(enumerate(o))
        elif hasattr(o, "__dict__") and not callable(o):
            items = list(vars(o).items())
        else:
            return
        for k, v in items:
            if isinstance(v, (bool, int, float)):
                found.append((o, k, v))
            else:
                walk(v, d - 1)

    walk(obj, depth)
    return found


def _restore_host_scalars(found):
    for o, k, v in found:
        if isinstance(o, (dict, list)):
            o[k] = v
        else:
            setattr(o, k, v)


class _labels_bound:
    """Points the runner's label buffer at an input slot's labels while one graph is captured (the
    kernels bake the pointer in), restoring the static buffer afterwards."""

    def __init__(self, runner, labels):
        self.runner, self.labels, self.saved = runner, labels, None

    def __enter__(self):
        if self.labels is not None:
            self.saved = self.runner.labels
            self.runner.labels = self.labels

    def __exit__(self, *exc):
        if self.saved is not None:
            self.runner.labels = self.saved
        return False


class GraphedTrainStep:
    """One hipGraph per step: seed advance, zero-grad, forward, backward, the data-parallel gradient
    mean (world_size > 1), optimizer.

    Inputs are copied into static buffers before each replay -- unless they are one of the
    ``inputs`` slots: ``inputs=(images [N, B, H, W, C] uint8, labels [N, B] int32)`` on the device is a
    ring of batch buffers that a loader fills in place, and each slot gets its own captured
    forward/backward graph reading that slot directly (no per-step copy launches, which cost a
    graph boundary plus two copy kernels, ~18 us, at ViT C2).  The warm-up launches that
    precede capture (lazy library setup) run on zero images; the params, optimizer state and
    seed they touch are snapshotted and restored, so construction does not train the model,
    and under data parallelism the warm-up gradients are all-reduced like a real step.

    Data parallelism (``reduce``, default world_size > 1): the gradient mean over ranks (and the
    BatchNorm running averages) sits between the backward and the optimizer.  On RCCL it is captured
    inside the step graph (``capture_reduce``, default: when dp.captured_reduce_works), so a step stays
    one replay, Muon's matrix-phase overlap included.  Otherwise (gloo, or a build whose collectives do
    not capture) each step replays the forward/backward graph, reduces eagerly and replays a second
    graph holding the optimizer's part of the step -- the overlap holds there too."""

    # each ring slot is one more captured forward/backward graph (construction time and graph memory
    # grow with the ring); the slot graphs share the copy-in graph's memory pool
    MAX_SLOTS = 8

    def __init__(self, state: TrainState, image_shape, warmup=2, inputs=None, overlap_opt=False,
                 reduce=None, capture_reduce=None):
        self.state = state
        # another step object's deferred matrix phase must land before this one snapshots the state
        # and replays its own gradient phase over the same moments / fp32 copies
        state.params.settle()
        self.runner = state.runner_for(image_shape)
        dev = state.params.device
        self.images = torch.zeros(tuple(image_shape), dtype=torch.uint8, device=dev)
        self.labels = self.runner.labels   # the runner's static label buffer (no second copy)
        self.slots = []
        if inputs is not None:
            xs, ys = inputs
            B = image_shape[0]
            if (xs.dtype != torch.uint8 or tuple(xs.shape[1:]) != tuple(image_shape) or ys.dtype != torch.int32 or
                    tuple(ys.shape) != (xs.shape[0], B) or not xs.is_cuda or not ys.is_cuda or
                    not xs.is_contiguous() or not ys.is_contiguous()):
                raise ValueError("inputs: (uint8 [N, *image_shape], int32 [N, B]) contiguous device tensors")
            if xs.shape[0] > self.MAX_SLOTS:
                raise ValueError(f"inputs: at most {self.MAX_SLOTS} ring slots (one captured graph each)")
            self.slots = [(xs[k], ys[k]) for k in range(xs.shape[0])]
        # reduce=True on a one-rank process group still launches the collective (tests of the
        # captured-reduce graph on one GPU); without a process group there is nothing to reduce over
        self.distributed = (dp.world_size() > 1) if reduce is None else bool(reduce and dp.is_initialized())
        # SOAP/Shampoo steps are host-driven (first step, refreshes, basis restarts): they run
        # eagerly after the captured forward/backward.
        self.opt_graphed = bool(getattr(state.tx, "graphable", True))
        # overlap_opt: an optimizer whose step splits into a gradient phase and a matrix phase (Muon:
        # momentum + Adam branch | Newton-Schulz + routed update) runs the matrix phase of step t on a
        # side stream at the start of step t+1, beside that step's forward up to the first read of a
        # routed weight (runner.forward(join=...)).  The phase order per step is step_()'s; the last
        # step's matrix phase runs in flush() (called by whoever reads the params next: bench, eval).
        self.overlap = bool(overlap_opt and self.opt_graphed and
                            getattr(self.runner, "supports_join", False) and
                            hasattr(state.tx, "split_capable") and state.tx.split_capable(state.opt_state))
        self.pending = False
        # the captured step always runs the backward, so its metrics come from there; the flag is set
        # only while this constructor warms up and captures (the runner's eager behaviour is unchanged)
        had_flag = hasattr(self.runner, "metrics_in_backward")
        old_flag = getattr(self.runner, "metrics_in_backward", None)
        if had_flag:
            self.runner.metrics_in_backward = True
        try:
            self._build(state, warmup, capture_reduce, dev)
        finally:
            if had_flag:
                self.runner.metrics_in_backward = old_flag
        self.metrics = self.runner.metrics

    def _build(self, state, warmup, capture_reduce, dev):
        self.stream = torch.cuda.Stream(device=dev)
        self.g_fb = torch.cuda.CUDAGraph()
        self.g_post = None
        s = self.stream
        store = state.params
        saved = [(st, st.clone()) for st in _device_storages([store.flat, store.shadow, self.runner.seed,
                                                              state.opt_state, state.batch_stats])]
        host = _host_scalars(state.opt_state)   # e.g. host_step, also inside wrapped (schedule-free) states
        # the snapshot clones run on the current stream: the warm-up stream waits for them, or the
        # warm-up's seed advance / optimizer step could land before the clone reads its source
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._fb()
                if self.distributed:
                    self._reduce()
                self._opt()
            torch.cuda.synchronize()
            for st, copy in saved:
                st.copy_(copy)
            torch.cuda.synchronize()
            _restore_host_scalars(host)
            if self.distributed and capture_reduce is None:
                capture_reduce = self.opt_graphed and dp.captured_reduce_works(dev, s)
            self.capture_reduce = bool(self.distributed and capture_reduce)
            # split: the step graph ends after the backward; the reduce and the optimizer's part run
            # after its replay (eager reduce, then g_post, or the eager optimizer)
            self.split = (self.distributed and not self.capture_reduce) or not self.opt_graphed
            # with a process group up, its watchdog thread polls events while we capture: under the
            # "global" mode a poll during capture invalidates the capture (seen once in a one-rank RCCL run,
            # "operation failed due to a previous error during capture"), so only this thread's calls
            # are checked then
            mode = "thread_local" if dp.is_initialized() else "global"
            self.g_slots = []
            after_first = None
            for images, labels in [(None, None)] + self.slots:   # the copy-in graph, then one per slot
                g = self.g_fb if images is None else torch.cuda.CUDAGraph()
                with _labels_bound(self.runner, labels):
                    # slot graphs replay one at a time on this stream, after the copy-in graph's capture:
                    # they can share its memory pool
                    with torch.cuda.graph(g, stream=s, pool=None if images is None else self.g_fb.pool(),
                                          capture_error_mode=mode):
                        self._body(images, steady=False)
                if images is None:
                    after_first = _host_scalars(state.opt_state)   # host state as after one capture
                else:
                    self.g_slots.append(g)
                    _restore_host_scalars(after_first)
            if self.overlap:
                # steady-state graphs: the previous step's matrix phase on a side stream beside this
                # step's forward head, joined before the first routed-weight read
                self.side = torch.cuda.Stream(device=dev)
                self.g_steady = []
                for images, labels in [(None, None)] + self.slots:
                    g = torch.cuda.CUDAGraph()
                    with _labels_bound(self.runner, labels):
                        with torch.cuda.graph(g, stream=s, pool=self.g_fb.pool(), capture_error_mode=mode):
                            self._body(images, steady=True)
                    self.g_steady.append(g)
                self.g_flush = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.g_flush, stream=s, pool=self.g_fb.pool(), capture_error_mode=mode):
                    state.tx.step_ns_phase_(store, state.opt_state)
            if self.split and self.opt_graphed:
                self.g_post = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.g_post, stream=s, pool=self.g_fb.pool(), capture_error_mode=mode):
                    self._post()
        torch.cuda.current_stream().wait_stream(s)

    def _body(self, images, steady):
        """What one step graph holds: [the previous step's matrix phase on the side stream, joined before
        the first routed-weight read] forward, backward, then -- unless split -- the reduce and the
        optimizer's part."""
        s, state = self.stream, self.state
        if steady:
            self.side.wait_stream(s)
            with torch.cuda.stream(self.side):
                state.tx.step_ns_phase_(state.params, state.opt_state)
            join = lambda i: s.wait_stream(self.side) if i == 0 else None  # noqa: E731
            self._fb(images, join=join)
            s.wait_stream(self.side)   # (a one-block model never joins at block 1)
        else:
            self._fb(images)
        if self.split:
            return
        if self.distributed:
            self._reduce()
        self._post()

    def _post(self):
        """The optimizer's part of a step: the gradient phase when the matrix phase is deferred."""
        if self.overlap:
            self.state.tx.step_grad_phase_(self.state.params, self.state.opt_state)
        else:
            self._opt()

    def _reduce(self):
        dp.all_reduce_grads(self.state.params, always=True)
        if self.state.batch_stats is not None:
            dp.all_reduce_mean_(self.state.batch_stats.flat, always=True)

    def _fb(self, images=None, join=None):
        K.zero_seed(self.state.params.grad_flat, self.runner.seed)   # zero grads + advance seed
        kw = {"join": join} if join is not None else {}
        self.runner.forward(self.images if images is None else images, None, train=True, need_grad=True, **kw)
        self.runner.backward(train=True)

    def flush(self):
        """Finish the last step's deferred matrix phase (overlap_opt): the params and optimizer state
        are then exactly those after the steps taken.  A no-op otherwise.  Also run by
        ParamStore.settle() (to_dict, load, the eager train / eval steps), so nothing reads the
        params with a phase still owed."""
        if self.pending:
            self.g_flush.replay()
            self.pending = False
        if self.state.params.pending == self.flush:
            self.state.params.pending = None

    def _slot_of(self, images, labels):
        """The input slot holding exactly this batch: both the images AND the labels must be that slot's
        tensors (or views of the same storage and shape); anything else goes through the copy-in graph."""
        if images is None or labels is None:
            return None

        def same(a, b):
            return a is b or (a.data_ptr() == b.data_ptr() and a.shape == b.shape and a.dtype == b.dtype)

        for k, (x, y) in enumerate(self.slots):
            if same(images, x) and same(labels, y):
                return k
        return None

    def _opt(self):
        self.state.tx.step_(self.state.params, self.state.opt_state)

    def __call__(self, images=None, labels=None):
        owed = self.state.params.pending
        if owed is not None and owed != self.flush:
            # another step object (e.g. the runner of a different batch shape) still owes its matrix
            # phase: run it before this step's gradient phase rewrites the moments it reads
            self.state.params.settle()
        k = self._slot_of(images, labels) if self.slots else None
        steady = self.overlap and self.pending
        if k is not None:
            # the batch is read in place from its input slot
            (self.g_steady[k + 1] if steady else self.g_slots[k]).replay()
        else:
            if images is not None:
                self.images.copy_(images, non_blocking=True)
            if labels is not None:
                self.labels.copy_(labels, non_blocking=True)
            (self.g_steady[0] if steady else self.g_fb).replay()
        if self.overlap:
            self.pending = True
            self.state.params.pending = self.flush
        if self.split:
            if self.distributed:
                self._reduce()
            if self.g_post is not None:
                self.g_post.replay()
            else:
                self._opt()
        self.state.step += 1
        return self.metrics
