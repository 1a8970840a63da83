"""Data parallelism: one process per GPU, gradient mean over RCCL/xGMI.

Replaces the reference's single-process ``jax.pmap`` + ``lax.pmean(grads)``
(train_lm.py:195-210, 256-271) and its collective probe with fallback
(train_lm.py:442-462, 485-492).  Each rank computes its own micro-batches; the
only exchange is the mean of the flat fp32 gradient buffer, done ONCE per
optimizer step (the reference reduces every micro-step; mean-of-sums equals
sum-of-means up to fp rounding), in contiguous buckets walked from the end of
the buffer (= the order the backward produces them).  Params/optimizer state
stay replicated; every rank runs the identical optimizer update.

Overlap (:class:`OverlappedReducer`): during the LAST micro-step's backward the runner reports,
layer by layer, the offset above which the flat gradient is final; once a bucket's worth is
final it is all-reduced on a side stream (RCCL over xGMI) while the backward continues on the
compute stream, ordered by HIP events -- so only the last bucket (the embedding's rows) is
exposed after the backward.
``torch.distributed`` backend "nccl" is RCCL on ROCm; "gloo" is used for the
CPU multi-process tests.
"""
import os

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 128 << 20


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def world_size():
    return dist.get_world_size() if is_initialized() else 1


def rank():
    return dist.get_rank() if is_initialized() else 0


def resolve_use_dp(cfg, world):
    """train_lm.py:476-506: ``use_pmap`` (None = auto) and ``force_single_device`` decide whether the
    visible devices train data-parallel.  Here the device count is the launcher's WORLD_SIZE (one
    process per GPU), so a config that asks for single-device training while N > 1 ranks were
    launched is rejected loudly instead of silently running N-way DP -- launch one process."""
    requested = getattr(cfg, "use_pmap", None)
    force_single = bool(getattr(cfg, "force_single_device", False))
    if requested is None:
        use_dp = world > 1 and not force_single
    else:
        use_dp = bool(requested) and world > 1 and not force_single
    if world > 1 and not use_dp:
        raise ValueError(
            f"config requests single-device training (use_pmap={requested!r}, force_single_device="
            f"{force_single}) but {world} ranks were launched; start one process (python train_lm.py ...) "
            "or drop the key")
    return use_dp


def init_from_env(backend=None):
    """torchrun-style env (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/PORT).  Returns
    (rank, local_rank, world_size, device)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(lr)
            dist.init_process_group(backend=backend, device_id=torch.device("cuda", lr))
        else:
            dist.init_process_group(backend=backend)
    dev = torch.device("cuda", lr) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    return rank(), lr, world_size(), dev


def probe_collectives(device):
    """psum(arange(n)) health check (train_lm.py:442-462).  Returns (ok, err)."""
    n = world_size()
    if n <= 1:
        return False, None
    try:
        x = torch.arange(n, dtype=torch.float32, device=device)
        dist.all_reduce(x)
        ok = torch.allclose(x.cpu(), torch.arange(n, dtype=torch.float32) * n)
        return bool(ok), None if ok else "psum mismatch"
    except Exception as exc:  # pragma: no cover - depends on the fabric
        return False, str(exc)


def _avg_supported(t):
    return t.is_cuda and dist.get_backend() == "nccl"


def all_reduce_mean_(t, bucket_bytes=DEFAULT_BUCKET_BYTES, always=False):
    """In-place mean of a flat tensor across ranks, bucketed back to front.  A one-rank group skips the
    collective unless ``always`` (a one-rank RCCL group still launches it: how the captured-reduce step
    graph is exercised on one GPU)."""
    n = world_size()
    if n <= 1 and not (always and is_initialized()):
        return t
    per = max(1, bucket_bytes // t.element_size())
    total = t.numel()
    end = total
    use_avg = _avg_supported(t)
    while end > 0:
        start = max(0, end - per)
        chunk = t[start:end]
        if use_avg:
            dist.all_reduce(chunk, op=dist.ReduceOp.AVG)
        else:
            dist.all_reduce(chunk, op=dist.ReduceOp.SUM)
            chunk.div_(n)
        end = start
    return t


def all_reduce_grads(store, bucket_bytes=DEFAULT_BUCKET_BYTES, always=False):
    if world_size() > 1 or always:
        all_reduce_mean_(store.grad_flat[: store.layout.size], bucket_bytes, always=always)


def captured_reduce_works(device, stream):
    """Whether an all-reduce captured into a hipGraph runs correctly on this process group.  Every rank
    captures one on ``stream``; the ranks agree (eagerly) that every capture succeeded before any rank
    replays, then replay once and agree the mean is right -- so all ranks take the same decision.  Only
    RCCL ("nccl") collectives are graph-capturable; gloo runs on the host."""
    if not is_initialized() or device.type != "cuda" or dist.get_backend() != "nccl":
        return False
    n = dist.get_world_size()
    t = torch.full((256,), float(rank() + 1), device=device)
    g = torch.cuda.CUDAGraph()
    ok = 1
    stream.wait_stream(torch.cuda.current_stream(device))
    try:
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
            all_reduce_mean_(t, always=True)
    except Exception:   # pragma: no cover - depends on the RCCL / HIP build
        ok = 0

    def agree(v):
        f = torch.tensor([v], dtype=torch.int32, device=device)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        return bool(f.item())

    if not agree(ok):
        return False
    g.replay()
    torch.cuda.synchronize(device)
    return agree(int(bool(torch.all(t == (n + 1) / 2.0).item())))


def all_reduce_metrics(m):
    """pmean of the [loss, acc] scalars (train_lm.py:208-209)."""
    if world_size() > 1:
        all_reduce_mean_(m)
    return m


class OverlappedReducer:
    """Bucketed gradient mean overlapped with the backward that produces the gradients.

    ``ready(offset)``: flat[offset:] is final (the backward walks the layout back to front);
    buckets of >= ``bucket_bytes`` are launched immediately on the communication stream after an
    event recorded on the compute stream.  ``finish()`` reduces the rest and makes the compute
    stream wait for every launched reduction.  With one rank it does nothing; on CPU (gloo tests)
    the reductions run synchronously with the same bucketing."""

    def __init__(self, flat, bucket_bytes=32 << 20):
        self.flat = flat
        self.bucket = max(1, bucket_bytes // flat.element_size())
        self.active = world_size() > 1
        self.cuda = flat.is_cuda
        self.comm = torch.cuda.Stream(device=flat.device) if (self.active and self.cuda) else None
        self.pending_end = None
        self.launched = 0

    def begin(self, end=None):
        self.pending_end = self.flat.numel() if end is None else int(end)
        self.launched = 0

    def _launch(self, start, end):
        chunk = self.flat[start:end]
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.flat.device))
            self.comm.wait_event(ev)
            with torch.cuda.stream(self.comm):
                all_reduce_mean_(chunk, bucket_bytes=(end - start) * self.flat.element_size())
        else:
            all_reduce_mean_(chunk, bucket_bytes=(end - start) * self.flat.element_size())
        self.launched += 1

    def ready(self, offset):
        if not self.active or self.pending_end is None:
            return
        if self.pending_end - offset >= self.bucket:
            self._launch(int(offset), self.pending_end)
            self.pending_end = int(offset)

    def finish(self):
        if not self.active or self.pending_end is None:
            return
        if self.pending_end > 0:
            self._launch(0, self.pending_end)
        self.pending_end = None
        if self.cuda:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.comm)
