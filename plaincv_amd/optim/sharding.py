"""Optimizer-work sharding across data-parallel replicas (second stage).

The reference's pmapped ``apply_grads`` (train_lm.py:316-353, flax_engine.py:110-111) runs every
routed matrix's preconditioner -- Muon's Newton-Schulz chain, SOAP's rotations / QR / eigh,
Shampoo's inverse roots -- on every replica: identical work N times.  Here each rank OWNS a
contiguous run of routed matrices in layout order, balanced by preconditioner cost, keeps only
their per-matrix state and runs only their preconditioner work.  After the step every rank's
span of the flat parameter buffer -- its matrices plus the replicated leaves lying between them,
which are bit-identical on all ranks anyway -- is broadcast from its owner (RCCL over xGMI; gloo
in the CPU tests) and the span's bf16 GEMM shadow is re-cast locally.  The Adam branch
(embeddings, norms, biases, 3-D attention kernels) stays replicated: it is HBM-bound elementwise
work that costs less than moving its result.

Result: the same update as the unsharded step (the owner runs the identical kernels on the
identical, already all-reduced gradients), replicas stay bit-identical (every rank ends with the
owner's bits), and the per-rank preconditioner work drops by ~N.  Payload per step: the routed
parameters once (a broadcast per rank), instead of zero -- worth it when the preconditioner
costs more than moving its result (Muon NS5 on the 124M / 420M LMs: 1.6 / 7.5 TFLOP per
replica per step; SOAP / Shampoo eigen work).
"""
from .. import kernels as K


def muon_cost(r, c):
    """Newton-Schulz FLOPs of one (r, c) matrix (min side first), per step."""
    r, c = min(r, c), max(r, c)
    return 10.0 * r * r * c + 4.0 * r ** 3


def soap_cost(r, c):
    """Gram updates, rotations, back-projections and the amortised refresh of one matrix."""
    return float(r) ** 3 + float(c) ** 3 + float(r) * c * (r + c)


def shampoo_cost(r, c):
    """Inverse roots of the two Kronecker factors (coupled-Newton iterations) dominate."""
    return float(r) ** 3 + float(c) ** 3


def partition(costs, world):
    """Owner rank of each unit (in order): unit i goes to the rank whose 1/world slice of the
    cumulative cost holds the unit's midpoint -- monotone, so every rank owns one contiguous run."""
    total = float(sum(costs))
    if world <= 1 or total <= 0.0:
        return [0] * len(costs)
    out, acc = [], 0.0
    for c in costs:
        out.append(min(world - 1, int((acc + 0.5 * c) * world / total)))
        acc += c
    return out


def resolve(shard):
    """``shard``: None/False (off), True/"auto" (this process group's rank and world when
    world > 1) or an explicit (rank, world) pair (tests)."""
    if shard is None or shard is False:
        return None
    if shard is True or shard == "auto":
        from ..engine import data_parallel as dp
        world = dp.world_size()
        return (dp.rank(), world) if world > 1 else None
    rank, world = (int(x) for x in shard)
    return (rank, world) if world > 1 else None


class RoutedShard:
    """Ownership of the routed matrices of one optimizer and the post-step exchange.

    Fused storage groups (the LM's interleaved fc_gate|fc_up, params.Layout.add_fused) are one
    unit: their members share storage rows, so they must have one owner."""

    def __init__(self, store, routed, cost_fn, rank, world):
        self.rank, self.world = int(rank), int(world)
        lay = store.layout
        units, seen = [], {}
        for k in routed:                      # layout order = forward order
            g = lay.leaves[k].group
            if g is not None and g in seen:
                units[seen[g]].append(k)
                continue
            if g is not None:
                seen[g] = len(units)
            units.append([k])
        costs = [sum(cost_fn(*store.params[k].shape) for k in u) for u in units]
        owners = partition(costs, self.world)
        self.owner = {k: o for u, o in zip(units, owners) for k in u}
        self.owned = [k for k in routed if self.owner[k] == self.rank]
        self.cost = [0.0] * self.world
        for c, o in zip(costs, owners):
            self.cost[o] += c
        # each rank's span of the flat storage: first to last storage element of its units
        self.spans = []
        for r in range(self.world):
            lo, hi = None, None
            for u, o in zip(units, owners):
                if o != r:
                    continue
                for k in u:
                    s, e = self._extent(lay, k)
                    lo = s if lo is None else min(lo, s)
                    hi = e if hi is None else max(hi, e)
            self.spans.append((lo, hi) if lo is not None else None)
        prev = -1
        for sp in self.spans:   # contiguous runs in layout order -> disjoint, ascending spans
            if sp is not None:
                assert sp[0] >= prev, self.spans
                prev = sp[1]

    @staticmethod
    def _extent(lay, k):
        lf = lay.leaves[k]
        if lf.group is not None:
            off, rows, row, _ = lay.groups[lf.group]
            return off, off + rows * row
        return lf.offset, lf.offset + lf.numel_storage

    def exchange(self, buf, shadow=None):
        """Broadcast every rank's span of ``buf`` (the fp32 params after an applied step, or the
        flat update buffer of ``update()``) from its owner; re-cast the bf16 shadow of the spans
        received (the owner's own shadow was written by its optimizer kernels)."""
        import torch.distributed as dist
        for r, sp in enumerate(self.spans):
            if sp is None:
                continue
            dist.broadcast(buf[sp[0]:sp[1]], src=r)
        if shadow is not None:
            for r, sp in enumerate(self.spans):
                if sp is not None and r != self.rank:
                    K.cast_f32_bf16(buf[sp[0]:sp[1]], shadow[sp[0]:sp[1]])

    def describe(self):
        return {"rank": self.rank, "world": self.world, "owned": len(self.owned),
                "cost_share": [round(c / max(1e-30, sum(self.cost)), 4) for c in self.cost]}


def setup(tx, store, routed, cost_fn):
    """Called from an optimizer's init: returns (routed matrices this rank works on, shard or
    None).  A sharded optimizer is not graph-captured (the broadcasts run eagerly)."""
    sh = resolve(getattr(tx, "shard", None))
    if sh is None:
        return list(routed), None
    rs = RoutedShard(store, routed, cost_fn, *sh)
    tx.graphable = False
    return rs.owned, rs


def finish(shard, store, st, apply):
    if shard is not None:
        shard.exchange(store.flat if apply else st.upd, store.shadow if apply else None)


__all__ = ["RoutedShard", "partition", "resolve", "setup", "finish", "muon_cost", "soap_cost", "shampoo_cost"]
