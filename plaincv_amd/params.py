"""Flat parameter / gradient storage laid out for the MI355X kernels.

Every model keeps ONE fp32 master buffer, ONE fp32 grad buffer with the same
layout, and ONE bf16 shadow (the GEMM operand copy, rewritten by the optimizer
kernels).  Each Flax leaf (``"EncoderBlock_0/SelfAttention_0/query/kernel"``,
``"layers_3/mlp/fc_up/kernel"`` ...) is a strided view with its Flax shape, so
the optimizer routing of optim/matrix_routing.py:27-40 applies to the same
names and shapes as in the reference, while the storage is chosen for the
kernels:

* the last axis of every leaf is padded to a multiple of 8 elements (16-B
  aligned bf16 rows for the MFMA loaders; pads stay exactly 0 under every
  optimizer because their gradients are 0);
* "fused" groups interleave sibling kernels along their output axis so the
  fused GEMM operand is a plain 2-D view: ViT q|k|v kernels -> W_qkv [D, 3*H*Dh],
  q|k|v biases -> [3*H*Dh], LM fc_gate|fc_up -> W_gu [D, 2*F];
* leaves start on 64-element boundaries; the order is the forward order so
  a reverse walk is the backward (DDP bucket) order.
"""
import math
from collections import OrderedDict

import torch

ALIGN = 64


def _pad8(n):
    return (n + 7) // 8 * 8


class Leaf:
    __slots__ = ("name", "shape", "offset", "strides", "numel_storage", "group")

    def __init__(self, name, shape, offset, strides, numel_storage, group=None):
        self.name, self.shape, self.offset, self.strides = name, tuple(shape), offset, tuple(strides)
        self.numel_storage, self.group = numel_storage, group


class Layout:
    """Builds the flat layout from (name, shape) specs and fused groups."""

    def __init__(self):
        self.leaves = OrderedDict()
        self.groups = {}  # group name -> (offset, rows, row_len_storage)
        self.size = 0

    def _alloc(self, n):
        off = (self.size + ALIGN - 1) // ALIGN * ALIGN
        self.size = off + n
        return off

    def add(self, name, shape):
        shape = tuple(shape)
        if len(shape) == 0:
            shape = (1,)
        last = shape[-1]
        ld = _pad8(last) if len(shape) >= 2 else last
        outer = int(math.prod(shape[:-1])) if len(shape) > 1 else 1
        n = outer * ld
        off = self._alloc(n)
        strides = []
        acc = ld
        for d in reversed(shape[:-1]):
            strides.insert(0, acc)
            acc *= d
        strides.append(1)
        self.leaves[name] = Leaf(name, shape, off, strides, n)
        return self.leaves[name]

    def add_fused(self, gname, names, shape, pad_each=False):
        """k sibling leaves of identical shape (rows, *tail), interleaved along
        the output axis: storage [rows, k, prod(tail)] with the row padded to 8;
        with ``pad_each`` every member's width is padded to 8 (so each half of
        [gate|up] starts 16-B aligned) and the group spans the padded width."""
        k = len(names)
        shape = tuple(shape)
        rows = shape[0]
        tail = shape[1:]
        tn0 = int(math.prod(tail))
        tn = _pad8(tn0) if pad_each else tn0
        row = _pad8(k * tn)
        off = self._alloc(rows * row)
        for i, nm in enumerate(names):
            strides = [row]
            acc = 1
            tstr = []
            for d in reversed(tail):
                tstr.insert(0, acc)
                acc *= d
            self.leaves[nm] = Leaf(nm, shape, off + i * tn, tuple(strides + tstr), rows * tn0, gname)
        self.groups[gname] = (off, rows, row, k * tn)


    def add_concat(self, gname, names, shape):
        """k sibling leaves of identical shape stored back to back (contiguous);
        the group is the 1-D concatenation (e.g. q|k|v biases -> [3*H*Dh])."""
        shape = tuple(shape)
        n = int(math.prod(shape))
        k = len(names)
        off = self._alloc(_pad8(k * n))
        strides = []
        acc = 1
        for d in reversed(shape):
            strides.insert(0, acc)
            acc *= d
        for i, nm in enumerate(names):
            self.leaves[nm] = Leaf(nm, shape, off + i * n, tuple(strides), n, gname)
        self.groups[gname] = (off, 1, _pad8(k * n), k * n)


class ParamStore:
    """Device storage for a Layout: fp32 params + grads, bf16 shadow."""

    def __init__(self, layout: Layout, device, with_grads=True):
        self.layout = layout
        self.device = torch.device(device)
        n = (layout.size + 255) // 256 * 256
        self.flat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.grad_flat = torch.zeros(n, dtype=torch.float32, device=self.device) if with_grads else None
        self.shadow = torch.zeros(n, dtype=torch.bfloat16, device=self.device)
        self.params = OrderedDict((k, self._view(self.flat, l)) for k, l in layout.leaves.items())
        self.grads = OrderedDict((k, self._view(self.grad_flat, l)) for k, l in layout.leaves.items()) \
            if with_grads else None
        self.bf16 = OrderedDict((k, self._view(self.shadow, l)) for k, l in layout.leaves.items())
        # bumped whenever the bf16 shadow changes (load, optimizer step), so derived
        # copies (e.g. the LM runner's transposed forward weights) know to refresh
        self.version = 0
        # a deferred optimizer phase still owed to these params (engine.GraphedTrainStep overlap_opt:
        # the last step's Newton-Schulz phase): settle() runs it; every reader that must see the
        # params as after the steps taken -- to_dict, load, the eager train / eval steps -- settles first
        self.pending = None

    @staticmethod
    def _view(buf, leaf):
        return buf.as_strided(leaf.shape, leaf.strides, leaf.offset)

    def group_view(self, buf, gname, dtype_buf=None):
        off, rows, row, used = self.layout.groups[gname]
        if rows == 1:
            return buf.as_strided((used,), (1,), off)
        return buf.as_strided((rows, used), (row, 1), off)

    def leaf(self, name):
        return self.layout.leaves[name]

    def settle(self):
        """Run the deferred optimizer phase, if one is pending (a no-op otherwise)."""
        fn, self.pending = self.pending, None
        if fn is not None:
            fn()

    def load(self, values):
        """Copy a {name: tensor(Flax shape)} dict into the master buffer (pads stay 0)."""
        self.settle()
        for k, v in values.items():
            self.params[k].copy_(torch.as_tensor(v, dtype=torch.float32))
        self.sync_shadow()

    def sync_shadow(self):
        from . import kernels
        kernels.cast_f32_bf16(self.flat, self.shadow)
        self.version += 1

    def to_dict(self):
        self.settle()
        return OrderedDict((k, v.detach().clone().cpu()) for k, v in self.params.items())

    def grads_dict(self):
        return OrderedDict((k, v.detach().clone().cpu()) for k, v in self.grads.items())

    def zero_grad(self):
        self.grad_flat.zero_()

    def chunks(self, names=None, chunk=4096):
        """Chunk table {start, len} covering the storage of `names` (all leaves by default)."""
        spans = []
        if names is None:
            spans = [(0, self.layout.size)]
        else:
            seen = set()
            for k in names:
                lf = self.layout.leaves[k]
                if lf.group is not None:
                    if lf.group in seen:
                        continue
                    seen.add(lf.group)
                    off, rows, row, used = self.layout.groups[lf.group]
                    members = [n for n, l in self.layout.leaves.items() if l.group == lf.group]
                    if not all(m in names for m in members):
                        raise ValueError(f"fused group {lf.group} split across optimizer routes")
                    spans.append((off, rows * row))
                else:
                    spans.append((lf.offset, lf.numel_storage))
        out = []
        for s, n in spans:
            for c in range(0, n, chunk):
                out.append((s + c, min(chunk, n - c)))
        t = torch.tensor(out, dtype=torch.int64).reshape(-1, 2)
        return t.to(self.device)
