"""Schedule-free wrapper (optim/factory.py:82-99, 801 -> optax.contrib.schedule_free, optax 0.2.6).

The params the model sees are y (where gradients are taken).  Each step the base optimizer's update
u (computed at y, already scaled by -lr) advances z; x is re-formed from y and the old z and mixed
with the new z by c_k = w_k / sum_j w_j (w = max_lr^weight_lr_power); y = b1 x + (1-b1) z:

    z' = z + u;  x = (1-c_k) (y - (1-b1) z)/b1 + c_k z';  y' = b1 x + (1-b1) z'

The base runs through ``update_into_`` (its update written to a buffer, its state advanced), then
one ``pcv_schedule_free_step`` launch (a 1-thread scalar prologue forms c_k on the device, so the
wrapped step replays from a hipGraph) rewrites y, z and the bf16 shadow.  Extra HBM traffic over
the base optimizer: 20 B/param read (y, z, u) + 10 B written (y, z, shadow).
"""
import torch

from .. import hip
from ..hip import ptr, stream_ptr
from .adamw import _views
from .base import GradientTransformation, OptState, ensure_grads


class ScheduleFree(GradientTransformation):
    def __init__(self, base, learning_rate, b1=0.9, weight_lr_power=2.0):
        if b1 == 0:
            raise ValueError("The current implementation of schedule_free requires b1 > 0.")
        self.base = base
        self.lr, self.b1, self.power = float(learning_rate), float(b1), float(weight_lr_power)

    @property
    def graphable(self):   # the base decides, after its init has seen the factor sizes
        return bool(getattr(self.base, "graphable", True))

    def init(self, store):
        st = OptState(store.device)
        st.base = self.base.init(store)
        st.tensors["z"] = store.flat.clone()
        st.sf = torch.zeros(3, dtype=torch.float32, device=store.device)     # weight_sum, max_lr, c_k
        st.step_count = torch.ones(1, dtype=torch.int32, device=store.device)
        st.upd = torch.zeros_like(store.flat)
        st.chunks = store.chunks(None)
        return st

    def _run(self, store, st, gscale, apply):
        u = self.base.update_into_(store, st.base, gscale)
        hip.call("pcv_schedule_free_step", ptr(store.flat), ptr(st.tensors["z"]), ptr(u),
                 ptr(store.shadow) if apply else None, None if apply else ptr(st.upd), ptr(st.chunks),
                 int(st.chunks.shape[0]), self.b1, self.lr, self.power, ptr(st.sf), ptr(st.step_count),
                 int(apply), stream_ptr())
        if apply:
            store.version += 1

    def update(self, grads, state, params=None):
        ensure_grads(params, grads)
        self._run(params, state, None, apply=False)
        return _views(params, state.upd), state

    def update_into_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=False)
        return state.upd

    def step_(self, store, state, gscale=None):
        self._run(store, state, gscale, apply=True)
