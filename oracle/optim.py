"""Optimizer semantics restated from optim/* and optax 0.2.6 (TEST INFRASTRUCTURE ONLY).

Every transformation is functional like an optax ``GradientTransformation``:
``init(params) -> state`` and ``update(grads, state, params) -> (updates, state)``
where ``updates`` are additive deltas already scaled by -lr (apply with
``oracle.engine.apply_updates``).  Params/grads are flat dicts keyed by the
Flax path.
"""
from types import SimpleNamespace

import torch


# ----------------------------------------------------------------------------
# routing (optim/matrix_routing.py:22-40, optim/shampoo.py:61-74)
# ----------------------------------------------------------------------------
def is_non_degenerate_2d_matrix(p):
    return p.ndim == 2 and p.shape[0] > 1 and p.shape[1] > 1


def should_use_matrix_preconditioner(name, p):
    if not is_non_degenerate_2d_matrix(p):
        return False
    name = name.lower()
    leaf = name.split("/")[-1] if name else ""
    if leaf != "kernel":
        return False
    if ("embed" in name) or ("embedding" in name) or ("lm_head" in name):
        return False
    if "norm" in name:
        return False
    return True


def should_use_shampoo(name, p):
    if not should_use_matrix_preconditioner(name, p):
        return False
    leaf = name.lower().split("/")[-1]
    return leaf not in {"bias", "scale"}


# ----------------------------------------------------------------------------
# AdamW (optim/factory.py:193-205 -> optax.adamw)
# ----------------------------------------------------------------------------
def _adam_direction(g, m, v, count, b1, b2, eps, eps_root=0.0, nesterov=False):
    """optax.scale_by_adam; returns (direction, m_new, v_new)."""
    m_new = b1 * m + (1.0 - b1) * g
    v_new = b2 * v + (1.0 - b2) * g * g
    if nesterov:
        m_hat = b1 * m_new / (1.0 - b1 ** (count + 1)) + (1.0 - b1) * g / (1.0 - b1 ** count)
    else:
        m_hat = m_new / (1.0 - b1 ** count)
    v_hat = v_new / (1.0 - b2 ** count)
    return m_hat / (torch.sqrt(v_hat + eps_root) + eps), m_new, v_new


def adamw(learning_rate, b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0, weight_decay=1e-4,
          nesterov=False, mask=None):
    """optax.adamw: chain(scale_by_adam, add_decayed_weights(wd), scale_by_learning_rate).
    Weight decay applies to every leaf when mask is None."""

    def init(params):
        return SimpleNamespace(count=0, mu={k: torch.zeros_like(p) for k, p in params.items()},
                               nu={k: torch.zeros_like(p) for k, p in params.items()})

    def update(grads, state, params):
        count = state.count + 1
        upd, mu, nu = {}, {}, {}
        for k, g in grads.items():
            d, mu[k], nu[k] = _adam_direction(g, state.mu[k], state.nu[k], count, b1, b2, eps,
                                              eps_root, nesterov)
            if weight_decay != 0.0 and (mask is None or mask(k)):
                d = d + weight_decay * params[k]
            upd[k] = -learning_rate * d
        return upd, SimpleNamespace(count=count, mu=mu, nu=nu)

    return SimpleNamespace(init=init, update=update)


# ----------------------------------------------------------------------------
# Muon (optim/factory.py:441-484 -> optax.contrib.muon)
# ----------------------------------------------------------------------------
def _bf(x):
    return x.to(torch.bfloat16).to(x.dtype)


def newton_schulz(x, coeffs=(3.4445, -4.7750, 2.0315), steps=5, eps=1e-8, bf16=False):
    """optax.contrib orthogonalize_via_newton_schulz for dimension numbers (0,1):
    transpose if rows > cols, X /= ||X||_F + eps, 5x {A=XX^T; B=bA+cA^2; X=aX+BX}.

    ``bf16=True`` is a NOISE MODEL of the device's one-workgroup NS (csrc/muon_fused.hip), not a
    reference semantic: the MFMA operands bf16(X) and A' = bf16(b X X^T) with fp32 accumulation,
    B = (c/b^2) A'A' + A' kept in fp32 (the kernel's hi + lo images), X carried in fp32 across
    iterations (X' = B bf16(X) + a X) -- the parity tests use it to size the rounding spread of a
    bf16-NS trajectory."""
    a, b, c = coeffs
    transposed = x.shape[0] > x.shape[1]
    if transposed:
        x = x.t()
    x = x / (torch.linalg.norm(x) + eps)
    for _ in range(steps):
        if bf16:
            xb = _bf(x)
            A1 = _bf(b * (xb @ xb.t()))
            B = (c / (b * b)) * (A1 @ A1) + A1
            x = a * x + B @ xb
        else:
            A = x @ x.t()
            B = b * A + c * (A @ A)
            x = a * x + B @ x
    return x.t() if transposed else x


def muon(learning_rate, ns_coeffs=(3.4445, -4.7750, 2.0315), ns_steps=5, beta=0.95, eps=1e-8,
         weight_decay=0.0, nesterov=True, adam_b1=0.9, adam_b2=0.999, adam_eps_root=0.0,
         adam_weight_decay=0.0, adam_nesterov=True, shape_scale=True, routed=None, adaptive=False, ns_bf16=False):
    """partition{'muon': chain(scale_by_muon, add_decayed_weights(wd), scale_by_lr),
    'adam': adamw(b1, b2, eps, eps_root, wd, nesterov)}; labels from
    optim/muon.py:120-129 (should_use_matrix_preconditioner).

    scale_by_muon: mu = beta*mu + (1-beta)*g; nesterov mu_hat = beta*mu/(1-beta^(t+1))
    + (1-beta)*g/(1-beta^t); NS5 orthogonalisation; adaptive (factory.py:457,475 muon_adaptive):
    O <- <mu_hat, O>_F * O, optax.contrib.muon's dual-norm scaling (einsum('ij,ij,ab->ab', mu_hat, O,
    O), arXiv 2409.20325; recalled from the optax source -- optax is absent here, so unpinned);
    x sqrt(max(1, fan_out/fan_in)).
    ``adam_nesterov``/``shape_scale`` are switches for the two recalled optax details
    (SURVEY.md §7 hard part (i)); ``ns_bf16``: newton_schulz's device noise model (tests only)."""
    routed = routed or should_use_matrix_preconditioner

    def init(params):
        return SimpleNamespace(count=0, mu={k: torch.zeros_like(p) for k, p in params.items()},
                               nu={k: torch.zeros_like(p) for k, p in params.items() if not routed(k, p)})

    def update(grads, state, params):
        count = state.count + 1
        upd, mu, nu = {}, {}, {}
        for k, g in grads.items():
            p = params[k]
            if routed(k, p):
                mu[k] = beta * state.mu[k] + (1.0 - beta) * g
                if nesterov:
                    mh = beta * mu[k] / (1.0 - beta ** (count + 1)) + (1.0 - beta) * g / (1.0 - beta ** count)
                else:
                    mh = mu[k] / (1.0 - beta ** count)
                o = newton_schulz(mh, ns_coeffs, ns_steps, eps, bf16=ns_bf16)
                if adaptive:
                    o = (mh * o).sum() * o
                if shape_scale:
                    o = o * max(1.0, p.shape[1] / p.shape[0]) ** 0.5
                if weight_decay != 0.0:
                    o = o + weight_decay * p
                upd[k] = -learning_rate * o
            else:
                d, mu[k], nu[k] = _adam_direction(g, state.mu[k], state.nu[k], count, adam_b1, adam_b2,
                                                  eps, adam_eps_root, adam_nesterov)
                if adam_weight_decay != 0.0:
                    d = d + adam_weight_decay * p
                upd[k] = -learning_rate * d
        return upd, SimpleNamespace(count=count, mu=mu, nu=nu)

    return SimpleNamespace(init=init, update=update)


# ----------------------------------------------------------------------------
# SOAP (optim/soap.py:136-368)
# ----------------------------------------------------------------------------
def _eigh_desc(mat):
    """soap.py:100-105."""
    m = 0.5 * (mat + mat.t())
    _, q = torch.linalg.eigh(m + 1e-30 * torch.eye(m.shape[0], dtype=m.dtype))
    return torch.flip(q, dims=[1])


def _refresh_qr_and_reindex_v(L, R, QL, QR, v):
    """soap.py:108-133."""
    est_l = torch.diag(QL.t() @ L @ QL)
    idx_l = torch.argsort(-est_l, stable=True)
    v_new = v[idx_l, :]
    QL_new, _ = torch.linalg.qr(L @ QL[:, idx_l], mode="reduced")
    est_r = torch.diag(QR.t() @ R @ QR)
    idx_r = torch.argsort(-est_r, stable=True)
    v_new = v_new[:, idx_r]
    QR_new, _ = torch.linalg.qr(R @ QR[:, idx_r], mode="reduced")
    return QL_new, QR_new, v_new


def soap(learning_rate, b1=0.95, b2=0.95, eps=1e-8, weight_decay=0.01, precondition_frequency=10,
         shampoo_beta2=None, correct_bias=True):
    """chain(scale_by_soap, scale_by_learning_rate) (soap.py:345-368)."""
    sb2 = b2 if shampoo_beta2 is None else shampoo_beta2

    def init(params):
        st = {}
        for k, p in params.items():
            s = SimpleNamespace(m=torch.zeros_like(p), v=torch.zeros_like(p), soap=False, step=0)
            if should_use_matrix_preconditioner(k, p):
                r, c = p.shape
                s.soap = True
                s.L = torch.zeros(r, r, dtype=p.dtype)
                s.R = torch.zeros(c, c, dtype=p.dtype)
                s.QL = torch.eye(r, dtype=p.dtype)
                s.QR = torch.eye(c, dtype=p.dtype)
                s.step = -1
            st[k] = s
        return st

    def _bc(step):
        return (1.0 - b1 ** step, 1.0 - b2 ** step) if correct_bias else (1.0, 1.0)

    def update(grads, state, params):
        upd, new = {}, {}
        for k, g in grads.items():
            s = state[k]
            p = params[k] if params is not None else None
            use_wd = p is not None and weight_decay != 0.0
            if s.soap:
                Lu, Ru = g @ g.t(), g.t() @ g
                L_new = sb2 * s.L + (1.0 - sb2) * Lu
                R_new = sb2 * s.R + (1.0 - sb2) * Ru
                if s.step < 0:
                    upd[k] = torch.zeros_like(g)
                    new[k] = SimpleNamespace(m=s.m, v=s.v, soap=True, L=L_new, R=R_new,
                                             QL=_eigh_desc(L_new), QR=_eigh_desc(R_new), step=0)
                    continue
                step = s.step + 1
                g_rot = s.QL.t() @ g @ s.QR
                m_new = b1 * s.m + (1.0 - b1) * g_rot
                v_new = b2 * s.v + (1.0 - b2) * g_rot * g_rot
                bc1, bc2 = _bc(step)
                n_rot = (m_new / bc1) / (torch.sqrt(v_new / bc2) + eps)
                n = s.QL @ n_rot @ s.QR.t()
                if use_wd:
                    n = n + weight_decay * p
                m_orig = s.QL @ m_new @ s.QR.t()
                if precondition_frequency > 0 and step % precondition_frequency == 0:
                    QL_new, QR_new, v_al = _refresh_qr_and_reindex_v(L_new, R_new, s.QL, s.QR, v_new)
                else:
                    QL_new, QR_new, v_al = s.QL, s.QR, v_new
                m_rep = QL_new.t() @ m_orig @ QR_new
                upd[k] = -learning_rate * n
                new[k] = SimpleNamespace(m=m_rep, v=v_al, soap=True, L=L_new, R=R_new, QL=QL_new,
                                         QR=QR_new, step=step)
            else:
                step = s.step + 1
                m_new = b1 * s.m + (1.0 - b1) * g
                v_new = b2 * s.v + (1.0 - b2) * g * g
                bc1, bc2 = _bc(step)
                n = (m_new / bc1) / (torch.sqrt(v_new / bc2) + eps)
                if use_wd:
                    n = n + weight_decay * p
                upd[k] = -learning_rate * n
                new[k] = SimpleNamespace(m=m_new, v=v_new, soap=False, step=step)
        return upd, new

    return SimpleNamespace(init=init, update=update)


# ----------------------------------------------------------------------------
# Shampoo (optim/shampoo.py:81-296)
# ----------------------------------------------------------------------------
def shampoo(learning_rate, eps=1e-4, exponent=0.25, weight_decay=0.0, adam_b1=0.9, adam_b2=0.999,
            adam_eps=1e-8):
    """chain(scale_by_shampoo, scale_by_learning_rate)."""

    def init(params):
        st = {}
        for k, p in params.items():
            s = SimpleNamespace(m=torch.zeros_like(p), v=torch.zeros_like(p), shampoo=False)
            if should_use_shampoo(k, p):
                r, c = p.shape
                s.shampoo = True
                s.L = eps * torch.eye(r, dtype=p.dtype)
                s.R = eps * torch.eye(c, dtype=p.dtype)
            st[k] = s
        return SimpleNamespace(count=0, per_param=st)

    def update(grads, state, params):
        count = state.count + 1
        m_bc = 1.0 - adam_b1 ** count
        v_bc = 1.0 - adam_b2 ** count
        upd, new = {}, {}
        for k, g in grads.items():
            s = state.per_param[k]
            p = params[k] if params is not None else None
            if s.shampoo:
                r, c = g.shape
                L_new = s.L + g @ g.t()
                R_new = s.R + g.t() @ g
                eL, UL = torch.linalg.eigh(L_new + eps * torch.eye(r, dtype=g.dtype))
                eR, UR = torch.linalg.eigh(R_new + eps * torch.eye(c, dtype=g.dtype))
                PL = (UL * torch.clamp(eL, min=eps) ** (-exponent)) @ UL.t()
                PR = (UR * torch.clamp(eR, min=eps) ** (-exponent)) @ UR.t()
                gp = PL @ g @ PR
                if p is not None and weight_decay != 0.0:
                    gp = gp + weight_decay * p
                upd[k] = -learning_rate * gp
                new[k] = SimpleNamespace(m=s.m, v=s.v, shampoo=True, L=L_new, R=R_new)
            else:
                m_new = (1.0 - adam_b1) * g + adam_b1 * s.m
                v_new = (1.0 - adam_b2) * g * g + adam_b2 * s.v
                u = (m_new / m_bc) / (torch.sqrt(v_new / v_bc) + adam_eps)
                if p is not None and weight_decay != 0.0:
                    u = u + weight_decay * p
                upd[k] = -learning_rate * u
                new[k] = SimpleNamespace(m=m_new, v=v_new, shampoo=False)
        return upd, SimpleNamespace(count=count, per_param=new)

    return SimpleNamespace(init=init, update=update)


# ----------------------------------------------------------------------------
# Signum (optim/signum.py:14-66)
# ----------------------------------------------------------------------------
def signum(learning_rate, momentum=0.9, nesterov=False, weight_decay=0.0):
    """m = mom m + (1-mom) g; d = (1-mom) g + mom m (nesterov) or m; u = -lr (sign(d) + wd p)."""
    if learning_rate < 0.0:
        raise ValueError(f"learning_rate must be >= 0, got {learning_rate}.")
    if momentum < 0.0 or momentum >= 1.0:
        raise ValueError(f"momentum must be in [0, 1), got {momentum}.")
    if weight_decay < 0.0:
        raise ValueError(f"weight_decay must be >= 0, got {weight_decay}.")

    def init(params):
        return SimpleNamespace(momentum_buffer={k: torch.zeros_like(p) for k, p in params.items()})

    def update(grads, state, params=None):
        buf, upd = {}, {}
        for k, g in grads.items():
            m = momentum * state.momentum_buffer[k] + (1.0 - momentum) * g
            buf[k] = m
            d = (1.0 - momentum) * g + momentum * m if nesterov else m
            u = torch.sign(d)
            if weight_decay > 0.0:
                if params is None:
                    raise ValueError("Signum with weight_decay requires current params.")
                u = u + weight_decay * params[k]
            upd[k] = -learning_rate * u
        return upd, SimpleNamespace(momentum_buffer=buf)

    return SimpleNamespace(init=init, update=update)


# ----------------------------------------------------------------------------
# schedule-free wrapper (optim/factory.py:82-99 -> optax.contrib.schedule_free, optax 0.2.6)
# ----------------------------------------------------------------------------
def schedule_free(base, learning_rate, b1=0.9, weight_lr_power=2.0):
    """optax.contrib.schedule_free (Defazio et al. 2024), restated: params are y (where gradients
    are taken); z (init = params) takes the base optimizer's steps; x is the weighted average with
    c_k = w_k / sum w, w_k = max_lr^weight_lr_power; y = b1 x + (1-b1) z.  x is recomputed from
    y and the old z each step: x_prev = (y - (1-b1) z_old) / b1.  Scalars in fp32 as optax keeps them."""
    if b1 == 0:
        raise ValueError("The current implementation of schedule_free requires b1 > 0.")
    f32 = torch.float32

    def init(params):
        return SimpleNamespace(b1=torch.tensor(b1, dtype=f32), weight_sum=torch.zeros((), dtype=f32),
                               step_count=1, max_lr=torch.zeros((), dtype=f32), base_state=base.init(params),
                               z={k: p.clone() for k, p in params.items()})

    def update(grads, state, params):
        lr = torch.tensor(learning_rate, dtype=f32)
        max_lr = torch.maximum(state.max_lr, lr)
        weight = max_lr ** weight_lr_power
        total = state.weight_sum + weight
        ck = torch.nan_to_num(weight / total, nan=0.0)
        if torch.isnan(weight) or torch.isnan(total):
            ck = torch.tensor(float("nan"), dtype=f32)
        base_upd, base_state = base.update(grads, state.base_state, params)
        z_new = {k: (state.z[k] + base_upd[k]).to(state.z[k].dtype) for k in params}
        upd = {}
        for k, y in params.items():
            prev_x = (y - (1.0 - state.b1) * state.z[k]) / state.b1
            x = (1.0 - ck) * prev_x + ck * z_new[k]
            upd[k] = (state.b1 * x + (1.0 - state.b1) * z_new[k]) - y
        return upd, SimpleNamespace(b1=state.b1, weight_sum=total, step_count=state.step_count + 1, max_lr=max_lr,
                                    base_state=base_state, z=z_new)

    return SimpleNamespace(init=init, update=update)


def get_optimizer(cfg, ns_bf16=False):
    """optim/factory.py:180-802 restricted to the hot-path branches (+ the schedule-free wrapper).
    ``ns_bf16``: Muon's Newton-Schulz through the device noise model (newton_schulz)."""
    name = str(getattr(cfg, "optim", "adamw")).lower()
    lr = float(cfg.lr)
    g = lambda k, d: getattr(cfg, k, d)  # noqa: E731
    if name in {"adam", "adamw"}:
        tx = adamw(lr, b1=g("beta1", 0.9), b2=g("beta2", 0.999), eps=g("eps", 1e-8),
                   weight_decay=g("weight_decay", 0.0))
    elif name == "muon":
        wd = g("weight_decay", 0.0)
        tx = muon(lr, ns_coeffs=tuple(g("muon_ns_coeffs", (3.4445, -4.7750, 2.0315))),
                  ns_steps=g("muon_ns_steps", 5), beta=g("muon_beta", 0.95), eps=g("eps", 1e-8),
                  weight_decay=wd, nesterov=g("muon_nesterov", True), adam_b1=g("beta1", 0.9),
                  adam_b2=g("beta2", 0.999), adam_eps_root=g("adam_eps_root", 0.0),
                  adam_weight_decay=wd, adam_nesterov=g("muon_nesterov", True),
                  adaptive=bool(g("muon_adaptive", False)), ns_bf16=ns_bf16)
    elif name == "soap":
        tx = soap(lr, b1=g("beta1", 0.95), b2=g("beta2", 0.95), eps=g("eps", 1e-8),
                  weight_decay=g("weight_decay", 0.01), precondition_frequency=g("precondition_frequency", 10),
                  shampoo_beta2=g("shampoo_beta2", None), correct_bias=g("correct_bias", True))
    elif name == "shampoo":
        tx = shampoo(lr, eps=g("eps", 1e-4), exponent=g("shampoo_exponent", 0.25),
                     weight_decay=g("weight_decay", 0.0), adam_b1=g("beta1", 0.9), adam_b2=g("beta2", 0.999),
                     adam_eps=g("adam_eps", 1e-8))
    elif name in {"signum", "sign_sgd", "sign-sgd", "signsgd"}:
        tx = signum(lr, momentum=g("signum_momentum", g("beta1", 0.9)), nesterov=g("signum_nesterov", False),
                    weight_decay=g("weight_decay", 0.0))
    else:
        raise ValueError(f"Unknown optimizer name: {cfg.optim}")
    if g("schedule_free", False):       # factory.py:82-99, 801
        tx = schedule_free(tx, g("schedule_free_lr", cfg.lr), b1=g("schedule_free_b1", 0.9),
                           weight_lr_power=g("schedule_free_weight_lr_power", 2.0))
    return tx
