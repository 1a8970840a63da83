"""Shared comparison helpers for the GPU parity tests (test infrastructure)."""
import torch

# SURVEY.md §8c bounds on one optimizer step given identical gradients
ADAM_TOL = 1e-5      # fp32 AdamW / Muon's Adam branch
MUON_TOL = 2e-2      # bf16-MFMA Newton-Schulz vs fp32 NS5, rel-Frobenius


def rel(a, b, floor=1e-30):
    a, b = a.double(), b.double()
    return (a - b).norm().item() / max(b.norm().item(), floor)


def step_rel(p0, p1, u, ulps=0.5):
    """Relative error of the applied step p1 - p0 against the expected update u, net of the
    fp32 rounding of p0 + u (`ulps` ulps of p1 per element: half an ulp for p + u; a few for
    schedule-free, whose y' = b1 x + (1 - b1) z' re-forms p from several rounded terms)."""
    p0, p1, u = p0.double(), p1.double(), u.double()
    err = (p1 - p0 - u).norm().item()
    p1f = p1.float()
    ulp = (torch.nextafter(p1f.abs(), torch.full_like(p1f, float("inf"))) - p1f.abs()).double()
    floor = ulps * ulp.norm().item()
    un = max(u.norm().item(), 1e-30)
    return max(0.0, err - floor) / un


def routed(name, p):
    from oracle.optim import should_use_matrix_preconditioner
    return should_use_matrix_preconditioner(name, p)


def step_bound(optim, name, p):
    """Bound on step_rel for one leaf: Muon's routed leaves carry the bf16 NS error."""
    return MUON_TOL if (optim == "muon" and routed(name, p)) else ADAM_TOL


def global_norm(grads):
    return torch.sqrt(sum((g.double() ** 2).sum() for g in grads.values())).item()
