"""Train/eval step semantics restated from engine/flax_engine.py and train_lm.py
(TEST INFRASTRUCTURE ONLY).  Gradients come from torch CPU autograd."""
import torch


def cross_entropy_loss(logits, labels):
    """engine/flax_engine.py:13-16: -mean(sum(one_hot * log_softmax))."""
    lp = torch.log_softmax(logits, dim=-1)
    return -lp.gather(-1, labels.long()[..., None]).squeeze(-1).mean()


def compute_metrics(logits, labels):
    """engine/flax_engine.py:19-22."""
    loss = cross_entropy_loss(logits, labels)
    acc = (logits.argmax(-1) == labels.long()).to(logits.dtype).mean()
    return {"loss": loss, "accuracy": acc}


def lm_loss_and_acc(logits, labels):
    """train_lm.py:181-186: fp32 softmax-CE with integer labels, mean; argmax acc."""
    lf = logits.float() if logits.dtype != torch.float64 else logits
    loss = (torch.logsumexp(lf, -1) - lf.gather(-1, labels.long()[..., None]).squeeze(-1)).mean()
    acc = (lf.argmax(-1) == labels.long()).float().mean()
    return loss, acc


def prepare_batch(input_ids, seq_len):
    """train_lm.py:134-146: inputs = ids[:, :-1], labels = ids[:, 1:]."""
    if input_ids.shape[1] != seq_len + 1:
        raise ValueError(f"Expected input_ids length {seq_len + 1} (seq_len+1) but got {input_ids.shape[1]}.")
    return input_ids[:, :-1], input_ids[:, 1:]


def global_norm(grads):
    """optax.global_norm: sqrt(sum of squares over all leaves)."""
    return torch.sqrt(sum((g.double() * g.double()).sum() for g in grads.values())).to(
        next(iter(grads.values())).dtype)


def clip_grads(grads, max_norm):
    """train_lm.py:173-178."""
    if max_norm is None:
        return grads
    g_norm = global_norm(grads)
    scale = torch.clamp(max_norm / (g_norm + 1e-6), max=1.0)
    return {k: g * scale for k, g in grads.items()}


def value_and_grad(loss_fn, params):
    """jax.value_and_grad over a flat param dict via torch autograd."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    out = loss_fn(leaves)
    loss = out[0] if isinstance(out, tuple) else out
    names = list(leaves)
    gs = torch.autograd.grad(loss, [leaves[k] for k in names], allow_unused=True)
    grads = {k: (g if g is not None else torch.zeros_like(leaves[k])).detach() for k, g in zip(names, gs)}
    return out, grads


def apply_updates(params, updates):
    """optax.apply_updates: (p + u).astype(p.dtype)."""
    return {k: (p + updates[k]).to(p.dtype) for k, p in params.items()}


def intra_doc_causal_mask(doc_boundaries, max_seq_length):
    """data/datasets/data_prep_utils.py:14-43: block-diagonal causal bool mask [T, T]."""
    if sum(doc_boundaries) != max_seq_length:
        raise ValueError("Sum of doc_boundaries does not match max_seq_length.")
    return torch.block_diag(*[torch.tril(torch.ones(n, n, dtype=torch.bool)) for n in doc_boundaries])


def build_attn_mask(docs_lengths, seq_len):
    """train_lm.py:97-131 (_trim_last_token + _build_attn_mask): (B, T, T) bool."""
    masks = []
    for boundaries in docs_lengths:
        b = [int(x) for x in boundaries]
        if b:
            b[-1] -= 1
            if b[-1] <= 0:
                b.pop()
        if sum(b) != seq_len:
            raise ValueError(f"Sum(doc_boundaries)={sum(b)} != seq_len={seq_len}.")
        masks.append(intra_doc_causal_mask(b, seq_len))
    return torch.stack(masks, 0)
