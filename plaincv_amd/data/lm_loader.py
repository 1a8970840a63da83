"""LM data loaders (mirrors data/lm_loader.py:17-118).

``get_dataloaders(cfg, rank=0, world=1)`` -> (train_iterable, valid_iterable or None).  The
datasets are the reference's on-disk HF format (``datasets.load_from_disk``): an ``input_ids``
column of length seq_len + 1 (int) and optionally ``docs_lengths`` (list of document lengths,
the intra-document mask input, train_lm.py:107-131).  Each batch is
``{"input_ids": np.int32 [B, T+1], "docs_lengths": list[list[int]]}`` (the reference's collate_fn);
the training loop moves input_ids to the GPU and the document lengths become the attention
kernels' per-token bounds (engine.lm.doc_bounds).  Sampler choice and resume offsets follow
``_get_sampler_jax`` (lm_loader.py:88-118); the DP rank split is RankInterleavedBatches.
"""
import numpy as np

from .lm_datasampler import (RandomSampler, RankInterleavedBatches, SequentialSampler, StatefulRandomSampler,
                             StatefulSequentialSampler)


def _g(cfg, k, d=None):
    return cfg.get(k, d) if isinstance(cfg, dict) else getattr(cfg, k, d)


def _load(path):
    from datasets import Dataset, load_from_disk
    ds = load_from_disk(path)
    if not isinstance(ds, Dataset):
        raise ValueError("dataset should be a datasets.Dataset")
    return ds


def get_sampler(train_set, cfg):
    """lm_loader.py:88-118."""
    name = _g(cfg, "sampler", "sequential")
    mb = int(_g(cfg, "micro_batch_size"))
    resume = bool(_g(cfg, "resume", False))
    start = int(_g(cfg, "resume_step", 0)) * int(_g(cfg, "grad_accumulation_steps", 1)) if resume else 0
    if name == "random":
        return RandomSampler(train_set, seed=_g(cfg, "sampler_seed", None))
    if name == "sequential":
        return SequentialSampler(train_set)
    if name == "stateful_random":
        return StatefulRandomSampler(train_set, batch_size=mb, shuffle=True, seed=_g(cfg, "sampler_seed", None),
                                     start_idx=start)
    if name == "stateful_sequential":
        return StatefulSequentialSampler(train_set, batch_size=mb, start_idx=start)
    raise NotImplementedError(f"Sampler {name} is not implemented.")


class BatchIterable:
    """Re-iterable (one pass per epoch) stream of collated micro-batches."""

    def __init__(self, dataset, sampler, batch_size, rank=0, world=1):
        self.dataset, self.batches = dataset, RankInterleavedBatches(sampler, batch_size, rank, world)
        self.has_docs = "docs_lengths" in dataset.column_names

    def __len__(self):
        return len(self.batches)

    def __iter__(self):
        for idx in self.batches:
            rows = self.dataset[idx]          # columnar slice: {"input_ids": [...], "docs_lengths": [...]}
            out = {"input_ids": np.asarray(rows["input_ids"], dtype=np.int32)}
            if self.has_docs:
                out["docs_lengths"] = [np.asarray(x).tolist() for x in rows["docs_lengths"]]
            yield out


def get_dataloaders(cfg, rank=0, world=1):
    train_set = _load(_g(cfg, "trainset_path"))
    mb = int(_g(cfg, "micro_batch_size"))
    train = BatchIterable(train_set, get_sampler(train_set, cfg), mb, rank, world)
    valid = None
    vpath = _g(cfg, "validset_path", None)
    if vpath:
        valid_set = _load(vpath)
        vt = _g(cfg, "valid_tokens", None)
        if vt:
            rows = int(vt) // (int(_g(cfg, "seq_len")) + 1)
            if rows > 0:
                valid_set = valid_set.select(range(min(rows, len(valid_set))))
        valid = BatchIterable(valid_set, SequentialSampler(valid_set), mb, rank, world)
    return train, valid


def next_batch(it, loader):
    """train_lm.py:151-159 (_next_batch with one device per process): restart at epoch end."""
    try:
        return next(it), it
    except StopIteration:
        it = iter(loader)
        return next(it), it
