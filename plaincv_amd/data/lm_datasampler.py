"""Samplers for the LM token datasets (mirrors data/lm_datasampler.py:19-162).

Same index streams as the reference's StatefulSequentialSampler / StatefulRandomSampler (resume
offsets in units of micro-batches; the random one draws a new numpy permutation per epoch from a
persistent default_rng(seed)).  Data parallelism is one process per GPU here, so the rank split
is a batch-level interleave (:class:`RankInterleavedBatches`): rank r takes micro-batches r,
r + world, r + 2 world, ... of the single index stream, which is exactly how the reference's
one-process pmap run hands consecutive loader batches to its devices (train_lm.py:134-170,
``_next_batch`` with ``num_batches = n_devices``).
"""
from typing import Iterator, Optional, Sized

import numpy as np


class StatefulSequentialSampler:
    """data/lm_datasampler.py:19-30."""

    def __init__(self, data_source: Sized, batch_size: int, start_idx: int = 0):
        self.data_source = data_source
        self.start = int(start_idx) * int(batch_size)

    def __iter__(self) -> Iterator[int]:
        return iter(range(self.start, len(self.data_source)))

    def __len__(self) -> int:
        return max(0, len(self.data_source) - self.start)


class StatefulRandomSampler:
    """data/lm_datasampler.py:33-69."""

    def __init__(self, data_source: Sized, batch_size: int, start_idx: int = 0, shuffle: bool = False,
                 seed: Optional[int] = None):
        self.data_source = data_source
        self.start = int(start_idx) * int(batch_size)
        self.shuffle = bool(shuffle)
        if self.shuffle:
            if seed is None:
                raise ValueError("Seed must be set if shuffle=True in a stateful sampler.")
            self.rng = np.random.default_rng(int(seed))
        else:
            self.rng = None

    def __iter__(self) -> Iterator[int]:
        indices = np.arange(len(self.data_source), dtype=np.int64)
        if self.shuffle:
            indices = self.rng.permutation(indices)
        return iter(indices[self.start:].tolist())

    def __len__(self) -> int:
        return max(0, len(self.data_source) - self.start)


class SequentialSampler:
    def __init__(self, data_source: Sized):
        self.data_source = data_source

    def __iter__(self):
        return iter(range(len(self.data_source)))

    def __len__(self):
        return len(self.data_source)


class RandomSampler:
    """torch.utils.data.RandomSampler(generator=manual_seed(seed)) order (factory call site
    lm_loader.py:96-100): a fresh torch randperm per epoch."""

    def __init__(self, data_source: Sized, seed: Optional[int] = None):
        import torch
        self.data_source = data_source
        self.gen = torch.Generator().manual_seed(int(seed)) if seed else None

    def __iter__(self):
        import torch
        return iter(torch.randperm(len(self.data_source), generator=self.gen).tolist())

    def __len__(self):
        return len(self.data_source)


class RankInterleavedBatches:
    """Micro-batches (lists of indices, drop_last) of one sampler, rank r taking batches
    r, r + world, ... -- the per-device batches of the reference's single-process pmap."""

    def __init__(self, sampler, batch_size: int, rank: int = 0, world: int = 1):
        self.sampler, self.batch_size, self.rank, self.world = sampler, int(batch_size), int(rank), int(world)

    def __iter__(self):
        batch, k = [], 0
        for idx in self.sampler:
            batch.append(int(idx))
            if len(batch) == self.batch_size:
                if k % self.world == self.rank:
                    yield batch
                batch, k = [], k + 1

    def __len__(self):
        nb = len(self.sampler) // self.batch_size
        return nb // self.world + (1 if self.rank < nb % self.world else 0)
