"""LM data path: samplers (data/lm_datasampler.py:19-162), loader over the
reference's on-disk HF format (data/lm_loader.py:17-118), rank interleave = the reference's
single-process pmap batch grouping (train_lm.py:151-170), and a tiny end-to-end train_lm run."""
import numpy as np
import pytest
import torch


def _dataset(tmp_path, n=24, T=8, docs=True):
    from datasets import Dataset
    ids = (np.arange(n * (T + 1)).reshape(n, T + 1) % 500).astype(np.int32)
    cols = {"input_ids": ids.tolist()}
    if docs:
        cols["docs_lengths"] = [[2, 3, T + 1 - 5]] * n
    path = str(tmp_path / "ds")
    Dataset.from_dict(cols).save_to_disk(path)
    return path, ids


def test_samplers_match_reference_semantics():
    from plaincv_amd.data.lm_datasampler import StatefulRandomSampler, StatefulSequentialSampler
    data = list(range(10))
    assert list(StatefulSequentialSampler(data, batch_size=3, start_idx=2)) == list(range(6, 10))
    s = StatefulRandomSampler(data, batch_size=2, start_idx=1, shuffle=True, seed=7)
    rng = np.random.default_rng(7)
    assert list(s) == rng.permutation(np.arange(10)).tolist()[2:]
    assert list(s) == rng.permutation(np.arange(10)).tolist()[2:]      # next epoch: next permutation
    with pytest.raises(ValueError):
        StatefulRandomSampler(data, batch_size=2, shuffle=True, seed=None)


def test_rank_interleave_equals_single_process_grouping(tmp_path):
    from plaincv_amd.data.lm_loader import get_dataloaders
    from utils import Config
    path, ids = _dataset(tmp_path)
    cfg = Config(trainset_path=path, micro_batch_size=4, sampler="sequential", seq_len=8)
    single, _ = get_dataloaders(cfg)
    seq = [b["input_ids"] for b in single]
    for world in (2, 3):
        per_rank = [[b["input_ids"] for b in get_dataloaders(cfg, rank=r, world=world)[0]] for r in range(world)]
        # reference: batch k goes to device k % world of optimizer step k // world
        for k, b in enumerate(seq[: len(seq) // world * world]):
            assert np.array_equal(per_rank[k % world][k // world], b)
    b0 = next(iter(single))
    assert b0["input_ids"].dtype == np.int32 and b0["docs_lengths"][0] == [2, 3, 4]
    with pytest.raises(NotImplementedError):
        from plaincv_amd.data.lm_loader import get_sampler
        get_sampler(list(range(4)), Config(sampler="nope", micro_batch_size=2))


@pytest.mark.gpu
def test_train_lm_end_to_end(dev, tmp_path, capsys):
    """train_lm.run on a tiny config: doc masking on, 2 micro-steps, clip, eval; loss finite and
    falling on a memorisable stream."""
    import train_lm
    from utils import Config
    path, _ = _dataset(tmp_path, n=16, T=64)
    cfg = Config(model="transformer", vocab_size=512, d_model=64, expand="8/3", n_layers=2, n_heads=2,
                 mlp_class="glu", seq_len=64, tie_embeddings=False, rope_theta=500000.0, dtype="bfloat16",
                 trainset_path=path, validset_path=path, valid_tokens=4 * 65, sampler="sequential",
                 micro_batch_size=4, grad_accumulation_steps=2, steps_budget=12, grad_clip=1.0, optim="adamw",
                 lr=3e-3, weight_decay=0.0, beta1=0.9, beta2=0.95, intra_doc_masking=True, log_every_steps=1,
                 eval_every_steps=12, seed=0)
    train_lm.run(cfg)
    out = capsys.readouterr().out
    losses = [float(l.split("train_loss: ")[1].split(" |")[0]) for l in out.splitlines() if "train_loss" in l]
    assert len(losses) == 12 and all(np.isfinite(losses))
    assert losses[-1] < losses[0]
    assert "eval_loss" in out and "Training complete." in out
