"""ViT data path: local-file Fashion-MNIST (IDX) and Tiny-ImageNet (JPEG tree)
loaders with the reference's contract (data/fashion_mnist.py:28-52, data/tiny_imagenet.py:36-203),
and the train.py epoch loop on the GPU."""
import gzip

import numpy as np
import pytest


def _write_idx(path, arr, gz=True):
    hdr = bytes([0, 0, 8, arr.ndim]) + b"".join(int(d).to_bytes(4, "big") for d in arr.shape)
    data = hdr + arr.astype(np.uint8).tobytes()
    with (gzip.open if gz else open)(path, "wb") as f:
        f.write(data)


def test_fashion_mnist_idx(tmp_path):
    from plaincv_amd.data.images import get_datasets
    g = np.random.default_rng(0)
    xtr, ytr = g.integers(0, 256, (10, 28, 28)), g.integers(0, 10, (10,))
    xte, yte = g.integers(0, 256, (7, 28, 28)), g.integers(0, 10, (7,))
    _write_idx(tmp_path / "train-images-idx3-ubyte.gz", xtr)
    _write_idx(tmp_path / "train-labels-idx1-ubyte.gz", ytr)
    _write_idx(tmp_path / "t10k-images-idx3-ubyte", xte, gz=False)
    _write_idx(tmp_path / "t10k-labels-idx1-ubyte", yte, gz=False)
    tr, te = get_datasets("fashion_mnist", 3, seed=5, data_root=tmp_path)
    trb, teb = list(tr), list(te)
    assert len(trb) == 3 and len(teb) == 2                      # drop_remainder
    assert trb[0][0].shape == (3, 28, 28, 1) and trb[0][0].dtype == np.uint8 and trb[0][1].dtype == np.int32
    assert np.array_equal(teb[0][0][..., 0], xte[:3]) and np.array_equal(teb[1][1], yte[3:6])   # eval in order
    seen = np.concatenate([b[1] for b in trb])
    order = np.random.default_rng(5).permutation(10)[:9]
    assert np.array_equal(seen, ytr[order])
    with pytest.raises(FileNotFoundError):
        get_datasets("fashion_mnist", 3, data_root=tmp_path / "nope")


def test_tiny_imagenet_tree(tmp_path):
    from PIL import Image
    from plaincv_amd.data.images import get_datasets
    d = tmp_path / "tiny-imagenet-200"
    wnids = ["n01", "n02", "n03"]
    (d / "val" / "images").mkdir(parents=True)
    (d / "wnids.txt").write_text("\n".join(wnids) + "\n")
    g = np.random.default_rng(1)
    for w in wnids:
        (d / "train" / w / "images").mkdir(parents=True)
        for i in range(2):
            Image.fromarray(g.integers(0, 256, (64, 64, 3), dtype=np.uint8)).save(d / "train" / w / "images" / f"{w}_{i}.JPEG")
    lines = []
    for i, w in enumerate(["n03", "n01", "n02", "n03"]):
        Image.fromarray(np.full((64, 64, 3), 10 * i, dtype=np.uint8)).save(d / "val" / "images" / f"val_{i}.JPEG")
        lines.append(f"val_{i}.JPEG\t{w}\t0\t0\t63\t63")
    (d / "val" / "val_annotations.txt").write_text("\n".join(lines))
    tr, va = get_datasets("tiny_imagenet", 2, seed=0, data_root=tmp_path)
    trb, vab = list(tr), list(va)
    assert len(trb) == 3 and trb[0][0].shape == (2, 64, 64, 3)
    assert sorted(np.concatenate([b[1] for b in trb]).tolist()) == [0, 0, 1, 1, 2, 2]
    assert np.concatenate([b[1] for b in vab]).tolist() == [2, 0, 1, 2]
    tr32, _ = get_datasets("tiny_imagenet", 2, seed=0, image_size=32, data_root=tmp_path)
    assert next(iter(tr32))[0].shape == (2, 32, 32, 3)


@pytest.mark.gpu
def test_train_vit_epochs(dev, capsys):
    import train
    from utils import Config
    cfg = Config(dataset="tiny_imagenet_synthetic", batch_size=16, num_epochs=2, image_size=32, seed=0,
                 model="vit_small", vit_patch_size=4, vit_hidden_size=64, vit_mlp_dim=128, vit_layers=2,
                 vit_heads=2, vit_dropout=0.1, vit_use_layernorm=True, optim="muon", lr=1e-3,
                 weight_decay=0.01, beta1=0.9, beta2=0.9)
    train.run(cfg)
    out = capsys.readouterr().out
    lines = [l for l in out.splitlines() if l.startswith("epoch")]
    assert len(lines) == 2 and "eval_accuracy" in lines[0]
    vals = [float(l.split("train_loss: ")[1].split(" |")[0]) for l in lines]
    assert all(np.isfinite(vals))
