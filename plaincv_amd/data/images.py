"""Image datasets for the ViT (mirrors data/fashion_mnist.py:19-52, data/tiny_imagenet.py:22-203).

Same contract as the reference: iterators of (images uint8 NHWC, labels int) batches, the train
split shuffled with ``seed`` (the reference varies it per epoch, train.py:369-374), the eval
split in file order, incomplete last batches dropped.  Sources are local files only -- the
reference's tfds / HTTP downloads are not available offline, so a missing dataset raises
FileNotFoundError naming the files it looked for:

* Fashion-MNIST: the IDX files (``train-images-idx3-ubyte[.gz]`` ...) under ``data_root``;
* Tiny-ImageNet: an extracted ``tiny-imagenet-200`` tree (wnids.txt, val/val_annotations.txt,
  train/<wnid>/images/*.JPEG), located like ``_find_dataset_dir`` (tiny_imagenet.py:36-53), JPEGs
  decoded with PIL, resized bilinearly when image_size != 64 (tiny_imagenet.py:22-33);
* ``tiny_imagenet_synthetic``: uniform uint8 images / labels of the Tiny-ImageNet shape (the
  benchmark's synthetic input, BASELINE configs[1]).
The reference's tf.data shuffle buffer is not reproducible outside TensorFlow; here a numpy
permutation of the whole split is used (same distribution of orders, not the same order).
"""
import gzip
import os
from pathlib import Path

import numpy as np

DEFAULT_ROOTS = {"fashion_mnist": Path.home() / "tensorflow_datasets" / "fashion_mnist",
                 "tiny_imagenet": Path.home() / "tensorflow_datasets" / "tiny_imagenet"}


def _read_idx(path):
    op = gzip.open if str(path).endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    if data[0] != 0 or data[1] != 0 or data[2] != 8:
        raise ValueError(f"{path}: not an unsigned-byte IDX file")
    nd = data[3]
    dims = [int.from_bytes(data[4 + 4 * i: 8 + 4 * i], "big") for i in range(nd)]
    arr = np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd)
    return arr.reshape(dims)


def _find(root, stem):
    for name in (stem, stem + ".gz"):
        p = Path(root) / name
        if p.exists():
            return p
    raise FileNotFoundError(f"Fashion-MNIST file {stem}[.gz] not found under {root} "
                            "(downloads are unavailable offline; place the IDX files there)")


def _batches(images, labels, batch_size, shuffle, seed):
    n = (len(images) // batch_size) * batch_size
    order = np.random.default_rng(seed).permutation(len(images)) if shuffle else np.arange(len(images))
    for i in range(0, n, batch_size):
        idx = order[i:i + batch_size]
        yield images[idx], labels[idx].astype(np.int32)


def fashion_mnist(batch_size, seed=0, data_root=None):
    """data/fashion_mnist.py:28-52: uint8 (B, 28, 28, 1), labels in [0, 10)."""
    root = Path(data_root) if data_root else DEFAULT_ROOTS["fashion_mnist"]
    xtr = _read_idx(_find(root, "train-images-idx3-ubyte"))[..., None]
    ytr = _read_idx(_find(root, "train-labels-idx1-ubyte"))
    xte = _read_idx(_find(root, "t10k-images-idx3-ubyte"))[..., None]
    yte = _read_idx(_find(root, "t10k-labels-idx1-ubyte"))
    return _batches(xtr, ytr, batch_size, True, seed), _batches(xte, yte, batch_size, False, seed)


def find_tiny_imagenet(data_root):
    """tiny_imagenet.py:36-53."""
    root = Path(data_root)
    cands = [root / "tiny-imagenet-200", root / "tiny_imagenet-200", root / "tiny-imagenet-200_extracted",
             root / "tiny-imagenet-200_extracted" / "tiny-imagenet-200"]
    if root.exists():
        cands += [p.parent for p in root.rglob("wnids.txt")]
    for p in cands:
        if p.exists() and (p / "train").exists() and (p / "val").exists() and (p / "wnids.txt").exists():
            return p
    raise FileNotFoundError(f"tiny-imagenet-200 not found under {root} (downloads are unavailable offline)")


def _decode(path, image_size):
    from PIL import Image
    with Image.open(path) as im:
        im = im.convert("RGB")
        if image_size and image_size != 64:
            im = im.resize((image_size, image_size), Image.BILINEAR)
        return np.asarray(im, dtype=np.uint8)


def tiny_imagenet(batch_size, seed=0, image_size=64, data_root=None):
    """data/tiny_imagenet.py:152-203: uint8 (B, S, S, 3), labels = wnids.txt order."""
    d = find_tiny_imagenet(data_root or DEFAULT_ROOTS["tiny_imagenet"])
    wnids = [l.strip() for l in (d / "wnids.txt").read_text().splitlines() if l.strip()]
    cls = {w: i for i, w in enumerate(wnids)}
    val = {}
    for line in (d / "val" / "val_annotations.txt").read_text().splitlines():
        parts = line.split("\t")
        if len(parts) >= 2:
            val[parts[0]] = cls[parts[1]]
    train = sorted((str(p), cls[p.parts[-3]]) for p in (d / "train").glob("*/images/*.JPEG"))
    valid = sorted((str(p), val[p.name]) for p in (d / "val" / "images").glob("*.JPEG"))

    def split(items, shuffle):
        n = (len(items) // batch_size) * batch_size
        order = np.random.default_rng(seed).permutation(len(items)) if shuffle else np.arange(len(items))
        for i in range(0, n, batch_size):
            sel = [items[j] for j in order[i:i + batch_size]]
            yield (np.stack([_decode(p, image_size) for p, _ in sel]),
                   np.asarray([l for _, l in sel], dtype=np.int32))
    return split(train, True), split(valid, False)


def synthetic(batch_size, seed=0, image_size=64, channels=3, num_classes=200, n_train=64, n_eval=8):
    g = np.random.default_rng(seed)

    def split(n):
        for _ in range(n):
            yield (g.integers(0, 256, (batch_size, image_size, image_size, channels), dtype=np.uint8),
                   g.integers(0, num_classes, (batch_size,), dtype=np.int32))
    return split(n_train), split(n_eval)


def get_datasets(dataset, batch_size, seed=0, image_size=None, data_root=None, **kw):
    """train.py:93-125's dataset switch (fashion_mnist, tiny_imagenet) + the synthetic input."""
    if dataset == "fashion_mnist":
        return fashion_mnist(batch_size, seed, data_root)
    if dataset == "tiny_imagenet":
        return tiny_imagenet(batch_size, seed, image_size or 64, data_root)
    if dataset == "tiny_imagenet_synthetic":
        return synthetic(batch_size, seed, image_size or 64, **kw)
    raise ValueError(f"Unknown dataset: {dataset}")
