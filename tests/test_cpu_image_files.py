"""On-disk image datasets (data/image_files.py): the reference's Tiny-ImageNet list files + JPEGs (decoded with PIL
as in ``tiny_imagenet/datasets.py:46-105``, optionally with its pixel scramble), the CIFAR-10/100 binary batches,
the decode cache, and the refusal of a ``data_dir`` that holds no dataset — on tiny fabricated trees."""
import os

import numpy as np
import pytest
import torch

from neuroimagedisttraining_amd.data import image_files as IF
from neuroimagedisttraining_amd.data import images


def _tiny_tree(root, n_train=5, n_val=3, seed=0):
    from PIL import Image
    d = os.path.join(root, "tiny-imagenet-200")
    rng = np.random.default_rng(seed)
    out = {}
    for split, n in (("train", n_train), ("val", n_val)):
        os.makedirs(os.path.join(d, split), exist_ok=True)
        lines, pix, labels = [], [], []
        for i in range(n):
            rel = "%s/img_%d.JPEG" % (split, i)
            img = rng.integers(0, 256, (64, 64, 3), dtype=np.uint8)
            Image.fromarray(img).save(os.path.join(d, rel), format="JPEG", quality=90)
            with Image.open(os.path.join(d, rel)) as im:  # what the reference's PIL decode yields (lossy JPEG)
                pix.append(np.asarray(im.convert("RGB")))
            lab = int(rng.integers(0, 200))
            labels.append(lab)
            lines.append("%s %d\n" % (rel, lab))
        with open(os.path.join(d, "%s_list.txt" % split), "w") as f:
            f.writelines(lines)
        out[split] = (np.stack(pix), np.asarray(labels))
    return out


def test_tiny_imagenet_decodes_reference_tree(tmp_path):
    ref = _tiny_tree(str(tmp_path))
    x, y = IF.read_tiny_imagenet(str(tmp_path), True)
    assert x.dtype == np.uint8 and x.shape == (5, 64, 64, 3)
    assert np.array_equal(x, ref["train"][0]) and np.array_equal(y, ref["train"][1])
    xv, yv = IF.read_tiny_imagenet(str(tmp_path), False)
    assert np.array_equal(xv, ref["val"][0]) and np.array_equal(yv, ref["val"][1])
    # the decode is cached as an .npz next to the lists and read back identically (no pickle)
    cache = os.path.join(str(tmp_path), "tiny-imagenet-200", "tinyTrue.npz")
    assert os.path.isfile(cache)
    x2, y2 = IF.read_tiny_imagenet(str(tmp_path), True)
    assert np.array_equal(x2, x) and np.array_equal(y2, y)
    # the reference's np.vstack(...).reshape(-1, 3, 64, 64).transpose(0, 2, 3, 1) scramble, behind the flag
    xs, _ = IF.read_tiny_imagenet(str(tmp_path), True, ref_pixel_order=True)
    want = np.vstack(list(ref["train"][0])).reshape(-1, 3, 64, 64).transpose((0, 2, 3, 1))
    assert np.array_equal(xs, want) and not np.array_equal(xs, x)
    # pointing at tiny-imagenet-200 itself works too
    x3, _ = IF.read_tiny_imagenet(os.path.join(str(tmp_path), "tiny-imagenet-200"), True)
    assert np.array_equal(x3, x)


def _cifar_records(n, nlab, rng):
    lab = rng.integers(0, 100 if nlab == 2 else 10, (n, nlab), dtype=np.uint8)
    pix = rng.integers(0, 256, (n, 3072), dtype=np.uint8)
    return np.concatenate([lab, pix], 1), lab[:, nlab - 1].astype(np.int64), pix.reshape(n, 3, 32, 32)


@pytest.mark.parametrize("name", ["cifar10", "cifar100"])
def test_cifar_binary_batches(tmp_path, name):
    rng = np.random.default_rng(1)
    sub, trn, tst, nlab = IF._CIFAR[name]
    d = tmp_path / sub
    d.mkdir()
    want = {}
    for split, files in (("train", trn), ("test", tst)):
        ys, xs = [], []
        for f in files:
            rec, y, x = _cifar_records(3, nlab, rng)
            rec.tofile(str(d / f))
            ys.append(y)
            xs.append(x)
        want[split] = (np.concatenate(xs).transpose(0, 2, 3, 1), np.concatenate(ys))
    x, y = IF.read_cifar_bin(name, str(tmp_path), True)
    assert x.shape == (3 * len(trn), 32, 32, 3) and x.dtype == np.uint8
    assert np.array_equal(x, want["train"][0]) and np.array_equal(y, want["train"][1])
    xt, yt = IF.read_cifar_bin(name, str(tmp_path), False)
    assert np.array_equal(xt, want["test"][0]) and np.array_equal(yt, want["test"][1])
    # the eager loader normalises the pixels exactly as ToTensor + Normalize(mean, std)
    xtr, ytr, _, _, ncls = images._load_arrays(name, str(tmp_path))
    mean, std = images.NORM[name]
    ref = (torch.from_numpy(want["train"][0]).permute(0, 3, 1, 2).float() / 255 - torch.tensor(mean).view(1, 3, 1, 1)) \
        / torch.tensor(std).view(1, 3, 1, 1)
    assert torch.allclose(xtr, ref, atol=1e-6) and ncls == (10 if name == "cifar10" else 100)
    assert torch.equal(ytr, torch.from_numpy(want["train"][1]))


def test_dataset_dir_without_files_raises(tmp_path):
    for name in ("cifar10", "cifar100", "tiny"):
        with pytest.raises(FileNotFoundError, match="holds no dataset files"):
            images._load_arrays(name, str(tmp_path))
    (tmp_path / "cifar-10-batches-py").mkdir()
    with pytest.raises(FileNotFoundError, match="never loaded"):
        images._load_arrays("cifar10", str(tmp_path))
    with pytest.raises(FileNotFoundError, match="does not exist"):
        images._load_arrays("cifar10", str(tmp_path / "nope"))
    # no data_dir at all: synthetic images of the dataset's shape
    xtr, ytr, xte, yte, n = images._load_arrays("cifar10", "", n_train=20, n_test=10)
    assert xtr.shape == (20, 3, 32, 32) and xtr.dtype == torch.float32 and n == 10


def test_uint8_npz_is_normalised_like_the_hip_path(tmp_path):
    """A uint8 HWC .npz: the eager loader normalises it (it used to feed raw 0..255 floats), and load_raw hands the
    HIP image engine the same uint8 pixels, which it normalises on device with the same NORM constants."""
    rng = np.random.default_rng(2)
    x = rng.integers(0, 256, (6, 32, 32, 3), dtype=np.uint8)
    y = rng.integers(0, 10, 6)
    p = str(tmp_path / "c.npz")
    np.savez(p, x_train=x, y_train=y, x_test=x[:2], y_test=y[:2])
    raw = images.load_raw("cifar10", p)
    assert raw[0].dtype == torch.uint8 and np.array_equal(raw[0].numpy(), x)
    xe = images._load_arrays("cifar10", p)[0]
    assert torch.allclose(xe, images.normalise_u8(torch.from_numpy(x), "cifar10"))
    assert float(xe.abs().max()) < 3.0
