"""CPU tests of the CLI's routing onto the client-batched executor for every model family (3DCNN / 3D ResNet-50 on
ABCD, ResNet-18-GN on CIFAR) and of the CIFAR image cohort of that path: same client splits as the eager loaders
(``data/images.load_partition_data``), uint8 pixels that the engine's normalisation maps back to the loader's
images, and one round of the ResNet-18-GN engine (fp32 CPU twin) through ``cli.run_hip``."""
import argparse
import logging

import numpy as np
import pytest
import torch


def _args(algo, argv):
    from neuroimagedisttraining_amd import cli
    args = cli.add_args(argparse.ArgumentParser(), algo).parse_args(argv)
    args.algo = algo
    args.identity = cli.identity(args, algo)
    return args


@pytest.mark.parametrize("algo,argv,fam", [
    ("sailentgrads", [], "alexnet3d"),
    ("dispfl", [], "alexnet3d"),
    ("subavg", [], "resnet2d"),
    ("ditto", ["--dataset", "cifar100"], "resnet2d"),
    ("fedavg", ["--model", "resnet3d_50"], "resnet3d"),
    ("subavg", ["--model", "vgg11"], "batched2d"),  # the other CIFAR models: vmapped client batches
    ("local", ["--dataset", "tiny"], "resnet2d"),  # tiny_resnet18 (64x64, 200 classes) on the same engine
    ("local", ["--dataset", "tiny", "--model", "vgg16"], None),
])
def test_hip_family_routes_reference_defaults(algo, argv, fam):
    from neuroimagedisttraining_amd import cli
    args = _args(algo, argv)
    assert cli.hip_family(args) == fam
    if fam is None:
        args.engine = "hip"
        with pytest.raises(RuntimeError):
            cli._use_hip(args, algo)
    args.engine = "torch"
    assert not cli._use_hip(args, algo)


@pytest.mark.parametrize("algo", ["subavg", "fedfomo"])
def test_image_cohort_matches_eager_loader_splits(algo):
    from neuroimagedisttraining_amd import cli
    from neuroimagedisttraining_amd.data import images
    from neuroimagedisttraining_amd.engine.resnet2d_hip import CIFAR_MEAN, CIFAR_STD
    from neuroimagedisttraining_amd.parallel.runtime import DistInfo
    args = _args(algo, ["--client_num_in_total", "5", "--synthetic_size", "500", "--seed", "3"])
    x8, y, splits, n_cls = cli.image_cohort(args, DistInfo(), with_val=algo == "fedfomo")
    ds = images.load_partition_data("cifar10", "", "dir", 0.3, 5, 16, n_train=500, n_test=100, seed=3,
                                    with_val=algo == "fedfomo", augment=False)  # un-augmented pixels to compare
    assert n_cls == 10 and x8.dtype == torch.uint8 and tuple(x8.shape) == (600, 32, 32, 3)
    num, trn = ds[4], ds[5]
    tst = ds[7] if algo == "fedfomo" else ds[6]
    for c in range(5):
        assert len(splits[c].train) == num[c] == len(trn[c].dataset)
        assert len(splits[c].test) == len(tst[c].dataset)
        if algo == "fedfomo":
            assert len(splits[c].val) == len(ds[6][c].dataset)
        # the client's train images: uint8 pixels normalised like the engine reproduce the loader's tensors
        xs = torch.stack([trn[c].dataset[i][0] for i in range(len(trn[c].dataset))])
        m_, s_ = torch.tensor(CIFAR_MEAN).view(1, 3, 1, 1), torch.tensor(CIFAR_STD).view(1, 3, 1, 1)
        xs = torch.maximum(torch.minimum(xs, (1 - m_) / s_), -m_ / s_)  # pixels saturate at 0 / 255
        mine = x8[torch.as_tensor(np.sort(splits[c].train))].float() / 255.0
        mine = ((mine - torch.tensor(CIFAR_MEAN)) / torch.tensor(CIFAR_STD)).permute(0, 3, 1, 2)
        # same multiset of images (loader order is shuffled): compare sorted per-image sums
        a = np.sort(xs.sum(dim=(1, 2, 3)).numpy())
        b = np.sort(mine.sum(dim=(1, 2, 3)).numpy())
        assert np.allclose(a, b, atol=2.0), np.abs(a - b).max()  # 8-bit rounding
    assert torch.equal(y[:500][torch.as_tensor(splits[0].train)].sort().values,
                       torch.as_tensor([trn[0].dataset[i][1] for i in range(num[0])]).sort().values)


def test_run_hip_resnet18_cifar_on_cpu_twin(tmp_path):
    from neuroimagedisttraining_amd import cli
    args = _args("subavg", ["--client_num_in_total", "4", "--synthetic_size", "160", "--comm_round", "1",
                            "--epochs", "1", "--batch_size", "16", "--frac", "0.5", "--log_dir", str(tmp_path)])
    out = cli.run_hip(args, "subavg", logging.getLogger("test"))
    vals = [v for k, v in out.items() if k.endswith("test_acc") and isinstance(v, list) and v]
    assert vals and all(0.0 <= x <= 1.0 for x in vals[0])


def test_alexnet_hip_routing_checks_the_cohort_volume_shape(tmp_path, caplog):
    """A cohort file whose volumes are not 1x121x145x121 cannot run on the AlexNet3D kernels: the entry point says so
    and runs eagerly (or refuses --engine hip) instead of failing inside the engine; ABCD-shape files route to HIP."""
    from neuroimagedisttraining_amd import cli
    from neuroimagedisttraining_amd.data.volume_file import write_volume_file
    g = np.random.default_rng(0)
    odd = write_volume_file(str(tmp_path / "odd.nidtvol"), g.integers(0, 255, (4, 20, 24, 20), dtype=np.uint8),
                            np.array([0, 1, 0, 1]), np.array([0, 0, 1, 1]))
    args = _args("sailentgrads", ["--data_dir", odd])
    args.synthetic_abcd = False
    assert cli._cohort_shape(args) == (20, 24, 20)
    assert cli.hip_family(args) is None
    args.engine = "hip"
    with pytest.raises(RuntimeError, match="AlexNet3D kernels need"):
        cli._use_hip(args, "sailentgrads")
    args.engine = "auto"
    with caplog.at_level(logging.WARNING):
        assert not cli._use_hip(args, "sailentgrads")
    assert "eager PyTorch engine" in caplog.text
    ok = write_volume_file(str(tmp_path / "abcd.nidtvol"), g.integers(0, 255, (2, 121, 145, 121), dtype=np.uint8),
                           np.array([0, 1]), np.array([0, 1]))
    args2 = _args("sailentgrads", ["--data_dir", ok])
    args2.synthetic_abcd = False
    assert cli.hip_family(args2) == "alexnet3d"
