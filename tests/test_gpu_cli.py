"""GPU tests of the reference entry points on the HIP executor: real-cohort data source (NIDTVOL1 site clients,
ADVICE r1: never substitute synthetic data) and every algorithm's entry point end to end."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cohort(tmp_path_factory):
    from neuroimagedisttraining_amd.data.volume_file import write_volume_file
    from neuroimagedisttraining_amd.data.volumes import make_synthetic_abcd
    n_sites, per = 22, 6
    site = np.repeat(np.arange(n_sites), per).astype(np.float32)
    st = make_synthetic_abcd(len(site), seed=3, device="cuda", site=site, n_sites=n_sites)
    path = str(tmp_path_factory.mktemp("abcd") / "alldatain8bitsnormalized.nidtvol")
    write_volume_file(path, st.volumes, st.labels, st.site)
    return path, st.labels.cpu().numpy(), site


def test_cli_hip_trains_on_the_real_cohort(cohort, tmp_path):
    from neuroimagedisttraining_amd import cli
    path, labels, site = cohort
    out = cli.main("sailentgrads", ["--synthetic_abcd", "0", "--data_dir", os.path.dirname(path), "--comm_round", "1",
                                    "--epochs", "1", "--batch_size", "4", "--engine", "hip",
                                    "--log_dir", str(tmp_path)])
    assert len(out["global_test_acc"]) >= 1
    log = next((tmp_path / "ABCD").glob("*.log")).read_text()
    assert "NIDTVOL1" in log and "21 clients" in log  # site clients of the file, first 21 sites (Q9)
    assert "train sizes [5, 5," in log  # 6 subjects per site -> 80/20 split: 5 train / 1 test


def test_cli_hip_refuses_missing_cohort(tmp_path):
    from neuroimagedisttraining_amd import cli
    with pytest.raises(FileNotFoundError):
        cli.main("sailentgrads", ["--synthetic_abcd", "0", "--data_dir", str(tmp_path), "--comm_round", "1",
                                  "--engine", "hip", "--log_dir", str(tmp_path)])


@pytest.mark.parametrize("algo", ["fedavg", "fedprox", "dispfl", "subavg", "ditto", "dpsgd", "fedfomo", "local"])
def test_cli_every_algorithm_runs_on_hip(algo, tmp_path):
    from neuroimagedisttraining_amd import cli
    argv = ["--model", "3DCNN", "--dataset", "ABCD", "--client_num_in_total", "4", "--comm_round", "2",
            "--epochs", "1", "--batch_size", "4", "--n_per_client", "20", "--frac", "0.5", "--engine", "hip",
            "--log_dir", str(tmp_path)]
    out = cli.main(algo, argv)
    vals = [v for k, v in out.items() if k.endswith("test_acc") and isinstance(v, list) and v]
    assert vals and all(0.0 <= x <= 1.0 for x in vals[0])


@pytest.mark.parametrize("algo", ["subavg", "dispfl", "ditto", "dpsgd", "fedfomo", "local", "fedavg"])
def test_cli_resnet18_cifar_runs_on_hip(algo, tmp_path):
    """The CIFAR entry points' default model (resnet18 = ResNet-18-GN, cifar10) runs on the client-batched
    ResNet engine (engine/resnet2d_hip.py), not the eager loop."""
    from neuroimagedisttraining_amd import cli
    argv = ["--model", "resnet18", "--dataset", "cifar10", "--client_num_in_total", "4", "--comm_round", "2",
            "--epochs", "1", "--batch_size", "16", "--synthetic_size", "640", "--frac", "0.5", "--engine", "hip",
            "--log_dir", str(tmp_path)]
    out = cli.main(algo, argv)
    vals = [v for k, v in out.items() if k.endswith("test_acc") and isinstance(v, list) and v]
    assert vals and all(0.0 <= x <= 1.0 for x in vals[0])
    log = next((tmp_path / "cifar10").glob("*.log")).read_text()
    assert "HIP cohort (resnet2d)" in log


@pytest.mark.parametrize("algo", ["subavg", "dispfl", "ditto", "dpsgd", "fedfomo", "local", "fedavg"])
def test_cli_resnet18_tiny_runs_on_hip(algo, tmp_path):
    """The Tiny-ImageNet presets (``fedml_experiments/standalone/*/tiny.sh``: resnet18 = tiny_resnet18, 64x64, 200
    classes) run on the client-batched ResNet engine with the fused augmentation."""
    from neuroimagedisttraining_amd import cli
    argv = ["--model", "resnet18", "--dataset", "tiny", "--client_num_in_total", "4", "--comm_round", "2",
            "--epochs", "1", "--batch_size", "16", "--synthetic_size", "400", "--frac", "0.5", "--engine", "hip",
            "--log_dir", str(tmp_path)]
    out = cli.main(algo, argv)
    vals = [v for k, v in out.items() if k.endswith("test_acc") and isinstance(v, list) and v]
    assert vals and all(0.0 <= x <= 1.0 for x in vals[0])
    log = next((tmp_path / "tiny").glob("*.log")).read_text()
    assert "HIP cohort (resnet2d)" in log


def test_cli_resnet3d50_runs_on_hip(tmp_path):
    """--model resnet3d_50 on ABCD-shape volumes runs on the client-batched 3D ResNet engine (config 5 family)."""
    from neuroimagedisttraining_amd import cli
    argv = ["--model", "resnet3d_50", "--dataset", "ABCD", "--client_num_in_total", "2", "--comm_round", "1",
            "--epochs", "1", "--batch_size", "2", "--n_per_client", "3", "--frac", "1.0", "--engine", "hip",
            "--log_dir", str(tmp_path)]
    out = cli.main("fedavg", argv)
    assert len(out["global_test_acc"]) >= 1
    log = next((tmp_path / "ABCD").glob("*.log")).read_text()
    assert "HIP cohort (resnet3d)" in log
