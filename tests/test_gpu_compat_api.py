"""The reference-compatible API classes on the client-batched MI355X executor: ``SailentGradsAPI`` and
``SubAvgAPI`` constructed exactly as the reference's ``main_sailentgrads.py:272-280`` / ``main_subavg.py:221-222``
do (loader tuple, model, ModelTrainer) run their ``train()`` on the HIP kernels (profiler trace: ``nidt::``
kernels), and ``engine = "torch"`` keeps the eager oracle."""
import types

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _args(**kw):
    a = dict(client_num_in_total=3, client_num_per_round=3, comm_round=2, epochs=1, batch_size=8, lr=0.05,
             lr_decay=0.998, wd=5e-4, momentum=0.0, client_optimizer="sgd", frequency_of_the_test=1, ci=0,
             seed=1, frac=1.0, dense_ratio=0.5, anneal_factor=0.5, active=1.0, cs="random", static=False,
             dis_gradient_check=False, uniform=False, different_initial=False, diff_spa=False, erk_power_scale=1.0,
             save_masks=False, each_prune_ratio=0.2, dist_thresh=1e-4, acc_thresh=0.0, lamda=0.5, local_epochs=1,
             itersnip_iteration=1, snip_mask=True, stratified_sampling=False, record_mask_diff=False)
    a.update(kw)
    return types.SimpleNamespace(**a)


def _nidt_kernels(prof):
    return sorted({e.name for e in prof.events() if "nidt::" in e.name})


def test_salientgrads_api_runs_on_hip_kernels():
    from neuroimagedisttraining_amd.algorithms.salientgrads import SailentGradsAPI
    from neuroimagedisttraining_amd.algorithms.trainers import VolumeTrainer
    from neuroimagedisttraining_amd.data.abcd import load_partition_data_abcd_synthetic
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    torch.manual_seed(1)
    dataset = load_partition_data_abcd_synthetic(3, "dir", 0.3, 8, n_per_client=10, seed=1)
    args = _args(model="3DCNN", dataset="ABCD")
    model = AlexNet3D_Dropout(num_classes=1).to(DEV)
    w0 = model.features[0].weight.detach().clone()
    api = SailentGradsAPI(dataset, DEV, args, VolumeTrainer(model, args))
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                            torch.profiler.ProfilerActivity.CUDA]) as prof:
        api.train()
        torch.cuda.synchronize()
    assert api.engine_used == "hip"
    ks = _nidt_kernels(prof)
    assert any("conv1" in k for k in ks), ks[:20]
    assert len(api.stat_info["global_test_acc"]) >= 2 and len(api.stat_info["person_test_acc"]) >= 2
    assert 0.0 <= api.stat_info["global_test_acc"][-1] <= 1.0
    # the final global model is loaded back into the caller's trainer
    assert not torch.equal(model.features[0].weight.detach(), w0)


def test_subavg_api_runs_on_hip_kernels():
    from neuroimagedisttraining_amd.algorithms.personalized import SubAvgAPI
    from neuroimagedisttraining_amd.algorithms.trainers import ClassificationTrainer
    from neuroimagedisttraining_amd.data.images import load_partition_data
    from neuroimagedisttraining_amd.models import customized_resnet18
    torch.manual_seed(1)
    dataset = load_partition_data("cifar10", "", "dir", 0.5, 3, 16, n_train=120, n_test=60, seed=1)
    args = _args(model="resnet18", dataset="cifar10", batch_size=16)
    model = customized_resnet18(class_num=10).to(DEV)
    api = SubAvgAPI(dataset, DEV, args, ClassificationTrainer(model, args))
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                            torch.profiler.ProfilerActivity.CUDA]) as prof:
        api.train()
        torch.cuda.synchronize()
    assert api.engine_used == "hip"
    assert _nidt_kernels(prof), "no nidt:: kernel in the trace"
    assert len(api.stat_info["person_test_acc"]) >= 1


def test_api_engine_torch_keeps_eager_oracle():
    from neuroimagedisttraining_amd.algorithms.fedavg import FedAvgAPI
    from neuroimagedisttraining_amd.algorithms.trainers import ClassificationTrainer
    from neuroimagedisttraining_amd.data.images import load_partition_data_synthetic_tabular
    from neuroimagedisttraining_amd.models import LogisticRegression
    ds = load_partition_data_synthetic_tabular(client_number=2, batch_size=32, n_per_client=100, dim=20, n_cls=5)
    args = _args(client_num_in_total=2, client_num_per_round=2, comm_round=1, engine="torch", final_finetune=False)
    api = FedAvgAPI(ds, DEV, args, ClassificationTrainer(LogisticRegression(20, 5).to(DEV), args))
    api.train()
    assert api.engine_used == "eager"
