"""CPU tests of the reference-compatibility surface added for drop-in use: wire-compatible gRPC protobuf
service, the MPI-style send/receive-thread manager (over torch.distributed gloo when mpi4py is absent),
truncated datasets, DARTS genotype graph export and the CNN complexity script."""
import os
import socket

import numpy as np
import pytest
import torch

from neuroimagedisttraining_amd.comm.message import Message


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_grpc_proto_wire_format_matches_protoc():
    from fedml_core.distributed.communication.gRPC import grpc_comm_manager_pb2 as pb2
    r = pb2.CommRequest(client_id=3, message="hi")
    # protoc encoding of {client_id: 3 (field 1 varint), message: "hi" (field 2 length-delimited)}
    assert r.SerializeToString() == b"\x08\x03\x12\x02hi"
    assert pb2.CommResponse.FromString(b"\x08\x07\x12\x01x").client_id == 7


def test_reference_style_stub_talks_to_grpc_manager():
    grpc = pytest.importorskip("grpc")
    from fedml_core.distributed.communication.gRPC import grpc_comm_manager_pb2 as pb2
    from fedml_core.distributed.communication.gRPC import grpc_comm_manager_pb2_grpc as pb2_grpc
    from neuroimagedisttraining_amd.comm import GRPCCommManager
    base = _free_port()
    srv = GRPCCommManager("127.0.0.1", None, client_id=0, base_port=base)
    try:
        m = Message(9, 1, 0)
        m.add_params("v", 5)
        with grpc.insecure_channel("127.0.0.1:%d" % base) as ch:  # what the reference's client code does
            resp = pb2_grpc.gRPCCommManagerStub(ch).sendMessage(pb2.CommRequest(client_id=1, message=m.to_json()),
                                                               timeout=10)
        assert resp.message == "message received"
        got = srv.q.get(timeout=10)
        assert got.get_type() == 9 and got.get("v") == 5
    finally:
        srv.stop_receive_message()


def _mpi_worker(rank, world, port, out):
    import torch.distributed as dist
    from neuroimagedisttraining_amd.comm.mpi_threads import MpiCommunicationManager, TorchP2PComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mgr = MpiCommunicationManager(TorchP2PComm(), rank, world, node_type="server" if rank == 0 else "client")
    got = []

    class Obs:
        def receive_message(self, t, msg):
            got.append((t, msg.get("payload")))

    mgr.add_observer(Obs())
    if rank == 1:
        m = Message(4, 1, 0)
        m.add_params("payload", torch.arange(5.0))
        mgr.send_message(m)
    else:
        assert mgr.poll_once(timeout=30.0)
        t, p = got[0]
        torch.save({"t": t, "p": p}, out)
    dist.barrier()
    mgr.stop_receive_message()
    dist.barrier()
    dist.destroy_process_group()


def test_mpi_style_manager_over_gloo(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "m.pt")
    mp.start_processes(_mpi_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    r = torch.load(out, weights_only=True)
    assert r["t"] == 4 and torch.equal(r["p"], torch.arange(5.0))


def test_truncated_datasets():
    from fedml_api.data_preprocessing.cifar10.datasets import CIFAR10_truncated
    from fedml_api.data_preprocessing.tiny_imagenet.datasets import tiny, tiny_truncated
    from neuroimagedisttraining_amd.data.datasets import ArrayData
    data = np.random.RandomState(0).rand(10, 32, 32, 3).astype(np.float32)
    cache = ArrayData(data, np.arange(10) % 3)
    ds = CIFAR10_truncated("unused", cache_data_set=cache, dataidxs=[7, 2, 5])
    assert len(ds) == 3 and list(ds.target) == [1, 2, 2]
    x, y = ds[0]
    assert x.shape == (3, 32, 32) and y == 1 and torch.allclose(x, torch.from_numpy(data[7]).permute(2, 0, 1))
    ds2 = CIFAR10_truncated("", dataidxs=[0, 1], n=16, transform=lambda im: torch.as_tensor(im).mean())
    assert len(ds2) == 2 and ds2[1][0].dim() == 0
    t = tiny("", n=8)  # no root: synthetic images of the real shape
    assert len(t) == 8 and t[0][0].shape == (3, 64, 64)
    tt = tiny_truncated("", dataidxs=[1, 3], n=8)
    assert len(tt) == 2
    with pytest.raises(FileNotFoundError):  # a root without dataset files is an error, not silent noise
        tiny("no/such/dir", n=8)


def test_genotype_dot_export(tmp_path):
    from neuroimagedisttraining_amd.nas import genotypes
    from fedml_api.model.cv.darts.visualize import plot, to_dot
    g = genotypes.DARTS.normal
    dot = to_dot(g)
    assert dot.count("->") == len(g) + len(g) // 2
    path = plot(g, str(tmp_path / "normal"))
    assert os.path.exists(str(tmp_path / "normal.dot")) and path


def test_cnn_dropout_complexity_script():
    import importlib.util
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("tcnn", os.path.join(here, "fedml_api/model/cv/test_cnn.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from fedml_api.model.cv.cnn import CNN_DropOut
    flops, params = mod.complexity(CNN_DropOut())
    assert params == 1199882 and flops > 0


def test_every_reference_import_line_resolves():
    """Each ``from fedml_api|fedml_core ... import ...`` line of the reference (tests/data/reference_imports.txt)
    imports against this repo, so the reference's scripts and modules find every public name they use."""
    path = os.path.join(os.path.dirname(__file__), "data", "reference_imports.txt")
    lines = [ln.strip() for ln in open(path) if ln.strip() and not ln.startswith("#")]
    assert len(lines) >= 60
    bad = []
    for ln in lines:
        try:
            exec(ln, {})
        except Exception as e:  # noqa: BLE001
            bad.append("%s -> %r" % (ln, e))
    assert not bad, "\n".join(bad)


def test_reference_snip_functions_match_monkeypatched_masks():
    """get_snip_scores / get_mask_from_grads / get_mean_snip_scores with the reference signatures: the scores equal
    |dL/dmask| of the reference's weight_mask monkey-patch (snip_forward_conv3d / snip_forward_linear), and the mask
    keeps the global top keep_ratio of the sum-normalised scores."""
    import copy
    import types
    from fedml_api.standalone.sailentgrads.snip import (
        get_mask_from_grads, get_mean_snip_scores, get_snip_scores, snip_forward_conv3d, snip_forward_linear)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.features = torch.nn.Sequential(torch.nn.Conv3d(1, 4, 3), torch.nn.ReLU())
            self.classifier = torch.nn.Linear(4 * 4 * 4 * 4, 1)

        def forward(self, x):
            return self.classifier(self.features(x).flatten(1))

    torch.manual_seed(0)
    owner = types.SimpleNamespace(model=Net())
    x, y = torch.randn(5, 6, 6, 6), torch.randint(0, 2, (5,))
    scores = get_snip_scores(owner, (x, y, None))
    # the reference's mechanism on a copy
    cp = copy.deepcopy(owner.model)
    for layer in cp.modules():
        if isinstance(layer, (torch.nn.Conv3d, torch.nn.Linear)):
            layer.weight_mask = torch.nn.Parameter(torch.ones_like(layer.weight))
            layer.weight.requires_grad = False
            f = snip_forward_conv3d if isinstance(layer, torch.nn.Conv3d) else snip_forward_linear
            layer.forward = types.MethodType(f, layer)
    loss = torch.nn.BCEWithLogitsLoss()(cp(x.unsqueeze(1)), y.unsqueeze(1).float())
    loss.backward()
    ref = [(n, m.weight_mask.grad.abs()) for n, m in cp.named_modules() if hasattr(m, "weight_mask")]
    assert [n for n, _ in scores] == [n for n, _ in ref]
    for (_, a), (_, b) in zip(scores, ref):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-8)
    mean = get_mean_snip_scores([scores, scores])
    keep, by_layer, final = get_mask_from_grads(owner, mean, 0.3, None)
    flat = torch.cat([v.flatten() for v in mean.values()])
    flat = flat / flat.sum()
    thr = torch.topk(flat, int(flat.numel() * 0.3)).values[-1]
    assert int(sum(int(v.sum()) for v in keep.values())) == int((flat >= thr).sum())
    assert set(final) == {n for n, _ in owner.model.named_parameters()}
    assert torch.equal(final["features.0.bias"], torch.ones(4))
    assert len(by_layer) == 2


def test_reference_helper_names():
    """dispflAPI / FEDFOMOAPI class names, slim_util.cosine_annealing(args, round) and print_model_param_nums."""
    import types
    from fedml_api.standalone.DisPFL.dispfl_api import dispflAPI
    from fedml_api.standalone.DisPFL.slim_util import cosine_annealing
    from fedml_api.standalone.fedfomo.fedfomo_api import FEDFOMOAPI
    from fedml_api.utils.main_flops_counter import print_model_param_nums
    from neuroimagedisttraining_amd.algorithms.personalized import DisPFLAPI, FedFomoAPI
    assert dispflAPI is DisPFLAPI and FEDFOMOAPI is FedFomoAPI
    args = types.SimpleNamespace(anneal_factor=0.5, comm_round=10)
    assert abs(cosine_annealing(args, 0) - 0.5) < 1e-12 and abs(cosine_annealing(args, 10)) < 1e-12
    assert abs(cosine_annealing(args, 5) - 0.25) < 1e-12
    net = torch.nn.Sequential(torch.nn.Conv2d(1, 2, 3), torch.nn.Conv3d(1, 2, 3), torch.nn.Linear(3, 4))
    with torch.no_grad():
        net[0].weight[0] = 0
    assert print_model_param_nums(net) == 9 + 12
