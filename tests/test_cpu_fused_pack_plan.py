"""Host-side planning of the optimizer-written weight images ([PACK-FUSE], resnet2d_hip.WeightPacker.fused_plan and
runner._pack_next) and of the depth-batched slab eligibility ([SLAB-BD]): pure host logic, no GPU."""
import numpy as np
import pytest
import torch

from neuroimagedisttraining_amd import ops

pytestmark = pytest.mark.skipif(not ops.available(), reason="HIP extension not built")


def _packer():
    from neuroimagedisttraining_amd.engine.executor import ParamLayout
    from neuroimagedisttraining_amd.engine.resnet2d_hip import GroupedResNet18GN
    from neuroimagedisttraining_amd.models import customized_resnet18
    m = customized_resnet18(class_num=10)
    lay = ParamLayout.from_tensors(list(m.named_parameters()))
    net = GroupedResNet18GN(lay, "cpu", hip=True)
    return net, lay


def test_fused_plan_covers_every_parameter_once():
    """Conv chunks (their theta spans) + the 'rest' ranges tile [0, P) exactly once, in blocks of <= 4096."""
    from neuroimagedisttraining_amd.engine.resnet2d_hip import WeightPacker
    net, lay = _packer()
    pk = WeightPacker(net.packer.convs, "cpu")
    key = (3, 8, True)
    pk._plan(3, True, key)
    tab, nd, nconv, rest, nrest, lds, buf = pk.fused_plan(key, lay.total)
    m = ops.ext()
    assert nd == len(pk.convs)
    assert nconv == sum(c.cout * m.pack_plain_chunks(c.cin_p, c.kt) for c in pk.convs)
    cover = np.zeros(lay.total, dtype=np.int32)
    for c in pk.convs:
        cover[c.off:c.off + c.numel] += 1
    r = rest.cpu().numpy()[:nrest]
    assert (r[:, 1] > 0).all() and (r[:, 1] <= 4096).all()
    for a, n in r:
        cover[a:a + n] += 1
    assert (cover == 1).all()
    assert lds == max(m.pack_plain_lds(c.cin_p, c.kt) for c in pk.convs)
    desc = np.frombuffer(tab.cpu().numpy().tobytes(), dtype=np.uint8).reshape(nd, -1)
    assert desc.shape[1] == m.pack_desc_bytes()


def test_pack_next_plan_rules():
    """Only a row group whose next entry in the epoch has the same shape, and whose shape no other group shares."""
    from neuroimagedisttraining_amd.engine.runner import FLRunner

    class E:
        fused_pack = True

    r = FLRunner.__new__(FLRunner)
    r.e = E()
    # (r0, r1, s, off, n, G, B): one group of 4 clients over three steps, last one partial
    plan = [(0, 4, 0, 0, 64, 4, 16), (0, 4, 1, 64, 64, 4, 16), (0, 4, 2, 128, 32, 4, 8)]
    assert r._pack_next(plan) == [True, False, False]
    # two groups of one shape share the image buffer: never
    plan2 = [(0, 4, 0, 0, 64, 4, 16), (4, 8, 0, 64, 64, 4, 16), (0, 4, 1, 128, 64, 4, 16), (4, 8, 1, 192, 64, 4, 16)]
    assert r._pack_next(plan2) == [False] * 4
    r.e = object()
    assert r._pack_next(plan) is None


@pytest.mark.parametrize("B,hw,c,ok", [(16, 8, 256, 1), (250, 8, 256, 1), (16, 4, 512, 1), (16, 4, 64, 0),
                                       (16, 16, 128, 0), (1022, 8, 64, 0)])
def test_slab_batched_depth_eligibility(B, hw, c, ok):
    """8x8 maps fit the 416-row union of 256-position blocks (4 padded samples); 4x4 maps take 128-position blocks
    (8 x 36 rows, 128-channel blocks only); 16x16 maps take the per-sample slab; the depth extent must stay below the
    10-bit plane code."""
    assert ops.ext().conv2d_fwd_slab_bd_ok(B, hw, hw, c, c) == ok
