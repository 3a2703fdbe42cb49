"""GPU test of the overlapped ingest pipeline: NIDTVOL1 file -> native gather -> pinned -> H2D on a copy stream
-> polyphase + patch-moment HIP kernels must equal the direct in-HBM path bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_stream_to_device_hip_store_matches_direct(tmp_path):
    from neuroimagedisttraining_amd.data.synthetic_fl import to_hip_store
    from neuroimagedisttraining_amd.data.volume_file import VolumeFile, stream_to_device, write_volume_file
    from neuroimagedisttraining_amd.data.volumes import make_synthetic_abcd
    st = make_synthetic_abcd(5, seed=3, device="cpu")
    p = write_volume_file(str(tmp_path / "c.nidtvol"), st.volumes, st.labels, st.site)
    vf = VolumeFile(p, threads=4)
    ix = [4, 0, 2, 3, 1]
    x8, mom = stream_to_device(vf, ix, "cuda", chunk=2, hip_store=True)
    x8_ref, mom_ref = to_hip_store(st.volumes[ix].cuda())
    torch.cuda.synchronize()
    assert torch.equal(x8, x8_ref)
    assert torch.equal(mom, mom_ref)
    raw = stream_to_device(vf, ix, "cuda", chunk=2)
    assert torch.equal(raw.cpu(), st.volumes[ix])
