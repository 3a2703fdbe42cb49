"""CPU tests of the native host runtime: the C++ NIDTVOL1 volume reader (``csrc/runtime/volume_io.cpp``) and
its Python pipeline / ABCD-loader integration."""
import os

import numpy as np
import pytest
import torch

from neuroimagedisttraining_amd.data.volume_file import VolumeFile, stream_to_device, write_volume_file


def _cohort(n=11, shape=(9, 13, 7), seed=0):
    rs = np.random.RandomState(seed)
    return (rs.randint(0, 256, size=(n,) + shape).astype(np.uint8), rs.randint(0, 2, n).astype(np.float32),
            rs.randint(0, 21, n).astype(np.float32))


def test_volume_file_roundtrip_and_gather(tmp_path):
    X, y, s = _cohort()
    p = write_volume_file(str(tmp_path / "c.nidtvol"), X, y, s, chunk=4)
    vf = VolumeFile(p, threads=3)
    assert len(vf) == 11 and vf.shape == (9, 13, 7)
    assert np.array_equal(vf.labels, y) and np.array_equal(vf.sites, s)
    ix = [10, 0, 3, 3, 7]
    got = vf.gather(ix)
    assert got.dtype == torch.uint8 and np.array_equal(got.numpy(), X[ix])
    out = torch.zeros((8,) + X.shape[1:], dtype=torch.uint8)
    vf.gather([2, 5], out=out)
    assert np.array_equal(out[:2].numpy(), X[[2, 5]]) and int(out[2:].sum()) == 0


def test_volume_file_async_tickets_and_large_subjects(tmp_path):
    # > 1 MiB per subject: each gather is split into several pieces across the worker pool
    X, y, s = _cohort(n=5, shape=(64, 130, 130), seed=1)
    vf = VolumeFile(write_volume_file(str(tmp_path / "big.nidtvol"), X, y, s), threads=4)
    a = torch.empty((3,) + X.shape[1:], dtype=torch.uint8)
    b = torch.empty((2,) + X.shape[1:], dtype=torch.uint8)
    ta = vf.submit([4, 1, 2], a)
    tb = vf.submit([0, 4], b)
    vf.prefetch([3])
    vf.wait(tb)
    vf.wait(ta)
    assert np.array_equal(a.numpy(), X[[4, 1, 2]]) and np.array_equal(b.numpy(), X[[0, 4]])


def test_volume_file_validation(tmp_path):
    X, y, s = _cohort(n=3)
    p = write_volume_file(str(tmp_path / "v.nidtvol"), X, y, s)
    vf = VolumeFile(p)
    with pytest.raises(IndexError):
        vf.gather([3])
    bad = tmp_path / "bad.nidtvol"
    bad.write_bytes(b"NOTAVOL!" + open(p, "rb").read()[8:])
    with pytest.raises(RuntimeError, match="bad magic"):
        VolumeFile(str(bad))
    trunc = tmp_path / "trunc.nidtvol"
    trunc.write_bytes(open(p, "rb").read()[:5000])
    with pytest.raises(RuntimeError, match="truncated"):
        VolumeFile(str(trunc))
    # floats are accepted only in the reference's k/255 form (quantised exactly); raw 0..255 floats are refused
    with pytest.raises(ValueError, match="k/255"):
        write_volume_file(str(tmp_path / "f.nidtvol"), X.astype(np.float32), y)


def test_stream_to_device_cpu_and_store(tmp_path):
    X, y, s = _cohort(n=7)
    vf = VolumeFile(write_volume_file(str(tmp_path / "c.nidtvol"), X, y, s))
    v = stream_to_device(vf, [6, 2], "cpu", chunk=1)
    assert np.array_equal(v.numpy(), X[[6, 2]])
    st = vf.to_store([1, 4, 5])
    assert len(st) == 3 and np.array_equal(st.volumes.numpy(), X[[1, 4, 5]])
    assert np.array_equal(st.labels.numpy(), y[[1, 4, 5]])


def test_abcd_loader_reads_volume_file_by_site(tmp_path):
    from neuroimagedisttraining_amd.data.abcd import load_partition_data_abcd
    rs = np.random.RandomState(3)
    n = 60
    X = rs.randint(0, 256, size=(n, 5, 6, 5)).astype(np.uint8)
    y = rs.randint(0, 2, n).astype(np.float32)
    site = (np.arange(n) % 4).astype(np.float32)
    p = write_volume_file(str(tmp_path / "abcd.nidtvol"), X, y, site)
    ds = load_partition_data_abcd(p, batch_size=4, max_clients=21)
    num, trn, tst = ds[4], ds[5], ds[6]
    assert sorted(num) == [0, 1, 2, 3] and sum(num.values()) + sum(len(t.indices) for t in tst.values()) == n
    store = trn[0].store
    assert tuple(store.shape) == (5, 6, 5)
    xb, yb, sb = next(iter(trn[0]))
    xv, yv = store.fetch(xb)
    assert xv.shape == (len(xb), 1, 5, 6, 5)
    assert np.array_equal(np.sort(yv.numpy()), np.sort(y[np.sort(xb.numpy().astype(int))]))


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_volume_reader_sanitizer_stress(san, tmp_path):
    """Race detection for the native runtime: the reader core (worker pool, ticket registry, completion
    signalling, destructor draining queued gathers) under ThreadSanitizer and AddressSanitizer+UBSan, host only."""
    import shutil
    import subprocess
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "stress")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-pthread", "-fsanitize=" + san, "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", os.path.join(root, "csrc/runtime/tests/volume_io_stress.cpp"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in b.stderr:
        pytest.skip("sanitizer runtime unavailable: " + b.stderr[-200:])
    assert b.returncode == 0, b.stderr[-2000:]
    r = subprocess.run([exe, str(tmp_path), "4", "25"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "volume_io_stress ok" in r.stdout, (r.stdout + r.stderr)[-3000:]


def test_abcd_preprocessing_matches_notebook_semantics(tmp_path):
    """Preprocess_ABCD.ipynb: mean-image > 0.2 mask, masked per-subject min-max, uint8 truncation, category codes
    for sex and LabelEncoder codes for site; written as a NIDTVOL1 file the native reader serves."""
    from neuroimagedisttraining_amd.data.preprocess import preprocess_cohort
    rs = np.random.RandomState(0)
    vols = rs.rand(5, 6, 7, 6).astype(np.float32) * 0.6
    vols[:, :2] = 0.05  # low-mean region falls outside the mask
    female = np.array(["1", "0", "1", "", "0"], dtype=object)
    site = np.array(["site21", "site02", "site02", "site10", "site21"])
    q, y, s = preprocess_cohort(vols, female, site, drop_missing=False)
    mask = vols.mean(0) > 0.2
    for i in range(5):
        v = vols[i].astype(np.float64) * mask
        ref = ((v - v.min()) / (v.max() - v.min()) * 255).astype(np.uint8)
        assert np.array_equal(q[i], ref)
    assert (q[:, :2] == 0).all()
    assert y.tolist() == [1, 0, 1, -1, 0] and s.tolist() == [2, 0, 0, 1, 2]
    # streamed into the file from a memory-mapped .npy; the subject with missing sex is dropped
    np.save(tmp_path / "X.npy", vols)
    _, y2, s2 = preprocess_cohort(np.load(tmp_path / "X.npy", mmap_mode="r"), female, site,
                                  out_path=str(tmp_path / "c.nidtvol"))
    assert y2.tolist() == [1, 0, 1, 0] and s2.tolist() == [2, 0, 0, 2]
    vf = VolumeFile(str(tmp_path / "c.nidtvol"))
    assert np.array_equal(vf.gather(np.array([3, 1])).numpy(), q[[4, 1]])
    assert np.asarray(vf.labels).tolist() == [1, 0, 1, 0]


def test_abcd_rescale_loader_reference_signature(tmp_path):
    """load_partition_data_abcd_rescale(data_dir, partition_method, partition_alpha, client_number, batch_size,
    logger) like ABCD/data_loader.py:216: every subject in exactly one train or test shard, contiguous equal
    train shards of the seeded 80/20 split."""
    import numpy as np
    import torch
    from neuroimagedisttraining_amd.data.abcd import load_partition_data_abcd_rescale
    from neuroimagedisttraining_amd.data.volume_file import write_volume_file
    n = 50
    vols = torch.randint(0, 256, (n, 6, 7, 6), dtype=torch.uint8)
    path = str(tmp_path / "alldatain8bitsnormalized.nidtvol")
    write_volume_file(path, vols, np.arange(n) % 2, np.arange(n) % 5)
    ds = load_partition_data_abcd_rescale(str(tmp_path), "site", 0.3, 4, 8, None)
    num, trn, tst = ds[4], ds[5], ds[6]
    tr = np.concatenate([trn[c].indices for c in range(4)])
    te = np.concatenate([tst[c].indices for c in range(4)])
    assert sorted(np.concatenate([tr, te]).tolist()) == list(range(n))
    assert len(te) == int(n * 0.2) and [num[c] for c in range(4)] == [10, 10, 10, 10]
