"""Real-cohort ingestion never silently zeroes the volumes (missing #1).

The reference stores the ABCD cohort as 8-bit-quantised maps divided by 255 (``Preprocess_ABCD.ipynb``:
``eight_bit_data = (...).astype(np.uint8) / 255.0``) and its trainer reads ``X`` back as float32
(``fedml_api/standalone/sailentgrads/my_model_trainer.py:185-199``).  The loaders here keep uint8 in HBM, so a float
``X`` must be quantised exactly (``round(X * 255)``) — or refused — never truncated by a plain cast.  h5py is not
installed here, so ``_read_h5`` is monkeypatched with in-memory cohorts of the three forms.
"""
import numpy as np
import pytest

from neuroimagedisttraining_amd.data import abcd
from neuroimagedisttraining_amd.data.volumes import quantize_cohort_volumes
from neuroimagedisttraining_amd.data.volume_file import VolumeFile, write_volume_file

SHAPE = (6, 7, 5)


def _cohort(n=40, seed=0):
    rs = np.random.RandomState(seed)
    q = rs.randint(0, 256, size=(n,) + SHAPE).astype(np.uint8)
    y = rs.randint(0, 2, size=n).astype(np.float32)
    site = (np.arange(n) % 4).astype(np.float32)
    return q, y, site


def _patched(monkeypatch, X, y, site):
    # the real _read_h5 quantises chunk-wise while the file is open; the stand-in returns the stored array as is
    monkeypatch.setattr(abcd, "_read_h5", lambda path: (X, y, site))


def _stored_bytes(ds):
    store = ds[5][0].store
    return store.volumes.cpu().numpy()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_float_k_over_255_cohort_is_quantised_exactly(monkeypatch, dtype):
    q, y, site = _cohort()
    X = (q.astype(np.float64) / 255.0).astype(dtype)  # the reference's stored form
    _patched(monkeypatch, X, y, site)
    ds = abcd.load_partition_data_abcd("cohort.h5", client_number=4, max_clients=4, batch_size=4)
    got = _stored_bytes(ds)
    assert got.dtype == np.uint8
    np.testing.assert_array_equal(got, q)
    assert got.max() > 0  # the r4 cast turned all of this into zeros


def test_uint8_cohort_is_taken_as_is(monkeypatch):
    q, y, site = _cohort(seed=1)
    _patched(monkeypatch, q, y, site)
    ds = abcd.load_partition_data_abcd("cohort.h5", client_number=4, max_clients=4, batch_size=4)
    np.testing.assert_array_equal(_stored_bytes(ds), q)
    # the rescale loader goes through the same ingestion
    ds2 = abcd.load_partition_data_abcd_rescale("cohort.h5", client_number=4, batch_size=4)
    np.testing.assert_array_equal(ds2[5][0].store.volumes.cpu().numpy(), q)


def test_non_quantised_float_cohort_is_refused(monkeypatch):
    q, y, site = _cohort(seed=2)
    X = q.astype(np.float32) / 255.0 + 0.3 / 255.0  # between the 8-bit levels: not the reference's data
    _patched(monkeypatch, X, y, site)
    with pytest.raises(ValueError) as ei:
        abcd.load_partition_data_abcd("cohort.h5", client_number=4, max_clients=4, batch_size=4)
    msg = str(ei.value)
    assert "float32" in msg and "range" in msg


def test_quantize_rejects_out_of_range_and_accepts_small_ints():
    with pytest.raises(ValueError):
        quantize_cohort_volumes(np.full((2,) + SHAPE, 300, np.int32))
    with pytest.raises(ValueError):
        quantize_cohort_volumes(np.full((2,) + SHAPE, 1.5, np.float32))  # 382.5 after x255: above 255, not a level
    v = np.arange(2 * 6 * 7 * 5, dtype=np.int16).reshape((2,) + SHAPE) % 256
    np.testing.assert_array_equal(quantize_cohort_volumes(v), v.astype(np.uint8))


def test_volume_file_convert_quantises_float_cohort(tmp_path):
    q, y, site = _cohort(n=9, seed=3)
    path = tmp_path / "c.nidtvol"
    write_volume_file(path, (q / 255.0).astype(np.float32), y, site, chunk=4)
    vf = VolumeFile(path)
    np.testing.assert_array_equal(vf.gather(np.arange(9)).numpy(), q)
    with pytest.raises(ValueError):
        write_volume_file(tmp_path / "bad.nidtvol", q.astype(np.float32) / 254.0 + 1e-2, y, site)
