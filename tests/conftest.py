import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# CLI runs inside tests record their stat_info into a scratch directory, not the working tree
if "NIDT_RESULTS_DIR" not in os.environ:
    import tempfile
    os.environ["NIDT_RESULTS_DIR"] = tempfile.mkdtemp(prefix="nidt_results_")
# pytest-xdist workers share the machine's cores: give each worker its share of intra-op threads (and the gloo ranks
# it spawns inherit the variable).  Unbounded, 6 workers x all-core OpenMP pools on 8 CPUs stalled small autograd
# graphs past the 900 s test timeout.
_XW = os.environ.get("PYTEST_XDIST_WORKER_COUNT")
if _XW and "OMP_NUM_THREADS" not in os.environ:
    os.environ["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 8) // max(1, int(_XW))))
    if "torch" in sys.modules:
        sys.modules["torch"].set_num_threads(int(os.environ["OMP_NUM_THREADS"]))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "extended: extra shapes of a kernel family already covered by the default GPU "
                                       "run (builder sessions: NIDT_EXTENDED_GPU_TESTS=1)")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("NIDT_EXTENDED_GPU_TESTS", "0") != "1":
        ext = pytest.mark.skip(reason="extended shape sweep (NIDT_EXTENDED_GPU_TESTS=1 runs it)")
        for it in items:
            if "extended" in it.keywords:
                it.add_marker(ext)
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
