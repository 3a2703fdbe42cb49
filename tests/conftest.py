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
