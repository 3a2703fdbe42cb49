"""Entry point (reference ``fedml_experiments/standalone/fedavg/main_fedavg.py``): same flags,
identity string and log file; see :mod:`neuroimagedisttraining_amd.cli` for the added MI355X flags."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

from neuroimagedisttraining_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    main('fedavg')
