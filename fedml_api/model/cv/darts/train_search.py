"""Compat shim: reference ``fedml_api/model/cv/darts/train_search.py``."""
from neuroimagedisttraining_amd.nas.train import run_search, search_args  # noqa: F401

if __name__ == "__main__":
    from neuroimagedisttraining_amd.nas.train import main
    import sys
    main(["search"] + sys.argv[1:])
