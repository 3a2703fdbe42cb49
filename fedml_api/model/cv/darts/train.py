"""Compat shim: reference ``fedml_api/model/cv/darts/train.py``."""
from neuroimagedisttraining_amd.nas.train import eval_args, run_eval  # noqa: F401

if __name__ == "__main__":
    from neuroimagedisttraining_amd.nas.train import main
    import sys
    main(["eval"] + sys.argv[1:])
