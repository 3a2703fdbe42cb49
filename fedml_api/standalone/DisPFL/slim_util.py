"""Compat shim: reference import path ``fedml_api/standalone/DisPFL/slim_util.py``."""
from neuroimagedisttraining_amd.algorithms.sparse import hamming_distance, model_difference  # noqa: F401
from neuroimagedisttraining_amd.algorithms.sparse import cosine_annealing as _cosine


def cosine_annealing(args, round):  # noqa: A002  (reference signature, slim_util.py:7)
    """``args.anneal_factor / 2 * (1 + cos(round * pi / args.comm_round))``."""
    return _cosine(args.anneal_factor, round, args.comm_round)
