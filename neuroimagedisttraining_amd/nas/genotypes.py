"""Cell genotypes (reference ``fedml_api/model/cv/darts/genotypes.py:1-91``).

The named genotypes are the published cells (NASNet-A, AmoebaNet-A, DARTS V1/V2, FedNAS V1), written in a
compact ``op@input`` notation and expanded at import time.
"""
from __future__ import annotations

from collections import namedtuple

from .ops import PRIMITIVES  # noqa: F401  (re-exported, reference import path)

Genotype = namedtuple("Genotype", "normal normal_concat reduce reduce_concat")


def _cell(spec):
    out = []
    for tok in spec.split():
        op, idx = tok.split("@")
        out.append((op, int(idx)))
    return out


def make_genotype(normal, normal_concat, reduce, reduce_concat):
    return Genotype(normal=_cell(normal), normal_concat=list(normal_concat),
                    reduce=_cell(reduce), reduce_concat=list(reduce_concat))


NASNet = make_genotype(
    "sep_conv_5x5@1 sep_conv_3x3@0 sep_conv_5x5@0 sep_conv_3x3@0 avg_pool_3x3@1 skip_connect@0 "
    "avg_pool_3x3@0 avg_pool_3x3@0 sep_conv_3x3@1 skip_connect@1", [2, 3, 4, 5, 6],
    "sep_conv_5x5@1 sep_conv_7x7@0 max_pool_3x3@1 sep_conv_7x7@0 avg_pool_3x3@1 sep_conv_5x5@0 "
    "skip_connect@3 avg_pool_3x3@2 sep_conv_3x3@2 max_pool_3x3@1", [4, 5, 6])

AmoebaNet = make_genotype(
    "avg_pool_3x3@0 max_pool_3x3@1 sep_conv_3x3@0 sep_conv_5x5@2 sep_conv_3x3@0 avg_pool_3x3@3 "
    "sep_conv_3x3@1 skip_connect@1 skip_connect@0 avg_pool_3x3@1", [4, 5, 6],
    "avg_pool_3x3@0 sep_conv_3x3@1 max_pool_3x3@0 sep_conv_7x7@2 sep_conv_7x7@0 avg_pool_3x3@1 "
    "max_pool_3x3@0 max_pool_3x3@1 conv_7x1_1x7@0 sep_conv_3x3@5", [3, 4, 6])

DARTS_V1 = make_genotype(
    "sep_conv_3x3@1 sep_conv_3x3@0 skip_connect@0 sep_conv_3x3@1 skip_connect@0 sep_conv_3x3@1 "
    "sep_conv_3x3@0 skip_connect@2", [2, 3, 4, 5],
    "max_pool_3x3@0 max_pool_3x3@1 skip_connect@2 max_pool_3x3@0 max_pool_3x3@0 skip_connect@2 "
    "skip_connect@2 avg_pool_3x3@0", [2, 3, 4, 5])

DARTS_V2 = make_genotype(
    "sep_conv_3x3@0 sep_conv_3x3@1 sep_conv_3x3@0 sep_conv_3x3@1 sep_conv_3x3@1 skip_connect@0 "
    "skip_connect@0 dil_conv_3x3@2", [2, 3, 4, 5],
    "max_pool_3x3@0 max_pool_3x3@1 skip_connect@2 max_pool_3x3@1 max_pool_3x3@0 skip_connect@2 "
    "skip_connect@2 max_pool_3x3@1", [2, 3, 4, 5])

DARTS = DARTS_V2

FedNAS_V1 = make_genotype(
    "sep_conv_3x3@1 sep_conv_3x3@0 sep_conv_3x3@2 sep_conv_5x5@0 sep_conv_3x3@1 sep_conv_5x5@3 "
    "dil_conv_5x5@3 sep_conv_3x3@4", range(2, 6),
    "max_pool_3x3@0 skip_connect@1 max_pool_3x3@0 max_pool_3x3@2 max_pool_3x3@0 dil_conv_5x5@1 "
    "max_pool_3x3@0 dil_conv_5x5@2", range(2, 6))

GENOTYPES = {"NASNet": NASNet, "AmoebaNet": AmoebaNet, "DARTS_V1": DARTS_V1, "DARTS_V2": DARTS_V2,
             "DARTS": DARTS, "FedNAS_V1": FedNAS_V1}


def genotype_from_string(s):
    """Parse ``str(Genotype(...))`` (as logged by a search run) or a registered name."""
    if s in GENOTYPES:
        return GENOTYPES[s]
    import ast
    body = s[s.index("(") + 1:s.rindex(")")]
    fields = {}
    for key in ("normal", "normal_concat", "reduce", "reduce_concat"):
        start = body.index(key + "=") + len(key) + 1
        rest = body[start:]
        depth, end = 0, len(rest)
        for i, ch in enumerate(rest):
            if ch in "[(":
                depth += 1
            elif ch in "])":
                depth -= 1
            elif ch == "," and depth == 0:
                end = i
                break
        val = rest[:end].strip()
        if val.startswith("range("):
            a, b = val[6:-1].split(",")
            fields[key] = list(range(int(a), int(b)))
        else:
            fields[key] = ast.literal_eval(val)
    return Genotype(normal=[tuple(x) for x in fields["normal"]], normal_concat=list(fields["normal_concat"]),
                    reduce=[tuple(x) for x in fields["reduce"]], reduce_concat=list(fields["reduce_concat"]))
