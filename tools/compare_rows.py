"""Compare the per-client rows two ``bench.py --dump-rows`` runs saved (e.g. 1 rank with ``--group 8`` against 8
ranks of 8 clients): prints how many clients' rows are bit-identical and the largest difference of the others.
Usage: ``python tools/compare_rows.py PREFIX_A PREFIX_B``."""
import glob
import sys

import torch


def load(prefix):
    rows = {}
    for f in sorted(glob.glob(prefix + ".rank*.pt")):
        rows.update(torch.load(f, weights_only=True))
    return rows


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    assert a and set(a) == set(b), (len(a), len(b))
    if -1 in a:  # the global masks (key -1): a different mask explains every row difference
        ma, mb = a.pop(-1), b.pop(-1)
        print("global mask: %d of %d entries differ" % (int((ma != mb).sum()), ma.numel()))
    same = [c for c in a if torch.equal(a[c], b[c])]
    diff = {c: float((a[c] - b[c]).abs().max()) for c in a if c not in same}
    print("clients %d  bit-identical %d  differing %d  max|diff| %.3e" %
          (len(a), len(same), len(diff), max(diff.values()) if diff else 0.0))
    return 0 if not diff else 1


if __name__ == "__main__":
    sys.exit(main())
