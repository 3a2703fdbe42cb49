"""Cell-genotype graph export (reference ``fedml_api/model/cv/darts/visualize.py:6-39``).

The reference renders with the ``graphviz`` package (not installed here).  :func:`to_dot` builds the same
graph (inputs ``c_{k-2}``/``c_{k-1}``, one node per intermediate step, op-labelled edges, concat into
``c_{k}``) as DOT text; :func:`plot` writes ``<filename>.dot`` and additionally renders ``<filename>.pdf``
when graphviz is importable.
"""
from __future__ import annotations

import sys


def to_dot(genotype):
    assert len(genotype) % 2 == 0
    steps = len(genotype) // 2
    lines = ["digraph {", "  rankdir=LR;",
             '  node [style=filled, shape=rect, align=center, fontsize=20, height=0.5, width=0.5, penwidth=2, '
             'fontname="times"];', '  edge [fontsize=20, fontname="times"];',
             '  "c_{k-2}" [fillcolor=darkseagreen2];', '  "c_{k-1}" [fillcolor=darkseagreen2];']
    for i in range(steps):
        lines.append('  "%d" [fillcolor=lightblue];' % i)
    for i in range(steps):
        for k in (2 * i, 2 * i + 1):
            op, j = genotype[k]
            u = "c_{k-2}" if j == 0 else "c_{k-1}" if j == 1 else str(j - 2)
            lines.append('  "%s" -> "%d" [label="%s", fillcolor=gray];' % (u, i, op))
    lines.append('  "c_{k}" [fillcolor=palegoldenrod];')
    for i in range(steps):
        lines.append('  "%d" -> "c_{k}" [fillcolor=gray];' % i)
    lines.append("}")
    return "\n".join(lines) + "\n"


def plot(genotype, filename):
    src = to_dot(genotype)
    with open(filename + ".dot", "w") as f:
        f.write(src)
    try:
        import graphviz
    except ImportError:
        return filename + ".dot"
    return graphviz.Source(src, format="pdf").render(filename)


if __name__ == "__main__":
    from . import genotypes
    if len(sys.argv) != 2:
        print("usage:\n python -m neuroimagedisttraining_amd.nas.visualize ARCH_NAME")
        sys.exit(1)
    g = getattr(genotypes, sys.argv[1], None)
    if g is None:  # attribute lookup instead of the reference's eval()
        print("{} is not specified in genotypes.py".format(sys.argv[1]))
        sys.exit(1)
    plot(g.normal, "normal")
    plot(g.reduce, "reduction")
