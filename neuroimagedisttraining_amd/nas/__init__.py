"""Differentiable architecture search (DARTS / GDAS) — reference ``fedml_api/model/cv/darts/``."""
from .architect import Architect  # noqa: F401
from .genotypes import GENOTYPES, PRIMITIVES, Genotype, genotype_from_string  # noqa: F401
from .network import AuxiliaryHeadCIFAR, AuxiliaryHeadImageNet, NetworkCIFAR, NetworkImageNet  # noqa: F401
from .search import ModelForModelSizeMeasure, Network, Network_GumbelSoftmax, derive_genotype  # noqa: F401
