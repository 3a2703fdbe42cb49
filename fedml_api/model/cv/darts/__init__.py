"""Compat shim: reference package ``fedml_api/model/cv/darts`` (its ``train.py:17`` imports ``NetworkCIFAR`` from
the package itself, which the reference's package, having no ``__init__``, does not provide)."""
from .model import NetworkCIFAR, NetworkImageNet  # noqa: F401
