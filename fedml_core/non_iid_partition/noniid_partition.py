"""Compat shim: reference import path ``fedml_core/non_iid_partition/noniid_partition.py`` -> ``neuroimagedisttraining_amd.core.partition``."""
from neuroimagedisttraining_amd.core.partition import (  # noqa: F401
    non_iid_partition_with_dirichlet_distribution, partition_class_samples_with_dirichlet_distribution,
    record_data_stats)
