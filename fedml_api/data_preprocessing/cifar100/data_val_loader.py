"""Compat shim: reference import path ``fedml_api/data_preprocessing/cifar100/data_val_loader.py`` -> ``neuroimagedisttraining_amd.data.images``."""
from neuroimagedisttraining_amd.data.images import load_partition_data_with_val


def load_partition_data_cifar100(data_dir, partition_method, partition_alpha, client_number, batch_size, logger=None,
                          **kw):
    """9-tuple loader (train/val/test) as in the reference's data_val_loader."""
    return load_partition_data_with_val('cifar100', data_dir, partition_method, partition_alpha, client_number,
                                        batch_size, logger, **kw)
