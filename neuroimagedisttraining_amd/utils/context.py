"""Failure-handling context managers (reference ``fedml_api/utils/context.py:9-35``).

The reference calls ``MPI.COMM_WORLD.Abort()`` on any exception.  With one process per GPU under
``torch.distributed`` the equivalent is to log, destroy the process group (so peers' collectives fail fast
instead of hanging) and re-raise; a non-zero exit then lets ``torchrun`` tear the job down.
"""
from __future__ import annotations

import contextlib
import logging
import threading
import traceback

log = logging.getLogger(__name__)


@contextlib.contextmanager
def raise_MPI_error():  # noqa: N802 (reference name)
    try:
        yield
    except Exception:
        log.error(traceback.format_exc())
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                dist.destroy_process_group()
        finally:
            raise


@contextlib.contextmanager
def raise_error_without_process():
    try:
        yield
    except Exception:
        log.error(traceback.format_exc())
        raise


_LOCK = threading.Lock()


@contextlib.contextmanager
def get_lock(lock=None):
    lk = lock or _LOCK
    lk.acquire()
    try:
        yield
    finally:
        lk.release()
