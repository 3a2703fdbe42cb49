"""Logging helpers (reference ``fedml_api/utils/logger.py:7-33`` and the entry points' file logger,
``main_sailentgrads.py:184-192,249-254``)."""
from __future__ import annotations

import logging
import os


def logging_config(args=None, process_id=0):
    """Rank-prefixed console logging."""
    root = logging.getLogger()
    for h in list(root.handlers):
        root.removeHandler(h)
    fmt = logging.Formatter(str(process_id) + " - %(asctime)s %(filename)s[line:%(lineno)d] %(levelname)s %(message)s",
                            "%a, %d %b %Y %H:%M:%S")
    h = logging.StreamHandler()
    h.setFormatter(fmt)
    root.addHandler(h)
    root.setLevel(logging.INFO if process_id == 0 else logging.WARNING)
    return root


def logger_config(log_path, logging_name):
    """File logger writing bare messages to ``log_path`` (the reference's LOG/<dataset>/<identity>.log)."""
    os.makedirs(os.path.dirname(os.path.abspath(log_path)), exist_ok=True)
    logger = logging.getLogger(logging_name)
    logger.setLevel(logging.DEBUG)
    for h in list(logger.handlers):
        logger.removeHandler(h)
    fh = logging.FileHandler(log_path, mode="w", encoding="UTF-8")
    fh.setLevel(logging.DEBUG)
    fh.setFormatter(logging.Formatter("%(message)s"))
    logger.addHandler(fh)
    ch = logging.StreamHandler()
    ch.setLevel(logging.INFO)
    ch.setFormatter(logging.Formatter("%(message)s"))
    logger.addHandler(ch)
    return logger
