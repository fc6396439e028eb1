"""Rank-aware logging.

Parity with the reference's logging setup (`train.py:16-29`): the same format
string, INFO level, and a filter that stamps `record.rank` from the `RANK`
environment variable (``?`` when unset).  Unlike the reference, the filter is
installed on a handler-independent logger factory so every framework module
can log with the rank prefix, not only ``__main__``.
"""
from __future__ import annotations

import logging
import os

LOG_FORMAT = "%(asctime)s - %(name)s - %(levelname)s - [Rank %(rank)s] %(message)s"

_configured = False


class RankLogFilter(logging.Filter):
    """Injects ``record.rank`` from ``$RANK`` (reference `train.py:22-25`)."""

    def filter(self, record: logging.LogRecord) -> bool:  # noqa: A003
        record.rank = os.environ.get("RANK", "?")
        return True


def setup_logging(level: int = logging.INFO) -> None:
    """Configure the root handler once with the reference format."""
    global _configured
    if _configured:
        return
    logging.basicConfig(level=level, format=LOG_FORMAT)
    # Records from loggers without the filter still need a ``rank`` field,
    # otherwise the formatter raises.  Attach the filter to root handlers.
    for h in logging.getLogger().handlers:
        h.addFilter(RankLogFilter())
    _configured = True


def get_logger(name: str) -> logging.Logger:
    setup_logging()
    logger = logging.getLogger(name)
    if not any(isinstance(f, RankLogFilter) for f in logger.filters):
        logger.addFilter(RankLogFilter())
    return logger
