"""Process/rank-tagged logging.

Parity with the reference's logger usage (`training.py:13,97-98` add a file handler at
`log/<...>.log`; `executor.py:25-26,36-37` stamp the executor name into every line so the
offline analysers can attribute lines, e.g. `analyze_log.py:55` matches `worker {id}.*train`).
Here one process drives a whole cohort of clients, so the *rank* is stamped into the record
and client-level lines carry the client name explicitly ("worker 3 ...").
"""

from __future__ import annotations

import logging
import os
import sys

_LOGGER_NAME = "dls_amd"
_configured = False


class _RankFilter(logging.Filter):
    def filter(self, record: logging.LogRecord) -> bool:
        record.rank = os.environ.get("RANK", "0")
        return True


def get_logger() -> logging.Logger:
    global _configured
    logger = logging.getLogger(_LOGGER_NAME)
    if not _configured:
        _configured = True
        handler = logging.StreamHandler(sys.stderr)
        handler.setFormatter(
            logging.Formatter(
                "%(asctime)s %(levelname)s [rank %(rank)s] %(message)s", "%H:%M:%S"
            )
        )
        handler.addFilter(_RankFilter())
        logger.addHandler(handler)
        logger.setLevel(os.environ.get("DLS_LOG_LEVEL", "INFO"))
        logger.propagate = False
    return logger


def set_level(level: str | int) -> None:
    get_logger().setLevel(level)


def add_file_handler(path: str) -> logging.Handler:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    handler = logging.FileHandler(path)
    handler.setFormatter(
        logging.Formatter("%(asctime)s %(levelname)s [rank %(rank)s] %(message)s")
    )
    handler.addFilter(_RankFilter())
    get_logger().addHandler(handler)
    return handler


def remove_handler(handler: logging.Handler) -> None:
    get_logger().removeHandler(handler)
    handler.close()
