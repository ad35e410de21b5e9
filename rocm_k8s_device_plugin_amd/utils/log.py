"""glog-style logging with verbosity levels and optional structured JSON.

Lines look like glog's (``I1015 22:04:05.123456   4242 manager.py:88] msg``)
so existing log scraping keeps working; ``--log-format=json`` switches to one
JSON object per line with structured fields (per-RPC latency etc.), which the
reference never had (SURVEY §5 "Tracing / profiling").
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from typing import Any

_LEVEL_CHAR = {logging.DEBUG: "I", logging.INFO: "I", logging.WARNING: "W", logging.ERROR: "E",
               logging.CRITICAL: "F"}
_THRESHOLDS = {"INFO": logging.INFO, "WARNING": logging.WARNING, "ERROR": logging.ERROR, "FATAL": logging.CRITICAL}

_verbosity = 0
LOGGER_NAME = "mi355x"


class GlogFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        t = record.created
        lt = time.localtime(t)
        us = int((t - int(t)) * 1e6)
        head = (f"{_LEVEL_CHAR.get(record.levelno, 'I')}{lt.tm_mon:02d}{lt.tm_mday:02d} "
                f"{lt.tm_hour:02d}:{lt.tm_min:02d}:{lt.tm_sec:02d}.{us:06d} {os.getpid():>7d} "
                f"{record.filename}:{record.lineno}] ")
        msg = record.getMessage()
        fields = getattr(record, "fields", None)
        if fields:
            msg += " " + " ".join(f"{k}={v}" for k, v in fields.items())
        if record.exc_info:
            msg += "\n" + self.formatException(record.exc_info)
        return head + msg


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": record.created, "level": logging.getLevelName(record.levelno), "src":
             f"{record.filename}:{record.lineno}", "msg": record.getMessage()}
        fields = getattr(record, "fields", None)
        if fields:
            d.update(fields)
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d, default=str)


def setup(verbosity: int = 0, json_format: bool = False, stderr_threshold: str = "INFO",
          logtostderr: bool = True) -> logging.Logger:
    global _verbosity
    _verbosity = int(verbosity)
    lg = logging.getLogger(LOGGER_NAME)
    lg.handlers.clear()
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(JsonFormatter() if json_format else GlogFormatter())
    lg.addHandler(h)
    lg.setLevel(logging.DEBUG if _verbosity > 0 else (logging.INFO if logtostderr else
                                                          _THRESHOLDS.get(stderr_threshold.upper(), logging.INFO)))
    lg.propagate = False
    return lg


def get(name: str = "") -> logging.Logger:
    return logging.getLogger(f"{LOGGER_NAME}.{name}" if name else LOGGER_NAME)


def V(level: int) -> bool:
    """glog.V(level): true if verbose logging at `level` is enabled."""
    return _verbosity >= level


def info_fields(logger: logging.Logger, msg: str, **fields: Any) -> None:
    logger.info(msg, extra={"fields": fields})
