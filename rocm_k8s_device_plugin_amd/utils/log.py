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
from typing import Any, Dict, List, Optional, Tuple

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


class _StderrHandler(logging.StreamHandler):
    """Writes to whatever sys.stderr is at emit time (not the object it was at
    setup: test capture, or a redirected stderr, may have replaced it)."""

    def __init__(self):
        super().__init__(sys.stderr)

    @property
    def stream(self):
        return sys.stderr

    @stream.setter
    def stream(self, _value):
        pass


class _GlogFileHandler(logging.Handler):
    """One glog severity file: ``<log_dir>/<prog>.<host>.<user>.log.<SEV>.<yyyymmdd-hhmmss>.<pid>``
    holding every record at or above SEV, created on the first such record
    with glog's header, plus the ``<prog>.<SEV>`` symlink to it
    (vendor/github.com/golang/glog/glog_file.go semantics)."""

    def __init__(self, log_dir: str, program: str, severity: str, level: int, formatter: logging.Formatter,
                 log_link: str = ""):
        super().__init__(level)
        self.log_dir, self.program, self.severity, self.log_link = log_dir, program, severity, log_link
        self.setFormatter(formatter)
        self._f = None
        self.path = ""

    def _open(self, created: float) -> None:
        import getpass
        import socket
        lt = time.localtime(created)
        stamp = time.strftime("%Y%m%d-%H%M%S", lt)
        try:
            user = getpass.getuser()
        except Exception:
            user = "unknownuser"
        host = socket.gethostname().split(".")[0] or "unknownhost"
        name = f"{self.program}.{host}.{user}.log.{self.severity}.{stamp}.{os.getpid()}"
        os.makedirs(self.log_dir, exist_ok=True)
        self.path = os.path.join(self.log_dir, name)
        self._f = open(self.path, "a", buffering=1)
        self._f.write(f"Log file created at: {time.strftime('%Y/%m/%d %H:%M:%S', lt)}\n"
                      f"Running on machine: {host}\n"
                      f"Binary: {self.program} (MI355X-native, Python {sys.version.split()[0]})\n"
                      "Log line format: [IWEF]mmdd hh:mm:ss.uuuuuu threadid file:line] msg\n")
        link = os.path.join(self.log_dir, f"{self.program}.{self.severity}")
        try:
            if os.path.islink(link) or os.path.exists(link):
                os.unlink(link)
            os.symlink(name, link)
        except OSError:
            pass
        if self.log_link:   # -log_link: a link to the full path (glog_file.go:133-137)
            link2 = os.path.join(self.log_link, f"{self.program}.{self.severity}")
            try:
                if os.path.islink(link2) or os.path.exists(link2):
                    os.unlink(link2)
                os.symlink(self.path, link2)
            except OSError:
                pass

    def emit(self, record: logging.LogRecord) -> None:
        try:
            if self._f is None:
                self._open(record.created)
            self._f.write(self.format(record) + "\n")
        except Exception:
            self.handleError(record)

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None
        super().close()


class _BacktraceAt(logging.Filter):
    """-log_backtrace_at=file.py:N: a record logged from that line carries the stack."""

    def __init__(self, spec: str):
        super().__init__()
        f, _, n = spec.rpartition(":")
        self.file, self.line = f, int(n) if n.isdigit() else -1

    def filter(self, record: logging.LogRecord) -> bool:
        if record.filename == self.file and record.lineno == self.line and not getattr(record, "_bt", False):
            import traceback
            record.msg = f"{record.msg}\n" + "".join(traceback.format_stack()[:-6]).replace("%", "%%")
            record._bt = True
        return True


_vmodule: List[Tuple[str, int]] = []
_vcache: Dict[str, int] = {}
_SEVERITIES = (("INFO", logging.DEBUG), ("WARNING", logging.WARNING), ("ERROR", logging.ERROR),
               ("FATAL", logging.CRITICAL))


def parse_vmodule(spec: str) -> List[Tuple[str, int]]:
    """glog -vmodule: comma-separated pattern=N (glob on the source file's base
    name without extension, or on the path when the pattern has a '/')."""
    out = []
    for part in (spec or "").split(","):
        part = part.strip()
        if not part:
            continue
        pat, sep, lvl = part.rpartition("=")
        if not sep or not pat or not lvl.lstrip("-").isdigit():
            raise ValueError(f"invalid -vmodule entry {part!r} (want pattern=N)")
        out.append((pat, int(lvl)))
    return out


def setup(verbosity: int = 0, json_format: bool = False, stderr_threshold: str = "ERROR",
          logtostderr: bool = True, alsologtostderr: bool = False, log_dir: str = "", vmodule: str = "",
          log_backtrace_at: str = "", program: Optional[str] = None, log_link: str = "") -> logging.Logger:
    """glog's output rules: -logtostderr sends everything to stderr and writes no
    files; otherwise every severity has its own file under -log_dir (default:
    the temp dir) and records at or above -stderrthreshold (everything with
    -alsologtostderr) are copied to stderr."""
    global _verbosity, _vmodule
    _verbosity = int(verbosity)
    _vmodule = parse_vmodule(vmodule)
    _vcache.clear()
    lg = logging.getLogger(LOGGER_NAME)
    for h in list(lg.handlers):
        h.close()
    lg.handlers.clear()
    lg.filters.clear()
    fmt = JsonFormatter() if json_format else GlogFormatter()
    h = _StderrHandler()
    h.setFormatter(fmt)
    if not logtostderr and not alsologtostderr:
        h.setLevel(_THRESHOLDS.get(stderr_threshold.upper(), logging.ERROR))
    lg.addHandler(h)
    if not logtostderr:
        prog = program or os.path.basename(sys.argv[0] or "mi355x-device-plugin").removesuffix(".py") or "python"
        d = log_dir or os.environ.get("TMPDIR") or "/tmp"
        for sev, level in _SEVERITIES:
            lg.addHandler(_GlogFileHandler(d, prog, sev, level, fmt, log_link))
    if log_backtrace_at:
        # on the handlers: logger filters do not see records of child loggers
        bt = _BacktraceAt(log_backtrace_at)
        for hd in lg.handlers:
            hd.addFilter(bt)
    lg.setLevel(logging.DEBUG if _verbosity > 0 or _vmodule else logging.INFO)
    lg.propagate = False
    return lg


def setup_from_flags(ns, program: str) -> logging.Logger:
    """setup() from the glog flags of utils.flags.add_glog_flags (+ -log_format)."""
    return setup(ns.v, json_format=getattr(ns, "log_format", "glog") == "json", stderr_threshold=ns.stderrthreshold,
                 logtostderr=ns.logtostderr, alsologtostderr=ns.alsologtostderr, log_dir=ns.log_dir,
                 vmodule=ns.vmodule, log_backtrace_at=ns.log_backtrace_at, program=program,
                 log_link=getattr(ns, "log_link", ""))


def get(name: str = "") -> logging.Logger:
    return logging.getLogger(f"{LOGGER_NAME}.{name}" if name else LOGGER_NAME)


def V(level: int) -> bool:
    """glog.V(level): true if verbose logging at `level` is enabled, globally
    (-v) or for the calling source file (-vmodule)."""
    if _verbosity >= level:
        return True
    if not _vmodule:
        return False
    fn = sys._getframe(1).f_code.co_filename
    lvl = _vcache.get(fn)
    if lvl is None:
        import fnmatch
        base = os.path.splitext(os.path.basename(fn))[0]
        stem = os.path.splitext(fn)[0]
        lvl = next((n for pat, n in _vmodule if fnmatch.fnmatchcase(stem if "/" in pat else base, pat)
                    or ("/" in pat and fnmatch.fnmatchcase(stem, "*/" + pat.lstrip("/")))), 0)
        _vcache[fn] = lvl
    return lvl >= level


def info_fields(logger: logging.Logger, msg: str, **fields: Any) -> None:
    logger.info(msg, extra={"fields": fields})
