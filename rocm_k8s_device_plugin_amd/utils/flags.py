"""Go ``flag``-compatible command line parsing.

The reference binaries use Go's ``flag`` package plus glog's flags
(cmd/k8s-device-plugin/main.go:50-57; vendor/github.com/golang/glog/glog_flags.go:388-397),
so existing DaemonSets pass arguments like ``-pulse=30``, ``-logtostderr=true``,
``-v=5`` or bare booleans like ``-vram``. This module accepts every one of
those spellings (single or double dash, ``=value`` or separate value, bare
bool) so the manifests stay drop-in.
"""
from __future__ import annotations

import argparse
from typing import Any, Callable, Optional, Sequence


def go_bool(v: Any) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "t", "true", "yes", "y", "on"):
        return True
    if s in ("0", "f", "false", "no", "n", "off"):
        return False
    raise argparse.ArgumentTypeError(f"invalid boolean value {v!r}")


class GoFlagParser(argparse.ArgumentParser):
    """argparse with Go-style flag registration helpers."""

    def __init__(self, *a, **kw):
        kw.setdefault("allow_abbrev", False)
        super().__init__(*a, **kw)

    def _names(self, name: str):
        return [f"-{name}", f"--{name}"]

    def add_int(self, name: str, default: int, help: str, dest: Optional[str] = None):
        self.add_argument(*self._names(name), type=int, default=default, help=help,
                          dest=dest or name.replace("-", "_"), metavar="N")

    def add_str(self, name: str, default: str, help: str, dest: Optional[str] = None):
        self.add_argument(*self._names(name), type=str, default=default, help=help,
                          dest=dest or name.replace("-", "_"), metavar="VALUE")

    def add_float(self, name: str, default: float, help: str, dest: Optional[str] = None):
        self.add_argument(*self._names(name), type=float, default=default, help=help,
                          dest=dest or name.replace("-", "_"), metavar="X")

    def add_bool(self, name: str, default: bool, help: str, dest: Optional[str] = None):
        # Go bool flags: "-x", "-x=true", "-x=false" (but not "-x false")
        self.add_argument(*self._names(name), type=go_bool, nargs="?", const=True, default=default, help=help,
                          dest=dest or name.replace("-", "_"), metavar="BOOL")


def add_glog_flags(p: GoFlagParser) -> None:
    """glog's standard flags (glog_flags.go:388-397, glog_file.go:44-46)."""
    p.add_int("v", 0, "log level for V logs")
    p.add_bool("logtostderr", True, "log to standard error instead of files")
    p.add_bool("alsologtostderr", False, "log to standard error as well as files")
    p.add_str("stderrthreshold", "ERROR", "logs at or above this threshold go to stderr")
    p.add_str("log_dir", "", "If non-empty, write log files in this directory")
    p.add_str("log_link", "", "If non-empty, add symbolic links in this directory to the log files")
    p.add_int("logbuflevel", 0, "Buffer log messages logged at this level or lower (accepted; records are "
              "written and flushed as they are logged)")
    p.add_str("vmodule", "", "comma-separated list of pattern=N settings for file-filtered logging")
    p.add_str("log_backtrace_at", "", "when logging hits line file:N, emit a stack trace")


def parse(p: argparse.ArgumentParser, argv: Optional[Sequence[str]] = None,
          validate: Optional[Callable[[argparse.Namespace], None]] = None) -> argparse.Namespace:
    ns = p.parse_args(argv)
    if validate:
        validate(ns)
    return ns
