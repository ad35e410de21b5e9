"""Sphinx configuration for the MI355X device plugin docs.

Builds the markdown pages under docs/ (MyST) with the table of contents in
sphinx/_toc.yml. Uses the ROCm docs theme when it is installed (readthedocs,
docs/sphinx/requirements.txt) and falls back to Sphinx's built-in theme, so a
plain ``sphinx-build docs docs/_build`` works offline too.
"""
import importlib.util
import os
import re

_here = os.path.dirname(os.path.abspath(__file__))


def _chart_app_version() -> str:
    with open(os.path.join(_here, "..", "helm", "amd-gpu", "Chart.yaml")) as f:
        m = re.search(r"^appVersion:\s*\"?([^\"\n]+)\"?", f.read(), re.M)
    return m.group(1) if m else "dev"


project = "MI355X Kubernetes Device Plugin"
version = _chart_app_version()
release = version
html_title = f"MI355X Device Plugin {version}"
author = "MI355X device plugin authors"

exclude_patterns = ["_build", ".venv", "sphinx/requirements.*"]
source_suffix = {".md": "markdown"}
root_doc = "index"

if importlib.util.find_spec("rocm_docs") is not None:
    extensions = ["rocm_docs"]
    html_theme = "rocm_docs_theme"
    html_theme_options = {"flavor": "instinct"}
    external_toc_path = "./sphinx/_toc.yml"
else:
    extensions = [e for e in ("myst_parser", "sphinx_external_toc") if importlib.util.find_spec(e) is not None]
    external_toc_path = "./sphinx/_toc.yml"
    html_theme = "alabaster"

# _toc.yml is generated from _toc.yml.in (the rocm_docs convention); do it here
# so a local build needs no extra step
_toc_in = os.path.join(_here, "sphinx", "_toc.yml.in")
_toc = os.path.join(_here, "sphinx", "_toc.yml")
if os.path.exists(_toc_in):
    with open(_toc_in) as f_in:
        _text = f_in.read()
    if not os.path.exists(_toc) or open(_toc).read() != _text:
        try:
            with open(_toc, "w") as f_out:
                f_out.write(_text)
        except OSError:
            pass
