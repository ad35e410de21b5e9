"""A small renderer for this repo's Helm chart (no helm binary in the image).

It implements the part of Go text/template and of Helm's sprig functions the
chart under helm/amd-gpu uses, with Go's semantics where they matter:

* actions ``{{ pipeline }}`` with ``{{-`` / ``-}}`` whitespace trimming and
  ``{{/* comments */}}``;
* ``if`` / ``else if`` / ``else`` / ``range`` / ``with`` / ``define`` / ``end``;
* pipelines (``a | f b`` passes ``a`` as f's last argument), parenthesised
  sub-pipelines, ``$var := ...`` declarations, ``.Field.Chains``, ``$``;
* truthiness of Go's ``if`` (false, 0, "", nil, empty list / map are false);
* functions: default, ternary, or, and, not, eq, ne, quote, toYaml, nindent,
  indent, include, printf (%s %d %v), trunc, trimSuffix, replace, contains,
  required;
* numbers from values print like Helm's float64 (10, not 10.0);
* a missing value prints as "" (Helm's ``<no value>`` replacement).

``render_chart(chart_dir, values_overrides)`` returns {template name: text}
for every template, with values merged over values.yaml as ``helm --set``
would (nested dicts merged, scalars replaced).
"""
from __future__ import annotations

import copy
import os
import re
from typing import Any, Dict, List, Optional, Tuple

import yaml


class TemplateError(Exception):
    pass


# ------------------------------------------------------------------ lexing
_ACTION = re.compile(r"\{\{(-?)(.*?)(-?)\}\}", re.S)


def _tokenize(src: str) -> List[Tuple[str, str]]:
    """[(kind, text)] with kind "text" or "action"; trim markers applied."""
    out: List[Tuple[str, str]] = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        ltrim, body, rtrim = m.group(1) == "-", m.group(2), m.group(3) == "-"
        out.append(("text", text.rstrip() if ltrim else text))
        out.append(("action", body.strip()))
        out.append(("rtrim", "1" if rtrim else ""))
        pos = m.end()
    out.append(("text", src[pos:]))
    # apply right trims to the following text
    res: List[Tuple[str, str]] = []
    trim_next = False
    for kind, val in out:
        if kind == "rtrim":
            trim_next = bool(val)
            continue
        if kind == "text" and trim_next:
            val = val.lstrip()
            trim_next = False
        res.append((kind, val))
    return res


# ------------------------------------------------------------------ expression parsing
_EXPR_TOK = re.compile(r'\s*(?:(?P<str>"(?:[^"\\]|\\.)*")|(?P<raw>`[^`]*`)|(?P<num>-?\d+(?:\.\d+)?)'
                       r'|(?P<decl>:=)|(?P<assign>=)|(?P<pipe>\|)|(?P<lp>\()|(?P<rp>\))'
                       r'|(?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)|(?P<field>(?:\.[A-Za-z0-9_]+)+|\.)'
                       r'|(?P<ident>[A-Za-z_][A-Za-z0-9_]*))')


def _lex_expr(s: str) -> List[Tuple[str, str]]:
    toks, pos = [], 0
    s = s.rstrip()
    while pos < len(s):
        m = _EXPR_TOK.match(s, pos)
        if not m or m.end() == pos:
            raise TemplateError(f"cannot parse {s!r} at {pos}")
        kind = m.lastgroup
        toks.append((kind, m.group(kind)))
        pos = m.end()
    return toks


class _Expr:
    """Parsed pipeline: optional declaration + list of commands (lists of operands)."""

    def __init__(self, text: str):
        toks = _lex_expr(text)
        self.decl: Optional[str] = None
        if len(toks) >= 2 and toks[0][0] == "var" and toks[1][0] in ("decl", "assign"):
            self.decl = toks[0][1]
            toks = toks[2:]
        self.cmds, rest = self._pipeline(toks)
        if rest:
            raise TemplateError(f"trailing tokens in {text!r}")

    def _pipeline(self, toks):
        cmds, cur = [], []
        while toks:
            k, v = toks[0]
            if k == "rp":
                break
            toks = toks[1:]
            if k == "pipe":
                cmds.append(cur)
                cur = []
            elif k == "lp":
                sub, toks = self._pipeline(toks)
                if not toks or toks[0][0] != "rp":
                    raise TemplateError("unbalanced (")
                toks = toks[1:]
                cur.append(("sub", sub))
            else:
                cur.append((k, v))
        cmds.append(cur)
        return cmds, toks


# ------------------------------------------------------------------ tree
class _Node:
    def __init__(self, kind: str, arg: str = ""):
        self.kind, self.arg = kind, arg
        self.body: List[Any] = []
        self.elifs: List[Tuple[str, List[Any]]] = []   # (condition, body)
        self.orelse: List[Any] = []


def _parse(tokens: List[Tuple[str, str]], defines: Dict[str, List[Any]]) -> List[Any]:
    root: List[Any] = []
    stack: List[Tuple[_Node, str]] = []          # (node, which list is open: body | elif | else)

    def cur_list():
        if not stack:
            return root
        node, where = stack[-1]
        if where == "body":
            return node.body
        if where == "else":
            return node.orelse
        return node.elifs[-1][1]

    for kind, val in tokens:
        if kind == "text":
            if val:
                cur_list().append(val)
            continue
        if val.startswith("/*"):
            continue
        word = val.split(None, 1)
        head, rest = word[0], (word[1] if len(word) > 1 else "")
        if head in ("if", "range", "with", "define"):
            n = _Node(head, rest)
            if head != "define":
                cur_list().append(n)
            stack.append((n, "body"))
        elif head == "else":
            node, _ = stack[-1]
            if rest.startswith("if "):
                node.elifs.append((rest[3:], []))
                stack[-1] = (node, "elif")
            else:
                stack[-1] = (node, "else")
        elif head == "end":
            node, _ = stack.pop()
            if node.kind == "define":
                defines[node.arg.strip().strip('"')] = node.body
        else:
            cur_list().append(("expr", val))
    if stack:
        raise TemplateError("unterminated block")
    return root


# ------------------------------------------------------------------ evaluation
def _truthy(v) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def _fmt(v) -> str:
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return str(int(v)) if v.is_integer() else repr(v)
    if isinstance(v, (dict, list)):
        return "map[...]" if isinstance(v, dict) else "[" + " ".join(_fmt(x) for x in v) + "]"
    return str(v)


def _go_numbers(v):
    """Helm's values are JSON numbers (float64); Go's YAML encoder writes an
    integral one without a fraction (3, not 3.0)."""
    if isinstance(v, dict):
        return {k: _go_numbers(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_go_numbers(x) for x in v]
    if isinstance(v, float) and v.is_integer() and abs(v) < 1e15:
        return int(v)
    return v


def _to_yaml(v) -> str:
    if v in ({}, [], None):
        return "{}" if v == {} or v is None else "[]"
    return yaml.safe_dump(_go_numbers(v), default_flow_style=False, sort_keys=True).rstrip("\n")


def _indent(n, s) -> str:
    pad = " " * int(n)
    return "\n".join(pad + line for line in str(s).split("\n"))


def _printf(fmt, *args) -> str:
    out, i = [], 0
    parts = re.split(r"(%[sdvq])", fmt)
    for p in parts:
        if p in ("%s", "%v"):
            out.append(_fmt(args[i]))
            i += 1
        elif p == "%d":
            out.append(str(int(args[i])))
            i += 1
        elif p == "%q":
            out.append('"' + _fmt(args[i]) + '"')
            i += 1
        else:
            out.append(p)
    return "".join(out)


class Renderer:
    def __init__(self, defines: Dict[str, List[Any]]):
        self.defines = defines
        self.funcs = {
            "default": lambda d, v=None: v if _truthy(v) else d,
            "ternary": lambda a, b, c: a if _truthy(c) else b,
            "or": lambda *a: next((x for x in a if _truthy(x)), a[-1] if a else None),
            "and": lambda *a: next((x for x in a if not _truthy(x)), a[-1] if a else None),
            "not": lambda a: not _truthy(a),
            "eq": lambda a, *b: any(a == x for x in b),
            "ne": lambda a, b: a != b,
            "mul": lambda *a: __import__("math").prod(int(x) for x in a),
            "quote": lambda *a: " ".join('"' + _fmt(x).replace('"', '\\"') + '"' for x in a),
            "toYaml": _to_yaml,
            "nindent": lambda n, s: "\n" + _indent(n, s),
            "indent": _indent,
            "printf": _printf,
            "trunc": lambda n, s: s[:int(n)],
            "trimSuffix": lambda suf, s: s[:-len(suf)] if suf and s.endswith(suf) else s,
            "replace": lambda old, new, s: s.replace(old, new),
            "contains": lambda sub, s: sub in s,
            "required": self._required,
        }

    @staticmethod
    def _required(msg, v):
        if not _truthy(v) and v is not False and v != 0:
            raise TemplateError(msg)
        return v

    def _lookup(self, base, chain: str):
        v = base
        for part in [p for p in chain.split(".") if p]:
            if isinstance(v, dict):
                v = v.get(part)
            else:
                v = getattr(v, part, None)
            if v is None:
                return None
        return v

    def _operand(self, tok, dot, env):
        k, v = tok
        if k == "str":
            return bytes(v[1:-1], "utf-8").decode("unicode_escape")
        if k == "raw":
            return v[1:-1]
        if k == "num":
            return float(v) if "." in v else int(v)
        if k == "field":
            return dot if v == "." else self._lookup(dot, v)
        if k == "var":
            name, _, chain = v.partition(".")
            if name not in env:
                raise TemplateError(f"undefined variable {name}")
            return self._lookup(env[name], chain) if chain else env[name]
        if k == "sub":
            return self._eval_cmds(tok[1], dot, env)
        if k == "ident":
            if v in ("true", "false"):
                return v == "true"
            if v == "nil":
                return None
            raise TemplateError(f"function {v} used as a value")
        raise TemplateError(f"unexpected {tok}")

    def _eval_cmd(self, cmd, dot, env, piped=(), has_piped=False):
        if not cmd:
            raise TemplateError("empty command")
        k, v = cmd[0]
        if k == "ident" and v not in ("true", "false", "nil"):
            args = [self._operand(t, dot, env) for t in cmd[1:]]
            if has_piped:
                args.append(piped)
            if v == "include":
                return self.include(args[0], args[1])
            if v not in self.funcs:
                raise TemplateError(f"unknown function {v}")
            return self.funcs[v](*args)
        if len(cmd) > 1 or has_piped:
            raise TemplateError(f"cannot call a non-function {cmd}")
        return self._operand(cmd[0], dot, env)

    def _eval_cmds(self, cmds, dot, env):
        val, has = None, False
        for c in cmds:
            val = self._eval_cmd(c, dot, env, val, has)
            has = True
        return val

    def eval(self, text: str, dot, env):
        e = _Expr(text)
        val = self._eval_cmds(e.cmds, dot, env)
        if e.decl:
            env[e.decl] = val
            return None, True
        return val, False

    def include(self, name, dot) -> str:
        if name not in self.defines:
            raise TemplateError(f"no template {name!r}")
        return self.run(self.defines[name], dot, {"$": dot})

    def run(self, nodes, dot, env) -> str:
        out = []
        for n in nodes:
            if isinstance(n, str):
                out.append(n)
            elif isinstance(n, tuple):
                val, decl = self.eval(n[1], dot, env)
                if not decl:
                    out.append(_fmt(val))
            elif n.kind == "if":
                branches = [(n.arg, n.body)] + n.elifs
                for cond, body in branches:
                    if _truthy(self.eval(cond, dot, dict(env))[0]):
                        out.append(self.run(body, dot, dict(env)))
                        break
                else:
                    out.append(self.run(n.orelse, dot, dict(env)))
            elif n.kind == "with":
                v = self.eval(n.arg, dot, dict(env))[0]
                out.append(self.run(n.body, v, dict(env)) if _truthy(v) else self.run(n.orelse, dot, dict(env)))
            elif n.kind == "range":
                v = self.eval(n.arg, dot, dict(env))[0]
                items = list(v.values()) if isinstance(v, dict) else list(v or [])
                if not items:
                    out.append(self.run(n.orelse, dot, dict(env)))
                for it in items:
                    out.append(self.run(n.body, it, dict(env)))
        return "".join(out)


def _merge(base: dict, over: dict) -> dict:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def _floats(v):
    """Helm reads numbers in values as float64."""
    if isinstance(v, bool):
        return v
    if isinstance(v, int):
        return float(v)
    if isinstance(v, dict):
        return {k: _floats(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_floats(x) for x in v]
    return v


def render_chart(chart_dir: str, values: Optional[dict] = None, release: str = "amd-gpu",
                 namespace: str = "kube-system") -> Dict[str, str]:
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        vals = _merge(yaml.safe_load(f) or {}, values or {})
    tdir = os.path.join(chart_dir, "templates")
    defines: Dict[str, List[Any]] = {}
    trees = {}
    for name in sorted(os.listdir(tdir)):
        with open(os.path.join(tdir, name)) as f:
            trees[name] = _parse(_tokenize(f.read()), defines)
    ctx = {"Values": _floats(vals),
           "Chart": {"Name": chart["name"], "Version": chart["version"], "AppVersion": chart.get("appVersion", "")},
           "Release": {"Name": release, "Namespace": namespace, "Service": "Helm"}}
    r = Renderer(defines)
    out = {}
    for name, tree in trees.items():
        if name.startswith("_") or not name.endswith((".yaml", ".yml")):
            continue
        out[name] = r.run(tree, ctx, {"$": ctx})
    return out


def rendered_objects(chart_dir: str, values: Optional[dict] = None) -> List[dict]:
    """Every Kubernetes object the chart renders with these values."""
    objs = []
    for text in render_chart(chart_dir, values).values():
        for doc in yaml.safe_load_all(text):
            if doc:
                objs.append(doc)
    return objs
