"""The native YAML reader (native/src/kube/yaml.cpp: kubeconfig and the device
plugin's -config file) against PyYAML on the same documents.

Hypothesis builds mappings of strings, booleans, nulls, lists and nested
mappings; PyYAML writes each one in block, flow and mixed style, with every
scalar quoting style and line widths that fold long scalars; the native reader
must return what ``yaml.safe_load`` returns. Plain scalars that are not
booleans or null stay strings in the native reader (configs read them as
text), so the generated documents hold no numbers: PyYAML quotes any string
that would resolve to one.

A second generator writes documents the way people write configs by hand
(per-level indentation, sequences at their key's column, comments after
values and on their own lines, blank lines, document markers, short flow
leaves); every one PyYAML accepts must read the same natively.

The suite runs these properties derandomized (the "ci" Hypothesis profile,
tests/conftest.py); tools/yaml_differential.py explores fresh draws.
"""
import json

import pytest
import yaml
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from rocm_k8s_device_plugin_amd.ops.native import core

# keys and values over characters that exercise quoting, escapes, comments and indicators
_CHARS = st.characters(codec="utf-8", exclude_categories=("Cs", "Cc"), exclude_characters="\ufeff\x85\u2028\u2029")
_TEXT = st.text(alphabet=st.one_of(st.sampled_from(list("ab -:#,[]{}'\"&*!|>%@`?\\\t/.0123456789")), _CHARS),
                max_size=24)
_KEY = st.text(alphabet=st.sampled_from(list("abcdefxyz_-./0123456789 :#'\"")), min_size=1, max_size=12)
_SCALAR = st.one_of(_TEXT, st.booleans(), st.none())
_VALUE = st.recursive(_SCALAR, lambda c: st.one_of(st.lists(c, max_size=4),
                                                   st.dictionaries(_KEY, c, max_size=4)), max_leaves=16)
_DOC = st.one_of(st.dictionaries(_KEY, _VALUE, min_size=1, max_size=6), st.lists(_VALUE, min_size=1, max_size=5))


def native(text):
    out, err = core().yaml_to_json(text)
    assert out is not None, f"native reader refused:\n{text}\n-> {err}"
    return json.loads(out)


@settings(deadline=None, suppress_health_check=[HealthCheck.too_slow])  # examples: the profile (conftest.py)
@given(doc=_DOC, flow=st.sampled_from([False, True, None]), style=st.sampled_from([None, '"', "'"]),
       width=st.integers(min_value=20, max_value=120), unicode=st.booleans())
def test_native_reader_equals_pyyaml(doc, flow, style, width, unicode):
    text = yaml.safe_dump(doc, default_flow_style=flow, default_style=style, width=width, allow_unicode=unicode,
                          sort_keys=False)
    assert native(text) == yaml.safe_load(text), text


@pytest.mark.parametrize("text", [
    # kubeconfig as kubectl writes it
    "apiVersion: v1\nkind: Config\nclusters:\n- cluster:\n    certificate-authority-data: QUJD\n"
    "    server: https://10.0.0.1:6443\n  name: c\ncontexts:\n- context:\n    cluster: c\n    user: u\n  name: x\n"
    "current-context: x\nusers:\n- name: u\n  user:\n    token: abc # trailing comment\n",
    # the device plugin's -config file
    "gpu:\n  device_count: 4\n",
    # block scalars with chomping indicators, comments, blank lines, nested sequences
    "a: |+\n  keep\n\n\nb: >\n  folded\n  line\n\n  para\nc: |-\n  strip\n# comment\nd:\n- - x\n  - y\n- z\n",
    # a JSON document read as YAML 1.1: an exponent needs a '.' and a sign to be a float (the
    # explore profile's find, profiles/r6/yaml_differential_10k.json)
    "[[0E0]]\n", "[1e3, 1.5e3]\n", "{\"a\": 0E0, \"b\": [1E2, 3.25e2]}\n",
    # quotes inside plain scalars are ordinary characters: keys `:'` / `:"`, `a'b`, a quote after a
    # flow indicator in block context (`:'` was read as an open quoted scalar)
    ":': ' #'\n", ":\": ' #'\n", ":': \" #\"\n", "a:': b # c\n", "a'b: c # d\n", "a: b'c # d\n",
    "a: b,'c # d'\n", "a: x:'y # z'\n", "- :' # c\n", "a: [b, 'c # d', \"e # f\"] # g\n",
    "{\"a\":'b # c'} # d\n", "a: &x 'v # w'\nb: *x\n", "a: !!str 'v # w'\n",
    # quoted scalars with escapes, and a multi-line plain scalar
    "e: \"tab\\tnl\\n\\u00e9 \\\"q\\\"\"\nf: 'it''s'\ng: plain scalar\n  continued here\n",
    # comment lines indented deeper than the scalar above them end it
    "gpu:\n  device_count: 2\n    # two GPUs\n", "- x\n    # note\n", "a: b\n  c\n    # z\n",
    "a: [1,\n  # c\n  2]\n", "a: \"b\n  # c\n  d\"\n", "a: !!str \"b\n  # c\n  d\"\n", "gpu:\n  device_count: 2  # two\n      # GPUs\nx: y\n",
    # sequence entries that are blocks, empty, or block scalars
    "-\n  a: 1\n-\n- b\n", "- |\n  text\n  more\n- >-\n  folded\n  text\n",
    # every double-quoted escape, an explicit indentation indicator, kept and folded blank lines
    "a: \"\\0\\a\\b\\v\\f\\r\\e\\N\\L\\P\\x41\\u00e9\\U0001F600\\_\\ \\/\"\n", "a: |2\n   x\n  y\n",
    "a: |+\n  x\n\n\nb: c\n", "a: >\n  one\n\n\n  two\n", "a: \"one\n\n\n  two\"\n",
    # single-pair mappings inside flow sequences
    "a: [b: c]\n", "a: [b: c, d, \"e\": [f: g], h:]\n", "[x: 1, y]\n", "a: {b:, c: [d:]}\n", "a: [http://x:80/y, z]\n",
    # anchors and aliases: on scalars, block and flow collections, keys, after/before a tag
    "a: &x v\nb: *x\n", "a: &x\n  b: v\nc: *x\n", "l1: &id001\n- x\nl2: *id001\n", "f: [&id001 [x, y], *id001]\n",
    "- &x [v]\n- *x\n", "- &s\n  - v\n- *s\n", "- &s |\n  text\n- *s\n", "a: &x >-\n  f\n  g\nb: *x\n",
    "a: !!str &x v\nb: *x\n", "a: &x !!str v\nb: *x\n", "a: !!map &m\n  k: v\nb: *m\n", "- &s !!seq\n  - a\n- *s\n",
    "- &a k: v\n- *a\n", "&k key: v\nother: *k\n", "a: &x k\n*x : v\n", "a: &x k\n*x: v\n", "a: {&q k: *q}\n",
    "a: &x\nb: *x\n", "a: &x-1_y z\nb: *x-1_y\n",
    # merge keys: one mapping, a list (the earlier mapping wins), own keys override, in flow
    "base: &b {x: p, y: q}\nd:\n  <<: *b\n  y: r\n", "a: &a {x: p}\nb: &b {x: q, y: r}\nc:\n  <<: [*a, *b]\n  z: s\n",
    "a: &a {x: p}\nc: {<<: *a, q: t}\n", "x: &a\n  <<: {p: q}\n  r: s\ny: *a\n", "- <<: {a: b}\n  c: d\n", "\"<<\": v\n",
    # one document with its markers and directives, a byte order mark, CRLF, Null / NULL,
    # scalars and flow collections on the lines below their key
    "---\ngpu:\n  device_count: 2\n", "--- # c\na: b\n", "a: b\n...\n", "%YAML 1.1\n---\na: b\n",
    "\ufeffa: b\n", "a: b\r\nc: d\r\n", "--- {a: b}\n", "--- [x,\n  y]\n", "---\n- x\n", "a: Null\nb: NULL\n",
    "a:    \n  b\n", "a:\n  b\n  c\nd: e\n", "a:\n  \"q\"\n", "a:\n  [x, y]\n", "- \n  {b: c}\n",
    # tags on block values
    "a: !!str |\n  x\n", "a: !!map\n  b: c\n", "a: !!seq\n- b\n", "a: !!str\n", "a: !!null\n", "- !!map\n  a: b\n",
])
def test_hand_written_documents(text):
    assert native(text) == _stringify(yaml.safe_load(text))


def _stringify(v):
    """PyYAML's ints become the native reader's strings (its plain scalars are text)."""
    if isinstance(v, dict):
        return {k: _stringify(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_stringify(x) for x in v]
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return str(v)
    return v


@pytest.mark.parametrize("text", ["a: [b, c\n", "a: 'open\n", "a:\n  - b\n c: d\n", "- a\nb: c\n", "{\"a\": 1",
                                  "a: \"x\\q\"\n", "a: !custom x\n", "a: |\n    x\n  y\n",
                                  # a mapping indicator inside a plain scalar (an indentation mistake)
                                  "a: b\n  c: d\n", "a: b c: d\n", "a: v:\n", "- b\n  c: d\n",
                                  # a plain scalar cannot go on past a comment line
                                  "a: b\n  # c\n  d\n",
                                  # aliases to nothing, bad anchor names, merges of non-mappings
                                  "a: *nope\n", "a: &x.y z\n", "a: &\n", "a: *\n", "a: &a v\nc:\n  <<: *a\n",
                                  "a: &a [v]\nc:\n  <<: *a\n", "- &s - v\n  - w\n- *s\n",
                                  # indicators that cannot start a plain scalar; tags on the wrong kind
                                  "a: , v\n", "a: %x\n", "a: @x\n", "a: `x\n", "a: [|]\n", "a: ]\n", "- ,\n",
                                  "a: [a, %b]\n", "a: !!str\n  b: c\n", "- !!seq\n- x\n",
                                  # a second document, directives without ---, a stray "- "
                                  "a: b\n---\nc: d\n", "a: b\n...\nc: d\n", "%YAML 1.1\na: b\n", "a: - b\n",
                                  "a: -\n", "a:\n  b\n   c: d\n"])
def test_malformed_documents_are_refused(text):
    """Documents PyYAML refuses are refused here too, with an error."""
    with pytest.raises(yaml.YAMLError):
        yaml.safe_load(text)
    out, err = core().yaml_to_json(text)
    assert out is None and err, (text, out)


@pytest.mark.parametrize("text", ["? a\n: b\n", "a: !!binary |\n  eA==\n"])
def test_unsupported_documents_are_refused(text):
    """What PyYAML reads but no config here needs (complex keys, bytes) is refused, not misread."""
    yaml.safe_load(text)
    out, err = core().yaml_to_json(text)
    assert out is None and err, (text, out)


@pytest.mark.parametrize("text, want", [
    # JSON: a repeated key keeps the last value (Python's json and Go's encoding/json agree)
    ('{"a": 1, "b": 2, "a": 3}', {"a": "3", "b": "2"}),
    # UTF-16 escapes: a pair is one code point, a lone surrogate U+FFFD (Go's encoding/json),
    # and an escape after a lone high surrogate is read on its own
    ('{"a": "\\ud83d\\ude00"}', {"a": "\U0001F600"}), ('{"a": "\\ud800"}', {"a": "\ufffd"}),
    ('{"a": "\\ud800\\u0041"}', {"a": "\ufffdA"}), ('{"a": "x\\udc00"}', {"a": "x\ufffd"}),
    # the same in YAML double-quoted scalars
    ('a: "\\ud83d\\ude00"\n', {"a": "\U0001F600"}), ('a: "\\ud800 x"\n', {"a": "\ufffd x"}),
])
def test_repeated_keys_and_surrogate_escapes(text, want):
    """Output is always valid UTF-8 and a repeated key reads as the readers the labeller
    replaces read it."""
    out, err = core().yaml_to_json(text)
    assert out is not None, err
    got = json.loads(out)
    assert {k: str(v) if isinstance(v, int) else v for k, v in got.items()} == want


@pytest.mark.parametrize("text", ["[1e3, 1.5e3, 1.5e+3, -2.0E-1, 7, -0.5]\n", "{\"a\": 0E0, \"b\": [1E+2, 3.25e-2]}\n"])
def test_json_numbers_resolve_as_yaml11(text):
    """A JSON document's numbers as PyYAML's YAML 1.1 resolvers read them: floats
    need a '.' and a signed exponent, the rest stays text."""
    assert native(text) == yaml.safe_load(text)


def test_anchor_redefinition_rebinds():
    """A later anchor of the same name rebinds it for the aliases after it (YAML 1.2 3.2.2.2,
    as go-yaml reads it); PyYAML refuses the document instead."""
    assert native("a: &x v\na2: &x w\nb: *x\n") == {"a": "v", "a2": "w", "b": "w"}


_SHARED = st.one_of(st.lists(_SCALAR, min_size=1, max_size=3), st.dictionaries(_KEY, _SCALAR, min_size=1, max_size=3))


@settings(deadline=None, suppress_health_check=[HealthCheck.too_slow])  # examples: the profile (conftest.py)
@given(doc=st.dictionaries(_KEY, _VALUE, max_size=4), shared=_SHARED, keys=st.lists(_KEY, min_size=2, max_size=4),
       flow=st.sampled_from([False, True, None]), nested=st.booleans())
def test_shared_nodes_equal_pyyaml(doc, shared, keys, flow, nested):
    """An object referenced more than once is written once with an anchor (&id001) and
    then as aliases (*id001); the native reader must expand them as PyYAML does."""
    doc = dict(doc)
    for n, k in enumerate(keys):
        doc[k] = [shared, n] if nested and n % 2 else shared
    text = yaml.safe_dump(doc, default_flow_style=flow, sort_keys=False)
    assert native(text) == _stringify(yaml.safe_load(text)), text


def test_alias_expansion_is_bounded():
    """Ten aliases of ten aliases of ... (a "billion laughs") are refused, not expanded."""
    lines = ["a0: &a0 [x, x, x, x, x, x, x, x, x, x]"]
    lines += [f"a{i}: &a{i} [" + ", ".join([f"*a{i - 1}"] * 10) + "]" for i in range(1, 12)]
    out, err = core().yaml_to_json("\n".join(lines) + "\n")
    assert out is None and "too large" in err
    assert len(native("\n".join(lines[:4]) + "\n")["a3"]) == 10  # small expansions stay fine


# ---- hand-written surface syntax -------------------------------------------------
# safe_dump writes one canonical layout. Config files and kubeconfigs written
# by hand vary indentation per level, put "- " entries at the key's own column,
# comment after values and on lines of their own, leave blank lines, mark the
# document, and use flow collections for short leaves. The native reader must
# read those as PyYAML does (a generated text PyYAML refuses is skipped).
# plain scalars PyYAML also reads as text (no 0b1 / 0x1 / 1_0 / 017 / 1:30 numbers:
# the native reader keeps every plain scalar as text, see the module docstring)
def _reads_as_text(t):
    try:
        return isinstance(yaml.safe_load(t), str)
    except (yaml.YAMLError, ValueError):  # PyYAML itself fails on "0x_" / "0b_"
        return False


_PLAIN = st.text(alphabet=st.sampled_from(list("abcxyz_-./0123456789")), min_size=1, max_size=8).filter(
    lambda t: t[0] not in "-." and _reads_as_text(t))
_LEAF = st.one_of(_PLAIN, st.sampled_from(["true", "false", "null", "~", "''", '""']),
                  st.tuples(st.sampled_from(["'", '"']), _TEXT.filter(lambda t: "\\" not in t and "\n" not in t
                                                                     and "\t" not in t)))
_TREE = st.recursive(_LEAF, lambda c: st.one_of(st.lists(c, min_size=1, max_size=3),
                                               st.dictionaries(_PLAIN, c, min_size=1, max_size=3)), max_leaves=10)


def _leaf_text(v):
    if isinstance(v, tuple):
        q, t = v
        return q + (t.replace("'", "''") if q == "'" else t.replace('"', '\\"')) + q
    return v


def _flow(v):
    if isinstance(v, list):
        return "[" + ", ".join(_flow(x) for x in v) + "]"
    if isinstance(v, dict):
        return "{" + ", ".join(f"{k}: {_flow(x)}" for k, x in v.items()) + "}"
    return _leaf_text(v)


@st.composite
def _hand_written(draw):
    tree = draw(st.dictionaries(_PLAIN, _TREE, min_size=1, max_size=4))
    lines = []
    if draw(st.booleans()):
        lines.append("---" + (" # start" if draw(st.booleans()) else ""))

    def comment():
        c = draw(st.sampled_from(["", "", " # note", "  # a: b", " #- x", " # 'q"]))
        return c

    def emit(v, indent):
        if isinstance(v, dict):
            for k, x in v.items():
                if draw(st.integers(0, 5)) == 0:
                    lines.append(" " * draw(st.integers(0, indent + 2)) + "# " + draw(_PLAIN))
                if draw(st.integers(0, 6)) == 0:
                    lines.append("")
                if isinstance(x, (dict, list)) and x and draw(st.integers(0, 3)):
                    lines.append(" " * indent + f"{k}:" + comment())
                    step = draw(st.integers(1, 4))
                    # a block sequence may sit at its key's own column
                    emit(x, indent if isinstance(x, list) and draw(st.booleans()) else indent + step)
                else:
                    lines.append(" " * indent + f"{k}: {_flow(x)}" + comment())
        else:
            for x in v:
                if isinstance(x, dict) and x and draw(st.booleans()):
                    items = list(x.items())
                    k0, x0 = items[0]
                    lines.append(" " * indent + f"- {k0}: {_flow(x0)}" + comment())
                    for k, y in items[1:]:
                        lines.append(" " * (indent + 2) + f"{k}: {_flow(y)}" + comment())
                elif isinstance(x, (dict, list)) and x and draw(st.booleans()):
                    lines.append(" " * indent + "-" + comment())
                    emit(x, indent + draw(st.integers(1, 3)))
                else:
                    lines.append(" " * indent + f"- {_flow(x)}" + comment())

    emit(tree, 0)
    if draw(st.booleans()):
        lines.append("..." if draw(st.booleans()) else "# end")
    return "\n".join(lines) + "\n"


@settings(deadline=None, suppress_health_check=[HealthCheck.too_slow, HealthCheck.filter_too_much])
@given(text=_hand_written())
def test_hand_written_layouts_equal_pyyaml(text):
    from hypothesis import assume
    try:
        want = yaml.safe_load(text)
    except yaml.YAMLError:
        assume(False)
    assert native(text) == _stringify(want), text
