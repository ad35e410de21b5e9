"""The native JSON reader / writer (native/src/kube/json.cpp: the labeller's
Node objects and watch events, JSON kubeconfigs) against Python's json module.

Generated documents, written by ``json.dumps`` in compact, indented and
ASCII-escaped forms, must read back to the same value after the native
parse + serialise round trip (numbers keep their source text, so a GET +
Update of a Node does not reformat it); documents Python refuses are refused.
"""
import json

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from rocm_k8s_device_plugin_amd.ops.native import core

_SCALAR = st.one_of(st.none(), st.booleans(), st.integers(min_value=-2**63, max_value=2**64),
                    st.floats(allow_nan=False, allow_infinity=False),
                    st.text(st.characters(codec="utf-8", exclude_categories=("Cs",)), max_size=20))
_VALUE = st.recursive(_SCALAR, lambda c: st.one_of(st.lists(c, max_size=5),
                                                   st.dictionaries(st.text(max_size=10), c, max_size=5)),
                      max_leaves=25)


def roundtrip(text):
    out, err = core().json_roundtrip(text)
    assert out is not None, f"native reader refused {text!r}: {err}"
    return out


@settings(deadline=None, suppress_health_check=[HealthCheck.too_slow])  # examples: the profile (conftest.py)
@given(v=_VALUE, indent=st.sampled_from([None, 0, 2]), ascii_=st.booleans())
def test_roundtrip_equals_python(v, indent, ascii_):
    text = json.dumps(v, indent=indent, ensure_ascii=ascii_)
    out = roundtrip(text)
    assert json.loads(out) == json.loads(text)
    # the writer's output reads back to itself (stable)
    assert roundtrip(out) == out


def test_numbers_keep_their_source_text():
    assert roundtrip('{"a": 1.50, "b": -0, "c": 1E+3, "d": 12345678901234567890123}') == \
        '{"a":1.50,"b":-0,"c":1E+3,"d":12345678901234567890123}'


@pytest.mark.parametrize("text", ['{"a": 1,}', '[1 2]', '{"a" 1}', '"\\x"', '01', '[1,]', '{"a": tru}', '"\\ud800"x',
                                  '{"a": 1}}', '', '   ', '"unterminated', '{"a": 1e}', '-', '1.', '.5', '+1', '1e+',
                                  '-01', '[1-2]', '0x10'])
def test_malformed_documents_are_refused(text):
    with pytest.raises(ValueError):
        json.loads(text)
    out, err = core().json_roundtrip(text)
    assert out is None and err, (text, out)


def test_nesting_is_bounded():
    """Deeper than 128 levels is refused (a hostile apiserver answer must not
    exhaust the stack); Python reads it."""
    deep = "[" * 129 + "]" * 129
    assert json.loads(deep)
    out, err = core().json_roundtrip(deep)
    assert out is None and "deep" in err
    assert core().json_roundtrip("[" * 128 + "]" * 128)[0] is not None
