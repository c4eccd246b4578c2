"""Canonical signing string M (the bytes every Plenum signature covers).

Restates common/serializers/signing_serializer.py:35-92 and
common/serializers/serialization.py:27-36:
  * str -> itself; None -> ""; dict -> "k:v" pairs sorted by key, joined by
    "|" (top-level keys in topLevelKeysToIgnore dropped, level 0 only);
    other iterables -> items joined by ","; anything else -> str(x)
  * only str/int/float/list/dict/None are acceptable (bool is an int);
    anything else raises Exception (common/error.py:1-9)
  * UTF-8 encoded at the top level
"""
from collections.abc import Iterable

ACCEPTABLE = (str, int, float, list, dict, type(None))


class SigningSerializer:
    def serialize(self, obj, level=0, objname=None, topLevelKeysToIgnore=None, toBytes=True):
        text = self._ser(obj, level, objname, topLevelKeysToIgnore)
        return text.encode('utf-8') if toBytes else text

    def _ser(self, obj, level, objname, ignore):
        if not isinstance(obj, ACCEPTABLE):
            raise Exception('invalid type found {}: {}'.format(objname, obj))
        if isinstance(obj, str):
            return obj
        if isinstance(obj, dict):
            skip = set(ignore or ()) if level == 0 else set()
            keys = sorted(k for k in obj.keys() if k not in skip)
            parts = []
            for k in keys:
                child = '.'.join([str(objname), str(k)]) if objname else k
                parts.append(str(k) + ':' + self._ser(obj[k], level + 1, child, None))
            return '|'.join(parts)
        if isinstance(obj, Iterable):
            return ','.join(self._ser(o, level + 1, objname, None) for o in obj)
        if obj is None:
            return ''
        return str(obj)


signing_serializer = SigningSerializer()


try:
    from . import _host   # native serializer (csrc/pv_host.cpp)
except ImportError:
    _host = None


def serialize_msg_for_signing(msg, topLevelKeysToIgnore=None):
    if _host is not None:
        try:
            return _host.serialize(msg, topLevelKeysToIgnore)
        except _host.Fallback:
            pass  # unacceptable/special input: the restatement raises or handles it exactly
    return signing_serializer.serialize(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)
