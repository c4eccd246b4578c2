"""ORACLE SHIM: just enough of jsonpickle for plenum/common/jsonpickle_util.py to import."""
