"""ORACLE SHIM: placeholder module."""
