"""ORACLE SHIM: ujson -> json."""
from json import *  # noqa
