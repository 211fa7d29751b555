"""Typed parameters with validators and JSON encode/decode.

Behavioural parity with the reference:
- ``Param`` identity is its name (``flink-ml-core/.../param/Param.java:80-91``).
- ``WithParams.set`` checks membership, type and validator (``param/WithParams.java:76-109``);
  ``get`` fails on a null value whose validator rejects null (``:119-129``).
- Every public ``Param`` attribute on a class (incl. mixins) is registered with its default
  value (``util/ParamUtils.java:41-88``).
- JSON encoding of the 16 param kinds matches the Java side so ``metadata`` files are
  interchangeable (vectors as ``{"values":..}`` / ``{"n","indices","values"}``, windows as
  ``{"class": <java class>, ...}``; ``param/VectorParam.java:43-67``, ``param/WindowsParam.java:43-94``).

Python-side setters/getters are generated from the Java camelCase names, in both
``set_features_col`` (snake, like the reference's pyflink API) and ``setFeaturesCol`` spellings.
"""
from __future__ import annotations

import math
import re
from typing import Any, Callable, Dict, Generic, Optional, Sequence, TypeVar

import numpy as np

from ..linalg.vectors import DenseVector, SparseVector, Vector

T = TypeVar("T")


class ParamValidator(Generic[T]):
    def __init__(self, fn: Callable[[Any], bool], desc: str = ""):
        self._fn = fn
        self.desc = desc

    def validate(self, value) -> bool:
        return bool(self._fn(value))

    def __call__(self, value) -> bool:
        return self.validate(value)


class ParamValidators:
    """Validator factories (reference ``param/ParamValidators.java:27-121``)."""

    @staticmethod
    def always_true():
        return ParamValidator(lambda v: True, "alwaysTrue")

    @staticmethod
    def gt(lower):
        return ParamValidator(lambda v: v is not None and float(v) > lower, "gt(%s)" % lower)

    @staticmethod
    def gt_eq(lower):
        return ParamValidator(lambda v: v is not None and float(v) >= lower, "gtEq(%s)" % lower)

    @staticmethod
    def lt(upper):
        return ParamValidator(lambda v: v is not None and float(v) < upper, "lt(%s)" % upper)

    @staticmethod
    def lt_eq(upper):
        return ParamValidator(lambda v: v is not None and float(v) <= upper, "ltEq(%s)" % upper)

    @staticmethod
    def in_range(lower, upper, lower_inclusive=True, upper_inclusive=True):
        def ok(v):
            if v is None:
                return False
            v = float(v)
            lo = v >= lower if lower_inclusive else v > lower
            hi = v <= upper if upper_inclusive else v < upper
            return lo and hi

        return ParamValidator(ok, "inRange(%s,%s)" % (lower, upper))

    @staticmethod
    def in_array(*allowed):
        if len(allowed) == 1 and isinstance(allowed[0], (list, tuple)):
            allowed = tuple(allowed[0])
        return ParamValidator(lambda v: v is not None and v in allowed, "inArray%s" % (allowed,))

    @staticmethod
    def not_null():
        return ParamValidator(lambda v: v is not None, "notNull")

    @staticmethod
    def non_empty_array():
        return ParamValidator(lambda v: v is not None and len(v) > 0, "nonEmptyArray")

    @staticmethod
    def is_sub_set(*allowed):
        if len(allowed) == 1 and isinstance(allowed[0], (list, tuple)):
            allowed = tuple(allowed[0])
        s = set(allowed)

        def ok(v):
            if v is None:
                return False
            v = list(v)
            return len(v) > 0 and len(set(v)) == len(v) and all(x in s for x in v)

        return ParamValidator(ok, "isSubSet")

    # camelCase aliases
    alwaysTrue = always_true
    gtEq = gt_eq
    ltEq = lt_eq
    inRange = in_range
    inArray = in_array
    notNull = not_null
    nonEmptyArray = non_empty_array
    isSubSet = is_sub_set


class Param(Generic[T]):
    """A named, typed, validated parameter."""

    kind = "object"

    def __init__(self, name: str, description: str = "", default_value: T = None,
                 validator: Optional[ParamValidator] = None):
        self.name = name
        self.description = description
        self.validator = validator if validator is not None else ParamValidators.always_true()
        self.default_value = self.convert(default_value) if default_value is not None else None
        if self.default_value is not None and not self.validator.validate(self.default_value):
            raise ValueError("Parameter %s is given an invalid value %s" % (name, default_value))

    # -- value coercion / type check -------------------------------------------------------
    def convert(self, value):
        return value

    def json_encode(self, value):
        return value

    def json_decode(self, obj):
        return self.convert(obj) if obj is not None else None

    def __eq__(self, other):
        return isinstance(other, Param) and other.name == self.name

    def __hash__(self):
        return hash(self.name)

    def __repr__(self):
        return self.name

    @property
    def snake_name(self) -> str:
        return camel_to_snake(self.name)


def _is_bool(v):
    return isinstance(v, (bool, np.bool_))


class BooleanParam(Param[bool]):
    kind = "bool"

    def convert(self, value):
        if value is None:
            return None
        if not _is_bool(value):
            raise TypeError("Parameter %s is given a value with incompatible class %s" % (self.name, type(value).__name__))
        return bool(value)


class IntParam(Param[int]):
    kind = "int"

    def convert(self, value):
        if value is None:
            return None
        if _is_bool(value) or not isinstance(value, (int, np.integer)):
            if isinstance(value, (float, np.floating)) and float(value).is_integer():
                return int(value)
            raise TypeError("Parameter %s is given a value with incompatible class %s" % (self.name, type(value).__name__))
        return int(value)


LongParam = type("LongParam", (IntParam,), {"kind": "long"})


class FloatParam(Param[float]):
    """Double-valued parameter (``DoubleParam``/``FloatParam`` in Java)."""

    kind = "double"

    def convert(self, value):
        if value is None:
            return None
        if _is_bool(value) or not isinstance(value, (int, float, np.integer, np.floating)):
            raise TypeError("Parameter %s is given a value with incompatible class %s" % (self.name, type(value).__name__))
        return float(value)

    def json_encode(self, value):
        if value is None:
            return None
        if math.isinf(value) or math.isnan(value):
            # Jackson writes these as strings when ALLOW_NON_NUMERIC is off
            return "NaN" if math.isnan(value) else ("Infinity" if value > 0 else "-Infinity")
        return value

    def json_decode(self, obj):
        if isinstance(obj, str):
            return float(obj)
        return super().json_decode(obj)


DoubleParam = FloatParam


class StringParam(Param[str]):
    kind = "string"

    def convert(self, value):
        if value is None:
            return None
        if not isinstance(value, str):
            raise TypeError("Parameter %s is given a value with incompatible class %s" % (self.name, type(value).__name__))
        return value


class _ArrayParam(Param):
    elem: Param = None

    def convert(self, value):
        if value is None:
            return None
        if isinstance(value, (str, bytes)) or not isinstance(value, (list, tuple, np.ndarray)):
            raise TypeError("Parameter %s expects an array, got %s" % (self.name, type(value).__name__))
        return tuple(self._conv_elem(v) for v in value)

    def _conv_elem(self, v):
        return v

    def json_encode(self, value):
        return None if value is None else [self._enc_elem(v) for v in value]

    def _enc_elem(self, v):
        return v


class IntArrayParam(_ArrayParam):
    kind = "int[]"

    def _conv_elem(self, v):
        return int(v)


class FloatArrayParam(_ArrayParam):
    kind = "double[]"

    def _conv_elem(self, v):
        return float(v)

    def _enc_elem(self, v):
        return FloatParam.json_encode(self, v)


DoubleArrayParam = FloatArrayParam
LongArrayParam = type("LongArrayParam", (IntArrayParam,), {"kind": "long[]"})


class StringArrayParam(_ArrayParam):
    kind = "string[]"

    def _conv_elem(self, v):
        if v is not None and not isinstance(v, str):
            raise TypeError("Parameter %s expects strings" % self.name)
        return v


class FloatArrayArrayParam(_ArrayParam):
    kind = "double[][]"

    def _conv_elem(self, v):
        return tuple(float(x) for x in v)

    def _enc_elem(self, v):
        return [FloatParam.json_encode(self, x) for x in v]


DoubleArrayArrayParam = FloatArrayArrayParam


class StringArrayArrayParam(_ArrayParam):
    kind = "string[][]"

    def _conv_elem(self, v):
        return tuple(v)

    def _enc_elem(self, v):
        return list(v)


class VectorParam(Param[Vector]):
    kind = "vector"

    def convert(self, value):
        if value is None:
            return None
        if isinstance(value, Vector):
            return value
        if isinstance(value, (list, tuple, np.ndarray)):
            return DenseVector(value)
        raise TypeError("Parameter %s expects a Vector" % self.name)

    def json_encode(self, value):
        if value is None:
            return None
        if isinstance(value, SparseVector):
            return {"n": value.n, "indices": [int(i) for i in value.indices], "values": [float(v) for v in value.values]}
        return {"values": [float(v) for v in value.values]}

    def json_decode(self, obj):
        if obj is None:
            return None
        if len(obj) == 1:
            return DenseVector(obj["values"])
        if len(obj) == 3:
            return SparseVector(obj["n"], obj["indices"], obj["values"])
        raise ValueError("Vector parameter is invalid.")


class WindowsParam(Param):
    kind = "windows"

    def convert(self, value):
        from ..common.window import Windows

        if value is None:
            return None
        if not isinstance(value, Windows):
            raise TypeError("Parameter %s expects Windows" % self.name)
        return value

    def json_encode(self, value):
        return None if value is None else value.to_json()

    def json_decode(self, obj):
        from ..common.window import Windows

        return None if obj is None else Windows.from_json(obj)


# -------------------------------------------------------------------------------------------
_CAMEL_RE1 = re.compile(r"(.)([A-Z][a-z]+)")
_CAMEL_RE2 = re.compile(r"([a-z0-9])([A-Z])")


def camel_to_snake(name: str) -> str:
    return _CAMEL_RE2.sub(r"\1_\2", _CAMEL_RE1.sub(r"\1_\2", name)).lower()


def snake_to_camel(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def _collect_params(cls) -> Dict[str, Param]:
    cache = cls.__dict__.get("_fmlx_param_cache")
    if cache is not None:
        return cache
    params: Dict[str, Param] = {}
    for klass in reversed(cls.__mro__):
        for attr, val in vars(klass).items():
            if isinstance(val, Param) and attr.isupper():
                params[val.name] = val
    setattr(cls, "_fmlx_param_cache", params)
    return params


class WithParams:
    """Mixin holding a param map (reference ``param/WithParams.java``).

    Parameters are declared as UPPER_CASE class attributes holding ``Param`` instances
    (e.g. ``FEATURES_COL = StringParam("featuresCol", ..., "features", not_null())``).
    """

    def __init__(self):
        self._param_map: Dict[Param, Any] = {}
        for p in _collect_params(type(self)).values():
            self._param_map[p] = p.default_value

    # -- core API ---------------------------------------------------------------------------
    def get_param_map(self) -> Dict[Param, Any]:
        return self._param_map

    def get_param(self, name: str) -> Optional[Param]:
        for p in self._param_map:
            if p.name == name:
                return p
        return None

    def set(self, param: Param, value):
        if param not in self._param_map:
            raise ValueError("Parameter %s is not defined on the class %s" % (param.name, type(self).__name__))
        value = param.convert(value)
        if not param.validator.validate(value):
            if value is None:
                raise ValueError("Parameter %s's value should not be null" % param.name)
            raise ValueError("Parameter %s is given an invalid value %s" % (param.name, value))
        self._param_map[param] = value
        return self

    def get(self, param: Param):
        if param not in self._param_map:
            raise ValueError("Parameter %s is not defined on the class %s" % (param.name, type(self).__name__))
        value = self._param_map.get(param)
        if value is None and not param.validator.validate(value):
            raise ValueError("Parameter %s's value should not be null" % param.name)
        return value

    # -- generated accessors ----------------------------------------------------------------
    def __getattr__(self, item: str):
        if item.startswith("_"):
            raise AttributeError(item)
        params = _collect_params(type(self))
        for prefix, is_set in (("set_", True), ("get_", False), ("set", True), ("get", False)):
            if item.startswith(prefix) and len(item) > len(prefix):
                rest = item[len(prefix):]
                if prefix.endswith("_"):
                    pname = snake_to_camel(rest)
                else:
                    if not rest[0].isupper():
                        continue
                    pname = rest[0].lower() + rest[1:]
                p = _lookup_param(params, pname)
                if p is None:
                    continue
                if is_set:
                    if isinstance(p, _ArrayParam):
                        # variadic like the reference Python API: set_input_cols('a', 'b')
                        def _set_arr(*values, _p=p):
                            if len(values) == 1 and (values[0] is None or isinstance(
                                    values[0], (list, tuple, np.ndarray))):
                                return self.set(_p, values[0])
                            return self.set(_p, values)
                        return _set_arr
                    return lambda value, _p=p: self.set(_p, value)
                return lambda _p=p: self.get(_p)
        # property-style access: obj.features_col
        pname = snake_to_camel(item)
        p = _lookup_param(params, pname)
        if p is not None:
            return self.get(p)
        raise AttributeError("%s has no attribute %s" % (type(self).__name__, item))


def _lookup_param(params: Dict[str, Param], name: str) -> Optional[Param]:
    """Exact name first, then case-insensitive (``get_min_df`` -> ``minDF``)."""
    p = params.get(name)
    if p is None:
        low = name.lower()
        for k, v in params.items():
            if k.lower() == low:
                return v
    return p


def update_existing_params(target: WithParams, param_map: Dict[Param, Any]) -> None:
    """Copies values for params that exist on ``target`` (``util/ReadWriteUtils.java:337-345``)."""
    for p, v in param_map.items():
        if p in target.get_param_map():
            target.set(p, v)
