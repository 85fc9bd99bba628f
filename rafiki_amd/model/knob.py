"""Hyper-parameter ("knob") space types and their JSON (de)serialisation.

Wire format is identical to the reference (`{"type": <class name>, "args": {...}}`,
rafiki/model/knob.py:14-34) so knob configs round-trip between the two systems.  Fixes the
reference's bool-typed CategoricalKnob being inferred as ``int`` (SURVEY §7.4 bug (i)).

Each knob also knows how to map itself to/from the unit hypercube, which is what the advisors
(GP-EI / random search) optimise over.
"""
from __future__ import annotations

import abc
import json
import math


def _value_type(v):
    if isinstance(v, bool):  # bool before int: isinstance(True, int) is True
        return bool
    if isinstance(v, int):
        return int
    if isinstance(v, float):
        return float
    if isinstance(v, str):
        return str
    raise TypeError('Only the following types are supported: `int`, `float`, `bool`, `str`')


class BaseKnob(abc.ABC):
    def __init__(self, knob_args=None):
        self._knob_args = dict(knob_args or {})

    def to_json(self):
        return json.dumps({'type': self.__class__.__name__, 'args': self._knob_args})

    @classmethod
    def from_json(cls, json_str):
        d = json.loads(json_str)
        if 'type' not in d or 'args' not in d:
            raise ValueError('Invalid JSON representation of knob: {}.'.format(json_str))
        for clazz in (CategoricalKnob, IntegerKnob, FloatKnob, FixedKnob):
            if clazz.__name__ == d['type']:
                return clazz(**d['args'])
        raise ValueError('Invalid knob type: {}'.format(d['type']))

    # --- unit-cube encoding used by the advisors ---
    @property
    def dims(self) -> int:
        return 1

    @abc.abstractmethod
    def encode(self, value) -> list:
        ...

    @abc.abstractmethod
    def decode(self, u: list):
        ...

    def __eq__(self, other):
        return type(self) is type(other) and self._knob_args == other._knob_args

    def __repr__(self):
        return '{}({})'.format(self.__class__.__name__, self._knob_args)


class CategoricalKnob(BaseKnob):
    """A value from ``values`` (all of one type: int, float, bool or str)."""

    def __init__(self, values):
        super().__init__({'values': values})
        if len(values) == 0:
            raise ValueError('Length of `values` should at least 1')
        self._values = list(values)
        self._value_type = _value_type(values[0])
        if any(_value_type(x) is not self._value_type for x in values):
            raise TypeError('`values` should have elements of the same type')

    value_type = property(lambda self: self._value_type)
    values = property(lambda self: self._values)

    @property
    def dims(self):
        return len(self._values)

    def encode(self, value):  # one-hot
        return [1.0 if v == value else 0.0 for v in self._values]

    def decode(self, u):
        best = max(range(len(self._values)), key=lambda i: u[i])
        return self._values[best]


class FixedKnob(BaseKnob):
    """A single fixed value (needs no tuning)."""

    def __init__(self, value):
        super().__init__({'value': value})
        self._value = value
        self._value_type = _value_type(value)

    value_type = property(lambda self: self._value_type)
    value = property(lambda self: self._value)

    @property
    def dims(self):
        return 0

    def encode(self, value):
        return []

    def decode(self, u):
        return self._value


class _RangeKnob(BaseKnob):
    def __init__(self, value_min, value_max, is_exp=False):
        super().__init__({'value_min': value_min, 'value_max': value_max, 'is_exp': is_exp})
        self._validate(value_min, value_max)
        if is_exp and value_min <= 0:
            raise ValueError('`is_exp` knobs need `value_min` > 0')
        self._value_min, self._value_max, self._is_exp = value_min, value_max, bool(is_exp)

    value_min = property(lambda self: self._value_min)
    value_max = property(lambda self: self._value_max)
    is_exp = property(lambda self: self._is_exp)

    def _fwd(self, v):
        return math.log(v) if self._is_exp else float(v)

    def encode(self, value):
        lo, hi = self._fwd(self._value_min), self._fwd(self._value_max)
        if hi == lo:
            return [0.5]
        return [min(1.0, max(0.0, (self._fwd(value) - lo) / (hi - lo)))]

    def _raw(self, u):
        lo, hi = self._fwd(self._value_min), self._fwd(self._value_max)
        x = lo + min(1.0, max(0.0, float(u[0]))) * (hi - lo)
        return math.exp(x) if self._is_exp else x


class IntegerKnob(_RangeKnob):
    """Any int in [value_min, value_max]; ``is_exp`` samples on a log scale."""

    @staticmethod
    def _validate(value_min, value_max):
        if not isinstance(value_min, int) or isinstance(value_min, bool):
            raise ValueError('`value_min` should be an `int`')
        if not isinstance(value_max, int) or isinstance(value_max, bool):
            raise ValueError('`value_max` should be an `int`')
        if value_min > value_max:
            raise ValueError('`value_max` should be at least `value_min`')

    def decode(self, u):
        return int(min(self._value_max, max(self._value_min, round(self._raw(u)))))


class FloatKnob(_RangeKnob):
    """Any float in [value_min, value_max]; ``is_exp`` samples on a log scale."""

    @staticmethod
    def _validate(value_min, value_max):
        for n, v in (('value_min', value_min), ('value_max', value_max)):
            if not isinstance(v, (int, float)) or isinstance(v, bool):
                raise ValueError('`{}` should be a `float` or `int`'.format(n))
        if value_min > value_max:
            raise ValueError('`value_max` should be at least `value_min`')

    def decode(self, u):
        return float(min(self._value_max, max(self._value_min, self._raw(u))))


def serialize_knob_config(knob_config):
    return json.dumps({name: knob.to_json() for (name, knob) in knob_config.items()})


def deserialize_knob_config(knob_config_str):
    return {name: BaseKnob.from_json(s) for (name, s) in json.loads(knob_config_str).items()}


def knob_space_dims(knob_config) -> int:
    return sum(k.dims for k in knob_config.values())


def encode_knobs(knob_config, knobs) -> list:
    out = []
    for name in sorted(knob_config):
        out.extend(knob_config[name].encode(knobs[name]))
    return out


def decode_knobs(knob_config, u) -> dict:
    knobs, i = {}, 0
    for name in sorted(knob_config):
        k = knob_config[name]
        knobs[name] = k.decode(list(u[i:i + k.dims]))
        i += k.dims
    return knobs
