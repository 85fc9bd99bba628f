"""BaseModel contract + local validation harness + dynamic model loading.

Reference parity: rafiki/model/model.py — ``BaseModel`` (:20-127), ``test_model_class``
(:129-219), ``load_model_class`` (:221-242), ``parse_model_install_command`` (:244-273).

Differences (MI355X node, no network):
  * ``load_model_class`` imports the uploaded source from an in-memory module (no temp file in
    the CWD) and aliases ``rafiki.*`` imports so reference-style model files load unchanged;
  * ``parse_model_install_command`` only emits commands for packages that are NOT importable
    already (there is no package index on the target) — workers run it under an allow-list.
"""
from __future__ import annotations

import abc
import importlib.util
import inspect
import json
import pickle
import sys
import types
import uuid

from ..constants import ModelDependency, TaskType
from .knob import BaseKnob, deserialize_knob_config, serialize_knob_config


class InvalidModelClassException(Exception):
    pass


class InvalidModelParamsException(Exception):
    pass


class BaseModel(abc.ABC):
    """Models implement train/evaluate/predict/dump_parameters/load_parameters/destroy plus the
    static ``get_knob_config()``; ``__init__(**knobs)`` receives one proposal from the advisor."""

    def __init__(self, **knobs):
        pass

    @staticmethod
    def get_knob_config():
        raise NotImplementedError()

    @abc.abstractmethod
    def train(self, dataset_uri):
        raise NotImplementedError()

    @abc.abstractmethod
    def evaluate(self, dataset_uri):
        """-> accuracy-like float in [0, 1] (higher is better)."""
        raise NotImplementedError()

    @abc.abstractmethod
    def predict(self, queries):
        """-> list of JSON-serialisable predictions, one per query."""
        raise NotImplementedError()

    @abc.abstractmethod
    def dump_parameters(self):
        """-> picklable dict that fully defines the trained state."""
        raise NotImplementedError()

    @abc.abstractmethod
    def load_parameters(self, params):
        raise NotImplementedError()

    def destroy(self):
        pass


# ------------------------------------------------------------------------------ dynamic loading
def _install_rafiki_alias():
    """Make ``import rafiki...`` resolve to this package for reference-style model files."""
    try:
        import rafiki  # noqa: F401  (the in-repo alias package)
    except Exception:
        pass


def load_model_class(model_file_bytes, model_class, temp_mod_name=None):
    _install_rafiki_alias()
    if isinstance(model_file_bytes, str):
        model_file_bytes = model_file_bytes.encode('utf-8')
    name = temp_mod_name or 'rafiki_user_model_{}'.format(uuid.uuid4().hex)
    mod = types.ModuleType(name)
    mod.__file__ = '<{}>'.format(name)
    sys.modules[name] = mod
    try:
        exec(compile(model_file_bytes, mod.__file__, 'exec'), mod.__dict__)
    except Exception:
        sys.modules.pop(name, None)
        raise
    if not hasattr(mod, model_class):
        raise InvalidModelClassException('Model class "{}" not found in model file'.format(model_class))
    return getattr(mod, model_class)


def load_model_class_from_file(path, model_class):
    with open(path, 'rb') as f:
        return load_model_class(f.read(), model_class)


_PIP_NAMES = {ModelDependency.SCIKIT_LEARN: 'sklearn', ModelDependency.PYTORCH: 'torch',
              ModelDependency.TENSORFLOW: 'tensorflow', ModelDependency.KERAS: 'keras',
              ModelDependency.SINGA: 'singa'}


def _importable(dep):
    mod = _PIP_NAMES.get(dep, dep)
    return importlib.util.find_spec(mod) is not None


def parse_model_install_command(dependencies, enable_gpu=False):
    """``{dep: version}`` -> shell command installing the missing ones ('' when all present)."""
    cmds = []
    for dep, ver in (dependencies or {}).items():
        if _importable(dep):
            continue
        if dep == ModelDependency.SINGA:
            cmds.append('conda install -y -c nusdbsystem singa={}'.format(ver))
        else:
            cmds.append('pip install {}=={}'.format(dep, ver))
    return '; '.join(cmds)


def _check_dependencies(dependencies):
    missing = [d for d in (dependencies or {}) if not _importable(d)]
    if missing:
        print('Missing model dependencies (install before training): {}'.format(', '.join(missing)))
    return missing


# ------------------------------------------------------------------------------------ validation
def _check_model_class(clazz):
    if not issubclass(clazz, BaseModel):
        raise InvalidModelClassException('Model should extend `rafiki_amd.model.BaseModel`')
    if inspect.isfunction(getattr(clazz, 'get_knob_config', None)) is False:
        raise InvalidModelClassException('`get_knob_config` should be a static method')


def _check_knob_config(knob_config):
    if not isinstance(knob_config, dict) or any(not isinstance(n, str) or not isinstance(k, BaseKnob)
                                                for n, k in knob_config.items()):
        raise InvalidModelClassException('`get_knob_config()` should return a dict[str, BaseKnob]')
    again = deserialize_knob_config(serialize_knob_config(knob_config))
    if again != knob_config:
        raise InvalidModelClassException('knob config does not survive JSON serialisation')


def test_model_class(model_file_path, model_class, task, dependencies, train_dataset_uri, test_dataset_uri,
                     queries=(), knobs=None, advisor_type=None):
    """Run the full train -> evaluate -> dump -> load -> predict -> ensemble flow locally."""
    from ..advisor import make_advisor
    from ..predictor.ensemble import ensemble_predictions

    _check_dependencies(dependencies)
    with open(model_file_path, 'rb') as f:
        clazz = load_model_class(f.read(), model_class)
    _check_model_class(clazz)
    knob_config = clazz.get_knob_config()
    _check_knob_config(knob_config)
    if knobs is None:
        knobs = make_advisor(knob_config, advisor_type).propose()
    print('Using knobs: {}'.format(knobs))
    model = clazz(**knobs)
    model.train(train_dataset_uri)
    score = model.evaluate(test_dataset_uri)
    if not isinstance(score, float):
        raise InvalidModelClassException('`evaluate()` should return a float, got {!r}'.format(score))
    print('Score: {}'.format(score))
    params = model.dump_parameters()
    try:
        blob = pickle.dumps(params)
        params = pickle.loads(blob)
    except Exception as e:
        raise InvalidModelParamsException('`dump_parameters()` output must be picklable: {}'.format(e))
    model.destroy()
    model = clazz(**knobs)
    model.load_parameters(params)
    predictions = model.predict(list(queries))
    try:
        json.dumps(predictions)
    except Exception as e:
        raise InvalidModelClassException('`predict()` output must be JSON serialisable: {}'.format(e))
    predictions = ensemble_predictions([predictions], task)
    model.destroy()
    print('Predictions: {}'.format(predictions))
    return predictions, score, knobs


__all__ = ['BaseModel', 'InvalidModelClassException', 'InvalidModelParamsException', 'load_model_class',
           'load_model_class_from_file', 'parse_model_install_command', 'test_model_class', 'TaskType']
