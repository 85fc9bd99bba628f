"""Import-compatibility alias: ``import rafiki.model`` / ``from rafiki.client import Client`` resolve
to ``rafiki_amd`` so model files and scripts written against the reference SDK run unchanged."""
import importlib
import sys

_SUBMODULES = ['constants', 'config', 'model', 'advisor', 'client', 'predictor', 'db', 'admin', 'container',
               'worker', 'utils', 'parallel', 'engine', 'ops', 'models']

for _name in _SUBMODULES:
    try:
        _mod = importlib.import_module('rafiki_amd.' + _name)
    except Exception:  # pragma: no cover - optional heavy deps
        continue
    sys.modules['rafiki.' + _name] = _mod
    globals()[_name] = _mod
