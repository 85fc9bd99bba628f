"""Import-compatibility alias: ``import rafiki.model`` / ``from rafiki.client import Client`` resolve
to ``rafiki_amd`` so model files and scripts written against the reference SDK run unchanged.

Submodules are aliased lazily (a meta-path finder + module ``__getattr__``): importing ``rafiki``
itself costs nothing, and a model file's ``from rafiki.model import BaseModel`` loads only
``rafiki_amd.model`` — not the HTTP client stack — so trial start-up stays fast.
"""
import importlib
import importlib.abc
import importlib.util
import sys


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target):
        self.target = target

    def create_module(self, spec):
        mod = importlib.import_module(self.target)
        self._spec = mod.__spec__
        return mod

    def exec_module(self, module):
        module.__spec__ = self._spec   # the import system re-labels it with the alias spec; undo


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(__name__ + '.'):
            return None
        real = 'rafiki_amd.' + fullname[len(__name__) + 1:]
        if importlib.util.find_spec(real) is None:
            return None
        return importlib.util.spec_from_loader(fullname, _AliasLoader(real))


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())


def __getattr__(name):
    try:
        return importlib.import_module(__name__ + '.' + name)
    except ImportError as e:
        raise AttributeError(name) from e
