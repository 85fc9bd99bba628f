"""gfx950 kernel bindings: ``functional`` (raw tensor ops) and ``autograd`` (differentiable ops)."""
from . import _lib  # noqa: F401
