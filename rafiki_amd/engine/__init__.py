"""Static-graph training engines (flat parameter arena, fused optimizers, hipGraph capture)."""
from .flat import FlatAdam, FlatParams, FlatSGD  # noqa: F401
