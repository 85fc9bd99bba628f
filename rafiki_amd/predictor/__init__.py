"""Predictor: batched top-k ensemble serving (reference rafiki.predictor)."""
from .ensemble import ensemble_predictions, ensemble_probabilities  # noqa: F401
from .predictor import ParamCache, Predictor  # noqa: F401
