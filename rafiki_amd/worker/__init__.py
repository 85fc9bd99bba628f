"""Workers (reference rafiki.worker): the trial-parallel TrainWorker group."""
from .train import TrainWorker  # noqa: F401
