"""rafiki_amd — an MI355X-native AutoML train-and-serve framework with Rafiki's capabilities.

Layers (see SURVEY.md §1 for the reference's layer map):
  client / admin / predictor  REST + SDK (wire-compatible with rafiki.client)
  advisor                     GP-EI Bayesian optimisation + random search, batch proposals
  worker / parallel           trial-parallel HPO over RCCL (one process per GPU), DP grad buckets
  model / models              BaseModel SDK + model zoo (VGG-small, MLP, PG-GAN, BiLSTM, sklearn, HMM)
  engine / ops                static-graph training engine + hand-written gfx950 HIP kernels
  db / cache / container      SQLite store, in-process queues, local GPU process manager
"""
import os as _os

# ProcessGroupNCCL's CUDA-event cache recycles a work's events into later works; an event recorded
# while a stream was being captured into a hipGraph (the PG-GAN data-parallel rounds) must never be
# handed to an eager work the watchdog polls.  Fresh events per work (a few us) sidestep that.
_os.environ.setdefault('TORCH_NCCL_CUDA_EVENT_CACHE', '0')

__version__ = "0.1.0"
