"""Mid-trial checkpoints: ``<params_dir>/<trial_id>.ckpt``.

The reference only pickles parameters at trial end, so a killed worker loses the trial.  Models
that support resuming call ``ctx.checkpoint.save(state, epoch)`` at epoch boundaries (atomic
rename) and ``ctx.checkpoint.load()`` at the start of ``train``; a restarted worker re-runs the
trial's knobs under the same trial id and the model continues from the last saved epoch.  The
file is deleted when the trial completes (its final params go to ``<trial_id>.model`` as before).
"""
from __future__ import annotations

import os
import pickle
import time
from typing import Optional


class TrialCheckpoint:
    def __init__(self, params_dir: str, trial_id: str, every_epochs: int = 1):
        self.path = os.path.join(params_dir, '{}.ckpt'.format(trial_id))
        self.every = max(1, int(every_epochs))
        self.resumed_from: Optional[int] = None

    def due(self, epoch: int) -> bool:
        return (epoch + 1) % self.every == 0

    def save(self, state: dict, epoch: int):
        tmp = self.path + '.tmp'
        with open(tmp, 'wb') as f:
            pickle.dump({'epoch': int(epoch), 'time': time.time(), 'state': state}, f,
                        protocol=pickle.HIGHEST_PROTOCOL)
        os.replace(tmp, self.path)

    def load(self) -> Optional[dict]:
        """-> {'epoch': last completed epoch, 'state': ...} or None.  Only files this framework
        wrote itself are ever unpickled (params dir of the worker)."""
        if not os.path.exists(self.path):
            return None
        with open(self.path, 'rb') as f:
            d = pickle.load(f)
        self.resumed_from = int(d['epoch'])
        return d

    def exists(self) -> bool:
        return os.path.exists(self.path)

    def remove(self):
        try:
            os.remove(self.path)
        except OSError:
            pass
