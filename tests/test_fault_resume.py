"""Failure paths: injected trial errors, a worker crash mid-trial, restart and
resume from the epoch checkpoint under the same trial id; heartbeat staleness detection."""
import os
import time

import pytest

from rafiki_amd.constants import TrialStatus
from rafiki_amd.models import model_file
from rafiki_amd.utils import faults

DATA = 'synthetic://image?n=256&size=8&channels=1&classes=3&seed=0'
TEST = 'synthetic://image?n=64&size=8&channels=1&classes=3&seed=1'


def _setup(tmp_path, budget):
    from rafiki_amd.db.database import Database
    from rafiki_amd.utils.auth import hash_password
    db = Database(str(tmp_path / 'db.sqlite3'))
    u = db.create_user('u@x', hash_password('p'), 'ADMIN')
    with open(model_file('FeedForward'), 'rb') as f:
        m = db.create_model(u.id, 'ff', 'IMAGE_CLASSIFICATION', f.read(), 'FeedForward', 'img', {}, 'PRIVATE')
    tj = db.create_train_job(u.id, 'app', 1, 'IMAGE_CLASSIFICATION', budget, DATA, TEST)
    sub = db.create_sub_train_job(tj.id, m.id, u.id)
    svc = db.create_service('TRAIN', 'test', 'img', 1, 0)
    db.create_train_job_worker(svc.id, sub.id)
    return db, svc.id, sub.id


@pytest.fixture(autouse=True)
def _cpu(monkeypatch, tmp_path):
    monkeypatch.setenv('RAFIKI_CPU_ONLY', '1')
    monkeypatch.setenv('WORKDIR_PATH', str(tmp_path))
    faults.reset()
    yield
    faults.reset()


def test_injected_trial_error_is_contained(tmp_path, monkeypatch):
    from rafiki_amd.worker.train import TrainWorker
    db, sid, sub_id = _setup(tmp_path, {'MODEL_TRIAL_COUNT': 3})
    monkeypatch.setenv('RAFIKI_FAULT_INJECT', 'train_step:step=2')
    w = TrainWorker(sid, 'w0', db=db, seed=0, params_dir=str(tmp_path / 'params'))
    w.start()
    trials = db.get_trials_of_sub_train_job(sub_id)
    st = sorted(t.status for t in trials)
    assert st == [TrialStatus.COMPLETED, TrialStatus.COMPLETED, TrialStatus.ERRORED], st
    assert db.get_sub_train_job(sub_id).datetime_stopped is not None


def test_crash_then_resume_from_checkpoint(tmp_path, monkeypatch):
    from rafiki_amd.worker.train import TrainWorker
    db, sid, sub_id = _setup(tmp_path, {'MODEL_TRIAL_COUNT': 1})
    params = str(tmp_path / 'params')
    monkeypatch.setenv('RAFIKI_FAULT_INJECT', 'crash:epoch=0')
    w = TrainWorker(sid, 'w0', db=db, seed=0, params_dir=params)
    # FeedForward runs 2 epochs (FixedKnob, the reference's); the crash fires right after epoch 0's checkpoint
    with pytest.raises(faults.WorkerCrash):
        w.start()
    (trial,) = db.get_trials_of_sub_train_job(sub_id)
    assert trial.status == TrialStatus.RUNNING
    assert os.path.exists(os.path.join(params, trial.id + '.ckpt'))
    # "restarted" worker: same service / worker id, no fault this time
    monkeypatch.setenv('RAFIKI_FAULT_INJECT', '')
    faults.reset()
    w2 = TrainWorker(sid, 'w0', db=db, seed=0, params_dir=params)
    w2.start()
    (t2,) = db.get_trials_of_sub_train_job(sub_id)
    assert t2.id == trial.id and t2.status == TrialStatus.COMPLETED
    assert not os.path.exists(os.path.join(params, trial.id + '.ckpt'))
    assert os.path.exists(t2.params_file_path)
    logs = [l.line if hasattr(l, 'line') else l for l in db.get_trial_logs(trial.id)]
    assert any('resumed from checkpoint after epoch 0' in str(x) for x in logs)


def test_heartbeat_staleness(tmp_path):
    from rafiki_amd.container.container_manager import LocalProcessManager
    from rafiki_amd.utils.service import heartbeat_path
    m = LocalProcessManager()
    m.heartbeat_timeout = 5.0
    svc = {'env': {'WORKDIR_PATH': str(tmp_path), 'RAFIKI_SERVICE_ID': 's1'}, 'world': 1,
           'started_at': time.time() - 100}
    assert m._stale(svc)  # never beat since start 100 s ago
    p = heartbeat_path(str(tmp_path), 's1', 0)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, 'w') as f:
        f.write(str(time.time()))
    assert not m._stale(svc)


def test_fault_rule_matching(monkeypatch):
    monkeypatch.setenv('RAFIKI_FAULT_INJECT', 'train_step:step=3,rank=1,times=2;nan_grad:step=0')
    faults.maybe_fail('train_step', step=5, rank=0)  # wrong rank: no fault
    with pytest.raises(faults.TrialFault):
        faults.maybe_fail('train_step', step=3, rank=1)
    with pytest.raises(faults.TrialFault):
        faults.maybe_fail('train_step', step=4, rank=1)
    faults.maybe_fail('train_step', step=9, rank=1)  # fired twice already
    import torch
    t = torch.zeros(3)
    assert faults.maybe_corrupt(t, step=0) and torch.isnan(t).all()
