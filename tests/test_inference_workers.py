"""``workers`` serving mode: InferenceWorker processes behind shared-memory queues (the reference's
Redis-based InferenceWorker/Predictor design), CPU, 2 processes."""
import os
import pickle
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from rafiki_amd.models import model_file

DATA = 'synthetic://image?n=300&size=8&channels=1&classes=3&seed=0'


def _worker_main(service_id, db_path, workdir):
    os.environ.update({'RAFIKI_CPU_ONLY': '1', 'WORKDIR_PATH': workdir})
    from rafiki_amd.cache import Cache
    from rafiki_amd.db.database import Database
    from rafiki_amd.worker.inference import InferenceWorker
    InferenceWorker(service_id, db=Database(db_path), cache=Cache(workdir)).start()


def _train(name, knobs, params_dir, db, sub, model, u):
    from rafiki_amd.model.model import load_model_class
    clazz = load_model_class(open(model_file(name), 'rb').read(), name)
    inst = clazz(**knobs)
    inst.train(DATA)
    t = db.create_trial(sub.id, model.id, 'w')
    db.mark_trial_as_running(t, knobs)
    path = os.path.join(params_dir, t.id + '.model')
    with open(path, 'wb') as f:
        f.write(pickle.dumps(inst.dump_parameters()))
    db.mark_trial_as_complete(t, 0.5, path)
    return t, inst


def test_inference_workers_fan_out(tmp_path, monkeypatch):
    monkeypatch.setenv('RAFIKI_CPU_ONLY', '1')
    monkeypatch.setenv('WORKDIR_PATH', str(tmp_path))
    from rafiki_amd.cache import Cache
    from rafiki_amd.db.database import Database
    from rafiki_amd.model.dataset import synthetic_images
    from rafiki_amd.predictor.predictor import Predictor
    from rafiki_amd.utils.auth import hash_password
    db_path = str(tmp_path / 'db.sqlite3')
    db = Database(db_path)
    u = db.create_user('u@x', hash_password('p'), 'ADMIN')
    tj = db.create_train_job(u.id, 'app', 1, 'IMAGE_CLASSIFICATION', {}, DATA, DATA)
    trials = []
    for name, knobs in (('SkDt', {'max_depth': 4, 'criterion': 'gini'}),
                        ('FeedForward', {'epochs': 1, 'hidden_layer_count': 1, 'hidden_layer_units': 16,
                                         'learning_rate': 0.01, 'batch_size': 32, 'image_size': 8})):
        m = db.create_model(u.id, name, 'IMAGE_CLASSIFICATION', open(model_file(name), 'rb').read(), name, 'img',
                            {}, 'PRIVATE')
        sub = db.create_sub_train_job(tj.id, m.id, u.id)
        trials.append(_train(name, knobs, str(tmp_path), db, sub, m, u))
    ij = db.create_inference_job(u.id, tj.id)
    svc_ids = []
    for t, _ in trials:
        svc = db.create_service('INFERENCE', 'test', 'img', 1, 0)
        db.create_inference_job_worker(svc.id, ij.id, t.id)
        svc_ids.append(svc.id)
    ctx = mp.get_context('spawn')
    procs = [ctx.Process(target=_worker_main, args=(sid, db_path, str(tmp_path)), daemon=True) for sid in svc_ids]
    for p in procs:
        p.start()
    cache = Cache(str(tmp_path))
    try:
        t0 = time.time()
        while len(cache.get_workers_of_inference_job(ij.id)) < 2 and time.time() - t0 < 120:
            time.sleep(0.2)
        assert sorted(cache.get_workers_of_inference_job(ij.id)) == sorted(svc_ids)
        pred = Predictor.from_inference_workers(ij.id, db=db, cache=cache, timeout_s=60)
        imgs, _ = synthetic_images(10, size=8, channels=1, classes=3, seed=5)
        q = imgs.tolist()
        got = np.asarray(pred.predict(q))
        want = np.mean([np.asarray(inst.predict(q)) for _, inst in trials], axis=0)
        assert got.shape == want.shape and np.allclose(got, want, atol=1e-4)
        # a dead worker is dropped from the ensemble after the timeout (partial-ensemble fallback)
        procs[1].terminate()
        procs[1].join(10)
        pred.timeout_s = 2.0
        got2 = np.asarray(pred.predict(q))
        assert np.allclose(got2, np.asarray(trials[0][1].predict(q)), atol=1e-4)
        assert pred.stats['errors'] >= 1
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(10)
        for sid in svc_ids:
            cache.clear_worker(sid)
