"""POS-tagging flow (reference examples/scripts/tasks/run_pos_tagging.py:13-65): upload the BigramHmm
and PyBiLstm models, train on a CORPUS dataset (synthetic unless --train/--test), deploy, predict."""
import argparse
import os
import sys
import time
import uuid

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from rafiki_amd.client import Client  # noqa: E402
from rafiki_amd.config import SUPERADMIN_EMAIL, SUPERADMIN_PASSWORD  # noqa: E402
from rafiki_amd.constants import TaskType  # noqa: E402
from rafiki_amd.model.dataset import synthetic_corpus, write_corpus_zip  # noqa: E402
from rafiki_amd.models import model_file  # noqa: E402

if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--host', default='127.0.0.1')
    ap.add_argument('--port', type=int, default=3000)
    ap.add_argument('--train', default=None)
    ap.add_argument('--test', default=None)
    a = ap.parse_args()
    os.makedirs('data', exist_ok=True)
    train = a.train or write_corpus_zip('data/pos_train.zip', synthetic_corpus(400, seed=0))
    test = a.test or write_corpus_zip('data/pos_test.zip', synthetic_corpus(100, seed=1))
    c = Client(admin_host=a.host, admin_port=a.port)
    c.login(SUPERADMIN_EMAIL, SUPERADMIN_PASSWORD)
    sfx = uuid.uuid4().hex[:6]
    ms = [c.create_model(n + '_' + sfx, TaskType.POS_TAGGING, model_file(n), n) for n in ('BigramHmm', 'PyBiLstm')]
    app = 'pos_tagging_' + sfx
    c.create_train_job(app, TaskType.POS_TAGGING, train, test, {'MODEL_TRIAL_COUNT': 2},
                       models=[m['id'] for m in ms])
    while c.get_train_job(app)['status'] not in ('STOPPED', 'ERRORED'):
        time.sleep(2)
    print(c.get_best_trials_of_train_job(app))
    ij = c.create_inference_job(app)
    print(c.predict(ij['predictor_host'], ['w1', 'w2', 'w3']))
    c.stop_inference_job(app)
