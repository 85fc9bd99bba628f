"""Quickstart: the reference's end-to-end flow (examples/scripts/quickstart.py:68-146) against a
running admin (scripts/start.sh): create users, upload models, train, inspect trials, deploy the
best trials and make predictions.  Uses synthetic Fashion-MNIST-shaped data unless --train/--test
point at IMAGE_FILES zips (examples/datasets/image_classification/load_mnist_format.py).

usage: python examples/scripts/quickstart.py [--host 127.0.0.1] [--port 3000] [--gpus 0]
"""
import argparse
import os
import sys
import time
import uuid

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path.insert(0, ROOT)

from rafiki_amd.client import Client  # noqa: E402
from rafiki_amd.config import SUPERADMIN_EMAIL, SUPERADMIN_PASSWORD  # noqa: E402
from rafiki_amd.constants import BudgetType, TaskType, UserType  # noqa: E402
from rafiki_amd.model.dataset import synthetic_images, write_image_files_zip  # noqa: E402
from rafiki_amd.models import model_file  # noqa: E402


def make_data(d):
    imgs, labels = synthetic_images(3000, size=28, channels=1, classes=10, seed=0)
    tr = write_image_files_zip(os.path.join(d, 'train.zip'), imgs[:2500], labels[:2500])
    te = write_image_files_zip(os.path.join(d, 'test.zip'), imgs[2500:], labels[2500:])
    return tr, te


def wait_until_train_job_has_stopped(client, app, timeout=3600):
    t0 = time.time()
    while time.time() - t0 < timeout:
        tj = client.get_train_job(app)
        if tj['status'] in ('STOPPED', 'ERRORED'):
            return tj
        time.sleep(2)
    raise TimeoutError(app)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--host', default='127.0.0.1')
    ap.add_argument('--port', type=int, default=3000)
    ap.add_argument('--gpus', type=int, default=0)
    ap.add_argument('--trials', type=int, default=4)
    ap.add_argument('--train', default=None)
    ap.add_argument('--test', default=None)
    ap.add_argument('--data_dir', default='data')
    a = ap.parse_args()
    os.makedirs(a.data_dir, exist_ok=True)
    train, test = (a.train, a.test) if a.train else make_data(a.data_dir)

    admin = Client(admin_host=a.host, admin_port=a.port)
    admin.login(SUPERADMIN_EMAIL, SUPERADMIN_PASSWORD)
    suffix = uuid.uuid4().hex[:6]
    dev_email, app_email = 'model_developer_{}@rafiki'.format(suffix), 'app_developer_{}@rafiki'.format(suffix)
    admin.create_user(dev_email, 'rafiki', UserType.MODEL_DEVELOPER)
    admin.create_user(app_email, 'rafiki', UserType.APP_DEVELOPER)

    dev = Client(admin_host=a.host, admin_port=a.port)
    dev.login(dev_email, 'rafiki')
    models = [dev.create_model('FeedForward_' + suffix, TaskType.IMAGE_CLASSIFICATION, model_file('FeedForward'),
                               'FeedForward', access_right='PUBLIC'),
              dev.create_model('SkDt_' + suffix, TaskType.IMAGE_CLASSIFICATION, model_file('SkDt'), 'SkDt',
                               access_right='PUBLIC')]
    print('models:', [m['name'] for m in models])

    app_c = Client(admin_host=a.host, admin_port=a.port)
    app_c.login(app_email, 'rafiki')
    app = 'fashion_mnist_app_' + suffix
    tj = app_c.create_train_job(app, TaskType.IMAGE_CLASSIFICATION, train, test,
                                {BudgetType.MODEL_TRIAL_COUNT: a.trials, BudgetType.GPU_COUNT: a.gpus},
                                models=[m['id'] for m in models])
    print('train job:', tj)
    tj = wait_until_train_job_has_stopped(app_c, app)
    print('train job finished:', tj['status'])
    for t in app_c.get_best_trials_of_train_job(app):
        print('best trial {} {} score={:.4f}'.format(t['id'][:8], t['model_name'], t['score']))
    ij = app_c.create_inference_job(app)
    print('inference job:', ij)
    imgs, labels = synthetic_images(5, size=28, channels=1, classes=10, seed=7)
    for img, lab in zip(imgs, labels):
        pred = app_c.predict(ij['predictor_host'], img.tolist())
        print('label {} -> predicted {} (p={:.3f})'.format(lab, max(range(len(pred)), key=pred.__getitem__),
                                                            max(pred)))
    app_c.stop_inference_job(app)


if __name__ == '__main__':
    main()
