"""Python SDK: every public method of the reference ``rafiki.client.Client`` (client.py:29-737).

Same method names, arguments, routes and return shapes; raises
``RafikiConnectionError`` on any non-200 response.  Extensions: ``predict``/``predict_batch``
against a running predictor, and ``create_inference_job(..., max_models=k)`` for top-k ensembles.
"""
from __future__ import annotations

import functools
import json
import os
import pickle
import warnings

import requests

from ..constants import ModelAccessRight


class RafikiConnectionError(ConnectionError):
    pass


def _removed(msg):
    """Method kept for API compatibility that only warns (reference client.py:14-27, 123-125, 278-284)."""
    def deco(func):
        @functools.wraps(func)
        def shim(*args, **kwargs):
            warnings.warn('{} (see docs/api.md)'.format(msg), DeprecationWarning, stacklevel=2)
            return None
        return shim
    return deco


class Client:
    def __init__(self, admin_host=os.environ.get('RAFIKI_ADDR', 'localhost'),
                 admin_port=os.environ.get('ADMIN_EXT_PORT', 3000),
                 advisor_host=os.environ.get('RAFIKI_ADDR', 'localhost'),
                 advisor_port=os.environ.get('ADVISOR_EXT_PORT', 3002), timeout=600):
        self._admin_host, self._admin_port = admin_host, admin_port
        self._advisor_host, self._advisor_port = advisor_host, advisor_port
        self._token = None
        self._user = None
        self._timeout = timeout
        self._session = requests.Session()

    # ------------------------------------------------------------------------------- users
    def login(self, email, password):
        data = self._post('/tokens', json={'email': email, 'password': password})
        self._token = data['token']
        self._user = {'id': data['user_id'], 'user_type': data['user_type']}
        return self._user

    def get_current_user(self):
        return self._user

    def logout(self):
        self._user = None
        self._token = None

    def create_user(self, email, password, user_type):
        return self._post('/users', json={'email': email, 'password': password, 'user_type': user_type})

    def get_users(self):
        return self._get('/users')

    def ban_user(self, email):
        return self._delete('/users', json={'email': email})

    @_removed('`create_users` has been removed; call `create_user` per user')
    def create_users(self, *args, **kwargs):
        pass

    # ------------------------------------------------------------------------------ models
    def create_model(self, name, task, model_file_path, model_class, dependencies=None,
                     access_right=ModelAccessRight.PRIVATE, docker_image=None):
        with open(model_file_path, 'rb') as f:
            blob = f.read()
        form = {'name': name, 'task': task, 'dependencies': json.dumps(dependencies or {}),
                'model_class': model_class, 'access_right': access_right}
        if docker_image:
            form['docker_image'] = docker_image
        return self._post('/models', files={'model_file_bytes': blob}, form_data=form)

    def get_model(self, model_id):
        return self._get('/models/{}'.format(model_id))

    def download_model_file(self, model_id, out_model_file_path):
        blob = self._get('/models/{}/model_file'.format(model_id))
        with open(out_model_file_path, 'wb') as f:
            f.write(blob)
        return self.get_model(model_id)

    def get_available_models(self, task=None):
        return self._get('/models/available', params={'task': task} if task else {})

    @_removed('`get_models` & `get_models_of_task` have been combined into `get_available_models`')
    def get_models(self, *args, **kwargs):
        pass

    @_removed('`get_models` & `get_models_of_task` have been combined into `get_available_models`')
    def get_models_of_task(self, *args, **kwargs):
        pass

    def delete_model(self, model_id):
        return self._delete('/models/{}'.format(model_id))

    # -------------------------------------------------------------------------- train jobs
    def create_train_job(self, app, task, train_dataset_uri, test_dataset_uri, budget, models=None):
        if models is None:
            models = [m['id'] for m in self.get_available_models(task)]
        return self._post('/train_jobs', json={'app': app, 'task': task, 'train_dataset_uri': train_dataset_uri,
                                               'test_dataset_uri': test_dataset_uri, 'budget': budget,
                                               'model_ids': models})

    def get_train_jobs_by_user(self, user_id):
        return self._get('/train_jobs', params={'user_id': user_id})

    def get_train_jobs_of_app(self, app):
        return self._get('/train_jobs/{}'.format(app))

    def get_train_job(self, app, app_version=-1):
        return self._get('/train_jobs/{}/{}'.format(app, app_version))

    def get_best_trials_of_train_job(self, app, app_version=-1, max_count=2):
        return self._get('/train_jobs/{}/{}/trials'.format(app, app_version),
                         params={'type': 'best', 'max_count': max_count})

    def get_trials_of_train_job(self, app, app_version=-1):
        return self._get('/train_jobs/{}/{}/trials'.format(app, app_version))

    def stop_train_job(self, app, app_version=-1):
        return self._post('/train_jobs/{}/{}/stop'.format(app, app_version))

    # ------------------------------------------------------------------------------ trials
    def get_trial(self, trial_id):
        return self._get('/trials/{}'.format(trial_id))

    def get_trial_logs(self, trial_id):
        return self._get('/trials/{}/logs'.format(trial_id))

    def get_trial_parameters(self, trial_id):
        """Unpickles the trial's saved params (trusted: written by this system's workers)."""
        return pickle.loads(self._get('/trials/{}/parameters'.format(trial_id)))

    def load_trial_model(self, trial_id, ModelClass):
        trial = self.get_trial(trial_id)
        params = self.get_trial_parameters(trial_id)
        model = ModelClass(**(trial.get('knobs') or {}))
        model.load_parameters(params)
        return model

    # ---------------------------------------------------------------------- inference jobs
    def create_inference_job(self, app, app_version=-1, max_models=None):
        body = {'app': app, 'app_version': app_version}
        if max_models is not None:
            body['max_models'] = int(max_models)
        return self._post('/inference_jobs', json=body)

    def get_inference_jobs_by_user(self, user_id):
        return self._get('/inference_jobs', params={'user_id': user_id})

    def get_inference_jobs_of_app(self, app):
        return self._get('/inference_jobs/{}'.format(app))

    def get_running_inference_job(self, app, app_version=-1):
        return self._get('/inference_jobs/{}/{}'.format(app, app_version))

    def stop_inference_job(self, app, app_version=-1):
        return self._post('/inference_jobs/{}/{}/stop'.format(app, app_version))

    # ---------------------------------------------------------------------------- predictor
    def predict(self, predictor_host, query):
        r = self._session.post('http://{}/predict'.format(predictor_host), json={'query': query},
                               timeout=self._timeout)
        return self._parse_response(r)['prediction']

    def predict_batch(self, predictor_host, queries):
        r = self._session.post('http://{}/predict_batch'.format(predictor_host), json={'queries': queries},
                               timeout=self._timeout)
        return self._parse_response(r)['predictions']

    def predict_array(self, predictor_host, array):
        """Binary batch prediction: a numpy batch in, a float32 numpy [Q, classes] out
        (``POST /predict_batch_npy``; no JSON for the pixels)."""
        import io
        import numpy as np
        buf = io.BytesIO()
        np.save(buf, np.asarray(array), allow_pickle=False)
        r = self._session.post('http://{}/predict_batch_npy'.format(predictor_host), data=buf.getvalue(),
                               headers={'Content-Type': 'application/octet-stream'}, timeout=self._timeout)
        if r.status_code != 200:
            raise RafikiConnectionError(r.text)
        return np.load(io.BytesIO(r.content), allow_pickle=False)

    # ----------------------------------------------------------------------------- advisors
    def _create_advisor(self, knob_config_str, advisor_id=None):
        return self._post('/advisors', target='advisor',
                          json={'knob_config_str': knob_config_str, 'advisor_id': advisor_id})

    def _generate_proposal(self, advisor_id):
        return self._post('/advisors/{}/propose'.format(advisor_id), target='advisor')

    def _feedback_to_advisor(self, advisor_id, knobs, score):
        return self._post('/advisors/{}/feedback'.format(advisor_id), target='advisor',
                          json={'score': score, 'knobs': knobs})

    def _delete_advisor(self, advisor_id):
        return self._delete('/advisors/{}'.format(advisor_id), target='advisor')

    # ------------------------------------------------------------------------------ admin
    def stop_all_jobs(self):
        return self._post('/actions/stop_all_jobs')

    def send_event(self, name, **params):
        return self._post('/event/{}'.format(name), json=params)

    # ---------------------------------------------------------------------------- plumbing
    def _get(self, path, params=None, target='admin'):
        r = self._session.get(self._make_url(path, target), headers=self._headers(), params=params or {},
                              timeout=self._timeout)
        return self._parse_response(r)

    def _post(self, path, params=None, files=None, form_data=None, json=None, target='admin'):
        r = self._session.post(self._make_url(path, target), headers=self._headers(), params=params or {},
                               files=files or None, data=form_data, json=json, timeout=self._timeout)
        return self._parse_response(r)

    def _delete(self, path, params=None, files=None, form_data=None, json=None, target='admin'):
        r = self._session.delete(self._make_url(path, target), headers=self._headers(), params=params or {},
                                 files=files or None, data=form_data, json=json, timeout=self._timeout)
        return self._parse_response(r)

    def _make_url(self, path, target='admin'):
        if target == 'admin':
            return 'http://{}:{}{}'.format(self._admin_host, self._admin_port, path)
        if target == 'advisor':
            return 'http://{}:{}{}'.format(self._advisor_host, self._advisor_port, path)
        raise ValueError('invalid target {}'.format(target))

    def _headers(self):
        return {'Authorization': 'Bearer ' + self._token} if self._token else {}

    @staticmethod
    def _parse_response(res):
        if res.status_code != 200:
            raise RafikiConnectionError(res.text)
        ctype = res.headers.get('content-type', '')
        if ctype.startswith('application/json'):
            return res.json()
        if ctype.startswith('application/octet-stream'):
            return res.content
        raise RafikiConnectionError('Invalid response content type: {}'.format(ctype))
