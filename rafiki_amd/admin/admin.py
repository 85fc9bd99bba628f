"""Admin: users, models, train/inference jobs, trials, events — returns JSON-able dicts.

Reference parity: rafiki/admin/admin.py (``Admin`` :29-674; method-by-method the same public
surface and response shapes).  Storage is the SQLite DAL, services run through the
node-local ``ServicesManager``.  Fixes reference bug (c) (None checks after dereference).
"""
from __future__ import annotations

import logging
import os

from .. import config
from ..constants import (BudgetType, InferenceJobStatus, ModelAccessRight, ServiceStatus, TrainJobStatus,
                         UserType)
from ..db.database import Database
from ..model.log import ModelLogger
from ..utils.auth import check_password, hash_password
from .services_manager import WORKER_IMAGE, ServicesManager

logger = logging.getLogger(__name__)


class UserExistsError(Exception):
    pass


class UserAlreadyBannedError(Exception):
    pass


class InvalidUserError(Exception):
    pass


class InvalidPasswordError(Exception):
    pass


class InvalidRunningInferenceJobError(Exception):
    pass


class InvalidModelError(Exception):
    pass


class InvalidTrainJobError(Exception):
    pass


class InvalidTrialError(Exception):
    pass


class RunningInferenceJobExistsError(Exception):
    pass


class NoModelsForTrainJobError(Exception):
    pass


class Admin:
    def __init__(self, db=None, container_manager=None):
        self._db = db or Database()
        if container_manager is None:
            from ..container.container_manager import LocalProcessManager
            container_manager = LocalProcessManager(logs_dir=config.get_config().path('logs'))
        self._cm = container_manager
        self._services_manager = ServicesManager(self._db, container_manager)
        if hasattr(container_manager, 'on_exit'):
            container_manager.on_exit(self._services_manager.on_container_exit)

    @property
    def db(self):
        return self._db

    @property
    def services_manager(self):
        return self._services_manager

    def seed(self):
        try:
            self._create_user(config.SUPERADMIN_EMAIL, config.SUPERADMIN_PASSWORD, UserType.SUPERADMIN)
        except UserExistsError:
            logger.info('superadmin exists')

    # -------------------------------------------------------------------------------- users
    @staticmethod
    def _user_dict(u, with_banned=True):
        d = {'id': u.id, 'email': u.email, 'user_type': u.user_type}
        if with_banned:
            d['banned_date'] = u.banned_date
        return d

    def authenticate_user(self, email, password):
        user = self._db.get_user_by_email(email)
        if user is None:
            raise InvalidUserError()
        if not check_password(password, user.password_hash):
            raise InvalidPasswordError()
        return self._user_dict(user)

    def create_user(self, email, password, user_type):
        return self._user_dict(self._create_user(email, password, user_type), with_banned=False)

    def get_users(self):
        return [self._user_dict(u) for u in self._db.get_users()]

    def get_user_by_email(self, email):
        u = self._db.get_user_by_email(email)
        return None if u is None else self._user_dict(u)

    def ban_user(self, email):
        user = self._db.get_user_by_email(email)
        if user is None:
            raise InvalidUserError()
        if user.banned_date is not None:
            raise UserAlreadyBannedError()
        self._db.ban_user(user)
        return self._user_dict(user)

    def _create_user(self, email, password, user_type):
        if self._db.get_user_by_email(email) is not None:
            raise UserExistsError()
        return self._db.create_user(email, hash_password(password), user_type)

    # ---------------------------------------------------------------------------- train jobs
    @staticmethod
    def _train_job_dict(x):
        return {'id': x.id, 'status': x.status, 'app': x.app, 'app_version': x.app_version, 'task': x.task,
                'train_dataset_uri': x.train_dataset_uri, 'test_dataset_uri': x.test_dataset_uri,
                'datetime_started': x.datetime_started, 'datetime_stopped': x.datetime_stopped, 'budget': x.budget}

    def create_train_job(self, user_id, app, task, train_dataset_uri, test_dataset_uri, budget, model_ids):
        if not model_ids:
            raise NoModelsForTrainJobError()
        existing = self._db.get_train_jobs_by_app(user_id, app)
        app_version = max([x.app_version for x in existing], default=0) + 1
        avail = {m.id for m in self._db.get_available_models(user_id, task)}
        for mid in model_ids:
            if mid not in avail:
                raise InvalidModelError('No model of ID "{}" is available for task "{}"'.format(mid, task))
        budget = dict(budget or {})
        budget.setdefault(BudgetType.MODEL_TRIAL_COUNT, config.DEFAULT_MODEL_TRIAL_COUNT)
        tj = self._db.create_train_job(user_id, app, app_version, task, budget, train_dataset_uri, test_dataset_uri)
        for mid in model_ids:
            self._db.create_sub_train_job(tj.id, mid, user_id)
        tj = self._services_manager.create_train_services(tj.id)
        return {'id': tj.id, 'app': tj.app, 'app_version': tj.app_version}

    def stop_train_job(self, user_id, app, app_version=-1):
        tj = self._db.get_train_job_by_app_version(user_id, app, app_version)
        if tj is None:
            raise InvalidTrainJobError()
        self._services_manager.stop_train_services(tj.id)
        return {'id': tj.id, 'app': tj.app, 'app_version': tj.app_version}

    def get_train_job(self, user_id, app, app_version=-1):
        tj = self._db.get_train_job_by_app_version(user_id, app, app_version)
        if tj is None:
            raise InvalidTrainJobError()
        workers = []
        for w in self._db.get_workers_of_train_job(tj.id):
            svc = self._db.get_service(w.service_id)
            model = self._db.get_model(self._db.get_sub_train_job(w.sub_train_job_id).model_id)
            workers.append({'service_id': svc.id, 'status': svc.status, 'replicas': svc.replicas,
                            'gpus': svc.gpus, 'datetime_started': svc.datetime_started,
                            'datetime_stopped': svc.datetime_stopped, 'model_name': model.name if model else None})
        d = self._train_job_dict(tj)
        d['workers'] = workers
        return d

    def get_train_jobs_by_app(self, user_id, app):
        return [self._train_job_dict(x) for x in self._db.get_train_jobs_by_app(user_id, app)]

    def get_train_jobs_by_user(self, user_id):
        return [self._train_job_dict(x) for x in self._db.get_train_jobs_by_user(user_id)]

    def _trial_dict(self, t, with_status=True, with_worker=False):
        model = self._db.get_model(t.model_id)
        d = {'id': t.id, 'knobs': t.knobs, 'datetime_started': t.datetime_started,
             'datetime_stopped': t.datetime_stopped, 'model_name': model.name if model else None, 'score': t.score}
        if with_status:
            d['status'] = t.status
        if with_worker:
            d['worker_id'] = t.worker_id
        return d

    def get_best_trials_of_train_job(self, user_id, app, app_version=-1, max_count=2):
        tj = self._db.get_train_job_by_app_version(user_id, app, app_version)
        if tj is None:
            raise InvalidTrainJobError()
        return [self._trial_dict(t, with_status=False)
                for t in self._db.get_best_trials_of_train_job(tj.id, max_count=max_count)]

    def get_trials_of_train_job(self, user_id, app, app_version=-1):
        tj = self._db.get_train_job_by_app_version(user_id, app, app_version)
        if tj is None:
            raise InvalidTrainJobError()
        trials = []
        for sub in self._db.get_sub_train_jobs_of_train_job(tj.id):
            trials.extend(self._db.get_trials_of_sub_train_job(sub.id))
        return [self._trial_dict(t) for t in trials]

    def stop_all_train_jobs(self):
        jobs = self._db.get_train_jobs_by_statuses([TrainJobStatus.STARTED, TrainJobStatus.RUNNING])
        for tj in jobs:
            self._services_manager.stop_train_services(tj.id)
        return [{'id': tj.id} for tj in jobs]

    # -------------------------------------------------------------------------------- trials
    def get_trial(self, trial_id):
        t = self._db.get_trial(trial_id)
        if t is None:
            raise InvalidTrialError()
        return self._trial_dict(t, with_worker=True)

    def get_trial_logs(self, trial_id):
        if self._db.get_trial(trial_id) is None:
            raise InvalidTrialError()
        lines = [x.line for x in self._db.get_trial_logs(trial_id)]
        messages, metrics, plots = ModelLogger.parse_logs(lines)
        return {'plots': plots, 'metrics': metrics, 'messages': messages}

    def get_trial_parameters(self, trial_id):
        t = self._db.get_trial(trial_id)
        if t is None or not t.params_file_path:
            raise InvalidTrialError()
        with open(t.params_file_path, 'rb') as f:
            return f.read()

    # ------------------------------------------------------------------------ inference jobs
    def create_inference_job(self, user_id, app, app_version=-1, max_models=None):
        tj = self._db.get_train_job_by_app_version(user_id, app, app_version)
        if tj is None:
            raise InvalidTrainJobError('Have you started a train job for this app?')
        if tj.status != TrainJobStatus.STOPPED:
            raise InvalidTrainJobError('Train job must be of status `STOPPED`.')
        if self._db.get_running_inference_job_by_train_job(tj.id) is not None:
            raise RunningInferenceJobExistsError()
        ij = self._db.create_inference_job(user_id, tj.id)
        ij, predictor = self._services_manager.create_inference_services(ij.id, max_models=max_models)
        return {'id': ij.id, 'train_job_id': tj.id, 'app': tj.app, 'app_version': tj.app_version,
                'predictor_host': self._host(predictor)}

    def stop_inference_job(self, user_id, app, app_version=-1):
        tj = self._db.get_train_job_by_app_version(user_id, app, app_version)
        if tj is None:
            raise InvalidRunningInferenceJobError()
        ij = self._db.get_running_inference_job_by_train_job(tj.id)
        if ij is None:
            raise InvalidRunningInferenceJobError()
        ij = self._services_manager.stop_inference_services(ij.id)
        return {'id': ij.id, 'train_job_id': tj.id, 'app': tj.app, 'app_version': tj.app_version}

    def get_running_inference_job(self, user_id, app, app_version=-1):
        tj = self._db.get_train_job_by_app_version(user_id, app, app_version)
        if tj is None:
            raise InvalidRunningInferenceJobError()
        ij = self._db.get_running_inference_job_by_train_job(tj.id)
        if ij is None:
            raise InvalidRunningInferenceJobError()
        workers = []
        for w in self._db.get_workers_of_inference_job(ij.id):
            svc = self._db.get_service(w.service_id)
            trial = self._db.get_trial(w.trial_id)
            model = self._db.get_model(trial.model_id)
            workers.append({'service_id': svc.id, 'status': svc.status, 'replicas': svc.replicas,
                            'datetime_started': svc.datetime_started, 'datetime_stopped': svc.datetime_stopped,
                            'trial': {'id': trial.id, 'score': trial.score, 'knobs': trial.knobs,
                                      'model_name': model.name if model else None}})
        return {'id': ij.id, 'status': ij.status, 'train_job_id': tj.id, 'app': tj.app,
                'app_version': tj.app_version, 'datetime_started': ij.datetime_started,
                'datetime_stopped': ij.datetime_stopped,
                'predictor_host': self._host(self._db.get_service(ij.predictor_service_id)), 'workers': workers}

    def _inference_job_list(self, jobs):
        out = []
        for ij in jobs:
            tj = self._db.get_train_job(ij.train_job_id)
            out.append({'id': ij.id, 'status': ij.status, 'train_job_id': tj.id, 'app': tj.app,
                        'app_version': tj.app_version, 'datetime_started': ij.datetime_started,
                        'datetime_stopped': ij.datetime_stopped,
                        'predictor_host': self._host(self._db.get_service(ij.predictor_service_id))})
        return out

    def get_inference_jobs_of_app(self, user_id, app):
        return self._inference_job_list(self._db.get_inference_jobs_of_app(user_id, app))

    def get_inference_jobs_by_user(self, user_id):
        return self._inference_job_list(self._db.get_inference_jobs_by_user(user_id))

    def stop_all_inference_jobs(self):
        jobs = self._db.get_inference_jobs_by_status(InferenceJobStatus.RUNNING)
        for ij in jobs:
            self._services_manager.stop_inference_services(ij.id)
        return [{'id': ij.id} for ij in jobs]

    # -------------------------------------------------------------------------------- models
    @staticmethod
    def _model_dict(m, full=True):
        d = {'id': m.id, 'user_id': m.user_id, 'name': m.name, 'task': m.task}
        if full:
            d.update({'model_class': m.model_class, 'datetime_created': m.datetime_created,
                      'docker_image': m.docker_image, 'dependencies': m.dependencies,
                      'access_right': m.access_right})
        return d

    def create_model(self, user_id, name, task, model_file_bytes, model_class, docker_image=None, dependencies=None,
                     access_right=ModelAccessRight.PRIVATE):
        m = self._db.create_model(user_id, name, task, model_file_bytes, model_class, docker_image or WORKER_IMAGE,
                                  dependencies or {}, access_right)
        return {'id': m.id, 'user_id': m.user_id, 'name': m.name}

    def delete_model(self, model_id):
        m = self._db.get_model(model_id)
        if m is None:
            raise InvalidModelError()
        self._db.delete_model(m)
        return {'id': m.id, 'user_id': m.user_id, 'name': m.name}

    def get_model_by_name(self, user_id, name):
        m = self._db.get_model_by_name(user_id, name)
        if m is None:
            raise InvalidModelError()
        return self._model_dict(m)

    def get_model(self, model_id):
        m = self._db.get_model(model_id)
        if m is None:
            raise InvalidModelError()
        return self._model_dict(m)

    def get_model_file(self, model_id):
        m = self._db.get_model(model_id)
        if m is None:
            raise InvalidModelError()
        return m.model_file_bytes

    def get_available_models(self, user_id, task=None):
        return [{'id': m.id, 'user_id': m.user_id, 'name': m.name, 'task': m.task,
                 'datetime_created': m.datetime_created, 'dependencies': m.dependencies,
                 'access_right': m.access_right} for m in self._db.get_available_models(user_id, task)]

    # -------------------------------------------------------------------------------- events
    def handle_event(self, name, **params):
        handlers = {'sub_train_job_budget_reached': self._on_budget_reached,
                    'train_job_worker_started': self._on_worker_changed,
                    'train_job_worker_stopped': self._on_worker_changed}
        if name not in handlers:
            logger.error('Unknown event: "%s"', name)
            return
        handlers[name](**params)

    def _on_budget_reached(self, sub_train_job_id):
        self._services_manager.stop_sub_train_job_services(sub_train_job_id)

    def _on_worker_changed(self, sub_train_job_id):
        sub = self._db.get_sub_train_job(sub_train_job_id)
        if sub is not None:
            self._services_manager.refresh_train_job_status(sub.train_job_id)

    # ------------------------------------------------------------------------------- helpers
    @staticmethod
    def _host(service):
        if service is None:
            return None
        return '{}:{}'.format(service.ext_hostname, service.ext_port)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def connect(self):
        pass

    def disconnect(self):
        self._db.flush_logs()
