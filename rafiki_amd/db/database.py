"""Metadata store: embedded SQLite (WAL) with the reference's tables and query surface.

Reference parity: rafiki/db/schema.py:18-133 (same tables/columns) and rafiki/db/database.py
(:43-480, one method per query).  PostgreSQL + SQLAlchemy are replaced by stdlib ``sqlite3`` —
one node, no separate DB container — and:
  * every method is its own short transaction (thread-safe; one writer lock), so there is no
    session object to leak between requests;
  * trial log lines are written by a batching writer (the reference commits one DB
    transaction per model log line);
  * rows come back as attribute-access records (``rec.status``), JSON columns decoded.
"""
from __future__ import annotations

import json
import os
import queue
import sqlite3
import threading
import time
import uuid
from datetime import datetime
from types import SimpleNamespace

from ..constants import (InferenceJobStatus, ModelAccessRight, ServiceStatus, TrainJobStatus, TrialStatus,
                         UserType)


class InvalidModelAccessRightError(Exception):
    pass


class DuplicateModelNameError(Exception):
    pass


class ModelUsedError(Exception):
    pass


class InvalidUserTypeError(Exception):
    pass


_SCHEMA = """
CREATE TABLE IF NOT EXISTS user (
  id TEXT PRIMARY KEY, email TEXT UNIQUE NOT NULL, password_hash BLOB NOT NULL, user_type TEXT NOT NULL,
  banned_date TEXT);
CREATE TABLE IF NOT EXISTS model (
  id TEXT PRIMARY KEY, datetime_created TEXT NOT NULL, user_id TEXT NOT NULL REFERENCES user(id),
  name TEXT NOT NULL, task TEXT NOT NULL, model_file_bytes BLOB NOT NULL, model_class TEXT NOT NULL,
  docker_image TEXT NOT NULL, dependencies TEXT NOT NULL, access_right TEXT NOT NULL,
  UNIQUE(name, user_id));
CREATE TABLE IF NOT EXISTS service (
  id TEXT PRIMARY KEY, service_type TEXT NOT NULL, status TEXT NOT NULL, docker_image TEXT NOT NULL,
  container_manager_type TEXT NOT NULL, replicas INTEGER NOT NULL, gpus INTEGER NOT NULL, ext_hostname TEXT,
  ext_port INTEGER, hostname TEXT, port INTEGER, container_service_name TEXT, container_service_id TEXT,
  container_service_info TEXT, datetime_started TEXT NOT NULL, datetime_stopped TEXT);
CREATE TABLE IF NOT EXISTS train_job (
  id TEXT PRIMARY KEY, app TEXT NOT NULL, app_version INTEGER NOT NULL, task TEXT NOT NULL, budget TEXT NOT NULL,
  train_dataset_uri TEXT NOT NULL, test_dataset_uri TEXT NOT NULL, user_id TEXT NOT NULL REFERENCES user(id),
  status TEXT NOT NULL, datetime_started TEXT NOT NULL, datetime_stopped TEXT,
  UNIQUE(app, app_version, user_id));
CREATE TABLE IF NOT EXISTS sub_train_job (
  id TEXT PRIMARY KEY, train_job_id TEXT REFERENCES train_job(id), model_id TEXT REFERENCES model(id),
  user_id TEXT NOT NULL, datetime_started TEXT NOT NULL, datetime_stopped TEXT);
CREATE TABLE IF NOT EXISTS train_job_worker (
  service_id TEXT PRIMARY KEY REFERENCES service(id), sub_train_job_id TEXT NOT NULL REFERENCES sub_train_job(id));
CREATE TABLE IF NOT EXISTS trial (
  id TEXT PRIMARY KEY, sub_train_job_id TEXT NOT NULL REFERENCES sub_train_job(id),
  model_id TEXT NOT NULL REFERENCES model(id), datetime_started TEXT NOT NULL, status TEXT NOT NULL,
  worker_id TEXT NOT NULL, knobs TEXT, score REAL DEFAULT 0, params_file_path TEXT, datetime_stopped TEXT);
CREATE TABLE IF NOT EXISTS trial_log (
  id TEXT PRIMARY KEY, datetime TEXT, trial_id TEXT NOT NULL REFERENCES trial(id), line TEXT NOT NULL,
  level TEXT);
CREATE INDEX IF NOT EXISTS trial_log_trial_id ON trial_log(trial_id);
CREATE TABLE IF NOT EXISTS inference_job (
  id TEXT PRIMARY KEY, datetime_started TEXT NOT NULL, train_job_id TEXT REFERENCES train_job(id),
  status TEXT NOT NULL, user_id TEXT NOT NULL, predictor_service_id TEXT REFERENCES service(id),
  datetime_stopped TEXT);
CREATE TABLE IF NOT EXISTS inference_job_worker (
  service_id TEXT PRIMARY KEY REFERENCES service(id), inference_job_id TEXT REFERENCES inference_job(id),
  trial_id TEXT NOT NULL REFERENCES trial(id));
"""

_JSON_COLS = {'dependencies', 'budget', 'knobs', 'container_service_info'}
_DT_COLS = {'banned_date', 'datetime_created', 'datetime_started', 'datetime_stopped', 'datetime'}


def _uuid():
    return str(uuid.uuid4())


def _now():
    return datetime.utcnow()


def _enc(k, v):
    if v is None:
        return None
    if k in _JSON_COLS:
        return json.dumps(v)
    if k in _DT_COLS and isinstance(v, datetime):
        return v.isoformat()
    return v


def _dec(k, v):
    if v is None:
        return None
    if k in _JSON_COLS:
        return json.loads(v)
    if k in _DT_COLS:
        return datetime.fromisoformat(v)
    return v


class Record(SimpleNamespace):
    """A row; attribute access, plus the table it came from."""


class Database:
    def __init__(self, path=None):
        from ..config import get_config
        self.path = path or os.environ.get('RAFIKI_DB_PATH') or get_config().resolved_db_path
        if self.path != ':memory:':
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        self._local = threading.local()
        self._wlock = threading.RLock()
        self._shared = None
        if self.path == ':memory:':  # one shared connection for in-memory DBs (tests)
            self._shared = sqlite3.connect(':memory:', check_same_thread=False, isolation_level=None)
            self._shared.row_factory = sqlite3.Row
        with self._wlock:
            self._conn().executescript(_SCHEMA)
        self._log_q: "queue.Queue" = queue.Queue()
        self._log_thread = None
        self._log_stop = threading.Event()

    # --------------------------------------------------------------------------- plumbing
    def _conn(self):
        if self._shared is not None:
            return self._shared
        c = getattr(self._local, 'conn', None)
        if c is None:
            c = sqlite3.connect(self.path, timeout=30.0, check_same_thread=False, isolation_level=None)
            c.row_factory = sqlite3.Row
            c.execute('PRAGMA journal_mode=WAL')
            c.execute('PRAGMA synchronous=NORMAL')
            c.execute('PRAGMA foreign_keys=OFF')
            self._local.conn = c
        return c

    def _rec(self, table, row):
        if row is None:
            return None
        r = Record(**{k: _dec(k, row[k]) for k in row.keys()})
        r._table = table
        return r

    def _insert(self, table, **cols):
        cols.setdefault('id', _uuid()) if table not in ('train_job_worker', 'inference_job_worker') else None
        keys = list(cols)
        sql = 'INSERT INTO {} ({}) VALUES ({})'.format(table, ','.join(keys), ','.join('?' * len(keys)))
        with self._wlock:
            try:
                self._conn().execute(sql, [_enc(k, cols[k]) for k in keys])
            except sqlite3.IntegrityError as e:
                if table == 'model' and 'UNIQUE' in str(e):
                    raise DuplicateModelNameError()
                raise
        r = Record(**cols)
        r._table = table
        return r

    def _update(self, rec, **cols):
        pk = 'service_id' if rec._table in ('train_job_worker', 'inference_job_worker') else 'id'
        keys = list(cols)
        sql = 'UPDATE {} SET {} WHERE {} = ?'.format(rec._table, ','.join('{} = ?'.format(k) for k in keys), pk)
        with self._wlock:
            self._conn().execute(sql, [_enc(k, cols[k]) for k in keys] + [getattr(rec, pk)])
        for k, v in cols.items():
            setattr(rec, k, v)
        return rec

    def _one(self, table, sql, params=()):
        return self._rec(table, self._conn().execute(sql, params).fetchone())

    def _all(self, table, sql, params=()):
        return [self._rec(table, r) for r in self._conn().execute(sql, params).fetchall()]

    # compatibility with the reference's session-style API
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def connect(self):
        pass

    def disconnect(self):
        self.flush_logs()

    def commit(self):
        pass

    def expire(self):
        pass

    def close(self):
        self.stop_log_writer()
        c = getattr(self._local, 'conn', None)
        if c is not None:
            c.close()
            self._local.conn = None

    # ------------------------------------------------------------------------------ users
    def create_user(self, email, password_hash, user_type):
        if user_type not in (UserType.SUPERADMIN, UserType.ADMIN, UserType.APP_DEVELOPER, UserType.MODEL_DEVELOPER):
            raise InvalidUserTypeError()
        return self._insert('user', email=email, password_hash=password_hash, user_type=user_type, banned_date=None)

    def ban_user(self, user):
        return self._update(user, banned_date=_now())

    def get_user_by_email(self, email):
        return self._one('user', 'SELECT * FROM user WHERE email = ?', (email,))

    def get_user(self, user_id):
        return self._one('user', 'SELECT * FROM user WHERE id = ?', (user_id,))

    def get_users(self):
        return self._all('user', 'SELECT * FROM user')

    # ------------------------------------------------------------------------- train jobs
    def create_train_job(self, user_id, app, app_version, task, budget, train_dataset_uri, test_dataset_uri):
        return self._insert('train_job', user_id=user_id, app=app, app_version=app_version, task=task, budget=budget,
                            train_dataset_uri=train_dataset_uri, test_dataset_uri=test_dataset_uri,
                            status=TrainJobStatus.STARTED, datetime_started=_now(), datetime_stopped=None)

    def get_train_jobs_by_app(self, user_id, app):
        return self._all('train_job', 'SELECT * FROM train_job WHERE app = ? AND user_id = ? '
                                      'ORDER BY app_version DESC', (app, user_id))

    def get_train_jobs_by_user(self, user_id):
        return self._all('train_job', 'SELECT * FROM train_job WHERE user_id = ? ORDER BY datetime_started',
                         (user_id,))

    def get_train_job(self, id):
        return self._one('train_job', 'SELECT * FROM train_job WHERE id = ?', (id,))

    def get_train_jobs_by_statuses(self, statuses):
        q = 'SELECT * FROM train_job WHERE status IN ({})'.format(','.join('?' * len(statuses)))
        return self._all('train_job', q, tuple(statuses))

    def get_train_job_by_app_version(self, user_id, app, app_version=-1):
        if app_version == -1:
            return self._one('train_job', 'SELECT * FROM train_job WHERE user_id = ? AND app = ? '
                                          'ORDER BY app_version DESC LIMIT 1', (user_id, app))
        return self._one('train_job', 'SELECT * FROM train_job WHERE user_id = ? AND app = ? AND app_version = ?',
                         (user_id, app, int(app_version)))

    def mark_train_job_as_running(self, train_job):
        return self._update(train_job, status=TrainJobStatus.RUNNING)

    def mark_train_job_as_errored(self, train_job):
        return self._update(train_job, status=TrainJobStatus.ERRORED, datetime_stopped=_now())

    def mark_train_job_as_stopped(self, train_job):
        return self._update(train_job, status=TrainJobStatus.STOPPED, datetime_stopped=_now())

    # --------------------------------------------------------------------- sub train jobs
    def create_sub_train_job(self, train_job_id, model_id, user_id):
        return self._insert('sub_train_job', train_job_id=train_job_id, model_id=model_id, user_id=user_id,
                            datetime_started=_now(), datetime_stopped=None)

    def get_sub_train_jobs_of_train_job(self, train_job_id):
        return self._all('sub_train_job', 'SELECT * FROM sub_train_job WHERE train_job_id = ?', (train_job_id,))

    def get_sub_train_job(self, id):
        return self._one('sub_train_job', 'SELECT * FROM sub_train_job WHERE id = ?', (id,))

    def mark_sub_train_job_as_stopped(self, sub_train_job):
        return self._update(sub_train_job, datetime_stopped=_now())

    # ------------------------------------------------------------------ train job workers
    def create_train_job_worker(self, service_id, sub_train_job_id):
        return self._insert('train_job_worker', service_id=service_id, sub_train_job_id=sub_train_job_id)

    def get_train_job_worker(self, service_id):
        return self._one('train_job_worker', 'SELECT * FROM train_job_worker WHERE service_id = ?', (service_id,))

    def get_workers_of_sub_train_job(self, sub_train_job_id):
        return self._all('train_job_worker', 'SELECT * FROM train_job_worker WHERE sub_train_job_id = ?',
                         (sub_train_job_id,))

    def get_workers_of_train_job(self, train_job_id):
        return self._all('train_job_worker', 'SELECT w.* FROM train_job_worker w JOIN sub_train_job s '
                                             'ON s.id = w.sub_train_job_id WHERE s.train_job_id = ?',
                         (train_job_id,))

    # --------------------------------------------------------------------- inference jobs
    def create_inference_job(self, user_id, train_job_id):
        return self._insert('inference_job', user_id=user_id, train_job_id=train_job_id,
                            status=InferenceJobStatus.STARTED, datetime_started=_now(), datetime_stopped=None,
                            predictor_service_id=None)

    def get_inference_job(self, id):
        return self._one('inference_job', 'SELECT * FROM inference_job WHERE id = ?', (id,))

    def get_inference_job_by_predictor(self, predictor_service_id):
        return self._one('inference_job', 'SELECT * FROM inference_job WHERE predictor_service_id = ?',
                         (predictor_service_id,))

    def get_running_inference_job_by_train_job(self, train_job_id):
        return self._one('inference_job', 'SELECT * FROM inference_job WHERE train_job_id = ? AND status = ?',
                         (train_job_id, InferenceJobStatus.RUNNING))

    def get_inference_jobs_by_user(self, user_id):
        return self._all('inference_job', 'SELECT * FROM inference_job WHERE user_id = ? ORDER BY datetime_started',
                         (user_id,))

    def update_inference_job(self, inference_job, predictor_service_id):
        return self._update(inference_job, predictor_service_id=predictor_service_id)

    def mark_inference_job_as_running(self, inference_job):
        return self._update(inference_job, status=InferenceJobStatus.RUNNING, datetime_stopped=None)

    def mark_inference_job_as_stopped(self, inference_job):
        return self._update(inference_job, status=InferenceJobStatus.STOPPED, datetime_stopped=_now())

    def mark_inference_job_as_errored(self, inference_job):
        return self._update(inference_job, status=InferenceJobStatus.ERRORED, datetime_stopped=_now())

    def get_inference_jobs_of_app(self, user_id, app):
        return self._all('inference_job', 'SELECT i.* FROM inference_job i JOIN train_job t ON i.train_job_id = t.id '
                                          'WHERE t.user_id = ? AND t.app = ? ORDER BY i.datetime_started DESC',
                         (user_id, app))

    def get_inference_jobs_by_status(self, status):
        return self._all('inference_job', 'SELECT * FROM inference_job WHERE status = ?', (status,))

    # -------------------------------------------------------------- inference job workers
    def create_inference_job_worker(self, service_id, inference_job_id, trial_id):
        return self._insert('inference_job_worker', service_id=service_id, inference_job_id=inference_job_id,
                            trial_id=trial_id)

    def get_inference_job_worker(self, service_id):
        return self._one('inference_job_worker', 'SELECT * FROM inference_job_worker WHERE service_id = ?',
                         (service_id,))

    def get_workers_of_inference_job(self, inference_job_id):
        return self._all('inference_job_worker', 'SELECT * FROM inference_job_worker WHERE inference_job_id = ?',
                         (inference_job_id,))

    # --------------------------------------------------------------------------- services
    def create_service(self, service_type, container_manager_type, docker_image, replicas, gpus):
        return self._insert('service', service_type=service_type, container_manager_type=container_manager_type,
                            docker_image=docker_image, replicas=replicas, gpus=gpus, status=ServiceStatus.STARTED,
                            datetime_started=_now(), datetime_stopped=None, ext_hostname=None, ext_port=None,
                            hostname=None, port=None, container_service_name=None, container_service_id=None,
                            container_service_info=None)

    def mark_service_as_deploying(self, service, container_service_name, container_service_id, hostname, port,
                                  ext_hostname, ext_port, container_service_info):
        return self._update(service, container_service_name=container_service_name,
                            container_service_id=container_service_id, hostname=hostname, port=port,
                            ext_hostname=ext_hostname, ext_port=ext_port,
                            container_service_info=container_service_info, status=ServiceStatus.DEPLOYING)

    def update_service_container_info(self, service, container_service_id, hostname, port, ext_hostname, ext_port,
                                      container_service_info):
        """Record where a launched service lives without touching its status."""
        return self._update(service, container_service_id=container_service_id, hostname=hostname, port=port,
                            ext_hostname=ext_hostname, ext_port=ext_port,
                            container_service_info=container_service_info)

    def mark_service_as_running(self, service):
        return self._update(service, status=ServiceStatus.RUNNING, datetime_stopped=None)

    def mark_service_as_errored(self, service):
        return self._update(service, status=ServiceStatus.ERRORED, datetime_stopped=_now())

    def mark_service_as_stopped(self, service):
        return self._update(service, status=ServiceStatus.STOPPED, datetime_stopped=_now())

    def get_service(self, service_id):
        return self._one('service', 'SELECT * FROM service WHERE id = ?', (service_id,))

    def get_services(self, status=None):
        if status is None:
            return self._all('service', 'SELECT * FROM service')
        return self._all('service', 'SELECT * FROM service WHERE status = ?', (status,))

    # ----------------------------------------------------------------------------- models
    def create_model(self, user_id, name, task, model_file_bytes, model_class, docker_image, dependencies,
                     access_right):
        if access_right not in (ModelAccessRight.PUBLIC, ModelAccessRight.PRIVATE):
            raise InvalidModelAccessRightError()
        return self._insert('model', user_id=user_id, name=name, task=task, model_file_bytes=model_file_bytes,
                            model_class=model_class, docker_image=docker_image, dependencies=dependencies,
                            access_right=access_right, datetime_created=_now())

    def delete_model(self, model):
        used = self._conn().execute('SELECT 1 FROM sub_train_job WHERE model_id = ? LIMIT 1', (model.id,)).fetchone()
        if used is not None:
            raise ModelUsedError()
        with self._wlock:
            self._conn().execute('DELETE FROM model WHERE id = ?', (model.id,))

    def get_available_models(self, user_id, task=None):
        q = 'SELECT * FROM model WHERE (access_right = ? OR user_id = ?)'
        args = [ModelAccessRight.PUBLIC, user_id]
        if task is not None:
            q += ' AND task = ?'
            args.append(task)
        return self._all('model', q + ' ORDER BY datetime_created', tuple(args))

    def get_model_by_name(self, user_id, name):
        return self._one('model', 'SELECT * FROM model WHERE user_id = ? AND name = ?', (user_id, name))

    def get_model(self, id):
        return self._one('model', 'SELECT * FROM model WHERE id = ?', (id,))

    # ----------------------------------------------------------------------------- trials
    def create_trial(self, sub_train_job_id, model_id, worker_id):
        return self._insert('trial', sub_train_job_id=sub_train_job_id, model_id=model_id, worker_id=worker_id,
                            status=TrialStatus.STARTED, datetime_started=_now(), knobs=None, score=0.0,
                            params_file_path=None, datetime_stopped=None)

    def claim_trial(self, sub_train_job_id, model_id, worker_id, max_trials):
        """Atomically create a trial if the sub-train-job still has budget: counts COMPLETED, ERRORED
        and in-flight (STARTED/RUNNING) trials inside one ``BEGIN IMMEDIATE`` transaction, so concurrent
        workers (threads or processes) can never overshoot MODEL_TRIAL_COUNT (the reference's budget
        race, worker/train.py:50).  Returns the new trial or None."""
        with self._wlock:
            c = self._conn()
            c.execute('BEGIN IMMEDIATE')
            try:
                n = c.execute('SELECT COUNT(*) FROM trial WHERE sub_train_job_id = ? AND status IN (?,?,?,?)',
                              (sub_train_job_id, TrialStatus.COMPLETED, TrialStatus.ERRORED, TrialStatus.STARTED,
                               TrialStatus.RUNNING)).fetchone()[0]
                if n >= max_trials:
                    c.execute('ROLLBACK')
                    return None
                tid = _uuid()
                c.execute('INSERT INTO trial (id, sub_train_job_id, model_id, worker_id, status, datetime_started, '
                          'knobs, score, params_file_path, datetime_stopped) VALUES (?,?,?,?,?,?,?,?,?,?)',
                          (tid, sub_train_job_id, model_id, worker_id, TrialStatus.STARTED, _enc('datetime_started',
                                                                                                _now()),
                           None, 0.0, None, None))
                c.execute('COMMIT')
            except Exception:
                c.execute('ROLLBACK')
                raise
        return self.get_trial(tid)

    def get_trial(self, id):
        return self._one('trial', 'SELECT * FROM trial WHERE id = ?', (id,))

    def get_trial_logs(self, id):
        self.flush_logs()
        return self._all('trial_log', 'SELECT * FROM trial_log WHERE trial_id = ? ORDER BY datetime, rowid', (id,))

    def get_best_trials_of_train_job(self, train_job_id, max_count=2):
        return self._all('trial', 'SELECT t.* FROM trial t JOIN sub_train_job s ON t.sub_train_job_id = s.id '
                                  'WHERE s.train_job_id = ? AND t.status = ? ORDER BY t.score DESC LIMIT ?',
                         (train_job_id, TrialStatus.COMPLETED, int(max_count)))

    def get_trials_of_sub_train_job(self, sub_train_job_id):
        return self._all('trial', 'SELECT * FROM trial WHERE sub_train_job_id = ? ORDER BY datetime_started DESC',
                         (sub_train_job_id,))

    def get_trials_of_train_job(self, train_job_id):
        return self._all('trial', 'SELECT t.* FROM trial t JOIN sub_train_job s ON t.sub_train_job_id = s.id '
                                  'WHERE s.train_job_id = ? ORDER BY t.datetime_started DESC', (train_job_id,))

    def get_trials_of_app(self, app):
        return self._all('trial', 'SELECT t.* FROM trial t JOIN sub_train_job s ON t.sub_train_job_id = s.id '
                                  'JOIN train_job j ON j.id = s.train_job_id WHERE j.app = ? '
                                  'ORDER BY t.datetime_started DESC', (app,))

    def count_trials_of_sub_train_job(self, sub_train_job_id, statuses):
        q = 'SELECT COUNT(*) FROM trial WHERE sub_train_job_id = ? AND status IN ({})'.format(
            ','.join('?' * len(statuses)))
        return int(self._conn().execute(q, (sub_train_job_id, *statuses)).fetchone()[0])

    def mark_trial_as_running(self, trial, knobs):
        return self._update(trial, status=TrialStatus.RUNNING, knobs=knobs)

    def mark_trial_as_errored(self, trial):
        return self._update(trial, status=TrialStatus.ERRORED, datetime_stopped=_now())

    def mark_trial_as_complete(self, trial, score, params_file_path):
        return self._update(trial, status=TrialStatus.COMPLETED, score=float(score), datetime_stopped=_now(),
                            params_file_path=params_file_path)

    def mark_trial_as_terminated(self, trial):
        return self._update(trial, status=TrialStatus.TERMINATED, datetime_stopped=_now())

    # ------------------------------------------------------------------ batched trial logs
    def add_trial_log(self, trial, line, level):
        """Enqueue a log line; a background writer commits them in batches."""
        tid = trial.id if hasattr(trial, 'id') else trial
        self._log_q.put((_uuid(), _now().isoformat(), tid, line, level))
        if self._log_thread is None:
            self._start_log_writer()

    def _start_log_writer(self):
        with self._wlock:
            if self._log_thread is not None:
                return
            self._log_stop.clear()
            t = threading.Thread(target=self._log_loop, name='rafiki-trial-log-writer', daemon=True)
            self._log_thread = t
            t.start()

    def _drain(self):
        batch = []
        try:
            while len(batch) < 4096:
                batch.append(self._log_q.get_nowait())
        except queue.Empty:
            pass
        if batch:
            with self._wlock:
                c = self._conn()
                c.execute('BEGIN')
                c.executemany('INSERT INTO trial_log (id, datetime, trial_id, line, level) VALUES (?,?,?,?,?)',
                              batch)
                c.execute('COMMIT')
        return len(batch)

    def _log_loop(self):
        while not self._log_stop.is_set():
            if self._drain() == 0:
                time.sleep(0.05)
        self._drain()

    def flush_logs(self):
        while self._drain():
            pass

    def stop_log_writer(self):
        if self._log_thread is not None:
            self._log_stop.set()
            self._log_thread.join(timeout=5)
            self._log_thread = None
        self.flush_logs()

    def clear_all_data(self):
        with self._wlock:
            for t in ('trial_log', 'trial', 'inference_job_worker', 'inference_job', 'train_job_worker',
                      'sub_train_job', 'train_job', 'service', 'model', 'user'):
                self._conn().execute('DELETE FROM {}'.format(t))
