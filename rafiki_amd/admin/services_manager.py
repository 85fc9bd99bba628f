"""Turns jobs into services on this node (reference rafiki/admin/services_manager.py:28-403).

Placement model (MI355X-first):
  * a train job's GPU budget (``GPU_COUNT``) is split evenly over its sub-train-jobs
    (reference :190-202); each sub-train-job gets ONE worker *group*: an SPMD service of
    ``gpus`` processes (one per GPU) that forms an RCCL process group.  Rank 0 hosts the
    sub-train-job's advisor and broadcasts one knob set per rank per round, so every GPU runs its
    own trial while sharing one GP posterior (fixes reference bug (d): one advisor per worker);
    a sub-train-job with 0 GPUs gets one CPU worker (reference :123-126);
  * an inference job is ONE predictor service holding all top-k models in HBM (288 GB/GPU) on
    RAFIKI_PREDICTOR_GPUS GPUs (default 1), as INFERENCE_WORKER_REPLICAS_PER_TRIAL replicas of the
    whole ensemble, with one logical ``INFERENCE`` service row per model for API parity.
"""
from __future__ import annotations

import logging
import os
import sys
import time
import traceback

from .. import config
from ..constants import BudgetType, ServiceStatus, ServiceType
from ..container.container_manager import ContainerManager, ContainerService, free_port
from ..model.model import parse_model_install_command

logger = logging.getLogger(__name__)

DEFAULT_TRAIN_GPU_COUNT = 0
WORKER_IMAGE = 'rafiki_amd/worker'
PREDICTOR_IMAGE = 'rafiki_amd/predictor'


class ServiceDeploymentError(Exception):
    pass


class ServicesManager:
    def __init__(self, db, container_manager: ContainerManager, wait_timeout_s: float = None):
        self._db = db
        self._cm = container_manager
        self._wait_timeout_s = wait_timeout_s or float(os.environ.get("RAFIKI_SERVICE_WAIT_TIMEOUT_S", "600"))
        self._cfg = config.get_config()

    # ---------------------------------------------------------------------------- inference
    def create_inference_services(self, inference_job_id, max_models=None):
        inference_job = self._db.get_inference_job(inference_job_id)
        k = int(max_models or config.INFERENCE_MAX_BEST_TRIALS)
        best_trials = self._db.get_best_trials_of_train_job(inference_job.train_job_id, max_count=k)
        if not best_trials:
            self._db.mark_inference_job_as_errored(inference_job)
            raise ServiceDeploymentError('no completed trials to serve')
        if os.environ.get('RAFIKI_INFERENCE_MODE', 'local') == 'workers':
            return self._create_inference_worker_services(inference_job, best_trials)
        try:
            workers = []
            for trial in best_trials:  # rows the predictor reads at start-up exist before it launches
                svc = self._db.create_service(ServiceType.INFERENCE, type(self._cm).__name__, PREDICTOR_IMAGE, 1, 0)
                self._db.mark_service_as_deploying(svc, 'in-predictor', None, None, None, None, None, None)
                self._db.create_inference_job_worker(svc.id, inference_job.id, trial.id)
                workers.append(svc)
            predictor = self._create_service(
                ServiceType.PREDICT, PREDICTOR_IMAGE, args=['-m', 'rafiki_amd.predictor.server'],
                environment_vars={'RAFIKI_INFERENCE_JOB_ID': inference_job.id},
                container_port=self._cfg.predictor_port, gpus=self._predictor_gpus(),
                before_launch=lambda s: self._db.update_inference_job(inference_job, predictor_service_id=s.id))
            for w in workers:
                self._db.update_service_container_info(w, predictor.container_service_id, None, None, None, None,
                                                       {'predictor_service_id': predictor.id})
            self._wait_until_services_running([predictor])
            for w in workers:
                self._db.mark_service_as_running(w)
            self._db.mark_inference_job_as_running(inference_job)
            return inference_job, self._db.get_service(predictor.id)
        except Exception:
            self._db.mark_inference_job_as_errored(inference_job)
            raise

    def _predictor_gpus(self):
        """GPUs for the predictor service: RAFIKI_PREDICTOR_GPUS (default 1); its replicas
        (INFERENCE_WORKER_REPLICAS_PER_TRIAL) are spread round-robin over them."""
        if not self._gpus_available():
            return 0
        return max(1, int(os.environ.get('RAFIKI_PREDICTOR_GPUS', '1')))

    def _create_inference_worker_services(self, inference_job, best_trials):
        """``workers`` mode: one InferenceWorker process per trial (its own GPU when free), then a
        predictor that fans out through the shared-memory Cache (reference services_manager.py:53-87)."""
        try:
            workers = []
            for trial in best_trials:
                gpus = 1 if self._gpus_available() else 0
                svc = self._create_service(
                    ServiceType.INFERENCE, WORKER_IMAGE, args=['-m', 'rafiki_amd.worker'],
                    environment_vars={'RAFIKI_SERVICE_TYPE': ServiceType.INFERENCE}, gpus=gpus,
                    before_launch=lambda s, t=trial: self._db.create_inference_job_worker(s.id, inference_job.id,
                                                                                         t.id))
                workers.append(svc)
            self._wait_until_services_running(workers)
            predictor = self._create_service(
                ServiceType.PREDICT, PREDICTOR_IMAGE, args=['-m', 'rafiki_amd.predictor.server'],
                environment_vars={'RAFIKI_INFERENCE_JOB_ID': inference_job.id, 'RAFIKI_INFERENCE_MODE': 'workers'},
                container_port=self._cfg.predictor_port, gpus=0,
                before_launch=lambda s: self._db.update_inference_job(inference_job, predictor_service_id=s.id))
            self._wait_until_services_running([predictor])
            self._db.mark_inference_job_as_running(inference_job)
            return inference_job, self._db.get_service(predictor.id)
        except Exception:
            self._db.mark_inference_job_as_errored(inference_job)
            raise

    def stop_inference_services(self, inference_job_id):
        inference_job = self._db.get_inference_job(inference_job_id)
        if inference_job.predictor_service_id:
            self._stop_service(self._db.get_service(inference_job.predictor_service_id))
        for w in self._db.get_workers_of_inference_job(inference_job_id):
            svc = self._db.get_service(w.service_id)
            if svc is not None and svc.container_service_id and svc.container_service_id != \
                    (self._db.get_service(inference_job.predictor_service_id).container_service_id
                     if inference_job.predictor_service_id else None):
                self._stop_service(svc)  # a real worker process (``workers`` mode)
            elif svc is not None and svc.status != ServiceStatus.STOPPED:
                self._db.mark_service_as_stopped(svc)
        return self._db.mark_inference_job_as_stopped(inference_job)

    # -------------------------------------------------------------------------------- train
    def create_train_services(self, train_job_id):
        train_job = self._db.get_train_job(train_job_id)
        subs = self._db.get_sub_train_jobs_of_train_job(train_job_id)
        total_gpus = int((train_job.budget or {}).get(BudgetType.GPU_COUNT, DEFAULT_TRAIN_GPU_COUNT))
        gpus_per_sub = self._split_gpus(total_gpus, len(subs))
        services = []
        try:
            for sub, gpus in zip(subs, gpus_per_sub):
                model = self._db.get_model(sub.model_id)
                env = {'WORKER_INSTALL_COMMAND': parse_model_install_command(model.dependencies, gpus > 0),
                       'RAFIKI_SUB_TRAIN_JOB_ID': sub.id}
                svc = self._create_service(ServiceType.TRAIN, model.docker_image, args=['-m', 'rafiki_amd.worker'],
                                           environment_vars=env, gpus=gpus, replicas=max(1, gpus),
                                           before_launch=lambda s, sub=sub: self._db.create_train_job_worker(
                                               s.id, sub.id))
                services.append(svc)
            self._wait_until_services_running(services, accept_stopped=True)
            self.refresh_train_job_status(train_job_id)
            tj = self._db.get_train_job(train_job_id)
            if tj.status == 'STARTED':
                self._db.mark_train_job_as_running(tj)
            return self._db.get_train_job(train_job_id)
        except Exception:
            logger.error(traceback.format_exc())
            for s in services:
                self._stop_service(self._db.get_service(s.id))
            self._db.mark_train_job_as_errored(train_job)
            raise

    def stop_train_services(self, train_job_id):
        train_job = self._db.get_train_job(train_job_id)
        for w in self._db.get_workers_of_train_job(train_job_id):
            self._stop_service(self._db.get_service(w.service_id))
        for sub in self._db.get_sub_train_jobs_of_train_job(train_job_id):
            if sub.datetime_stopped is None:
                self._db.mark_sub_train_job_as_stopped(sub)
        self._db.mark_train_job_as_stopped(train_job)
        return train_job

    def stop_sub_train_job_services(self, sub_train_job_id):
        sub = self._db.get_sub_train_job(sub_train_job_id)
        for w in self._db.get_workers_of_sub_train_job(sub_train_job_id):
            self._stop_service(self._db.get_service(w.service_id))
        if sub.datetime_stopped is None:
            self._db.mark_sub_train_job_as_stopped(sub)
        self.refresh_train_job_status(sub.train_job_id)
        return sub

    def refresh_train_job_status(self, train_job_id):
        """Roll service states up into the train job (reference :160-184)."""
        train_job = self._db.get_train_job(train_job_id)
        services = [self._db.get_service(w.service_id) for w in self._db.get_workers_of_train_job(train_job_id)]
        services = [s for s in services if s is not None]
        statuses = [s.status for s in services]
        if any(s == ServiceStatus.ERRORED for s in statuses):
            self._db.mark_train_job_as_errored(train_job)
        elif services and all(s == ServiceStatus.STOPPED for s in statuses):
            self._db.mark_train_job_as_stopped(train_job)
        elif any(s == ServiceStatus.RUNNING for s in statuses):
            self._db.mark_train_job_as_running(train_job)
        return train_job

    def on_container_exit(self, container_service_id, exit_codes):
        """Container-manager callback: a service's processes all exited."""
        for svc in self._db.get_services():
            if svc.container_service_id == container_service_id and svc.status != ServiceStatus.STOPPED:
                if any(c != 0 for c in exit_codes):
                    self._db.mark_service_as_errored(svc)
                else:
                    self._db.mark_service_as_stopped(svc)
                w = self._db.get_train_job_worker(svc.id)
                if w is not None:
                    sub = self._db.get_sub_train_job(w.sub_train_job_id)
                    self.refresh_train_job_status(sub.train_job_id)

    # ------------------------------------------------------------------------------ private
    @staticmethod
    def _split_gpus(total, n):
        if n == 0:
            return []
        base, extra = divmod(total, n)
        return [base + 1] * extra + [base] * (n - extra)

    def _gpus_available(self):
        ledger = getattr(self._cm, 'ledger', None)
        return bool(ledger and ledger.free)

    def _create_service(self, service_type, docker_image, args, environment_vars, container_port=None, gpus=0,
                        replicas=1, before_launch=None):
        """DB row -> (caller's rows) -> DEPLOYING -> launch -> record container info.  Everything the
        service reads at start-up exists before it is launched, and the launched service is the
        only writer of its later statuses (RUNNING/STOPPED/ERRORED)."""
        svc = self._db.create_service(service_type, type(self._cm).__name__, docker_image, replicas, gpus)
        if before_launch is not None:
            before_launch(svc)
        env = {'RAFIKI_SERVICE_ID': svc.id, 'RAFIKI_SERVICE_TYPE': service_type, 'WORKDIR_PATH': self._cfg.workdir,
               'RAFIKI_DB_PATH': self._db.path, 'PYTHONPATH': os.pathsep.join(p for p in sys.path if p)}
        env.update(environment_vars)
        publish = None
        if container_port is not None:
            publish = (free_port(), container_port)
        name = 'rafiki-{}-{}'.format(service_type.lower(), svc.id[:8])
        self._db.mark_service_as_deploying(svc, name, None, None, None, None, None, None)
        try:
            cs: ContainerService = self._cm.create_service(name, docker_image, args, env, None, replicas, publish, gpus)
        except Exception:
            self._db.mark_service_as_errored(svc)
            raise
        self._db.update_service_container_info(svc, cs.id, cs.hostname, cs.port,
                                               self._cfg.admin_host if cs.port else None, cs.port, cs.info)
        return svc

    def _stop_service(self, service):
        if service is None or service.status == ServiceStatus.STOPPED:
            return
        try:
            self._cm.destroy_service(ContainerService(service.container_service_id, service.hostname, service.port,
                                                      service.container_service_info))
        except Exception:
            logger.info('error stopping service %s (maybe already stopped)', service.id)
        self._db.mark_service_as_stopped(service)

    def _wait_until_services_running(self, services, accept_stopped=False):
        deadline = time.time() + self._wait_timeout_s
        for s in services:
            while True:
                cur = self._db.get_service(s.id)
                if cur.status == ServiceStatus.RUNNING or (accept_stopped and cur.status == ServiceStatus.STOPPED):
                    break
                if cur.status in (ServiceStatus.ERRORED, ServiceStatus.STOPPED):
                    raise ServiceDeploymentError('service {} is {}'.format(s.id, cur.status))
                if time.time() > deadline:
                    raise ServiceDeploymentError('timeout waiting for service {}'.format(s.id))
                time.sleep(min(config.SERVICE_STATUS_WAIT, 0.1))
