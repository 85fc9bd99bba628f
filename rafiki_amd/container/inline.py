"""Run services inside the current process (threads): CPU-only deployments and end-to-end tests.

Used with ``InProcessManager``: ``InProcessManager(InlineServiceRunner(db_path))``.  TRAIN
services run a single-rank ``TrainWorker``; PREDICT services serve the predictor's Flask app on
the published port from a background thread.
"""
from __future__ import annotations

import logging
import threading
import traceback

logger = logging.getLogger(__name__)


class InlineServiceRunner:
    def __init__(self, db_path):
        self.db_path = db_path
        self.servers = {}

    def __call__(self, env):
        from ..constants import ServiceType
        from ..db.database import Database
        db = Database(self.db_path)
        sid = env['RAFIKI_SERVICE_ID']
        stype = env.get('RAFIKI_SERVICE_TYPE')
        try:
            if stype == ServiceType.TRAIN:
                from ..parallel.dist import DistInfo
                from ..worker.train import TrainWorker
                db.mark_service_as_running(db.get_service(sid))
                TrainWorker(sid, 'inline', db=db, dist_info=DistInfo(), offer_resident=True).start()
                db.mark_service_as_stopped(db.get_service(sid))
                w = db.get_train_job_worker(sid)
                if w is not None:
                    from ..admin.services_manager import ServicesManager
                    sub = db.get_sub_train_job(w.sub_train_job_id)
                    ServicesManager(db, None).refresh_train_job_status(sub.train_job_id)
            elif stype == ServiceType.PREDICT:
                from ..predictor.nativeserve import make_server
                from ..predictor.predictor import Predictor
                predictor = Predictor.from_inference_job(env['RAFIKI_INFERENCE_JOB_ID'], db=db)
                srv = make_server(predictor, '127.0.0.1', int(env['RAFIKI_SERVICE_PORT'])).start()
                self.servers[sid] = srv
                db.mark_service_as_running(db.get_service(sid))
        except Exception:
            logger.error('inline service %s failed:\n%s', sid, traceback.format_exc())
            db.mark_service_as_errored(db.get_service(sid))

    def shutdown_service(self, service_id):
        srv = self.servers.pop(service_id, None)
        if srv is not None:
            threading.Thread(target=srv.shutdown, daemon=True).start()

    def shutdown(self):
        for srv in self.servers.values():
            threading.Thread(target=srv.shutdown, daemon=True).start()
