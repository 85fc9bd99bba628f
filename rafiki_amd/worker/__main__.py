"""Worker process entry: ``python -m rafiki_amd.worker`` (reference scripts/start_worker.py:1-34).

Reads RAFIKI_SERVICE_ID / RAFIKI_SERVICE_TYPE and the torchrun-style RANK/WORLD_SIZE env set by
``LocalProcessManager``.  TRAIN services join an RCCL (or gloo) process group and run the
``TrainWorker`` trial loop.  ``WORKER_INSTALL_COMMAND`` is NOT executed blindly (there is no
package index on the node): missing dependencies are only reported.
"""
import logging
import os
import sys


def main():
    from ..config import get_config
    from ..constants import ServiceType
    from ..db.database import Database
    from ..parallel import dist as D
    from ..utils.service import run_worker

    service_id = os.environ['RAFIKI_SERVICE_ID']
    service_type = os.environ.get('RAFIKI_SERVICE_TYPE', ServiceType.TRAIN)
    install = os.environ.get('WORKER_INSTALL_COMMAND', '')
    if install:
        logging.getLogger(__name__).warning('missing model dependencies (not installed, offline node): %s', install)
    db = Database()
    cfg = get_config()
    if service_type == ServiceType.TRAIN:
        from .train import TrainWorker
        backend = 'gloo' if os.environ.get('RAFIKI_CPU_ONLY') == '1' else None
        info = D.init_distributed(backend=backend)
        host = os.environ.get('HOSTNAME', 'localhost')
        worker_id = host if info.world_size == 1 else '{}-r{}'.format(host, info.rank)  # per-rank (resume)
        worker = TrainWorker(service_id, worker_id, db=db, dist_info=info)
        try:
            run_worker(db, lambda sid, cid: worker.start(), worker.stop, service_id=service_id, rank=info.rank,
                       workdir=cfg.workdir)
        finally:
            D.destroy(info)
    elif service_type == ServiceType.INFERENCE:
        from .inference import InferenceWorker
        worker = InferenceWorker(service_id, db=db)
        run_worker(db, lambda sid, cid: worker.start(), worker.stop, service_id=service_id, workdir=cfg.workdir)
    else:
        raise SystemExit('unknown service type {}'.format(service_type))


if __name__ == '__main__':
    sys.exit(main())
