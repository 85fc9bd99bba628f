"""Process wrapper for dynamic services: logging, SIGTERM/SIGINT, DB status transitions.

Reference parity: rafiki/utils/service.py:10-46 (``run_worker``): mark RUNNING, run, mark
STOPPED on clean exit and ERRORED on exception; signal handlers call ``stop``.  Extension: a
heartbeat thread stamps ``<workdir>/heartbeats/<service_id>`` so a supervisor can detect hangs
(SURVEY §5.3), and only rank 0 of an SPMD group writes service status.
"""
from __future__ import annotations

import logging
import os
import signal
import sys
import threading
import time
import traceback

from .log import configure_logging

logger = logging.getLogger(__name__)


def heartbeat_path(workdir, service_id, rank=0):
    return os.path.join(workdir, 'heartbeats', '{}.r{}'.format(service_id, rank))


def _heartbeat_loop(path, stop: threading.Event, period=2.0):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    while not stop.is_set():
        try:
            with open(path, 'w') as f:
                f.write(str(time.time()))
        except OSError:
            pass
        stop.wait(period)


def last_heartbeat(workdir, service_id, rank=0):
    try:
        with open(heartbeat_path(workdir, service_id, rank)) as f:
            return float(f.read().strip())
    except (OSError, ValueError):
        return None


def run_worker(db, start_worker, stop_worker, service_id=None, rank=0, workdir=None):
    service_id = service_id or os.environ.get('RAFIKI_SERVICE_ID')
    container_id = os.environ.get('HOSTNAME', 'localhost')
    configure_logging('service-{}-worker-{}-r{}'.format(service_id, container_id, rank))
    stop_hb = threading.Event()
    if workdir:
        threading.Thread(target=_heartbeat_loop, args=(heartbeat_path(workdir, service_id, rank), stop_hb),
                         daemon=True).start()

    def on_signal(signum, frame):
        logger.warning('received signal %s, stopping worker', signum)
        try:
            stop_worker()
        finally:
            stop_hb.set()
            sys.exit(0)

    signal.signal(signal.SIGTERM, on_signal)
    signal.signal(signal.SIGINT, on_signal)
    service = db.get_service(service_id) if service_id else None
    if service is not None and rank == 0:
        db.mark_service_as_running(service)
    try:
        start_worker(service_id, container_id)
        stop_worker()
        if service is not None and rank == 0:
            db.mark_service_as_stopped(db.get_service(service_id))
    except Exception:
        logger.error('worker failed:\n%s', traceback.format_exc())
        if service is not None:
            db.mark_service_as_errored(db.get_service(service_id))
        try:
            stop_worker()
        finally:
            stop_hb.set()
        raise
    stop_hb.set()
