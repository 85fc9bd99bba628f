"""Service orchestration on one MI355X node (replaces Docker Swarm).

Reference parity: rafiki/container/container_manager.py (:7-45, abstract ``ContainerManager``
contract: restart on non-zero exit, not on exit 0) and docker_swarm.py (:14-181, GPU ledger kept
in node labels).

``LocalProcessManager`` runs every service as a process group on this node:
  * a GPU ledger hands out physical GPU ids (replaces `available_gpus` node labels);
  * a service with ``gpus = N > 1`` is an SPMD group of N processes (one per GPU) with
    torchrun-style env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR=127.0.0.1/MASTER_PORT) so the group
    can form an RCCL process group over xGMI — trial-parallel HPO or data-parallel training;
  * ``HIP_VISIBLE_DEVICES`` lists the group's GPUs; rank r uses device r;
  * a monitor thread restarts a replica that exits non-zero (bounded retries) and reports exits;
  * ``InProcessManager`` runs a service's entry function in threads (tests, CPU-only).
"""
from __future__ import annotations

import abc
import itertools
import logging
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import uuid
from contextlib import closing
from typing import Callable, Dict, List, Optional

logger = logging.getLogger(__name__)


class ContainerService:
    def __init__(self, id, hostname, port, info=None):
        self.id = id
        self.hostname = hostname
        self.port = port
        self.info = info or {}


class ContainerManager(abc.ABC):
    @abc.abstractmethod
    def create_service(self, service_name, docker_image, args, environment_vars, mounts=None, replicas=1,
                       publish_port=None, gpus=0) -> ContainerService:
        """Start a service; if it exits non-zero it is restarted, on exit 0 it is not."""

    @abc.abstractmethod
    def destroy_service(self, service: ContainerService):
        """Stop a service and release its resources."""


def free_port(host='127.0.0.1') -> int:
    with closing(socket.socket(socket.AF_INET, socket.SOCK_STREAM)) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


class GpuLedger:
    """Which physical GPUs of this node are in use (thread-safe)."""

    def __init__(self, gpu_ids: Optional[List[int]] = None):
        if gpu_ids is None:
            n = int(os.environ.get('RAFIKI_GPUS_PER_NODE', '0') or 0)
            if n == 0:
                try:
                    import torch
                    n = torch.cuda.device_count()
                except Exception:
                    n = 0
            gpu_ids = list(range(n))
        self._free = list(gpu_ids)
        self._lock = threading.Lock()

    def acquire(self, n: int) -> List[int]:
        with self._lock:
            if n > len(self._free):
                raise RuntimeError('requested {} GPUs, {} free'.format(n, len(self._free)))
            got, self._free = self._free[:n], self._free[n:]
            return got

    def release(self, ids: List[int]):
        with self._lock:
            self._free = sorted(set(self._free) | set(ids))

    @property
    def free(self):
        with self._lock:
            return list(self._free)


class LocalProcessManager(ContainerManager):
    def __init__(self, gpu_ids: Optional[List[int]] = None, logs_dir: Optional[str] = None, max_restarts: int = 2,
                 python: str = sys.executable):
        self.ledger = GpuLedger(gpu_ids)
        self.logs_dir = logs_dir
        self.max_restarts = max_restarts
        self.python = python
        self._services: Dict[str, dict] = {}
        self._lock = threading.Lock()
        self._exit_callbacks: List[Callable] = []

    def on_exit(self, cb: Callable):
        self._exit_callbacks.append(cb)

    def create_service(self, service_name, docker_image, args, environment_vars, mounts=None, replicas=1,
                       publish_port=None, gpus=0):
        gpu_ids = self.ledger.acquire(gpus) if gpus > 0 else []
        world = max(1, gpus, replicas if gpus == 0 else gpus)
        master_port = free_port()
        host_port = None
        if publish_port is not None:
            host_port = int(publish_port[0]) if publish_port[0] else free_port()
        svc = {'name': service_name, 'gpus': gpu_ids, 'procs': [], 'restarts': 0, 'stopped': False,
               'args': list(args or []), 'env': dict(environment_vars or {}), 'world': world,
               'master_port': master_port, 'host_port': host_port}
        sid = 'local-' + uuid.uuid4().hex[:12]
        for r in range(world):
            svc['procs'].append(self._spawn(svc, r))
        with self._lock:
            self._services[sid] = svc
        threading.Thread(target=self._monitor, args=(sid,), daemon=True, name='svc-monitor-' + sid).start()
        info = {'gpus': gpu_ids, 'pids': [p.pid for p in svc['procs']], 'world_size': world,
                'master_port': master_port, 'node_id': socket.gethostname()}
        return ContainerService(sid, '127.0.0.1', host_port, info)

    def _spawn(self, svc, rank):
        env = dict(os.environ)
        env.update({k: str(v) for k, v in svc['env'].items()})
        env.update({'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(svc['world']),
                    'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(svc['master_port'])})
        env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
        if env.get('RAFIKI_DEBUG_SYNC', '0') not in ('', '0'):
            # race/fault triage: every kernel launch serialised and synchronous, so a
            # faulting kernel is reported at its own launch instead of at a later sync point
            env['AMD_SERIALIZE_KERNEL'] = '3'
            env['AMD_SERIALIZE_COPY'] = '3'
            env['HIP_LAUNCH_BLOCKING'] = '1'
        if svc['gpus']:
            env['HIP_VISIBLE_DEVICES'] = ','.join(str(g) for g in svc['gpus'])
        else:
            env['HIP_VISIBLE_DEVICES'] = ''
            env['RAFIKI_CPU_ONLY'] = '1'
        if svc['host_port'] is not None:
            env['RAFIKI_SERVICE_PORT'] = str(svc['host_port'])
        out = subprocess.DEVNULL
        if self.logs_dir:
            os.makedirs(self.logs_dir, exist_ok=True)
            out = open(os.path.join(self.logs_dir, '{}-r{}.log'.format(svc['name'], rank)), 'ab')
        return subprocess.Popen([self.python, *svc['args']], env=env, stdout=out, stderr=subprocess.STDOUT,
                                start_new_session=True)

    def _monitor(self, sid):
        while True:
            with self._lock:
                svc = self._services.get(sid)
            if svc is None or svc['stopped']:
                return
            codes = [p.poll() for p in svc['procs']]
            if all(c is not None for c in codes):
                if any(c != 0 for c in codes) and svc['restarts'] < self.max_restarts and not svc['stopped']:
                    svc['restarts'] += 1
                    logger.warning('service %s exited %s; restart %d', sid, codes, svc['restarts'])
                    svc['master_port'] = free_port()
                    svc['started_at'] = time.time()
                    svc['procs'] = [self._spawn(svc, r) for r in range(svc['world'])]
                    continue
                for cb in self._exit_callbacks:
                    try:
                        cb(sid, codes)
                    except Exception:
                        logger.exception('exit callback failed')
                self._release(sid)
                return
            if any(c is not None and c != 0 for c in codes):
                # one rank died: tear the group down so collectives cannot hang, then restart
                for p in svc['procs']:
                    if p.poll() is None:
                        self._kill(p)
            elif self._stale(svc):
                # a live process whose heartbeat stopped (hung collective, wedged kernel): kill the
                # group; the non-zero exit then goes through the restart policy above
                logger.warning('service %s heartbeat stale for > %.0fs; killing it', sid, self.heartbeat_timeout)
                for p in svc['procs']:
                    if p.poll() is None:
                        self._kill(p)
            time.sleep(0.5)

    heartbeat_timeout = float(os.environ.get('RAFIKI_HEARTBEAT_TIMEOUT_S', '600'))

    def _stale(self, svc):
        """True when any rank of a heartbeating service has been silent for heartbeat_timeout."""
        from ..utils.service import last_heartbeat
        workdir = svc['env'].get('WORKDIR_PATH') or os.environ.get('WORKDIR_PATH')
        sid = svc['env'].get('RAFIKI_SERVICE_ID')
        if not workdir or not sid or self.heartbeat_timeout <= 0:
            return False
        now = time.time()
        started = svc.setdefault('started_at', now)
        for r in range(svc['world']):
            hb = last_heartbeat(workdir, sid, r)
            ref = hb if hb is not None and hb >= started else started
            if now - ref > self.heartbeat_timeout:
                return True
        return False

    @staticmethod
    def _kill(p, grace=10.0):
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except (ProcessLookupError, PermissionError):
            return
        try:
            p.wait(timeout=grace)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass

    def _release(self, sid):
        with self._lock:
            svc = self._services.pop(sid, None)
        if svc is not None:
            self.ledger.release(svc['gpus'])

    def destroy_service(self, service: ContainerService):
        with self._lock:
            svc = self._services.get(service.id)
        if svc is None:
            return
        svc['stopped'] = True
        for p in svc['procs']:
            if p.poll() is None:
                self._kill(p)
        self._release(service.id)

    def is_running(self, service_id) -> bool:
        with self._lock:
            svc = self._services.get(service_id)
        return svc is not None and any(p.poll() is None for p in svc['procs'])


class InProcessManager(ContainerManager):
    """Runs ``target(service_env)`` in daemon threads — for tests and CPU-only deployments."""

    def __init__(self, target: Callable[[dict], None]):
        self.target = target
        self._threads: Dict[str, list] = {}
        self._envs: Dict[str, dict] = {}
        self._ids = itertools.count()

    def create_service(self, service_name, docker_image, args, environment_vars, mounts=None, replicas=1,
                       publish_port=None, gpus=0):
        sid = 'inproc-{}'.format(next(self._ids))
        threads = []
        for r in range(max(1, replicas if gpus == 0 else 1)):
            env = dict(environment_vars or {})
            env.update({'RANK': '0', 'WORLD_SIZE': '1', 'LOCAL_RANK': '0'})
            if publish_port is not None:
                env['RAFIKI_SERVICE_PORT'] = str(publish_port[0])
            t = threading.Thread(target=self.target, args=(env,), daemon=True, name='{}-{}'.format(service_name, r))
            t.start()
            threads.append(t)
        self._threads[sid] = threads
        self._envs[sid] = dict(environment_vars or {})
        return ContainerService(sid, '127.0.0.1', publish_port[0] if publish_port else None, {'threads': len(threads)})

    def destroy_service(self, service):
        self._threads.pop(service.id, None)
        env = self._envs.pop(service.id, {})
        shutdown = getattr(self.target, 'shutdown_service', None)
        if shutdown is not None and 'RAFIKI_SERVICE_ID' in env:
            shutdown(env['RAFIKI_SERVICE_ID'])
