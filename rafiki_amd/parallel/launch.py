"""Single-node rank launcher: one child process per GPU, spawned before the parent touches HIP.

The reference's unit of scale is one worker container per GPU of the ``GPU_COUNT`` budget
(rafiki/admin/services_manager.py:107-135, pinned through CUDA_VISIBLE_DEVICES in
container/docker_swarm.py:124-126).  Here the unit is one OS process per MI355X, joined into one
``torch.distributed`` group over RCCL/xGMI.  ``torchrun`` already provides that; this module is the
self-contained path used when a program (``bench.py --gpus N``) is started WITHOUT a launcher:

* children are started with ``subprocess`` (never ``exec``: replacing a process that has
  initialised the GPU is forbidden on this pool) and get RANK / LOCAL_RANK / WORLD_SIZE /
  MASTER_ADDR=127.0.0.1 / a free MASTER_PORT;
* the parent never initialises HIP (``torch.cuda.device_count()`` does not on this image);
* rank 0's stdout is relayed line by line, every other rank's stdout is prefixed; stderr is
  inherited;
* the parent exits non-zero as soon as any child fails, terminating the others (a rank that died
  would otherwise leave its peers blocked inside a collective until the RCCL timeout).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Sequence


def free_port(host: str = '127.0.0.1') -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def under_launcher() -> bool:
    """True when torchrun (or this module) already set up the rank environment."""
    return 'WORLD_SIZE' in os.environ and 'RANK' in os.environ


def rank_env(rank: int, world: int, port: int, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    # a parent started by torchrun: its elastic-agent variables would make the children's rendezvous
    # look for the agent's store (TORCHELASTIC_USE_AGENT_STORE) on a port nobody serves
    for k in [k for k in env if k.startswith('TORCHELASTIC_')]:
        del env[k]
    env.update({
        'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(world),
        'LOCAL_WORLD_SIZE': str(world), 'GROUP_RANK': '0',
        'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port),
        # dmabuf IPC: RCCL peer buffers on this host driver need it
        'HSA_ENABLE_IPC_MODE_LEGACY': env.get('HSA_ENABLE_IPC_MODE_LEGACY', '0'),
        'PYTHONUNBUFFERED': '1',
    })
    return env


def _pump(stream, rank: int, out, lock: threading.Lock):
    for line in iter(stream.readline, ''):
        with lock:
            if rank == 0:
                out.write(line)
            else:
                out.write('[rank{}] {}'.format(rank, line))
            out.flush()
    stream.close()


def spawn(cmd: Sequence[str], world: int, port: Optional[int] = None, out=None,
          poll_s: float = 0.05, env: Optional[Dict[str, str]] = None, timeout_s: Optional[float] = None) -> int:
    """Run ``cmd`` as ``world`` ranks; return 0 iff every rank exited 0.

    On the first failing rank the others are terminated (then killed after 10 s) and that rank's
    exit code is returned (1 for a signal).  With ``timeout_s``, ranks still running at the deadline
    are terminated the same way and 124 is returned (a hung collective ends the call, not the caller).
    """
    out = out or sys.stdout
    port = port or free_port()
    lock = threading.Lock()
    procs: List[subprocess.Popen] = []
    pumps = []
    for r in range(world):
        p = subprocess.Popen(list(cmd), env=rank_env(r, world, port, env), stdout=subprocess.PIPE,
                             text=True, bufsize=1, start_new_session=False)
        procs.append(p)
        t = threading.Thread(target=_pump, args=(p.stdout, r, out, lock), daemon=True)
        t.start()
        pumps.append(t)
    rc = 0
    failed = None
    deadline_all = None if timeout_s is None else time.time() + timeout_s
    while True:
        alive = 0
        for r, p in enumerate(procs):
            code = p.poll()
            if code is None:
                alive += 1
            elif code != 0 and failed is None:
                failed = r
                rc = code if code > 0 else 1
        if failed is not None or alive == 0:
            break
        if deadline_all is not None and time.time() > deadline_all:
            failed, rc = -1, 124
            break
        time.sleep(poll_s)
    if failed is not None:
        if failed < 0:
            sys.stderr.write('launch: ranks still running after {:.0f} s; terminating them\n'.format(timeout_s))
        else:
            sys.stderr.write('launch: rank {} exited with {}; terminating the other ranks\n'.format(
                failed, procs[failed].returncode))
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    for t in pumps:
        t.join(timeout=5)
    return rc


def check_devices(world: int, backend: str) -> None:
    """RCCL needs one GPU per rank: fail loudly instead of silently measuring fewer GPUs."""
    if backend != 'nccl':
        return
    import torch
    n = torch.cuda.device_count()   # does not initialise HIP on this image
    if n < world:
        raise SystemExit('launch: --gpus {} needs {} visible GPUs for the RCCL backend, found {} '
                         '(set RAFIKI_DIST_BACKEND=gloo to rehearse the control path with ranks sharing '
                         'one GPU)'.format(world, world, n))
