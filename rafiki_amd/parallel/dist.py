"""Process-group plumbing for one MI355X node: one process per GPU, RCCL over xGMI.

``torch.distributed`` with backend ``"nccl"`` IS RCCL on ROCm.  CPU tests use ``"gloo"`` with the
same code path.  Knob sets and scores are exchanged as small packed tensors (a few hundred bytes:
latency-bound, ~10-20 us on xGMI), replacing the reference's HTTP advisor round trips
(worker/train.py:84-119).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from ..model.knob import CategoricalKnob, FixedKnob, FloatKnob, IntegerKnob


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = 'none'

    @property
    def is_main(self):
        return self.rank == 0


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600) -> DistInfo:
    """Initialise from torchrun-style env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', str(rank)))
    if ws <= 1:
        return DistInfo(0, 1, local, 'none')
    if backend is None:
        # NodeConfig.dist_backend (RAFIKI_DIST_BACKEND; gloo rehearses multi-rank control paths on a
        # one-GPU box, ranks sharing the device); RCCL needs one GPU per rank, so a host without GPUs
        # falls back to gloo
        from ..config import NodeConfig
        backend = NodeConfig().dist_backend
        if backend == 'nccl' and not torch.cuda.is_available():
            backend = 'gloo'
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29500')
    if backend == 'nccl':
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=rank, world_size=ws, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == 'nccl':
            kw['device_id'] = torch.device('cuda', local)
        dist.init_process_group(**kw)
    return DistInfo(rank, ws, local, backend)


def comm_device(info: DistInfo) -> torch.device:
    return torch.device('cuda', info.local_rank) if info.backend == 'nccl' else torch.device('cpu')


def barrier(info: DistInfo):
    if info.world_size > 1:
        if info.backend == 'nccl':
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


# ---------------------------------------------------------------------------- knob packing
def _knob_to_float(knob, value) -> float:
    if isinstance(knob, FixedKnob):
        return 0.0
    if isinstance(knob, CategoricalKnob):
        return float(knob.values.index(value))
    return float(value)


def _float_to_knob(knob, f: float):
    if isinstance(knob, FixedKnob):
        return knob.value
    if isinstance(knob, CategoricalKnob):
        return knob.values[int(round(f))]
    if isinstance(knob, IntegerKnob):
        return int(round(f))
    if isinstance(knob, FloatKnob):
        return float(f)
    raise TypeError(type(knob))


def pack_knobs(knob_config, proposals: List[dict]) -> torch.Tensor:
    """[Q, n_knobs] float64, columns in sorted knob-name order."""
    names = sorted(knob_config)
    rows = [[_knob_to_float(knob_config[n], p[n]) for n in names] for p in proposals]
    return torch.tensor(rows, dtype=torch.float64).reshape(len(proposals), len(names))


def unpack_knobs(knob_config, t: torch.Tensor) -> List[dict]:
    names = sorted(knob_config)
    out = []
    for row in t.detach().cpu().tolist():
        out.append({n: _float_to_knob(knob_config[n], v) for n, v in zip(names, row)})
    return out


def broadcast_proposals(info: DistInfo, knob_config, proposals: Optional[List[dict]]) -> List[dict]:
    """Rank 0 supplies ``world_size`` proposals; every rank gets the full list."""
    n = len(knob_config)
    if info.world_size == 1:
        return proposals
    dev = comm_device(info)
    if info.is_main:
        buf = pack_knobs(knob_config, proposals).to(dev)
    else:
        buf = torch.zeros((info.world_size, n), dtype=torch.float64, device=dev)
    dist.broadcast(buf, src=0)
    return unpack_knobs(knob_config, buf)


def gather_floats(info: DistInfo, values: List[float]) -> Optional[torch.Tensor]:
    """all_gather a small fp64 vector per rank -> [world, len] on every rank."""
    t = torch.tensor(values, dtype=torch.float64, device=comm_device(info))
    if info.world_size == 1:
        return t.unsqueeze(0).cpu()
    out = [torch.zeros_like(t) for _ in range(info.world_size)]
    dist.all_gather(out, t)
    return torch.stack(out).cpu()


def all_reduce_max(info: DistInfo, v: float) -> float:
    if info.world_size == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=comm_device(info))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_object(info: DistInfo, obj):
    """Rank 0's picklable ``obj`` on every rank (control-plane metadata: ids, small configs)."""
    if info.world_size == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=0, device=comm_device(info))
    return lst[0]


def world_size(info: DistInfo) -> int:
    """The process group's own size (not the env's claim); 1 without a group."""
    if info.world_size > 1 and dist.is_initialized():
        return dist.get_world_size()
    return 1


def destroy(info: DistInfo):
    if info.world_size > 1 and dist.is_initialized():
        dist.destroy_process_group()


def preflight(info: DistInfo, timeout_s: float = 120.0, group=None) -> dict:
    """Exercise every communication pattern a multi-rank job uses, once, before any timed or trial
    work: barrier, all_reduce (max), broadcast, all_gather and broadcast_object on the default group,
    then point-to-point rows rank 0 <-> every peer in both directions on ``group`` (the knob exchange's
    control group; its communicators are created here, not lazily mid-trial).  A watchdog ends the
    process with a message naming the step that did not complete within ``timeout_s`` (exit code 3)
    instead of hanging the node; returns {'ok', 'seconds', 'steps': {name: ms}}."""
    import sys
    import threading
    import time
    if info.world_size <= 1:
        return {'ok': True, 'seconds': 0.0, 'steps': {}, 'world_size': 1}
    state = {'step': 'start'}
    done = threading.Event()

    def watchdog():
        if not done.wait(timeout_s):
            sys.stderr.write('rafiki preflight: rank {} stuck in step {!r} for {:.0f} s (backend {}, world {}): '
                             'a peer is missing or the interconnect is not usable; aborting\n'.format(
                                 info.rank, state['step'], timeout_s, info.backend, info.world_size))
            sys.stderr.flush()
            os._exit(3)
    threading.Thread(target=watchdog, name='rafiki-preflight-watchdog', daemon=True).start()
    dev = comm_device(info)
    steps = {}
    t_all = time.perf_counter()

    def step(name, fn):
        state['step'] = name
        t0 = time.perf_counter()
        out = fn()
        if dev.type == 'cuda':
            torch.cuda.synchronize(dev)
        steps[name] = round((time.perf_counter() - t0) * 1e3, 3)
        return out
    try:
        step('barrier', lambda: barrier(info))
        mx = step('all_reduce_max', lambda: all_reduce_max(info, float(info.rank)))
        if mx != float(info.world_size - 1):
            raise RuntimeError('preflight: all_reduce max {} != {}'.format(mx, info.world_size - 1))

        def bcast():
            t = torch.full((4,), float(info.rank), dtype=torch.float64, device=dev)
            dist.broadcast(t, src=0)
            return float(t[0].item())
        if step('broadcast', bcast) != 0.0:
            raise RuntimeError('preflight: broadcast from rank 0 lost')
        table = step('all_gather', lambda: gather_floats(info, [float(info.rank)]))
        if table[:, 0].tolist() != [float(r) for r in range(info.world_size)]:
            raise RuntimeError('preflight: all_gather rows out of order: {}'.format(table[:, 0].tolist()))
        if step('broadcast_object', lambda: broadcast_object(info, 'rafiki' if info.is_main else None)) != 'rafiki':
            raise RuntimeError('preflight: broadcast_object lost')
        g = group if group is not None else dist.group.WORLD

        def p2p():
            for peer in range(1, info.world_size):
                if info.rank == peer:
                    t = torch.full((8,), float(peer), dtype=torch.float64, device=dev)
                    dist.send(t, dst=0, group=g)
                    r = torch.empty(8, dtype=torch.float64, device=dev)
                    dist.recv(r, src=0, group=g)
                    if float(r[0].item()) != -float(peer):
                        raise RuntimeError('preflight: rank 0 -> {} row corrupted'.format(peer))
                elif info.is_main:
                    r = torch.empty(8, dtype=torch.float64, device=dev)
                    dist.recv(r, src=peer, group=g)
                    if float(r[0].item()) != float(peer):
                        raise RuntimeError('preflight: rank {} -> 0 row corrupted'.format(peer))
                    dist.send(-r, dst=peer, group=g)
        step('p2p_rank0_pairs', p2p)
        step('barrier_end', lambda: barrier(info))
    finally:
        done.set()
    return {'ok': True, 'seconds': round(time.perf_counter() - t_all, 4), 'steps': steps,
            'world_size': info.world_size, 'backend': info.backend}
