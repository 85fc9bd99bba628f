"""Environment-driven fault injection for failure-path tests.

``RAFIKI_FAULT_INJECT`` holds ';'-separated rules ``<point>[:key=value,...]``; a rule fires when
the code reaches ``maybe_fail(point, **ctx)`` and every key given in the rule matches ``ctx``
(``step`` / ``epoch`` compare with >=, other keys by string equality).  Points and effects:

  train_step   -> raise TrialFault (ordinary Exception: the trial is marked ERRORED)
  crash        -> raise WorkerCrash (BaseException: unwinds past the trial handler like a killed
                  process would; with ``exit=1`` the process calls os._exit(17) instead)
  nan_grad     -> maybe_corrupt(tensor) fills a gradient with NaN (tests the non-finite skip)

Rules fire at most ``times`` times per process (default 1).  Example:
``RAFIKI_FAULT_INJECT="crash:epoch=1,rank=0"`` — rank 0 dies after finishing epoch 1.
"""
from __future__ import annotations

import os
import threading

_lock = threading.Lock()
_fired = {}


class TrialFault(Exception):
    pass


class WorkerCrash(BaseException):
    pass


def _rules():
    spec = os.environ.get('RAFIKI_FAULT_INJECT', '').strip()
    out = []
    for i, part in enumerate(p for p in spec.split(';') if p.strip()):
        point, _, args = part.strip().partition(':')
        kv = {}
        for a in args.split(','):
            if '=' in a:
                k, v = a.split('=', 1)
                kv[k.strip()] = v.strip()
        out.append((i, point.strip(), kv))
    return out


def _matches(kv, ctx):
    for k, v in kv.items():
        if k in ('times', 'exit'):
            continue
        if k not in ctx:
            return False
        if k in ('step', 'epoch'):
            if float(ctx[k]) < float(v):
                return False
        elif str(ctx[k]) != v:
            return False
    return True


def _take(i, kv):
    with _lock:
        n = _fired.get(i, 0)
        if n >= int(kv.get('times', 1)):
            return False
        _fired[i] = n + 1
        return True


def should_fire(point, **ctx) -> bool:
    for i, p, kv in _rules():
        if p == point and _matches(kv, ctx) and _take(i, kv):
            return True
    return False


def maybe_fail(point, **ctx):
    for i, p, kv in _rules():
        if p != point or not _matches(kv, ctx) or not _take(i, kv):
            continue
        if point == 'crash':
            if kv.get('exit') == '1':
                os._exit(17)
            raise WorkerCrash('injected crash at {} {}'.format(point, ctx))
        raise TrialFault('injected fault at {} {}'.format(point, ctx))


def maybe_corrupt(tensor, **ctx):
    if should_fire('nan_grad', **ctx):
        tensor.fill_(float('nan'))
        return True
    return False


def reset():
    with _lock:
        _fired.clear()
