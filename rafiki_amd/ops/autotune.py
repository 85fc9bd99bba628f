"""Per-shape kernel-config autotuning for the igemm engine (find-once, replay-forever).

The best (tile shape, staging variant, split-K) differs per layer shape (measured on MI355X with
scripts/dev/bench_igemm.py: e.g. the LDS-DMA 2-stage ring wins on 16x16/8x8 layers, 64x64 register
staging on the 4x4x512 layers).  The first time a shape is seen outside hipGraph capture, every
candidate runs a few times under HIP events and the fastest is cached.  During capture only
cached/heuristic configs are used, so captured graphs never contain tuning launches.

The cache is a node-wide tuning database (MIOpen's perf-db idea), keyed by what the timings depend on:

* file ``<WORKDIR>/tune/<gfx arch>-<kernel source hash>.json`` (``RAFIKI_TUNE_CACHE`` overrides the
  path, ``RAFIKI_TUNE_CACHE=off`` keeps it in memory only).  A rebuilt kernel library or another GPU
  architecture starts a fresh file, so stale picks are never replayed;
* every worker process of the node shares it: a miss re-reads the file if another rank wrote it
  since, and writes are merged under an exclusive ``flock`` (read + merge + atomic replace), so
  concurrent ranks never drop each other's entries;
* a read-only database shipped in the package (``rafiki_amd/tune/<arch>-<hash>.json``) seeds it,
  so a fresh node whose kernel library matches starts warm.
"""
from __future__ import annotations

import fcntl
import hashlib
import json
import os
import sys
import threading

import torch

from .graphs import LOCK as _GRAPH_LOCK, capture as _capture

_lock = threading.Lock()
_cache = {}
_loaded = False
_disk_mtime = [None]
stats = {'tuned': 0, 'seconds': 0.0, 'candidates': 0, 'loaded': 0, 'reloads': 0}
_last_note = [0.0]
ENABLED = os.environ.get('RAFIKI_AUTOTUNE', '1') != '0'
REPS = 3      # timed replays per candidate and pass (at least 5 when timing a captured graph)
PASSES = 2    # sweeps over the candidates, min per candidate (the first also absorbs clock ramp-up)
SHIPPED_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tune')
_ident = {}


def _arch() -> str:
    if 'arch' not in _ident:
        try:
            name = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
            _ident['arch'] = name.split(':')[0]
        except Exception:
            _ident['arch'] = os.environ.get('RAFIKI_OFFLOAD_ARCH', 'gfx950')
    return _ident['arch']


_SRC_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), 'csrc',
                        'kernels')


def lib_hash() -> str:
    """Hash of the kernel library the picks were timed with (12 hex digits): of the kernel SOURCES when the
    tree has them (hipcc output is not byte-reproducible — it embeds temporary file names — so a rebuild
    of unchanged sources keeps its database), else of the library bytes."""
    if 'lib' not in _ident:
        h = hashlib.sha1()
        try:
            srcs = sorted(f for f in os.listdir(_SRC_DIR) if f.endswith(('.hip', '.h')))
        except OSError:
            srcs = []
        try:
            if srcs:
                for f in srcs:
                    h.update(f.encode())
                    with open(os.path.join(_SRC_DIR, f), 'rb') as fh:
                        h.update(fh.read())
                _ident['lib'] = 's' + h.hexdigest()[:11]
            else:
                from ._lib import loaded_path as lib_path
                with open(lib_path(), 'rb') as f:
                    for chunk in iter(lambda: f.read(1 << 20), b''):
                        h.update(chunk)
                _ident['lib'] = h.hexdigest()[:12]
        except OSError:
            _ident['lib'] = 'nolib'
    return _ident['lib']


# switches that change the candidate sets (not the kernels): a non-default setting tunes into its own
# database file, so a pick made among more candidates is never replayed where they are switched off
_CAND_SWITCHES = ('RAFIKI_X6', 'RAFIKI_PT_MAX_HW', 'RAFIKI_WINOGRAD', 'RAFIKI_WINOGRAD4')


def db_name() -> str:
    tag = ','.join('{}={}'.format(k, os.environ[k]) for k in _CAND_SWITCHES if k in os.environ)
    suffix = '-' + hashlib.sha1(tag.encode()).hexdigest()[:8] if tag else ''
    return '{}-{}{}.json'.format(_arch(), lib_hash(), suffix)


def _path():
    p = os.environ.get('RAFIKI_TUNE_CACHE')
    if p is not None and p.lower() in ('off', '0', 'none', ''):
        return ''
    if p:
        return p
    from ..config import get_config
    return os.path.join(get_config().workdir, 'tune', db_name())


def _tup(v):
    """JSON lists back to the (nested) tuples used as cache keys / configs."""
    return tuple(_tup(x) for x in v) if isinstance(v, list) else v


def _read(path):
    try:
        with open(path) as f:
            return {_tup(json.loads(k)): _tup(v) for k, v in json.load(f).items()}
    except (OSError, ValueError):
        return {}


def _load():
    global _loaded
    if _loaded:
        return
    _loaded = True
    shipped = os.path.join(SHIPPED_DIR, db_name())
    if os.path.exists(shipped):
        got = _read(shipped)
        _cache.update(got)
        stats['loaded'] += len(got)
    _refresh(force=True)


def _refresh(force=False):
    """Merge entries other processes wrote to the node database since we last looked."""
    p = _path()
    if not p:
        return
    try:
        m = os.stat(p).st_mtime_ns
    except OSError:
        return
    if not force and m == _disk_mtime[0]:
        return
    _disk_mtime[0] = m
    got = _read(p)
    for k, v in got.items():
        _cache.setdefault(k, v)
    stats['loaded'] += len(got)
    stats['reloads'] += 1


def _save():
    p = _path()
    if not p:
        return
    try:
        os.makedirs(os.path.dirname(p) or '.', exist_ok=True)
        with open(p + '.lock', 'a+') as lf:
            fcntl.flock(lf, fcntl.LOCK_EX)
            try:
                merged = _read(p)
                merged.update(_cache)       # this process's fresh timings win on a clash
                tmp = '{}.{}.tmp'.format(p, os.getpid())
                with open(tmp, 'w') as f:
                    json.dump({json.dumps(k): v for k, v in merged.items()}, f)
                os.replace(tmp, p)
                _disk_mtime[0] = os.stat(p).st_mtime_ns
                for k, v in merged.items():
                    _cache.setdefault(k, v)
            finally:
                fcntl.flock(lf, fcntl.LOCK_UN)
    except OSError:
        pass


def lookup(key):
    with _lock:
        _load()
        hit = _cache.get(key)
        if hit is None:
            _refresh()
            hit = _cache.get(key)
        return hit


def can_tune():
    if not ENABLED or not torch.cuda.is_available():
        return False
    try:
        return not torch.cuda.is_current_stream_capturing()
    except Exception:
        return False


def _time_graph(cfg, run, reps):
    """GPU time of ``reps`` back-to-back launches, captured into a hipGraph so host launch overhead
    (10-20 us per op from Python) does not swamp kernels that take a few microseconds."""
    run(cfg)  # warm: first-touch allocations happen outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with _capture(g):
        for _ in range(reps):
            run(cfg)
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    g.replay()
    e.record()
    e.synchronize()
    t = s.elapsed_time(e) / (2 * reps)
    del g
    return t


def _time_eager(cfg, run, reps):
    run(cfg)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        run(cfg)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def _valid(hit, candidates):
    """A stored pick is used only if it is still one of this call's candidates (a database written by other
    candidate-generation code, or for a key whose candidate set changed, is never replayed blindly)."""
    return hit is not None and tuple(hit) in {tuple(c) for c in candidates}


def tune(key, candidates, run):
    """candidates: list of config tuples; run(cfg) launches the op once.  Returns the best cfg."""
    hit = lookup(key)
    if _valid(hit, candidates):
        return tuple(hit)
    if hit is not None:
        stats['stale'] = stats.get('stale', 0) + 1
    if not can_tune():
        return candidates[0]
    with _GRAPH_LOCK:   # sweeps time captured graphs: never interleave with another thread's capture
        hit = lookup(key)
        if _valid(hit, candidates):
            return tuple(hit)
        return _tune_locked(key, candidates, run)


def _tune_locked(key, candidates, run):
    import time as _time
    t_start = _time.perf_counter()
    use_graph = True   # candidates timed inside a captured hipGraph (host launch overhead excluded)
    # PASSES sweeps over the candidates, min per candidate: the first sweep also absorbs clock
    # ramp-up after idle, which otherwise penalises whichever candidates happen to run first
    times = {}
    for _ in range(PASSES):
        for cfg in candidates:
            if times.get(cfg, 0.0) == float('inf'):
                continue
            try:
                t = _time_graph(cfg, run, max(REPS, 5)) if use_graph else _time_eager(cfg, run, REPS)
            except (NameError, TypeError, AttributeError, KeyError, IndexError, UnboundLocalError):
                raise   # a bug in the candidate's Python path, never "this config does not apply here"
            except Exception as e:   # KernelError (unsupported shape), capture / launch failures, asserts
                try:
                    torch.cuda.synchronize()
                except Exception:
                    pass
                t = float('inf')
                stats['failed'] = stats.get('failed', 0) + 1
                if os.environ.get('RAFIKI_AUTOTUNE_VERBOSE'):
                    print('autotune: candidate {} of {} failed: {!r}'.format(cfg, key, e), flush=True)
            times[cfg] = min(times.get(cfg, float('inf')), t)
    best = min(candidates, key=lambda c: times.get(c, float('inf')))
    best_t = times.get(best, float('inf'))
    log = os.environ.get('RAFIKI_AUTOTUNE_LOG', '')
    if log:
        try:
            with open(log, 'a') as f:
                f.write(json.dumps({'key': [str(k) for k in key], 'best': list(best), 'us': round(best_t * 1e3, 2),
                                    'first_us': round(times.get(candidates[0], float('inf')) * 1e3, 2),
                                    'all': {str(list(c)): round(t * 1e3, 2) for c, t in times.items()}}) + '\n')
        except OSError:
            pass
    with _lock:
        _cache[key] = tuple(best)
        _save()
        stats['tuned'] += 1
        stats['candidates'] += len(candidates)
        stats['seconds'] += _time.perf_counter() - t_start
        now = _time.perf_counter()
        if now - _last_note[0] > 30.0:   # a long in-process tuning pass says it is alive (stderr)
            _last_note[0] = now
            sys.stderr.write('[autotune] {} shapes tuned in {:.0f} s\n'.format(stats['tuned'], stats['seconds']))
            sys.stderr.flush()
    return best


def clear():
    with _lock:
        _cache.clear()


def snapshot():
    with _lock:
        return dict(_cache)
