"""CPU tests of the node-wide autotune database (ops/autotune.py): keyed by arch + kernel-library
hash, shared by concurrent worker processes with flock-merged writes, seeded from a shipped db."""
import json
import multiprocessing as mp
import os

import pytest

from rafiki_amd.ops import autotune as A


@pytest.fixture
def fresh(monkeypatch, tmp_path):
    monkeypatch.setenv('WORKDIR_PATH', str(tmp_path))
    monkeypatch.delenv('RAFIKI_TUNE_CACHE', raising=False)
    monkeypatch.setattr(A, '_ident', {'arch': 'gfx950', 'lib': 'abc123def456'})
    monkeypatch.setattr(A, '_cache', {})
    monkeypatch.setattr(A, '_loaded', False)
    monkeypatch.setattr(A, '_disk_mtime', [None])
    monkeypatch.setattr(A, 'SHIPPED_DIR', str(tmp_path / 'shipped'))
    return tmp_path


def test_default_path_is_keyed_by_arch_and_library(fresh):
    assert A._path() == os.path.join(str(fresh), 'tune', 'gfx950-abc123def456.json')
    A._ident['lib'] = 'ffffffffffff'
    assert A._path().endswith('gfx950-ffffffffffff.json')


def test_off_disables_persistence(fresh, monkeypatch):
    monkeypatch.setenv('RAFIKI_TUNE_CACHE', 'off')
    assert A._path() == ''


def _writer(workdir, i, n):
    os.environ['WORKDIR_PATH'] = workdir
    os.environ.pop('RAFIKI_TUNE_CACHE', None)
    A._ident.update({'arch': 'gfx950', 'lib': 'abc123def456'})
    for j in range(n):
        with A._lock:
            A._cache[('conv', i, j)] = (i, j, 1)
        A._save()


def test_concurrent_processes_merge_not_clobber(fresh):
    ctx = mp.get_context('fork')
    ps = [ctx.Process(target=_writer, args=(str(fresh), i, 25)) for i in range(4)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    with open(A._path()) as f:
        d = json.load(f)
    assert len(d) == 100
    # a process that starts afterwards sees every entry
    assert A.lookup(('conv', 3, 24)) == (3, 24, 1)


def test_miss_rereads_entries_written_by_another_process(fresh):
    assert A.lookup(('gemm', 1)) is None
    p = mp.get_context('fork').Process(target=_writer, args=(str(fresh), 7, 1))
    p.start()
    p.join(60)
    assert A.lookup(('conv', 7, 0)) == (7, 0, 1)
    assert A.stats['reloads'] >= 1


def test_shipped_db_seeds_the_cache(fresh):
    os.makedirs(fresh / 'shipped')
    with open(fresh / 'shipped' / 'gfx950-abc123def456.json', 'w') as f:
        json.dump({json.dumps(['gemm', 64, 64]): [128, 0, 1]}, f)
    assert A.lookup(('gemm', 64, 64)) == (128, 0, 1)
