"""CPU tests of the single-node rank launcher behind ``bench.py --gpus N`` (rafiki_amd/parallel/launch.py)."""
import io
import json
import os
import subprocess
import sys
import textwrap

from rafiki_amd.parallel import launch as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent('''
    import json, os, sys
    rank = int(os.environ['RANK'])
    env = {k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT',
                                      'HSA_ENABLE_IPC_MODE_LEGACY')}
    print(json.dumps(env), flush=True)
    fail = int(sys.argv[1]) if len(sys.argv) > 1 else -1
    if rank == fail:
        sys.exit(3)
    if fail >= 0:
        import time; time.sleep(60)   # a healthy peer blocked "in a collective": must be terminated
''')


def _script(tmp_path):
    p = tmp_path / 'child.py'
    p.write_text(CHILD)
    return str(p)


def test_spawn_sets_rank_env_and_relays_rank0(tmp_path):
    out = io.StringIO()
    rc = L.spawn([sys.executable, _script(tmp_path)], 2, port=29911, out=out)
    assert rc == 0
    lines = out.getvalue().strip().splitlines()
    assert len(lines) == 2
    r0 = [json.loads(s) for s in lines if not s.startswith('[rank')]
    r1 = [json.loads(s.split('] ', 1)[1]) for s in lines if s.startswith('[rank1] ')]
    assert len(r0) == 1 and len(r1) == 1
    for r, e in ((0, r0[0]), (1, r1[0])):
        assert e['RANK'] == str(r) and e['LOCAL_RANK'] == str(r)
        assert e['WORLD_SIZE'] == '2'
        assert e['MASTER_ADDR'] == '127.0.0.1' and e['MASTER_PORT'] == '29911'
        assert e['HSA_ENABLE_IPC_MODE_LEGACY'] == '0'


def test_spawn_fails_fast_and_terminates_peers(tmp_path):
    import time
    t = time.time()
    rc = L.spawn([sys.executable, _script(tmp_path), '1'], 3, out=io.StringIO())
    assert rc == 3
    assert time.time() - t < 30   # the sleeping ranks were terminated, not waited for


def test_under_launcher(monkeypatch):
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.delenv('RANK', raising=False)
    assert not L.under_launcher()
    monkeypatch.setenv('WORLD_SIZE', '2')
    monkeypatch.setenv('RANK', '0')
    assert L.under_launcher()


def test_bench_gpus2_without_gpus_fails_loudly():
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'RAFIKI_DIST_BACKEND'):
        env.pop(k, None)
    env['HIP_VISIBLE_DEVICES'] = ''
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--steps', '1',
                        '--warmup', '0'], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert 'needs 2 visible GPUs' in (r.stderr + r.stdout)


def test_bench_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE='2', RANK='0', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '4'], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert 'WORLD_SIZE=2 but --gpus 4' in (r.stderr + r.stdout)


def test_spawn_timeout_terminates_hung_ranks(tmp_path, monkeypatch):
    """A hung child group (e.g. a collective that never completes) ends at the deadline with 124, and a
    torchrun parent's elastic-agent variables are not passed to the children (their rendezvous would
    look for the agent's store)."""
    import time
    p = tmp_path / 'hang.py'
    p.write_text('import json, os, sys, time\n'
                 'print(json.dumps(sorted(k for k in os.environ if k.startswith("TORCHELASTIC_"))), flush=True)\n'
                 'time.sleep(60)\n')
    monkeypatch.setenv('TORCHELASTIC_USE_AGENT_STORE', 'True')
    out = io.StringIO()
    t = time.time()
    rc = L.spawn([sys.executable, str(p)], 2, out=out, timeout_s=3)
    assert rc == 124
    assert time.time() - t < 30
    r0 = [ln for ln in out.getvalue().splitlines() if ln.startswith('[')and not ln.startswith('[rank')]
    assert r0 and all(json.loads(ln) == [] for ln in r0), out.getvalue()
