"""Host C++ runtime under AddressSanitizer + UBSan: build csrc/tests/test_runtime.cpp
(which includes the runtime sources) with -fsanitize=address,undefined and run its round-trip and
fuzz checks.  CPU only; sanitizers are applied to host code only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which('g++') is None, reason='g++ not available')
def test_runtime_asan_ubsan(tmp_path):
    exe = str(tmp_path / 'rt_test')
    src = os.path.join(ROOT, 'csrc', 'tests', 'test_runtime.cpp')
    subprocess.run(['g++', '-std=c++17', '-O1', '-g', '-fsanitize=address,undefined', '-fno-omit-frame-pointer',
                    '-fno-sanitize-recover=all', src, '-o', exe], check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: tolerate libraries the environment preloads ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=1:verify_asan_link_order=0',
               UBSAN_OPTIONS='print_stacktrace=1')
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'runtime tests ok' in r.stdout


def test_pylist_u8_matches_numpy():
    import numpy as np
    from rafiki_amd import runtime
    rng = np.random.default_rng(0)
    q = rng.integers(-20, 300, (5, 7, 3)).tolist()
    got = runtime.pylist_u8(q)
    assert got is not None and got.dtype == np.uint8
    assert (got == np.clip(np.asarray(q), 0, 255).astype(np.uint8)).all()
    f = (rng.random((4, 6)) * 400 - 50).tolist()
    assert (runtime.pylist_u8(f) == np.clip(np.asarray(f), 0, 255).astype(np.uint8)).all()
    assert runtime.pylist_u8([[1, 2], [3]]) is None          # ragged
    assert runtime.pylist_u8([['a', 'b']]) is None           # non-numeric
    assert runtime.pylist_u8(((1, 2), (3, 4))).tolist() == [[1, 2], [3, 4]]


def test_pylist_u8_caps_adversarial_shapes():
    """the first-element chain of a small ragged query must not size a huge allocation."""
    from rafiki_amd import runtime
    if runtime._pylib() is None:
        import pytest
        pytest.skip('pylist extension not built')
    q = [[list(range(3))] * 100000] + [[]] * 100000
    assert runtime.pylist_u8(q) is None          # refused without allocating 3e10 bytes
    assert runtime.pylist_u8([[1, 2], [3, 4]]).tolist() == [[1, 2], [3, 4]]
