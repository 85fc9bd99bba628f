"""The shipped autotune seed matches the kernel sources in the tree (CPU).

The seed is keyed by a hash of csrc/kernels/*.hip|*.h (ops.autotune.lib_hash); a kernel edit without
``python scripts/ship_tune_db.py --rekey`` (or a fresh capture) would leave the package without picks,
and every first call on a GPU box would tune from scratch.
"""
import json
import os

from rafiki_amd.ops import autotune


def test_shipped_seed_matches_kernel_sources(monkeypatch):
    for k in autotune._CAND_SWITCHES:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setitem(autotune._ident, 'arch', 'gfx950')
    monkeypatch.delitem(autotune._ident, 'lib', raising=False)
    name = autotune.db_name()
    assert name.startswith('gfx950-s'), name   # keyed by the sources, not the library bytes
    path = os.path.join(autotune.SHIPPED_DIR, name)
    shipped = sorted(f for f in os.listdir(autotune.SHIPPED_DIR) if f.startswith('gfx950-'))
    assert shipped == [name], 'seed {} vs kernel sources {}: run scripts/ship_tune_db.py --rekey'.format(
        shipped, name)
    with open(path) as f:
        entries = json.load(f)
    assert len(entries) > 100
