"""Model SDK: knobs, logger, datasets, advisors, ensemble (CPU)."""
import json
import math
import os

import numpy as np
import pytest

from rafiki_amd.advisor import Advisor, GpAdvisor, RandomAdvisor, make_advisor
from rafiki_amd.constants import AdvisorType, TaskType
from rafiki_amd.model import (CategoricalKnob, FixedKnob, FloatKnob, IntegerKnob, ModelLogger, dataset_utils,
                              decode_knobs, deserialize_knob_config, encode_knobs, serialize_knob_config,
                              synthetic_images, write_corpus_zip, write_image_files_zip)
from rafiki_amd.predictor.ensemble import ensemble_predictions

KC = {
    'lr': FloatKnob(1e-4, 1e-1, is_exp=True),
    'units': IntegerKnob(2, 128),
    'bs': CategoricalKnob([16, 32, 64]),
    'flag': CategoricalKnob([True, False]),
    'act': CategoricalKnob(['relu', 'tanh']),
    'epochs': FixedKnob(3),
}


def test_knob_json_roundtrip_matches_reference_wire_format():
    s = serialize_knob_config(KC)
    d = json.loads(s)
    assert json.loads(d['lr']) == {'type': 'FloatKnob', 'args': {'value_min': 1e-4, 'value_max': 0.1, 'is_exp': True}}
    assert deserialize_knob_config(s) == KC


def test_bool_categorical_is_bool():  # reference bug (i)
    assert KC['flag'].value_type is bool
    assert KC['bs'].value_type is int


def test_knob_validation():
    with pytest.raises(ValueError):
        IntegerKnob(5, 1)
    with pytest.raises(TypeError):
        CategoricalKnob([1, 'a'])
    with pytest.raises(ValueError):
        FloatKnob(0.0, 1.0, is_exp=True)


def test_encode_decode_roundtrip():
    knobs = {'lr': 1e-3, 'units': 37, 'bs': 32, 'flag': False, 'act': 'tanh', 'epochs': 3}
    u = encode_knobs(KC, knobs)
    back = decode_knobs(KC, u)
    assert back['units'] == 37 and back['bs'] == 32 and back['flag'] is False and back['act'] == 'tanh'
    assert math.isclose(back['lr'], 1e-3, rel_tol=1e-9)


@pytest.mark.parametrize('kind', [AdvisorType.RANDOM, AdvisorType.BTB_GP])
def test_advisor_proposals_in_range(kind):
    a = make_advisor(KC, kind, seed=0)
    for _ in range(8):
        p = a.propose()
        assert 1e-4 <= p['lr'] <= 0.1 and 2 <= p['units'] <= 128 and p['bs'] in (16, 32, 64)
        assert isinstance(p['flag'], bool) and p['epochs'] == 3
        a.feedback(p, -abs(math.log10(p['lr']) + 2))


def test_gp_advisor_beats_random_on_smooth_objective():
    kc = {'x': FloatKnob(0.0, 1.0), 'y': FloatKnob(0.0, 1.0)}

    def f(p):
        return -((p['x'] - 0.3) ** 2 + (p['y'] - 0.7) ** 2)

    best = {}
    for name, cls in (('gp', GpAdvisor), ('rand', RandomAdvisor)):
        vals = []
        for seed in range(3):
            a = cls(kc, seed=seed)
            for _ in range(6):
                for p in a.propose_batch(4):
                    a.feedback(p, f(p))
            vals.append(a.best[1])
        best[name] = np.mean(vals)
    assert best['gp'] > best['rand']
    assert best['gp'] > -0.01


def test_batch_proposals_distinct_and_pending_respected():
    a = GpAdvisor({'x': FloatKnob(0.0, 1.0)}, seed=1)
    for p in a.propose_batch(4):
        a.feedback(p, p['x'])
    batch = a.propose_batch(8)
    xs = [round(p['x'], 6) for p in batch]
    assert len(set(xs)) == len(xs)


def test_reference_shaped_advisor_facade():
    a = Advisor(KC, AdvisorType.BTB_GP)
    p = a.propose()
    a.feedback(p, 0.5)
    assert len(a.history) == 1


def test_logger_roundtrip():
    lines = []

    class H:
        def info(self, line):
            lines.append(line)

    lg = ModelLogger()
    lg.set_logger(H())
    lg.define_loss_plot()
    lg.log('hello')
    lg.log_loss(0.5, 1)
    lg.log(acc=0.9, epoch=1)
    lines.append('not json')
    msgs, metrics, plots = ModelLogger.parse_logs(lines)
    assert plots == [{'title': 'Loss Over Epochs', 'metrics': ['loss'], 'x_axis': 'epoch', 'time': plots[0]['time']}]
    assert [m['message'] for m in msgs] == ['hello', 'not json']
    assert metrics[0]['loss'] == 0.5 and metrics[1]['acc'] == 0.9 and 'time' in metrics[0]


def test_image_files_zip_roundtrip(tmp_path):
    imgs, labels = synthetic_images(20, size=8, channels=1, classes=3, seed=0)
    p = write_image_files_zip(str(tmp_path / 'd.zip'), imgs, labels)
    ds = dataset_utils.load_dataset_of_image_files(p)
    x, y = ds.as_arrays()
    assert x.shape == (20, 8, 8) and np.array_equal(x, imgs) and np.array_equal(y, labels)
    assert ds.classes == int(labels.max()) + 1


def test_corpus_zip_roundtrip(tmp_path):
    sents = [[['a', 1], ['b', 2]], [['c', 0]]]
    p = write_corpus_zip(str(tmp_path / 'c.zip'), sents)
    ds = dataset_utils.load_dataset_of_corpus(p)
    assert ds.size == 2 and ds[0] == sents[0] and ds.tag_num_classes == [3] and ds.max_sent_len == 2


def test_synthetic_uris():
    ds = dataset_utils.load_dataset_of_image_files('synthetic://image?n=10&size=16&channels=3&classes=4')
    assert ds.images.shape == (10, 16, 16, 3)
    c = dataset_utils.load_dataset_of_corpus('synthetic://corpus?n=5')
    assert c.size == 5


def test_ensemble_predictions():
    preds = [[[0.2, 0.8], [1.0, 0.0]], [[0.6, 0.4], [0.0, 1.0]]]
    out = ensemble_predictions(preds, TaskType.IMAGE_CLASSIFICATION)
    assert np.allclose(out, [[0.4, 0.6], [0.5, 0.5]])
    assert ensemble_predictions([[[1, 2]], [[3, 4]]], TaskType.POS_TAGGING) == [[1, 2]]
    assert ensemble_predictions([], TaskType.IMAGE_CLASSIFICATION) == []


def test_graph_utils():
    from types import SimpleNamespace as NS
    from rafiki_amd.utils import graph as G
    subs = [NS(id='a', model_id='m1'), NS(id='b', model_id='m2'), NS(id='e', model_id='ens')]
    adj = G.build_dag(subs, NS(id='ens'))
    assert adj == {'a': ['e'], 'b': ['e'], 'e': []}
    assert G.topological_order(adj) == ['a', 'b', 'e'] and G.validate_dag(adj)
    assert G.get_parents('e', adj) == ['a', 'b'] and G.get_children('a', adj) == ['e']
    assert G.get_nodes_with_zero_incoming_degrees(adj) == ['a', 'b']
    assert not G.validate_dag({'x': ['y'], 'y': ['x']})
    assert G.build_dag(subs, None) == {'a': [], 'b': [], 'e': []}


def test_decoded_dataset_cache(tmp_path, monkeypatch):
    """A worker's trials decode an IMAGE_FILES dataset once; cached arrays are read-only, a
    rewritten file is re-decoded, and the byte budget evicts least-recently-used entries."""
    import os
    import numpy as np
    from rafiki_amd.model.dataset import ModelDatasetUtils, synthetic_images, write_image_files_zip
    du = ModelDatasetUtils()
    uri = 'synthetic://image?n=64&size=8&channels=3&classes=4&seed=0'
    a = du.load_dataset_of_image_files(uri)
    b = du.load_dataset_of_image_files(uri)
    assert a.images is b.images and not a.images.flags.writeable
    imgs, labels = synthetic_images(16, size=8, channels=1, classes=3, seed=2)
    path = str(tmp_path / 'd.zip')
    write_image_files_zip(path, imgs, labels)
    c = du.load_dataset_of_image_files(path)
    np.testing.assert_array_equal(c.images, imgs)
    write_image_files_zip(path, imgs[:8], labels[:8])
    os.utime(path, ns=(1, 10 ** 18))  # force a new mtime
    assert du.load_dataset_of_image_files(path).size == 8
    monkeypatch.setenv('RAFIKI_DATASET_CACHE_MB', '0')
    du.clear_cache()
    d = du.load_dataset_of_image_files(uri)
    assert d.images.flags.writeable and du._decoded_bytes == 0


def test_autotune_cache_file_roundtrip(tmp_path, monkeypatch):
    """Tuned picks (tuple keys / nested tuple configs) survive a JSON cache file."""
    from rafiki_amd.ops import autotune
    monkeypatch.setenv('RAFIKI_TUNE_CACHE', str(tmp_path / 'tune.json'))
    saved = autotune.snapshot()
    try:
        autotune.clear()
        autotune._cache[('cf', 4096, 512, 4608, 4, 4, 512, 9, 'acc')] = ('h', 0, 512)
        autotune._cache[('cw', 64, 576, 262144, False)] = (67, 256)
        autotune._save()
        autotune.clear()
        autotune._loaded = False
        assert autotune.lookup(('cf', 4096, 512, 4608, 4, 4, 512, 9, 'acc')) == ('h', 0, 512)
        assert autotune.lookup(('cw', 64, 576, 262144, False)) == (67, 256)
    finally:
        autotune.clear()
        autotune._cache.update(saved)
