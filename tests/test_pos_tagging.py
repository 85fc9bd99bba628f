"""POS_TAGGING models on CPU: BigramHmm and PyBiLstm train / evaluate / predict / params round trip,
and PyBiLstm mid-trial checkpoint + crash-resume (reference PyBiLstm.py:66-84 saves model and
optimizer state; here a restarted trial continues from its last epoch)."""
import pytest
import torch

from rafiki_amd.parallel.context import TrialContext, use_context

TR = 'synthetic://corpus?n=300&seed=0'
TE = 'synthetic://corpus?n=80&seed=1'
KNOBS = dict(epochs=4, word_embed_dims=16, word_rnn_hidden_size=16, word_dropout=0.05, learning_rate=0.05,
             batch_size=32)


def test_bigram_hmm_cpu():
    from rafiki_amd.models.pos_tagging import BigramHmm
    m = BigramHmm()
    m.train(TR)
    acc = m.evaluate(TE)
    assert 0.5 < acc <= 1.0
    m2 = BigramHmm()
    m2.load_parameters(m.dump_parameters())
    q = [['w1', 'w2', 'w3']]
    assert m2.predict(q) == m.predict(q)


def test_pybilstm_cpu_params_round_trip():
    from rafiki_amd.models.pos_tagging import PyBiLstm
    torch.manual_seed(0)
    with use_context(TrialContext(device=torch.device('cpu'))):
        m = PyBiLstm(**KNOBS)
        m.train(TR)
        acc = m.evaluate(TE)
        m2 = PyBiLstm(**KNOBS)
        m2.load_parameters(m.dump_parameters())
        assert m2.evaluate(TE) == acc
    assert acc > 0.3


def _weights(m):
    return {k: v.clone() for k, v in m._net.state_dict().items()}


def test_pybilstm_crash_resume_matches_uninterrupted(tmp_path, monkeypatch):
    from rafiki_amd.models.pos_tagging import PyBiLstm
    from rafiki_amd.utils import faults
    from rafiki_amd.utils.checkpoint import TrialCheckpoint
    torch.manual_seed(0)
    with use_context(TrialContext(device=torch.device('cpu'))):
        a = PyBiLstm(**KNOBS)
        a.train(TR)
    ck = TrialCheckpoint(str(tmp_path), 'bilstm1')
    monkeypatch.setenv('RAFIKI_FAULT_INJECT', 'crash:epoch=1')
    faults.reset()
    torch.manual_seed(0)
    with use_context(TrialContext(device=torch.device('cpu'), checkpoint=ck)):
        with pytest.raises(faults.WorkerCrash):
            PyBiLstm(**KNOBS).train(TR)
        assert ck.exists()
        monkeypatch.setenv('RAFIKI_FAULT_INJECT', '')
        faults.reset()
        torch.manual_seed(123)   # the restarted process's global RNG differs; the checkpoint restores it
        b = PyBiLstm(**KNOBS)
        b.train(TR)
    assert ck.resumed_from == 1
    wa, wb = _weights(a), _weights(b)
    for k in wa:
        assert torch.equal(wa[k], wb[k]), k


def test_tagger_pack_batch_layout():
    """Host packing of a tagger batch (engine/tagger.py): time-major ids / labels, stable-sorted runs
    with the padding id marked -1, and 1/#labelled tokens as float bits."""
    import numpy as np
    from rafiki_amd.engine.tagger import pack_batch
    x = np.array([[3, 1, 0], [1, 3, 2]])
    y = np.array([[5, 6, -100], [7, 8, 9]])
    w = pack_batch(x, y)
    n = 6
    assert w[:n].tolist() == [3, 1, 1, 3, 0, 2]
    assert w[n:2 * n].tolist() == [5, 7, 6, 8, -100, 9]
    assert w[2 * n:3 * n].tolist() == [4, 1, 2, 5, 0, 3]
    assert w[3 * n:3 * n + 4].tolist() == [-1, 1, 2, 3]
    assert w[4 * n:4 * n + 5].tolist() == [0, 1, 3, 4, 6]
    assert w[5 * n + 1] == 4
    assert w[5 * n + 2:].view(np.float32)[0] == np.float32(0.2)
