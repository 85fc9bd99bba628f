"""POS-tagging models: BigramHmm (count-based bigram HMM + Viterbi) and PyBiLstm (BiLSTM tagger).

Reference: examples/models/pos_tagging/BigramHmm.py:17-187 (counts :73-126, Viterbi :128-187)
and PyBiLstm.py:19-274 (Embedding -> Dropout -> BiLSTM -> Linear; knobs :24-32).

Task I/O (tasks.rst): a query is a list of tokens, a prediction is a list of integer tags.
Differences: Viterbi runs vectorised in numpy log-space; the BiLSTM applies cross-entropy to
logits (the reference applies it to softmax outputs, bug (k)) and batches sentences bucketed by
length.  On a GPU the BiLSTM's training step and prediction run on the native tagger engine
(engine/tagger.py: in-tree kernels only, one hipGraph per bucket shape, any knob value); on the CPU
the same network runs as torch modules.
"""
import math

import numpy as np

from rafiki_amd.constants import TaskType  # noqa: F401
from rafiki_amd.model import (BaseModel, CategoricalKnob, FixedKnob, FloatKnob, IntegerKnob, dataset_utils,
                              logger)
from rafiki_amd.engine.convnet import default_dtype
from rafiki_amd.parallel.context import current as trial_context
from rafiki_amd.utils import faults


def _to_cpu(obj):
    """Nested state dicts with every tensor on the host (picklable, device-independent)."""
    import torch
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def _accuracy(sents, preds):
    tot = ok = 0
    for s, p in zip(sents, preds):
        for tok, t in zip(s, p):
            tot += 1
            ok += int(tok[1] == t)
    return ok / max(1, tot)


class BigramHmm(BaseModel):
    @staticmethod
    def get_knob_config():
        return {'smoothing': FloatKnob(1e-3, 1.0, is_exp=True)}

    def __init__(self, **knobs):
        super().__init__(**knobs)
        self._alpha = float(knobs.get('smoothing', 0.01))
        self._vocab = {}
        self._log_trans = self._log_emit = self._log_start = None

    def train(self, dataset_uri):
        ds = dataset_utils.load_dataset_of_corpus(dataset_uri)
        sents = [ds[i] for i in range(len(ds))]
        T = ds.tag_num_classes[0]
        self._vocab = {}
        for s in sents:
            for tok in s:
                self._vocab.setdefault(tok[0], len(self._vocab))
        V = len(self._vocab) + 1  # last id = unknown word
        start = np.full(T, self._alpha)
        trans = np.full((T, T), self._alpha)
        emit = np.full((T, V), self._alpha)
        for s in sents:
            prev = None
            for tok in s:
                w, t = self._vocab[tok[0]], tok[1]
                emit[t, w] += 1
                if prev is None:
                    start[t] += 1
                else:
                    trans[prev, t] += 1
                prev = t
        self._log_start = np.log(start / start.sum())
        self._log_trans = np.log(trans / trans.sum(1, keepdims=True))
        self._log_emit = np.log(emit / emit.sum(1, keepdims=True))
        logger.log('Train accuracy: {}'.format(_accuracy(sents, self._tag([[t[0] for t in s] for s in sents]))))

    def _tag(self, sents_tokens):
        out = []
        unk = self._log_emit.shape[1] - 1
        for toks in sents_tokens:
            if not toks:
                out.append([])
                continue
            ids = [self._vocab.get(w, unk) for w in toks]
            score = self._log_start + self._log_emit[:, ids[0]]
            back = []
            for w in ids[1:]:
                cand = score[:, None] + self._log_trans  # [prev, cur]
                back.append(cand.argmax(0))
                score = cand.max(0) + self._log_emit[:, w]
            best = [int(score.argmax())]
            for bp in reversed(back):
                best.append(int(bp[best[-1]]))
            out.append(best[::-1])
        return out

    def evaluate(self, dataset_uri):
        ds = dataset_utils.load_dataset_of_corpus(dataset_uri)
        sents = [ds[i] for i in range(len(ds))]
        return float(_accuracy(sents, self._tag([[t[0] for t in s] for s in sents])))

    def predict(self, queries):
        return self._tag(queries)

    def dump_parameters(self):
        return {'vocab': self._vocab, 'start': self._log_start, 'trans': self._log_trans, 'emit': self._log_emit}

    def load_parameters(self, params):
        self._vocab = params['vocab']
        self._log_start, self._log_trans, self._log_emit = params['start'], params['trans'], params['emit']


class PyBiLstm(BaseModel):
    @staticmethod
    def get_knob_config():
        return {
            'epochs': FixedKnob(10),
            'word_embed_dims': IntegerKnob(16, 128),
            'word_rnn_hidden_size': IntegerKnob(16, 128),
            'word_dropout': FloatKnob(1e-3, 2e-1, is_exp=True),
            'learning_rate': FloatKnob(1e-2, 1e-1, is_exp=True),
            'batch_size': CategoricalKnob([16, 32, 64, 128]),
        }

    def __init__(self, **knobs):
        super().__init__(**knobs)
        self._knobs = knobs
        self._net = None
        self._engine = None
        self._word_dict = {}
        self._tag_count = 0
        self.device = trial_context().device

    def _create(self):
        import torch
        import torch.nn as nn
        from rafiki_amd.ops.autograd import dense
        from rafiki_amd.ops.lstm import bilstm, embedding
        k = self._knobs
        V = len(self._word_dict) + 2  # 0 = pad, 1 = unknown

        class Net(nn.Module):
            def __init__(s):
                super().__init__()
                s.emb = nn.Embedding(V, int(k.get('word_embed_dims', 64)), padding_idx=0)
                s.drop = nn.Dropout(float(k.get('word_dropout', 0.1)))
                s.lstm = nn.LSTM(int(k.get('word_embed_dims', 64)), int(k.get('word_rnn_hidden_size', 64)),
                                 batch_first=True, bidirectional=True)
                s.out = nn.Linear(2 * int(k.get('word_rnn_hidden_size', 64)), self._tag_count)
                s.rec_dtype = k.get('dtype') or default_dtype()   # fp32 (reference precision) unless opted into bf16

            def forward(s, x):
                # gfx950 kernels on GPU: embedding gather / sorted scatter-sum gradient, persistent-recurrence
                # BiLSTM with its GEMMs on sgemm (rafiki_amd.ops.lstm), the output layer on sgemm
                h = bilstm(s.drop(embedding(x, s.emb)), s.lstm, dtype=s.rec_dtype)
                o = s.out
                if h.is_cuda and h.dtype == torch.float32 and o.in_features % 4 == 0 and o.out_features % 4 == 0:
                    return dense(h.reshape(-1, o.in_features), o.weight, o.bias).reshape(h.shape[:-1] + (-1,))
                return o(h)

        return Net().to(self.device)

    def _encode(self, sents_tokens):
        return [[self._word_dict.get(w, 1) for w in s] for s in sents_tokens]

    @staticmethod
    def _batches_np(ids, tags, bs, shuffle, rng):
        order = np.argsort([len(s) for s in ids], kind='stable')  # bucket by length
        chunks = [order[i:i + bs] for i in range(0, len(order), bs)]
        if shuffle:
            rng.shuffle(chunks)
        for ch in chunks:
            L = max(1, max(len(ids[i]) for i in ch))
            x = np.zeros((len(ch), L), np.int64)
            y = np.full((len(ch), L), -100, np.int64)
            for r, i in enumerate(ch):
                x[r, :len(ids[i])] = ids[i]
                if tags is not None:
                    y[r, :len(tags[i])] = tags[i]
            yield ch, x, y

    def _batches(self, ids, tags, bs, shuffle, rng):
        import torch
        for ch, x, y in self._batches_np(ids, tags, bs, shuffle, rng):
            yield ch, torch.from_numpy(x).to(self.device), torch.from_numpy(y).to(self.device)

    def _native(self) -> bool:
        """The native engine runs the GPU step for every knob value of the search space (hidden <= 128)."""
        return (self.device.type == 'cuda' and int(self._knobs.get('word_rnn_hidden_size', 64)) <= 128
                and (self._knobs.get('dtype') or default_dtype()) != 'bf16')

    def train(self, dataset_uri):
        import torch
        import torch.nn.functional as F
        ds = dataset_utils.load_dataset_of_corpus(dataset_uri)
        sents = [ds[i] for i in range(len(ds))]
        self._word_dict = {}
        for s in sents:
            for tok in s:
                self._word_dict.setdefault(tok[0], len(self._word_dict) + 2)
        self._tag_count = ds.tag_num_classes[0]
        self._net = self._create()
        ids = self._encode([[t[0] for t in s] for s in sents])
        tags = [[t[1] for t in s] for s in sents]
        rng = np.random.default_rng(0)
        logger.define_loss_plot()
        epochs = int(self._knobs.get('epochs', 10))
        ck = trial_context().checkpoint
        saved = ck.load() if ck is not None else None
        if self._native():
            return self._train_native(ids, tags, rng, epochs, ck, saved)
        opt = torch.optim.Adam(self._net.parameters(), lr=float(self._knobs.get('learning_rate', 0.05)))
        start = 0
        if saved is not None:
            self._restore_ckpt(saved['state'], opt, rng)
            start = int(saved['epoch']) + 1
            logger.log('resumed from checkpoint after epoch {}'.format(saved['epoch']))
        for ep in range(start, epochs):
            self._net.train()
            tot = torch.zeros((), device=self.device)
            n = 0
            for _, x, y in self._batches(ids, tags, int(self._knobs.get('batch_size', 32)), True, rng):
                logits = self._net(x)
                loss = F.cross_entropy(logits.reshape(-1, self._tag_count), y.reshape(-1), ignore_index=-100)
                opt.zero_grad()
                loss.backward()
                opt.step()
                tot += loss.detach()   # summed on the device: one host sync per epoch
                n += 1
            logger.log_loss(loss=float(tot.item()) / max(1, n), epoch=ep)
            if ck is not None and ck.due(ep) and ep + 1 < epochs:
                ck.save(self._ckpt_state(opt, rng), ep)
            faults.maybe_fail('crash', epoch=ep, rank=0)

    def _train_native(self, ids, tags, rng, epochs, ck, saved):
        """The GPU training loop on the native engine: Adam over the padded arena, dropout from the
        engine's Philox stream (seeded from the trial's numpy generator), one graph per bucket shape."""
        from rafiki_amd.engine.tagger import TaggerEngine
        eng = TaggerEngine(self._net, float(self._knobs.get('learning_rate', 0.05)),
                           float(self._knobs.get('word_dropout', 0.1)), seed=int(rng.integers(1 << 62)))
        start = 0
        if saved is not None:
            st = saved['state']
            if 'engine' in st:
                eng.load_state(st['engine'])
            else:   # a checkpoint of the torch path: weights carry over, Adam restarts
                self._net.load_state_dict(st['net'])
                eng.load_module(self._net)
            rng.bit_generator.state = st['np_rng']
            start = int(saved['epoch']) + 1
            logger.log('resumed from checkpoint after epoch {}'.format(saved['epoch']))
        bs = int(self._knobs.get('batch_size', 32))
        eng.take_loss()
        for ep in range(start, epochs):
            n = 0
            for _, x, y in self._batches_np(ids, tags, bs, True, rng):
                eng.step(x, y)
                n += 1
            logger.log_loss(loss=eng.take_loss() / max(1, n), epoch=ep)   # one host sync per epoch
            if ck is not None and ck.due(ep) and ep + 1 < epochs:
                eng.store_module(self._net)
                ck.save({'engine': eng.state(), 'np_rng': rng.bit_generator.state,
                         'net': _to_cpu(self._net.state_dict())}, ep)
            faults.maybe_fail('crash', epoch=ep, rank=0)
        eng.store_module(self._net)
        eng.close()   # the step graphs are done; the engine stays for predict
        self._engine = eng

    # ----------------------------------------------------------------- checkpoint / resume
    def _ckpt_state(self, opt, rng):
        """Weights, Adam moments, and every RNG the epoch loop draws from (batch shuffling, dropout):
        the reference saves model + optimizer state (PyBiLstm.py:66-84)."""
        import torch
        st = {'net': _to_cpu(self._net.state_dict()), 'opt': _to_cpu(opt.state_dict()),
              'np_rng': rng.bit_generator.state, 'torch_rng': torch.get_rng_state()}
        if self.device.type == 'cuda':
            st['cuda_rng'] = torch.cuda.get_rng_state(self.device)
        return st

    def _restore_ckpt(self, st, opt, rng):
        import torch
        self._net.load_state_dict(st['net'])
        opt.load_state_dict(st['opt'])
        rng.bit_generator.state = st['np_rng']
        torch.set_rng_state(st['torch_rng'])
        if self.device.type == 'cuda' and 'cuda_rng' in st:
            torch.cuda.set_rng_state(st['cuda_rng'], self.device)

    def _predict(self, sents_tokens):
        import torch
        self._net.eval()
        ids = self._encode(sents_tokens)
        out = [None] * len(ids)
        eng = None
        if self._native():
            from rafiki_amd.engine.tagger import TaggerEngine
            eng = getattr(self, '_engine', None)
            if eng is None:
                eng = self._engine = TaggerEngine(self._net, 0.0, 0.0)
        with torch.no_grad():
            for ch, x, _ in self._batches_np(ids, None, 256, False, None):
                if eng is not None:
                    logits = eng.logits(x)
                else:
                    logits = self._net(torch.from_numpy(x).to(self.device))
                pred = logits.argmax(-1).cpu().numpy()
                for r, i in enumerate(ch):
                    out[i] = [int(t) for t in pred[r, :len(ids[i])]]
        return out

    def evaluate(self, dataset_uri):
        ds = dataset_utils.load_dataset_of_corpus(dataset_uri)
        sents = [ds[i] for i in range(len(ds))]
        return float(_accuracy(sents, self._predict([[t[0] for t in s] for s in sents])))

    def predict(self, queries):
        return self._predict(queries)

    def dump_parameters(self):
        return {'net_state_dict': {k: v.cpu() for k, v in self._net.state_dict().items()},
                'word_dict': self._word_dict, 'tag_count': self._tag_count}

    def load_parameters(self, params):
        self._word_dict = params['word_dict']
        self._tag_count = params['tag_count']
        self._net = self._create()
        self._net.load_state_dict(params['net_state_dict'])
        self._engine = None
