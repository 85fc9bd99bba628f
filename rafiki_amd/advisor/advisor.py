"""Hyper-parameter advisors: GP-EI Bayesian optimisation and random search.

Reference parity: rafiki/advisor/advisor.py (``Advisor.propose/feedback`` :26-62) and
btb_gp_advisor.py (BTB GP tuner, :7-61).  BTB is not available offline, so the Bayesian optimiser
is written here: Matern-5/2 GP over the unit-cube encoding of the knob space (log scale for
``is_exp`` range knobs, one-hot for categoricals, fixed knobs dropped), hyper-parameters chosen by
maximising the log marginal likelihood over a small grid, expected-improvement acquisition
maximised over random + local candidates.

Extensions for 8-way trial parallelism on one node:
  * ``propose_batch(q)`` — q distinct proposals via the constant-liar heuristic;
  * proposals that are out (proposed, no feedback yet) are treated as pending with a "lie" so
    concurrent workers never get the same point;
  * ``feedback`` is idempotent per proposal id and tolerates failed trials (score=None).
"""
from __future__ import annotations

import math
import threading

import numpy as np

from ..constants import AdvisorType
from ..model.knob import (CategoricalKnob, FixedKnob, FloatKnob, IntegerKnob, decode_knobs, encode_knobs,
                          knob_space_dims)


def _simplify(v):
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, np.bool_):
        return bool(v)
    return v


class BaseAdvisor:
    def __init__(self, knob_config, seed=None):
        self.knob_config = dict(knob_config)
        self.rng = np.random.default_rng(seed)
        self._lock = threading.Lock()
        self.history = []  # (knobs, score)
        self._pending = []

    def propose(self):
        with self._lock:
            knobs = self._propose_locked(1)[0]
            self._pending.append(knobs)
            return knobs

    def propose_batch(self, q):
        with self._lock:
            out = self._propose_locked(q)
            self._pending.extend(out)
            return out

    def feedback(self, knobs, score):
        with self._lock:
            knobs = {k: _simplify(v) for k, v in knobs.items()}
            for i, p in enumerate(self._pending):
                if p == knobs:
                    del self._pending[i]
                    break
            if score is not None and math.isfinite(float(score)):
                self.history.append((knobs, float(score)))

    def _random_knobs(self):
        knobs = {}
        for name, k in self.knob_config.items():
            if isinstance(k, FixedKnob):
                knobs[name] = k.value
            elif isinstance(k, CategoricalKnob):
                knobs[name] = _simplify(k.values[self.rng.integers(len(k.values))])
            elif isinstance(k, (IntegerKnob, FloatKnob)):
                knobs[name] = k.decode([self.rng.random()])
            else:
                raise TypeError('unknown knob type {}'.format(type(k)))
        return knobs

    def _propose_locked(self, q):
        return [self._random_knobs() for _ in range(q)]

    @property
    def best(self):
        if not self.history:
            return None
        return max(self.history, key=lambda t: t[1])


class RandomAdvisor(BaseAdvisor):
    """Uniform random search on the (log-)scaled knob space."""


class _GP:
    """Minimal GP regressor with a Matern-5/2 kernel (numpy, float64)."""

    def __init__(self, ls=0.3, sf2=1.0, sn2=1e-4):
        self.ls, self.sf2, self.sn2 = ls, sf2, sn2

    def _k(self, A, B):
        d = np.sqrt(np.maximum(((A[:, None, :] - B[None, :, :]) ** 2).sum(-1), 0.0)) / self.ls
        s5 = math.sqrt(5.0)
        return self.sf2 * (1.0 + s5 * d + 5.0 / 3.0 * d * d) * np.exp(-s5 * d)

    def fit(self, X, y):
        self.X = X
        self.ym, self.ys = float(y.mean()), float(y.std() + 1e-9)
        yn = (y - self.ym) / self.ys
        best = None
        for ls in (0.08, 0.15, 0.3, 0.6, 1.2):
            for sn2 in (1e-6, 1e-3, 1e-2, 1e-1):
                self.ls, self.sn2 = ls, sn2
                K = self._k(X, X) + sn2 * np.eye(len(X))
                try:
                    L = np.linalg.cholesky(K)
                except np.linalg.LinAlgError:
                    continue
                alpha = np.linalg.solve(L.T, np.linalg.solve(L, yn))
                lml = -0.5 * yn @ alpha - np.log(np.diag(L)).sum()
                if best is None or lml > best[0]:
                    best = (lml, ls, sn2, L, alpha)
        if best is None:  # pathological: fall back to heavy noise
            self.ls, self.sn2 = 0.3, 1.0
            K = self._k(X, X) + np.eye(len(X))
            L = np.linalg.cholesky(K)
            best = (0, 0.3, 1.0, L, np.linalg.solve(L.T, np.linalg.solve(L, yn)))
        _, self.ls, self.sn2, self.L, self.alpha = best
        return self

    def predict(self, Xs):
        Ks = self._k(Xs, self.X)
        mu = Ks @ self.alpha
        v = np.linalg.solve(self.L, Ks.T)
        var = np.maximum(self.sf2 - (v * v).sum(0), 1e-12)
        return mu * self.ys + self.ym, np.sqrt(var) * self.ys


def _norm_cdf(z):
    return 0.5 * (1.0 + np.vectorize(math.erf)(z / math.sqrt(2.0)))


def _norm_pdf(z):
    return np.exp(-0.5 * z * z) / math.sqrt(2 * math.pi)


class GpAdvisor(BaseAdvisor):
    """GP-EI Bayesian optimisation with constant-liar batch proposals."""

    def __init__(self, knob_config, seed=None, n_init=3, n_candidates=1500, xi=0.01):
        super().__init__(knob_config, seed)
        self.n_init, self.n_candidates, self.xi = n_init, n_candidates, xi
        self.dims = knob_space_dims(self.knob_config)

    def _encode(self, knobs):
        return np.asarray(encode_knobs(self.knob_config, knobs), dtype=np.float64)

    def _candidates(self, top):
        cands = [self._random_knobs() for _ in range(self.n_candidates)]
        for knobs in top:  # local perturbations around the incumbents
            for _ in range(max(1, self.n_candidates // (4 * max(1, len(top))))):
                u = self._encode(knobs)
                j = 0
                new = dict(knobs)
                for name in sorted(self.knob_config):
                    k = self.knob_config[name]
                    if isinstance(k, (IntegerKnob, FloatKnob)):
                        new[name] = k.decode([float(np.clip(u[j] + self.rng.normal(0, 0.08), 0, 1))])
                    elif isinstance(k, CategoricalKnob) and self.rng.random() < 0.2:
                        new[name] = _simplify(k.values[self.rng.integers(len(k.values))])
                    j += k.dims
                cands.append(new)
        return cands

    def _propose_locked(self, q):
        if self.dims == 0:
            return [self._random_knobs() for _ in range(q)]
        out = []
        obs = list(self.history)
        if len(obs) < self.n_init:
            n_rand = min(q, self.n_init - len(obs))
            out.extend(self._random_knobs() for _ in range(n_rand))
            if len(out) == q or len(obs) < 2:
                while len(out) < q:
                    out.append(self._random_knobs())
                return out
        scores = np.array([s for _, s in obs])
        lie = float(scores.mean())
        pending = [p for p in self._pending] + list(out)
        top = [k for k, _ in sorted(obs, key=lambda t: -t[1])[:3]]
        while len(out) < q:
            X = np.stack([self._encode(k) for k, _ in obs] + [self._encode(p) for p in pending])
            y = np.concatenate([scores, np.full(len(pending), lie)])
            gp = _GP().fit(X, y)
            cands = self._candidates(top)
            C = np.stack([self._encode(c) for c in cands])
            mu, sd = gp.predict(C)
            best = float(scores.max())
            z = (mu - best - self.xi) / sd
            ei = (mu - best - self.xi) * _norm_cdf(z) + sd * _norm_pdf(z)
            seen = {tuple(np.round(x, 6)) for x in X}
            order = np.argsort(-ei)
            pick = None
            for i in order:
                if tuple(np.round(C[i], 6)) not in seen:
                    pick = cands[i]
                    break
            if pick is None:
                pick = self._random_knobs()
            out.append(pick)
            pending.append(pick)
        return out


def make_advisor(knob_config, advisor_type=None, seed=None) -> BaseAdvisor:
    if advisor_type in (None, AdvisorType.BTB_GP, AdvisorType.GP_EI):
        return GpAdvisor(knob_config, seed=seed)
    if advisor_type == AdvisorType.RANDOM:
        return RandomAdvisor(knob_config, seed=seed)
    raise ValueError('Unknown advisor type: {}'.format(advisor_type))


class Advisor:
    """Reference-shaped facade: ``Advisor(knob_config, advisor_type).propose()/feedback()``."""

    def __init__(self, knob_config, advisor_type=AdvisorType.BTB_GP, seed=None):
        self._advisor = make_advisor(knob_config, advisor_type, seed)

    def propose(self):
        return {k: _simplify(v) for k, v in self._advisor.propose().items()}

    def propose_batch(self, q):
        return [{k: _simplify(v) for k, v in p.items()} for p in self._advisor.propose_batch(q)]

    def feedback(self, knobs, score):
        self._advisor.feedback(knobs, score)

    @property
    def history(self):
        return self._advisor.history

    def decode(self, u):
        return decode_knobs(self._advisor.knob_config, u)
