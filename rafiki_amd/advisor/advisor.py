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
from scipy.linalg import solve_triangular
from scipy.special import ndtr

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


PROPOSALS = [0]   # knob sets proposed by any advisor in this process (tests assert where GPs run)


class BaseAdvisor:
    def __init__(self, knob_config, seed=None):
        self.knob_config = dict(knob_config)
        self.rng = np.random.default_rng(seed)
        self._lock = threading.Lock()    # history / pending
        self._plock = threading.Lock()   # one proposal computation at a time (rng, GP state)
        self.history = []  # (knobs, score)
        self._pending = []

    def propose(self):
        return self.propose_batch(1)[0]

    def propose_batch(self, q):
        # the GP fit runs on a snapshot, outside the lock: feedback() from another thread never waits
        # behind a fit; proposals of concurrent callers are serialised by the proposal lock only
        with self._plock:
            with self._lock:
                PROPOSALS[0] += q
                history, pending = list(self.history), list(self._pending)
            out = self._propose_from(q, history, pending)
            with self._lock:
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

    def _propose_from(self, q, history, pending):
        return [self._random_knobs() for _ in range(q)]

    @property
    def best(self):
        if not self.history:
            return None
        return max(self.history, key=lambda t: t[1])


class RandomAdvisor(BaseAdvisor):
    """Uniform random search on the (log-)scaled knob space."""


def _tri(L, b, lower):
    return solve_triangular(L, b, lower=lower, check_finite=False)


class _GP:
    """Minimal GP regressor with a Matern-5/2 kernel (numpy, float64)."""

    def __init__(self, ls=0.3, sf2=1.0, sn2=1e-4):
        self.ls, self.sf2, self.sn2 = ls, sf2, sn2

    @staticmethod
    def _dist(A, B):
        # |a|^2 + |b|^2 - 2 a.b: one GEMM instead of an [n, m, d] broadcast
        d2 = (A * A).sum(1)[:, None] + (B * B).sum(1)[None, :] - 2.0 * (A @ B.T)
        return np.sqrt(np.maximum(d2, 0.0))

    def _kd(self, D):
        d = D / self.ls
        s5 = math.sqrt(5.0)
        return self.sf2 * (1.0 + s5 * d + 5.0 / 3.0 * d * d) * np.exp(-s5 * d)

    def _k(self, A, B):
        return self._kd(self._dist(A, B))

    def fit(self, X, y):
        self.X = X
        self.ym, self.ys = float(y.mean()), float(y.std() + 1e-9)
        yn = (y - self.ym) / self.ys
        D = self._dist(X, X)  # shared by every hyper-parameter candidate
        eye = np.eye(len(X))
        best = None
        for ls in (0.08, 0.15, 0.3, 0.6, 1.2):
            self.ls = ls
            Kls = self._kd(D)
            for sn2 in (1e-6, 1e-3, 1e-2, 1e-1):
                try:
                    L = np.linalg.cholesky(Kls + sn2 * eye)
                except np.linalg.LinAlgError:
                    continue
                alpha = _tri(L.T, _tri(L, yn, True), False)
                lml = -0.5 * yn @ alpha - np.log(np.diag(L)).sum()
                if best is None or lml > best[0]:
                    best = (lml, ls, sn2, L, alpha)
        if best is None:  # pathological: fall back to heavy noise
            self.ls, self.sn2 = 0.3, 1.0
            L = np.linalg.cholesky(self._k(X, X) + eye)
            best = (0, 0.3, 1.0, L, _tri(L.T, _tri(L, yn, True), False))
        _, self.ls, self.sn2, self.L, self.alpha = best
        return self

    def predict(self, Xs):
        Ks = self._k(Xs, self.X)
        mu = Ks @ self.alpha
        v = _tri(self.L, Ks.T, True)
        var = np.maximum(self.sf2 - (v * v).sum(0), 1e-12)
        return mu * self.ys + self.ym, np.sqrt(var) * self.ys


def _norm_cdf(z):
    return ndtr(z)


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

    def _snap(self, U):
        """Raw unit-cube samples [n, dims] -> encodings of valid knob values (the vectorised
        ``encode(decode(u))``: integers rounded on their own (log) scale, categoricals one-hot)."""
        out = np.empty_like(U)
        j = 0
        for name in sorted(self.knob_config):
            k = self.knob_config[name]
            d = k.dims
            if d == 0:
                continue
            u = U[:, j:j + d]
            if isinstance(k, CategoricalKnob):
                oh = np.zeros_like(u)
                oh[np.arange(len(u)), np.argmax(u, 1)] = 1.0
                out[:, j:j + d] = oh
            elif isinstance(k, IntegerKnob):
                lo, hi = k._fwd(k.value_min), k._fwd(k.value_max)
                if hi == lo:
                    out[:, j] = 0.5
                else:
                    x = lo + np.clip(u[:, 0], 0.0, 1.0) * (hi - lo)
                    v = np.clip(np.round(np.exp(x) if k.is_exp else x), k.value_min, k.value_max)
                    out[:, j] = np.clip(((np.log(v) if k.is_exp else v) - lo) / (hi - lo), 0.0, 1.0)
            else:
                out[:, j] = np.clip(u[:, 0], 0.0, 1.0)
            j += d
        return out

    def _candidates(self, top):
        """Encoded candidates [n, dims]: uniform samples plus local perturbations of the incumbents."""
        parts = [self.rng.random((self.n_candidates, self.dims))]
        cat_cols = []
        j = 0
        for name in sorted(self.knob_config):
            k = self.knob_config[name]
            if isinstance(k, CategoricalKnob):
                cat_cols.append((j, k.dims))
            j += k.dims
        per = max(1, self.n_candidates // (4 * max(1, len(top))))
        for knobs in top:
            u = np.tile(self._encode(knobs), (per, 1)) + self.rng.normal(0, 0.08, (per, self.dims))
            for (c, d) in cat_cols:  # a categorical is re-drawn with probability 0.2
                flip = self.rng.random(per) < 0.2
                u[flip, c:c + d] = self.rng.random((int(flip.sum()), d))
                keep = ~flip
                u[keep, c:c + d] = self._encode(knobs)[c:c + d]
            parts.append(u)
        # discrete knobs snap many samples onto the same point: score each distinct point once
        return np.unique(self._snap(np.concatenate(parts)), axis=0)

    def _propose_from(self, q, history, pending_in):
        if self.dims == 0:
            return [self._random_knobs() for _ in range(q)]
        out = []
        obs = list(history)
        if len(obs) < self.n_init:
            n_rand = min(q, self.n_init - len(obs))
            out.extend(self._random_knobs() for _ in range(n_rand))
            if len(out) == q or len(obs) < 2:
                while len(out) < q:
                    out.append(self._random_knobs())
                return out
        scores = np.array([s for _, s in obs])
        lie = float(scores.mean())
        pending = list(pending_in) + list(out)
        top = [k for k, _ in sorted(obs, key=lambda t: -t[1])[:3]]
        X = np.stack([self._encode(k) for k, _ in obs] + [self._encode(p) for p in pending])
        y = np.concatenate([scores, np.full(len(pending), lie)])
        best = float(scores.max())
        while len(out) < q:
            gp = _GP().fit(X, y)
            C = self._candidates(top)
            mu, sd = gp.predict(C)
            z = (mu - best - self.xi) / sd
            ei = (mu - best - self.xi) * _norm_cdf(z) + sd * _norm_pdf(z)
            # never re-propose an observed or pending point
            d2 = _GP._dist(C, X).min(1)
            ei[d2 < 1e-6] = -np.inf
            i = int(np.argmax(ei))
            pick = decode_knobs(self.knob_config, C[i]) if np.isfinite(ei[i]) else self._random_knobs()
            pick = {k: _simplify(v) for k, v in pick.items()}
            out.append(pick)
            X = np.vstack([X, self._encode(pick)[None]])
            y = np.append(y, lie)  # constant liar for the next proposal of this batch
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
