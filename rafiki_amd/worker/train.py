"""TrainWorker: the trial loop of one sub-train-job, run by an SPMD worker group (one rank per GPU).

Reference parity: rafiki/worker/train.py (``TrainWorker.start`` :37-132, ``stop`` :134-148,
``_train_and_evaluate_model`` :150-186): budget check -> create trial -> propose knobs ->
train/evaluate -> pickle params to ``<workdir>/params/<trial_id>.model`` -> report score.

MI355X-native redesign:
  * rank 0 owns the sub-train-job's ONE advisor (GP-EI); every rank trains its own trial on its own
    GPU.  Default (``async``) scheduling: a rank that finishes a trial claims the next budget slot
    atomically in the SQLite store, then exchanges one packed fp64 row with rank 0 over RCCL
    point-to-point — its (score, ok, seconds) in, its next knob set out, proposed with every
    in-flight trial as a constant-liar point (``parallel/exchange.py``).  No round barrier, no HTTP
    in the loop, one GP posterior, and the budget can never overshoot (the reference's budget race,
    train.py:50 / SURVEY §5.2);
  * ``rounds`` scheduling (lock-step): rank 0 proposes one knob set per rank per round, broadcast as
    one packed tensor over RCCL; scores come back by all_gather;
  * models that declare ``DATA_PARALLEL = True`` train ONE trial per round on all ranks jointly
    (bucketed gradient all-reduce inside the model), e.g. the PG-GAN;
  * a failed trial is marked ERRORED and the loop continues (bounded by ``max_trial_errors``)
    instead of killing the worker (reference bug (f));
  * trial log lines go through the DB's batched writer.
"""
from __future__ import annotations

import logging
import math
import os
import pickle
import time
import traceback

import torch

from ..advisor.advisor import make_advisor
from ..constants import BudgetType, TrialStatus
from ..model.log import logger as model_logger
from ..model.model import load_model_class
from ..parallel import dist as D
from ..parallel.context import TrialContext, default_device, use_context
from ..utils.checkpoint import TrialCheckpoint

logger = logging.getLogger(__name__)


class _TrialLogHandler(logging.Handler):
    def __init__(self, db, trial_id):
        super().__init__(level=logging.INFO)
        self.db, self.trial_id = db, trial_id

    def emit(self, record):
        try:
            self.db.add_trial_log(self.trial_id, record.getMessage(), record.levelname)
        except Exception:
            pass


class TrainWorker:
    def __init__(self, service_id, worker_id, db=None, dist_info: D.DistInfo = None, params_dir=None,
                 max_trial_errors=3, advisor_type=None, seed=None, checkpoint_every_epochs=1, scheduling=None,
                 offer_resident=None):
        from ..config import get_config
        from ..db.database import Database
        self._service_id = service_id
        self._worker_id = worker_id
        self._db = db or Database()
        self._dist = dist_info or D.DistInfo()
        cfg = get_config()
        self._params_dir = params_dir or os.path.join(cfg.workdir, cfg.params_dir)
        os.makedirs(self._params_dir, exist_ok=True)
        self._max_trial_errors = max_trial_errors
        self._ckpt_every = checkpoint_every_epochs
        # 'async' : ranks pull trials independently — an atomic budget claim in the store, then the
        #           knobs from rank 0's single GP-EI advisor over RCCL (in-flight trials as constant-
        #           liar points); no round barrier, so heterogeneous trial lengths (epochs / batch size /
        #           width knobs) never idle a GPU.  The default ('auto') for every non-data-parallel model.
        # 'rounds': rank 0 proposes one knob set per rank per round, broadcast over RCCL (lock-step;
        #           every round waits for its slowest trial).  Data-parallel models always use it.
        self._scheduling = scheduling or os.environ.get('RAFIKI_TRIAL_SCHEDULING', 'auto')
        # keep finished models resident in HBM for a predictor IN THIS PROCESS (inline services, the
        # bench, notebooks); a service-mode worker's predictor runs elsewhere and could never take them
        self._offer_resident = (os.environ.get('RAFIKI_OFFER_RESIDENT', '0') == '1' if offer_resident is None
                                else bool(offer_resident))
        self._advisor_type = advisor_type
        self._seed = seed
        self._trial_id = None
        self._stop = False
        self.completed_trials = []
        self.busy_s = 0.0  # wall seconds spent inside trials (train + evaluate + dump), for idle accounting
        self.first_trial_t = None   # perf_counter at the first / after the last trial (idle accounting)
        self.last_trial_end_t = None
        self.gap_parts = {'claim': 0.0, 'propose': 0.0}  # async-loop seconds outside trials
        self.trial_records = []   # per completed trial: claim / propose / train / evaluate / dump seconds

    # ------------------------------------------------------------------------------ main loop
    def start(self):
        info = self._dist
        worker = self._db.get_train_job_worker(self._service_id)
        if worker is None:
            raise RuntimeError('no train job worker for service {}'.format(self._service_id))
        sub = self._db.get_sub_train_job(worker.sub_train_job_id)
        train_job = self._db.get_train_job(sub.train_job_id)
        model = self._db.get_model(sub.model_id)
        budget = train_job.budget or {}
        max_trials = int(budget.get(BudgetType.MODEL_TRIAL_COUNT, 5))
        deadline = None
        if BudgetType.TIME_HOURS in budget:
            deadline = time.time() + float(budget[BudgetType.TIME_HOURS]) * 3600.0
        clazz = load_model_class(model.model_file_bytes, model.model_class)
        knob_config = clazz.get_knob_config()
        data_parallel = bool(getattr(clazz, 'DATA_PARALLEL', False)) and info.world_size > 1
        device = default_device()
        if self._scheduling in ('async', 'auto') and not data_parallel:
            return self._start_async(clazz, model, sub, train_job, knob_config, max_trials, deadline, device)
        advisor = make_advisor(knob_config, self._advisor_type, self._seed) if info.is_main else None
        errors = 0
        # trials this worker was running when its previous incarnation died, with a checkpoint to
        # resume from; re-run first, under their original ids and knobs
        resume = self._orphaned_trials(sub.id) if (info.is_main and not data_parallel) else []
        while not self._stop:
            # ---- rank 0 decides this round (budget is enforced by exactly one process)
            if info.is_main:
                done = self._db.count_trials_of_sub_train_job(sub.id, [TrialStatus.COMPLETED, TrialStatus.ERRORED])
                remaining = max(0, max_trials - done)
                if deadline is not None and time.time() > deadline:
                    remaining = 0
                if errors >= self._max_trial_errors:
                    remaining = 0
                n_active = min(remaining, 1 if data_parallel else info.world_size)
                resumed = resume[:n_active]
                resume = resume[n_active:]
                props = [k for _, k in resumed]
                if n_active > len(props):
                    props += advisor.propose_batch(n_active - len(props))
                resume_ids = [t for t, _ in resumed] + [None] * (info.world_size - len(resumed))
                padded = props + [props[0] if props else advisor._random_knobs()] * (info.world_size - len(props))
            else:
                n_active, padded, resume_ids = 0, None, None
            n_active = self._broadcast_int(n_active)
            if n_active == 0:
                break
            proposals = D.broadcast_proposals(info, knob_config, padded) if info.world_size > 1 else padded
            resume_ids = self._broadcast_obj(resume_ids)
            my = 0 if data_parallel else info.rank
            active = my < n_active
            ctx = TrialContext(device=device, dist=info, data_parallel=data_parallel)
            score, ok, secs = float('nan'), 0.0, 0.0
            if active:
                record = (not data_parallel) or info.is_main
                knobs = proposals[my]
                t0 = time.time()
                score, ok = self._run_trial(clazz, model, sub, knobs, train_job, ctx, record,
                                            resume_id=None if data_parallel else resume_ids[my])
                secs = time.time() - t0
                self.busy_s += secs
            table = D.gather_floats(info, [score if ok else float('nan'), ok, secs, float(active)])
            if info.is_main:
                for r in range(info.world_size):
                    if table[r, 3] > 0 and (not data_parallel or r == 0):
                        s = float(table[r, 0])
                        advisor.feedback(proposals[0 if data_parallel else r], s if table[r, 1] > 0 else None)
                        errors = errors + 1 if table[r, 1] == 0 else 0
        if info.is_main:
            logger.info('sub-train-job %s budget reached', sub.id)
            self._db.mark_sub_train_job_as_stopped(self._db.get_sub_train_job(sub.id))

    # ------------------------------------------------------------------ asynchronous scheduling
    def _start_async(self, clazz, model, sub, train_job, knob_config, max_trials, deadline, device):
        """Asynchronous trial scheduling: every rank pulls its next trial as
        soon as its GPU is free — no round barrier, so one slow trial never idles the other GPUs.

        * budget: an atomic claim in the store (``Database.claim_trial``), taken BEFORE asking for knobs;
        * knobs/scores: ONE GP-EI advisor on rank 0 (``parallel.exchange.KnobExchange``).  A rank that
          finishes a trial rings a doorbell in the rendezvous store and exchanges one packed fp64 row
          with rank 0 over RCCL point-to-point (its score in, its next knob set out); rank 0 proposes
          with every in-flight trial as a constant-liar pending point;
        * end: a failed claim reports the last score and leaves; rank 0's server exits once every
          peer has left, then a last barrier and rank 0 closes the sub-train-job."""
        from ..parallel.exchange import KnobExchange
        info = self._dist
        errors = 0
        history = []
        if info.is_main:   # a restarted job's GP starts from the durable record
            history = [(dict(t.knobs), float(t.score)) for t in self._db.get_trials_of_sub_train_job(sub.id)
                       if t.status == TrialStatus.COMPLETED and t.knobs]
        ex = KnobExchange(info, knob_config, lambda: make_advisor(knob_config, self._advisor_type, self._seed),
                          tag=str(sub.id), history=history)
        self.exchange = ex
        prev = None
        try:
            # trials this worker was running when its previous incarnation died, with a checkpoint to
            # resume from: they keep their ids, knobs and budget slot, and run first
            for tid, knobs in self._orphaned_trials(sub.id):
                if self._stop:
                    break
                ctx = TrialContext(device=device, dist=info, data_parallel=False)
                t0 = time.perf_counter()
                score, ok = self._run_trial(clazz, model, sub, knobs, train_job, ctx, True, resume_id=tid)
                secs = time.perf_counter() - t0
                self.busy_s += secs
                errors = errors + 1 if not ok else 0
                if prev is not None:   # fold the previous orphan's score in without asking for knobs
                    ex.report(prev)
                prev = (knobs, score, ok > 0, secs)
            while not self._stop and errors < self._max_trial_errors:
                if deadline is not None and time.time() > deadline:
                    break
                tc = time.perf_counter()
                trial = self._db.claim_trial(sub.id, model.id, self._worker_id, max_trials)
                claim_s = time.perf_counter() - tc
                self.gap_parts['claim'] += claim_s
                if trial is None:
                    break
                th = time.perf_counter()
                knobs = ex.request(prev)
                propose_s = time.perf_counter() - th
                self.gap_parts['propose'] += propose_s
                self._next_gap = {'claim': claim_s, 'propose': propose_s}
                ctx = TrialContext(device=device, dist=info, data_parallel=False)
                t0 = time.perf_counter()
                if self.first_trial_t is None:
                    self.first_trial_t = t0
                score, ok = self._run_trial(clazz, model, sub, knobs, train_job, ctx, True, resume_id=trial.id)
                self.last_trial_end_t = time.perf_counter()
                secs = self.last_trial_end_t - t0
                self.busy_s += secs
                errors = errors + 1 if not ok else 0
                prev = (knobs, score, ok > 0, secs)
        finally:
            ex.finish(prev)
            ex.close()
        if info.world_size > 1:
            D.barrier(info)
        if info.is_main:
            logger.info('sub-train-job %s budget reached (async, %s)', sub.id, ex.stats)
            self._db.mark_sub_train_job_as_stopped(self._db.get_sub_train_job(sub.id))

    def _orphaned_trials(self, sub_id):
        out = []
        for t in self._db.get_trials_of_sub_train_job(sub_id):
            if t.status in (TrialStatus.STARTED, TrialStatus.RUNNING, TrialStatus.TERMINATED) and t.knobs and \
                    t.worker_id == self._worker_id and TrialCheckpoint(self._params_dir, t.id).exists():
                out.append((t.id, dict(t.knobs)))
        if out:
            logger.info('resuming %d checkpointed trial(s): %s', len(out), [t for t, _ in out])
        return out

    def _broadcast_obj(self, obj):
        if self._dist.world_size == 1:
            return obj
        lst = [obj]
        torch.distributed.broadcast_object_list(lst, src=0)
        return lst[0]

    def _broadcast_int(self, v):
        info = self._dist
        if info.world_size == 1:
            return int(v)
        t = torch.tensor([v], dtype=torch.int64, device=D.comm_device(info))
        torch.distributed.broadcast(t, src=0)
        return int(t.item())

    # -------------------------------------------------------------------------------- trial
    def _run_trial(self, clazz, model, sub, knobs, train_job, ctx, record, resume_id=None):
        trial = None
        if record:
            trial = self._db.get_trial(resume_id) if resume_id else None
            if trial is None:
                trial = self._db.create_trial(sub.id, model.id, self._worker_id)
            self._trial_id = trial.id
            ctx.trial_id = trial.id
            ctx.checkpoint = TrialCheckpoint(self._params_dir, trial.id, self._ckpt_every)
            self._db.mark_trial_as_running(trial, knobs)
        handler = _TrialLogHandler(self._db, trial.id) if record else None
        prev_logger = model_logger.get_logger()
        trial_logger = logging.getLogger('rafiki_amd.trial.{}'.format(trial.id if trial else 'dp'))
        trial_logger.setLevel(logging.INFO)
        trial_logger.propagate = False
        if handler:
            trial_logger.addHandler(handler)
        model_logger.set_logger(trial_logger)
        inst = None
        try:
            rec = dict(getattr(self, '_next_gap', None) or {})
            self._next_gap = None
            t_start = time.perf_counter()
            with use_context(ctx):
                inst = clazz(**knobs)
                with model_logger.phase('train'):
                    inst.train(train_job.train_dataset_uri)
                t_train = time.perf_counter()
                with model_logger.phase('evaluate'):
                    score = float(inst.evaluate(train_job.test_dataset_uri))
                t_eval = time.perf_counter()
                if not math.isfinite(score):
                    raise ValueError('non-finite score {}'.format(score))
                params_path = None
                if record:
                    with model_logger.phase('dump_parameters'):
                        blob = pickle.dumps(inst.dump_parameters())
                    params_path = os.path.join(self._params_dir, '{}.model'.format(trial.id))
                    tmp = params_path + '.tmp'
                    with open(tmp, 'wb') as f:
                        f.write(blob)
                    os.replace(tmp, params_path)
            t_dump = time.perf_counter()
            if record:
                self._db.mark_trial_as_complete(trial, score, params_path)
                self.completed_trials.append((trial.id, score))
                # per-trial breakdown (bench phase 2): the model's own phases (load / build / upload /
                # capture / train loop / prepare_eval) when it reports them
                rec.update(train=t_train - t_start, evaluate=t_eval - t_train, dump=t_dump - t_eval,
                           record=time.perf_counter() - t_dump, model=dict(getattr(inst, 'timings', {}) or {}))
                self.trial_records.append(rec)
                ctx.checkpoint.remove()
                # in-process trainer -> predictor handoff: a kept model stays resident in HBM (the
                # params file above remains the durable copy)
                from ..predictor.resident import STORE
                if self._offer_resident and not ctx.data_parallel and STORE.offer(trial.id, inst, score):
                    inst = None
            return score, 1.0
        except Exception:
            logger.error('trial failed:\n%s', traceback.format_exc())
            if record and trial is not None:
                self._db.add_trial_log(trial.id, traceback.format_exc(), 'ERROR')
                self._db.mark_trial_as_errored(trial)
                ctx.checkpoint.remove()
            return float('nan'), 0.0
        finally:
            if inst is not None:
                from ..ops.graphs import quiesced
                with quiesced():   # no other thread may be capturing while the model's graphs die
                    try:
                        inst.destroy()
                    except Exception:
                        pass
                    inst = None
            model_logger.set_logger(prev_logger)
            if handler:
                trial_logger.removeHandler(handler)
            self._db.flush_logs()
            self._trial_id = None

    def stop(self):
        self._stop = True
        if self._trial_id is not None:
            t = self._db.get_trial(self._trial_id)
            if t is not None and t.status in (TrialStatus.STARTED, TrialStatus.RUNNING):
                self._db.mark_trial_as_terminated(t)
        self._db.flush_logs()
