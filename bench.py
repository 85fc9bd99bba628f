#!/usr/bin/env python3
"""Headline benchmark: VGG-small 32x32x3 HPO trials, one trial per MI355X GPU, fp32 (the reference's
precision; ``--dtype bf16`` opts into the bf16 engine).

Metric (BASELINE.json): "trials/hour + images/sec/trial, VGG-small 32x32x3; predictor ensemble QPS".
Every part of it is measured in this run, none extrapolated:

  phase 1  images/sec/trial (the JSON ``value`` = aggregate over all GPUs, weak scaling: per-GPU work
           is fixed): rank 0's GP-EI advisor proposes one knob set per rank (broadcast over RCCL as
           packed fp64 when N > 1), every rank captures its VGG-small training step (device-side minibatch
           gather + fwd + bwd + fused SGD) into one hipGraph and replays it on a device-resident
           synthetic dataset; W untimed warmup steps, then K timed steps bracketed by barrier +
           synchronize on both sides, max over ranks.
  phase 2  trials/hour: the real AutoML loop — ``TrainWorker`` (async trial scheduling, atomic budget
           claims in the SQLite store, knobs/scores exchanged with rank 0's single GP-EI advisor over
           RCCL, constant-liar pending points) runs propose -> train -> evaluate -> pickle params ->
           record score for ``--trials`` trials per GPU of the ``VggSmallTrial`` definition (10 epochs
           over 50k non-separable synthetic CIFAR-shaped images, evaluated on 10k), after one untimed
           warm-up trial per GPU; wall time max over ranks; per-trial breakdown of rank 0.
  phase 2b overhead probe: ``--probe-trials`` trials per GPU of ``VggSmallProbe`` (2 epochs x 8192
           images), where per-trial fixed costs dominate.
  phase 3  predictor ensemble QPS (rank 0, 1 GPU): the top-4 trials of phase 2 loaded from their
           params files into one ``Predictor``; hipGraph-captured forwards on 4 HIP streams + the
           on-device ensemble mean, device-resident uint8 batches of 256 (plus the batch-1 latency
           and the host-array API path); then POST /predict through the native HTTP front end under
           64 closed-loop JSON clients and 8 .npy batch-128 clients from a separate load-generator
           process (``ensemble_http_qps`` with p50 / p99, rafiki_amd/predictor/loadgen.py).
  phase 4  the other BASELINE.json configs (rafiki_amd/utils/benchmarks.py), each with its own config and
           dtype in the JSON (``baseline_configs``):
             #5 PG-GAN train rounds, reference architecture, fp32, graphed: lod 3 (4x4, mb 512, the
                reference's total_kimg=2 schedule) and lod 0 (32x32, mb 64, whole network).  N = 1:
                in-process; N > 1: rank 0 starts N fresh ranks (their own RCCL group, bounded by a
                timeout) running the DATA-PARALLEL round over all N GPUs (global minibatch split, bucketed
                all-reduce overlapped with the graphed backward) while the bench's ranks wait;
             #2 FeedForward (TfFeedForward-style MLP) trial on 1 GPU (N = 1 only);
             #1 SkDt random-search trials on the CPU (N = 1 only).

``python bench.py`` defaults to 1 GPU and finishes in a few minutes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

# multi-process GPU work on this host needs dmabuf IPC (RCCL peer buffers); set before HIP initialises
os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# phase 2 headline trial: CIFAR-10-sized synthetic splits (50k train / 10k test, 32x32x3, 10 classes)
TRAIN_URI = 'synthetic://image?n=50000&size=32&channels=3&classes=10&seed=0&noise=64&flip=0.1'
TEST_URI = 'synthetic://image?n=10000&size=32&channels=3&classes=10&seed=1&noise=64&flip=0.1'
# phase 2b overhead probe: ~64 training steps per trial
PROBE_TRAIN_URI = 'synthetic://image?n=8192&size=32&channels=3&classes=10&seed=0&noise=64&flip=0.1'
PROBE_TEST_URI = 'synthetic://image?n=2048&size=32&channels=3&classes=10&seed=1&noise=64&flip=0.1'


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch', type=int, default=256, help='per-trial (per-GPU) batch size')
    ap.add_argument('--dataset-size', type=int, default=50000)
    ap.add_argument('--trials', type=int, default=2, help='timed VggSmallTrial trials per GPU in phase 2 (0: skip)')
    ap.add_argument('--probe-trials', type=int, default=4, help='timed overhead-probe trials per GPU (0: skip)')
    ap.add_argument('--no-serving', action='store_true', help='skip phase 3')
    ap.add_argument('--configs', default='auto',
                    help="phase 4: comma list of pggan,mlp,skdt (auto: all at N = 1, pggan at N > 1; none: skip)")
    ap.add_argument('--skdt-trials', type=int, default=3)
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--dtype', default=os.environ.get('RAFIKI_DTYPE', 'fp32'), choices=('fp32', 'bf16'),
                    help='compute dtype (fp32 = the reference precision; bf16 is opt-in)')
    return ap.parse_args()


def phase_throughput(args, info, dev):
    from rafiki_amd.advisor.advisor import GpAdvisor
    from rafiki_amd.engine.convnet import ConvNetEngine
    from rafiki_amd.model.dataset import synthetic_images
    from rafiki_amd.model.knob import FixedKnob, FloatKnob
    from rafiki_amd.ops import f32 as S
    from rafiki_amd.ops import functional as F
    from rafiki_amd.parallel import dist as D

    world = info.world_size
    knob_config = {
        'lr': FloatKnob(1e-3, 2e-1, is_exp=True),
        'momentum': FloatKnob(0.8, 0.95),
        'weight_decay': FloatKnob(1e-5, 1e-3, is_exp=True),
        'batch_size': FixedKnob(args.batch),
    }
    advisor = GpAdvisor(knob_config, seed=args.seed) if info.is_main else None
    proposals = advisor.propose_batch(world) if info.is_main else None
    proposals = D.broadcast_proposals(info, knob_config, proposals)
    knobs = proposals[info.rank]

    eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=32, device=dev, seed=args.seed + info.rank,
                        lr=knobs['lr'], momentum=knobs['momentum'], weight_decay=knobs['weight_decay'],
                        dtype=args.dtype)
    # synthetic CIFAR-shaped data, resident in HBM as packed NHWC in the engine's dtype
    imgs, labels = synthetic_images(args.dataset_size, size=32, channels=3, classes=10, seed=args.seed + info.rank)
    x_u8 = torch.from_numpy(imgs).permute(0, 3, 1, 2).contiguous().to(dev)
    pack = S.pack_nhwc if eng.f32 else F.pack_nhwc
    data = pack(x_u8, eng.cin_p, 1.0 / 127.5, -1.0)
    del x_u8
    y_all = torch.from_numpy(labels).to(dev, torch.int32)
    B = args.batch
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + 17 * info.rank)
    total_steps = args.warmup + args.steps
    idx = torch.randint(0, args.dataset_size, (total_steps, B), device=dev, generator=gen)
    xb = torch.empty((B, 32, 32, eng.cin_p), dtype=eng.act_dtype, device=dev)
    yb = torch.empty((B,), dtype=torch.int32, device=dev)
    use_graph = not args.no_graph
    if use_graph:
        # one hipGraph per step: minibatch gather (device-side step counter) + fwd + bwd + optimizer
        eng.capture_scheduled(data, y_all, total_steps, B)
        eng.set_schedule(idx)

    def step(i):
        if use_graph:
            eng.replay()
            return
        torch.index_select(data, 0, idx[i], out=xb)
        torch.index_select(y_all, 0, idx[i], out=yb)
        eng.train_step(xb, yb)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    D.barrier(info)
    torch.cuda.synchronize()
    eng.reset_metrics()
    t0 = time.perf_counter()
    for i in range(args.warmup, total_steps):
        step(i)
    torch.cuda.synchronize()
    D.barrier(info)
    torch.cuda.synchronize()
    own = time.perf_counter() - t0
    elapsed = D.all_reduce_max(info, own)
    seen = max(1, int(eng.seen.item()))
    loss = float(eng.loss_sum.item()) / seen
    acc = float(eng.correct.item()) / seen
    table = D.gather_floats(info, [loss, acc])
    if info.is_main:
        for r in range(world):  # training accuracy over the timed window as the trial signal
            advisor.feedback(proposals[r], float(table[r, 1]))
    out = dict(elapsed=elapsed, own_elapsed=own, loss=loss, acc=acc, knobs=proposals[0], dtype=eng.dtype,
               train_flops_per_image=eng.train_flops_per_image(), use_graph=use_graph)
    del eng, data, y_all
    torch.cuda.empty_cache()
    return out


def _setup_job(db, budget, model_name, model_class, train_uri, test_uri):
    from rafiki_amd.models import model_file
    from rafiki_amd.utils.auth import hash_password
    u = db.get_user_by_email('bench@rafiki') or db.create_user('bench@rafiki', hash_password('bench'), 'ADMIN')
    tag = str(time.time_ns())
    with open(model_file(model_name), 'rb') as f:
        m = db.create_model(u.id, model_class + '_' + tag, 'IMAGE_CLASSIFICATION', f.read(), model_class,
                            'rafiki_amd', {}, 'PRIVATE')
    tj = db.create_train_job(u.id, 'bench_' + tag, 1, 'IMAGE_CLASSIFICATION', budget, train_uri, test_uri)
    sub = db.create_sub_train_job(tj.id, m.id, u.id)
    svc = db.create_service('TRAIN', 'bench', 'rafiki_amd', 1, 1)
    db.create_train_job_worker(svc.id, sub.id)
    return svc.id, sub.id


def _mean_breakdown(records):
    """Mean per-trial seconds: worker phases + the model's own phases (build / capture / loop / ...)."""
    if not records:
        return {}
    out = {}
    for k in ('claim', 'propose', 'train', 'evaluate', 'dump', 'record'):
        vals = [r[k] for r in records if k in r]
        if vals:
            out[k] = round(sum(vals) / len(vals), 4)
    mk = sorted({k for r in records for k in r.get('model', {})})
    for k in mk:
        vals = [r['model'][k] for r in records if k in r.get('model', {})]
        out['train.' + k] = round(sum(vals) / len(vals), 4)
    return out


def phase_trials(args, info, root, model_class, per_gpu, train_uri, test_uri, warm=True):
    """Timed sub-train-job of ``per_gpu`` trials per GPU (after an untimed warm-up one: one trial per
    GPU).  Returns wall time (max over ranks), completed count, scores and rank 0's breakdown."""
    from rafiki_amd.db.database import Database
    from rafiki_amd.parallel import dist as D
    from rafiki_amd.worker.train import TrainWorker
    world = info.world_size
    db_path = os.path.join(root, 'bench.sqlite3')
    params = os.path.join(root, 'params')
    os.environ['WORKDIR_PATH'] = root
    os.environ['RAFIKI_DTYPE'] = args.dtype
    ids = None
    if info.is_main:
        os.makedirs(params, exist_ok=True)
        db = Database(db_path)
        w_ids = _setup_job(db, {'MODEL_TRIAL_COUNT': world}, model_class, model_class, train_uri, test_uri) \
            if warm else (None, None)
        timed = _setup_job(db, {'MODEL_TRIAL_COUNT': world * per_gpu}, model_class, model_class, train_uri, test_uri)
        ids = [w_ids[0], w_ids[1], timed[0], timed[1]]
    ids = D.broadcast_object(info, ids)
    db = Database(db_path)
    first = None
    if warm:
        t0 = time.perf_counter()
        w = TrainWorker(ids[0], 'bench-w{}'.format(info.rank), db=db, dist_info=info, seed=args.seed,
                        scheduling='async', params_dir=params, offer_resident=True)
        w.start()
        first = dict(_mean_breakdown(w.trial_records), wall=round(time.perf_counter() - t0, 3))
    D.barrier(info)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    w = TrainWorker(ids[2], 'bench-w{}'.format(info.rank), db=db, dist_info=info, seed=args.seed + 1,
                    scheduling='async', params_dir=params, offer_resident=True)
    w.start()
    torch.cuda.synchronize()
    mine = time.perf_counter() - t0
    D.barrier(info)
    wall = D.all_reduce_max(info, mine)
    busy = D.gather_floats(info, [mine, w.busy_s, len(w.completed_trials)])
    trials = db.get_trials_of_sub_train_job(ids[3])
    done = [t for t in trials if t.status == 'COMPLETED']
    scores = sorted((float(t.score) for t in done), reverse=True)
    steady = _mean_breakdown(w.trial_records)
    ex = getattr(w, 'exchange', None)
    return dict(wall=wall, n=len(done), errored=len(trials) - len(done), scores=scores, sub=ids[3], db=db,
                busy=[float(b) for b in busy[:, 1]], per_rank=[int(c) for c in busy[:, 2]], first=first,
                steady=steady, exchange=dict(ex.stats) if (ex is not None and info.is_main) else None)


def phase_serving(db, sub_id, dev, k=4, batch=256, iters=30, http_seconds=3.0):
    import pickle

    import numpy as np

    from rafiki_amd.model.model import load_model_class
    from rafiki_amd.predictor.predictor import Predictor
    trials = [t for t in db.get_trials_of_sub_train_job(sub_id) if t.status == 'COMPLETED']
    trials.sort(key=lambda t: -float(t.score))
    top = trials[:k]
    if len(top) < k:
        return None
    from rafiki_amd.predictor.resident import STORE
    models = []
    from_hbm = 0
    t_load = time.perf_counter()
    for t in top:
        inst = STORE.take(t.id)   # trained in this process: still resident in HBM (no params-file read)
        if inst is not None and str(getattr(inst, 'device', '')) == str(dev):
            from_hbm += 1
        else:
            mrec = db.get_model(db.get_sub_train_job(t.sub_train_job_id).model_id)
            clazz = load_model_class(mrec.model_file_bytes, mrec.model_class)
            inst = clazz(**(t.knobs or {}))
            with open(t.params_file_path, 'rb') as f:
                inst.load_parameters(pickle.loads(f.read()))
        models.append((t.id, inst))
    t_load = time.perf_counter() - t_load
    pred = Predictor(models, max_batch=512)
    rng = np.random.default_rng(0)
    sig = models[0][1].input_signature()
    out = {'models': k, 'load_s': round(t_load, 3), 'loaded_from_hbm': from_hbm}

    def timed(fn, n):
        fn()
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n

    for b in (1, batch):
        x = torch.from_numpy(rng.integers(0, 256, (b, 32, 32, 3), dtype=np.uint8)).to(dev)
        dt = timed(lambda: pred.predict_proba_device({sig: x}), iters)
        out['device_b{}'.format(b)] = {'qps': round(b / dt, 1), 'ms': round(dt * 1e3, 3)}
    arr = rng.integers(0, 256, (batch, 32, 32, 3), dtype=np.uint8)
    dt = timed(lambda: pred.predict_array(arr), max(3, iters // 3))
    out['host_array_b{}'.format(batch)] = {'qps': round(batch / dt, 1), 'ms': round(dt * 1e3, 3)}
    # the BASELINE metric's own path: POST /predict through the native HTTP front end, loaded from a separate
    # process (64 single-query JSON clients, then 8 clients posting .npy batches of 128)
    from rafiki_amd.predictor import loadgen
    if loadgen.available():
        pred.start()
        try:
            out['http'] = loadgen.http_load(pred, seconds=http_seconds, json_sweep=(16, 256), npy_sweep=(16,),
                                            sweep_seconds=2.0)
        except Exception as e:   # the device numbers above stand; say why HTTP is missing
            out['http'] = {'error': '{}: {}'.format(type(e).__name__, e)[:300]}
        finally:
            pred.stop()
    return out


def _progress(info, msg):
    """A progress line on stderr (rank 0; stdout carries only the final JSON line)."""
    if info.is_main:
        sys.stderr.write('[bench {:.0f}s] {}\n'.format(time.perf_counter() - _T0, msg))
        sys.stderr.flush()


_T0 = time.perf_counter()


def _configs(args, world):
    if args.configs == 'none':
        return []
    if args.configs == 'auto':
        return ['pggan', 'mlp', 'skdt'] if world == 1 else ['pggan']
    return [c for c in args.configs.split(',') if c]


def phase_pg_gan(args, info, dev):
    """BASELINE #5 (see the module docstring).  Returns the phase's JSON dict (or an error record)."""
    from rafiki_amd.utils.benchmarks import pg_gan_rounds
    if info.world_size == 1:
        try:
            return pg_gan_rounds(dev, lods=(3.0, 0.0), steps=20, warmup=3, dtype='fp32')
        except Exception as e:   # the other phases' numbers stand; say why this one is missing
            return {'error': '{}: {}'.format(type(e).__name__, e)[:300]}
    # N > 1: N fresh ranks (own process group) so a hung collective is bounded by the spawn timeout and
    # the bench's own ranks are untouched; they wait on the rendezvous store, not in a collective
    import io
    from torch.distributed import distributed_c10d as c10d

    from rafiki_amd.parallel import launch as L
    store = c10d._get_default_store()
    key = 'rafiki/bench/pggan_dp_done'
    res = None
    if info.is_main:
        buf = io.StringIO()
        timeout = float(os.environ.get('RAFIKI_BENCH_PGGAN_DP_TIMEOUT_S', '420'))
        t0 = time.perf_counter()
        rc = L.spawn([sys.executable, '-u', os.path.join(ROOT, 'scripts', 'bench_pg_gan.py'), '--lods', '3,0',
                      '--steps', '20', '--warmup', '3'], info.world_size, out=buf, timeout_s=timeout)
        lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith('{')]
        res = json.loads(lines[-1]) if (rc == 0 and lines) else {'error': 'rc={} after {:.0f} s'.format(
            rc, time.perf_counter() - t0), 'tail': buf.getvalue()[-500:]}
        store.set(key, '1')
    else:
        store.wait([key], __import__('datetime').timedelta(seconds=900))
    return res


def phase_small_configs(args, dev, which):
    from rafiki_amd.utils.benchmarks import mlp_trial, skdt_trials
    out = {}
    if 'mlp' in which:
        try:
            out['mlp'] = mlp_trial(dev)
        except Exception as e:
            out['mlp'] = {'error': '{}: {}'.format(type(e).__name__, e)[:300]}
    if 'skdt' in which and args.skdt_trials > 0:
        try:
            out['skdt'] = skdt_trials(trials=args.skdt_trials)
        except Exception as e:
            out['skdt'] = {'error': '{}: {}'.format(type(e).__name__, e)[:300]}
    return out


def main():
    args = parse()
    from rafiki_amd.config import NodeConfig
    from rafiki_amd.parallel import dist as D
    from rafiki_amd.parallel import launch as L

    backend = NodeConfig().dist_backend
    if not L.under_launcher():
        if args.gpus > 1:
            # started without torchrun: spawn one rank per GPU before this process touches HIP
            L.check_devices(args.gpus, backend)
            sys.exit(L.spawn([sys.executable, '-u', os.path.abspath(__file__)] + sys.argv[1:], args.gpus))
    elif int(os.environ['WORLD_SIZE']) != args.gpus:
        raise SystemExit('bench: WORLD_SIZE={} but --gpus {}'.format(os.environ['WORLD_SIZE'], args.gpus))
    elif args.gpus > 1:
        L.check_devices(args.gpus, backend)

    info = D.init_distributed()
    world = info.world_size
    assert world == args.gpus, (world, args.gpus)
    ndev = max(1, torch.cuda.device_count())
    # one GPU per rank; the gloo rehearsal backend wraps ranks onto the GPUs present
    gpu = info.local_rank if info.backend == 'nccl' else info.local_rank % ndev
    torch.cuda.set_device(gpu)
    dev = torch.device('cuda', gpu)
    n_devices = world if info.backend in ('nccl', 'none') else min(world, ndev)

    pre = None
    if world > 1:
        # bounded-time check of every collective and rank-0 <-> peer P2P pair before any timed work (a
        # missing peer or unusable link ends the run with a named step instead of a hang)
        from rafiki_amd.parallel.exchange import control_group
        pre = D.preflight(info, timeout_s=float(os.environ.get('RAFIKI_PREFLIGHT_TIMEOUT_S', '120')),
                          group=control_group(info))

    _progress(info, 'phase 1: VGG-small training step (capture + {} warmup + {} timed)'.format(args.warmup,
                                                                                               args.steps))
    th = phase_throughput(args, info, dev)
    _progress(info, 'phase 1 done: {:.4f} ms/step'.format(th['elapsed'] * 1000.0 / args.steps))
    B = args.batch
    ms = th['elapsed'] * 1000.0 / args.steps
    ips_trial = B * args.steps / th['elapsed']
    ips_total = ips_trial * world if n_devices == world else None  # no aggregate when ranks share a GPU
    # per-rank rates from each rank's own timed window (the headline uses the max-over-ranks time)
    per_rank = D.gather_floats(info, [B * args.steps / th['own_elapsed']])[:, 0].tolist()

    trials = probe = None
    serving = None
    tag = os.environ.get('MASTER_PORT', '0') if world > 1 else str(os.getpid())
    root = os.path.join(tempfile.gettempdir(), 'rafiki_bench_{}'.format(tag))
    if args.trials > 0:
        _progress(info, 'phase 2: VggSmallTrial trials')
        trials = phase_trials(args, info, root, 'VggSmallTrial', args.trials, TRAIN_URI, TEST_URI)
    if args.probe_trials > 0:
        _progress(info, 'phase 2b: overhead-probe trials')
        probe = phase_trials(args, info, root, 'VggSmallProbe', args.probe_trials, PROBE_TRAIN_URI, PROBE_TEST_URI,
                             warm=False)
    src = probe or trials
    if src is not None and info.is_main and not args.no_serving:
        _progress(info, 'phase 3: ensemble serving (device, then HTTP)')
        serving = phase_serving(src['db'], src['sub'], dev)

    which = _configs(args, world)
    cfgs = {}
    # ranks sharing a GPU (gloo rehearsal) skip it unless RAFIKI_BENCH_PGGAN_REHEARSAL=1 (the spawn / store path)
    if 'pggan' in which and (n_devices == world or os.environ.get('RAFIKI_BENCH_PGGAN_REHEARSAL') == '1'):
        D.barrier(info)
        _progress(info, 'phase 4: PG-GAN rounds' + (' (data parallel x{})'.format(world) if world > 1 else ''))
        cfgs['pg_gan'] = phase_pg_gan(args, info, dev)
    if info.is_main and world == 1 and ('mlp' in which or 'skdt' in which):
        _progress(info, 'phase 4: FeedForward trial, SkDt trials')
        cfgs.update(phase_small_configs(args, dev, which))
    _progress(info, 'done')

    if info.is_main:
        out = {
            'metric': 'images/sec aggregate over concurrent VGG-small 32x32x3 HPO trials (1 trial/GPU)',
            'value': round(ips_total, 1) if ips_total is not None else None,
            'unit': 'images/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': th['dtype'],
            'data': 'synthetic (class-conditional 32x32x3 images, random-init weights)',
            'config': {'model': 'VGG-small 32x32x3 (8 conv3x3+BN+ReLU, 4 maxpool, FC512, FC10)',
                       'global_batch': B * world, 'per_trial_batch': B, 'seq_len': None,
                       'parallelism': 'trial-parallel x{} (1 trial/GPU)'.format(world) if world > 1 else
                       'single trial, 1 GPU',
                       'optimizer': 'SGD nesterov momentum + wd (fused flat-arena kernel)',
                       'hipgraph': th['use_graph']},
            'backend': info.backend,
            'world_size': D.world_size(info),
            'n_devices': n_devices,
            # ranks sharing GPUs (gloo rehearsal of the control path on a smaller box): no aggregate
            'rehearsal': n_devices < world,
            'images_per_sec_per_rank_min': round(min(per_rank), 1),
            'images_per_sec_per_rank_max': round(max(per_rank), 1),
            'images_per_sec_per_trial': round(ips_trial, 1),
            # direct-computation model FLOPs / time (the Winograd convs execute 4/9 of the conv MACs)
            'model_tflops': round(th['train_flops_per_image'] * ips_trial * n_devices / 1e12, 2),
            'train_loss': round(th['loss'], 4),
            'train_acc': round(th['acc'], 4),
            'knobs_rank0': th['knobs'],
        }
        if trials is not None:
            out['trials_per_hour_measured'] = round(trials['n'] * 3600.0 / trials['wall'], 1)
            out['trials_measured'] = trials['n']
            out['trials_errored'] = trials['errored']
            out['trials_wall_s'] = round(trials['wall'], 3)
            out['trials_per_rank'] = trials['per_rank']
            out['trial_busy_s_per_rank'] = [round(b, 3) for b in trials['busy']]
            via = ('from rank 0 over {} point-to-point'.format('RCCL' if info.backend == 'nccl' else info.backend)
                   if world > 1 else 'from the in-process advisor (1 rank: no collective in the path)')
            out['trial_definition'] = ('VggSmallTrial: GP-EI knobs (lr, momentum, wd) {}, '
                                       '10 epochs x 50000 synthetic CIFAR-shaped images, batch 256 + eval on '
                                       '10000, params pickled; async scheduling; after 1 untimed warm-up trial/GPU'
                                       .format(via))
            out['trial_scores'] = [round(s, 4) for s in trials['scores']]
            out['trial_breakdown_s'] = {'first_trial_rank0': trials['first'], 'steady_mean_rank0': trials['steady']}
            if trials['exchange'] is not None:
                out['knob_exchange'] = {k: (round(v, 4) if isinstance(v, float) else v)
                                        for k, v in trials['exchange'].items()}
        if probe is not None:
            out['probe_trials_per_hour'] = round(probe['n'] * 3600.0 / probe['wall'], 1)
            out['probe_trials_measured'] = probe['n']
            out['probe_definition'] = 'VggSmallProbe: 2 epochs x 8192 images + eval 2048 (~64 steps; overhead probe)'
            out['probe_breakdown_s'] = probe['steady']
        if pre is not None:
            out['preflight'] = pre
        if serving is not None:
            out['ensemble_qps'] = serving['device_b256']['qps']
            http = serving.get('http') or {}
            if 'json_single_query' in http:
                js, nb = http['json_single_query'], http.get('npy_batch128', {})
                out['ensemble_http_qps'] = js['qps']
                out['ensemble_http_p50_ms'], out['ensemble_http_p99_ms'] = js['p50_ms'], js['p99_ms']
                out['ensemble_http_npy_b128_qps'] = nb.get('qps')
                best = max([nb] + http.get('npy_sweep', []), key=lambda r: r.get('qps') or 0)
                out['ensemble_http_npy_b128_qps_max'] = {'qps': best.get('qps'), 'clients': best.get('clients')}
                for key, rows in (('json', [js] + http.get('json_sweep', [])), ('npy_b128', [nb] + http.get('npy_sweep', []))):
                    out['ensemble_http_{}_sweep'.format(key)] = sorted(
                        ({'clients': r.get('clients'), 'qps': r.get('qps'), 'p50_ms': r.get('p50_ms'),
                          'p99_ms': r.get('p99_ms'), 'mean_batch': r.get('mean_batch')} for r in rows if r),
                        key=lambda r: r['clients'] or 0)
            out['ensemble'] = serving
        if cfgs:
            pg = cfgs.get('pg_gan') or {}
            for lod, k in (('3.0', 'pg_gan_lod3_img_s'), ('0.0', 'pg_gan_lod0_img_s')):
                if lod in pg.get('lods', {}):
                    out[k] = pg['lods'][lod]['images_per_sec']
            if 'value' in cfgs.get('mlp', {}):
                out['mlp_img_s'] = cfgs['mlp']['value']
            if 'value' in cfgs.get('skdt', {}):
                out['skdt_trials_per_hour'] = cfgs['skdt']['value']
            out['baseline_configs'] = cfgs
        print(json.dumps(out), flush=True)
    D.destroy(info)


if __name__ == '__main__':
    main()
