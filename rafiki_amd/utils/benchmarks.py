"""Measurement phases for the BASELINE.json configs other than the VGG-small headline (bench.py runs them
after its own phases; scripts/bench_configs.py and scripts/bench_pg_gan.py run them stand-alone).

  #1 ``skdt_trials``      SkDt single-trial random-search advisor on CPU: trials/hour through
                          propose -> train -> evaluate -> dump_parameters -> feedback
                          (reference examples/models/image_classification/SkDt.py:12-84)
  #2 ``mlp_trial``        TfFeedForward-style MLP, one trial on one GPU: training images/s
                          (reference TfFeedForward.py:141-164; Flatten -> BN -> Dense+ReLU x L -> Dense, Adam)
  #5 ``pg_gan_rounds``    PG-GAN training rounds (D step with WGAN-GP double backward + Gs EMA + G step) at a
                          fixed level of detail, graphed, one GPU or data-parallel over a process group
                          (reference pg_gans.py:263-343 train loop, :1093-1225 multi-GPU optimizer)

All use synthetic data of the reference shapes and random-init weights.
"""
from __future__ import annotations

import pickle
import time
from typing import Optional, Sequence

import torch

FMNIST_TRAIN = 'synthetic://image?n={n}&size=28&channels=1&classes=10&seed=0'
FMNIST_TEST = 'synthetic://image?n={n}&size=28&channels=1&classes=10&seed=1'


def skdt_trials(n_train: int = 60000, n_test: int = 10000, trials: int = 3, seed: int = 0) -> dict:
    """BASELINE #1 on the CPU: ``trials`` SkDt trials from the random-search advisor (Fashion-MNIST
    shaped synthetic data, 28x28x1, 10 classes); the data is generated once before the timed trials."""
    from rafiki_amd.advisor.advisor import make_advisor
    from rafiki_amd.constants import AdvisorType
    from rafiki_amd.model import dataset_utils
    from rafiki_amd.model.model import load_model_class
    from rafiki_amd.models import model_file
    from rafiki_amd.parallel.context import TrialContext, use_context
    with open(model_file('SkDt'), 'rb') as f:
        clazz = load_model_class(f.read(), 'SkDt')
    adv = make_advisor(clazz.get_knob_config(), AdvisorType.RANDOM, seed=seed)
    train, test = FMNIST_TRAIN.format(n=n_train), FMNIST_TEST.format(n=n_test)
    dataset_utils.load_dataset_of_image_files(train, image_size=28)   # generator cache, as a job's 2nd trial
    dataset_utils.load_dataset_of_image_files(test, image_size=28)
    times, scores, depths = [], [], []
    with use_context(TrialContext(device=torch.device('cpu'))):
        for _ in range(trials):
            t0 = time.perf_counter()
            knobs = adv.propose()
            m = clazz(**knobs)
            m.train(train)
            s = m.evaluate(test)
            pickle.dumps(m.dump_parameters())
            adv.feedback(knobs, s)
            times.append(time.perf_counter() - t0)
            scores.append(float(s))
            depths.append(knobs.get('max_depth'))
    per = sum(times) / len(times)
    return {'config': '#1 SkDt single-trial random-search advisor, CPU', 'metric': 'trials/hour',
            'value': round(3600.0 / per, 1), 'seconds_per_trial': round(per, 3), 'trials': trials,
            'max_depths': depths, 'best_score': round(max(scores), 4),
            'data': 'synthetic Fashion-MNIST-shaped {}+{} 28x28x1'.format(n_train, n_test)}


def mlp_trial(dev: torch.device, n_train: int = 60000, n_test: int = 10000, epochs: int = 2,
              units: int = 128, layers: int = 2, batch_size: int = 128) -> dict:
    """BASELINE #2: one FeedForward trial (the reference's Fixed(2) epochs, the largest knob values:
    2 hidden layers x 128 units, batch 128) on one GPU; images/s over the training epochs including
    the dataset's decode and upload, plus the trial's wall time with evaluation."""
    from rafiki_amd.model import dataset_utils
    from rafiki_amd.model.model import load_model_class
    from rafiki_amd.models import model_file
    from rafiki_amd.parallel.context import TrialContext, use_context
    with open(model_file('FeedForward'), 'rb') as f:
        clazz = load_model_class(f.read(), 'FeedForward')
    knobs = {'epochs': epochs, 'hidden_layer_count': layers, 'hidden_layer_units': units, 'learning_rate': 1e-3,
             'batch_size': batch_size, 'image_size': 28}
    train, test = FMNIST_TRAIN.format(n=n_train), FMNIST_TEST.format(n=n_test)
    dataset_utils.load_dataset_of_image_files(train, image_size=28)
    dataset_utils.load_dataset_of_image_files(test, image_size=28)
    with use_context(TrialContext(device=dev)):
        m = clazz(**knobs)
        t0 = time.perf_counter()
        m.train(train)
        if dev.type == 'cuda':
            torch.cuda.synchronize()
        t_train = time.perf_counter() - t0
        s = m.evaluate(test)
        t_trial = time.perf_counter() - t0
        dtype = m._meta.get('dtype', 'fp32') if hasattr(m, '_meta') else 'fp32'
        m.destroy()
    return {'config': '#2 TfFeedForward-style MLP, 1 trial on 1 {}'.format('MI355X' if dev.type == 'cuda' else 'CPU'),
            'metric': 'training images/s (incl. dataset decode + upload)', 'value': round(n_train * epochs / t_train, 1),
            'trial_seconds': round(t_trial, 3), 'score': round(float(s), 4), 'knobs': knobs, 'dtype': dtype,
            'data': 'synthetic Fashion-MNIST-shaped {}+{} 28x28x1'.format(n_train, n_test)}


def pg_gan_rounds(dev: torch.device, lods: Sequence[float] = (3.0, 0.0), steps: int = 10, warmup: int = 3,
                  minibatch: int = 0, graph: bool = True, dtype: str = 'fp32', force_allreduce: bool = False,
                  info=None, bucket_mb: Optional[float] = None) -> dict:
    """BASELINE #5: PG-GAN rounds (D_repeats=1: one D step + Gs EMA + one G step) of the reference
    architecture (fmap_base 8192, fmap_max 512, latent 512, 32x32x1) at fixed levels of detail:
    lod 3 = 4x4 (the only LOD the reference's total_kimg=2 schedule reaches), lod 0 = 32x32 (whole
    network, the conv-transpose / stride-2 resampling convs active).  ``minibatch`` 0 = the reference
    schedule's GLOBAL minibatch for the resolution (minibatch_base 16: 512 at 4x4, 64 at 32x32).

    With ``info`` of world N > 1 (or ``force_allreduce`` on one rank) the round is the data-parallel
    one PgGan.train runs: each rank draws its shard of the global minibatch (strong scaling, as the
    reference's towers split it, pg_gans.py:290-293), gradients are bucket-all-reduced while the
    backward still replays (parallel/grad_bucket.py BucketedGrads), then mean + Adam + EMA.  Timed
    windows are bracketed by barrier + synchronize; the reported time is the max over ranks."""
    from rafiki_amd.engine.flat import FlatAdam
    from rafiki_amd.models.pg_gan import GraphedRounds, PgGan, TrainingSchedule, TrialRng, grad_bucket_mb
    from rafiki_amd.ops import _lib
    from rafiki_amd.parallel import dist as D
    from rafiki_amd.parallel.context import TrialContext, use_context
    from rafiki_amd.parallel.grad_bucket import FlatGradAllReduce
    if dev.type == 'cuda':
        _lib.lib()
    world = info.world_size if info is not None else 1
    dp = world > 1 or force_allreduce
    ctx = TrialContext(device=dev, dist=info, data_parallel=True) if info is not None else TrialContext(device=dev)
    with use_context(ctx):
        m = PgGan(D_repeats=1, minibatch_base=16, G_lrate=1e-3, D_lrate=1e-3, dtype=dtype)
        m._build([1, 32, 32], 0)
    nets = m.nets
    G_opt = FlatAdam(nets.G, 1e-3, betas=(0.0, 0.99))
    D_opt = FlatAdam(nets.D, 1e-3, betas=(0.0, 0.99))
    for o in (G_opt, D_opt):
        o.skip_flag = torch.zeros(1, dtype=torch.int32, device=dev)
    rng = TrialRng(dev, 0)
    g_ar = d_ar = None
    if dp:
        bmb = float(bucket_mb if bucket_mb is not None else grad_bucket_mb())
        g_ar = FlatGradAllReduce(nets.G.grad, nets.G.param_ranges(), list(nets.g_params.values()), world,
                                 force=world == 1, bucket_mb=bmb)
        d_ar = FlatGradAllReduce(nets.D.grad, nets.D.param_ranges(), list(nets.d_params.values()), world,
                                 force=world == 1, bucket_mb=bmb)
    acc = torch.zeros(6, device=dev)
    res = {'metric': 'PG-GAN train rounds (images/s through D + G steps)', 'params_G': nets.G.num_params(),
           'params_D': nets.D.num_params(), 'dtype': nets.dtype, 'world_size': world,
           'data': 'synthetic uint8 32x32x1, random-init weights', 'lods': {}}
    if dp:
        res['grad_bucket_mb'] = g_ar.bucket_mb
        res['parallelism'] = 'data parallel x{} (bucketed all-reduce overlapped with the graphed backward)'.format(
            world) if world > 1 else 'data-parallel round on a 1-rank group (collectives issued)'
    for lod in lods:
        lod = float(lod)
        r = 2 ** (5 - int(lod))
        g_mb = minibatch or TrainingSchedule.MINIBATCH_DICTS[16].get(r, 16)
        mb = g_mb // world
        level = torch.randint(0, 256, (4096, 1, r, r), dtype=torch.uint8, device=dev)
        labels = torch.zeros((4096, 0), device=dev)
        graphs = GraphedRounds(graph and dev.type == 'cuda')
        m.set_lod_live(lod)
        for ar in (g_ar, d_ar):
            if ar is not None:
                ar.clear_plans()

        def step():
            if dp:
                graphs.run_segments(lod, m.round_segments(lod, mb, level, labels, rng, G_opt, D_opt, acc,
                                                          d_ar=d_ar, g_ar=g_ar, tag=lod))
            else:
                graphs.run(lod, lambda: m.train_round(lod, mb, level, labels, rng, G_opt, D_opt, acc))
        t_setup = time.perf_counter()
        for _ in range(max(2, warmup)):
            step()
        if dev.type == 'cuda':
            torch.cuda.synchronize()
        t_setup = time.perf_counter() - t_setup
        D.barrier(info) if info is not None else None
        if dev.type == 'cuda':
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        if dev.type == 'cuda':
            torch.cuda.synchronize()
        D.barrier(info) if info is not None else None
        if dev.type == 'cuda':
            torch.cuda.synchronize()
        own = time.perf_counter() - t0
        dt = (D.all_reduce_max(info, own) if info is not None else own) / steps
        res['lods'][str(lod)] = {'resolution': r, 'global_minibatch': g_mb, 'minibatch_per_rank': mb,
                                 'ms_per_round': round(dt * 1e3, 3), 'images_per_sec': round(g_mb / dt, 1),
                                 'rounds_timed': steps, 'warmup_rounds_s': round(t_setup, 2),
                                 'hipgraph': graphs.enabled, 'graphs_captured': graphs.captures}
        del level, graphs
    for ar in (g_ar, d_ar):
        if ar is not None:
            ar.remove()
    return res
