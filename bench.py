#!/usr/bin/env python3
"""Headline benchmark: concurrent VGG-small 32x32x3 HPO trials, one trial per MI355X GPU.

Metric (BASELINE.json): "trials/hour + images/sec/trial, VGG-small 32x32x3; predictor ensemble QPS".
``value`` = aggregate training images/sec over all concurrent trials (= n_gpus x images/sec/trial,
weak scaling: per-GPU work is fixed).  Derived fields: images/sec/trial and trials/hour for the
documented trial definition (``--trial-epochs`` passes over a 50k-image train split).

Flow per rank (torchrun, one process per GPU, RCCL over xGMI):
  1. rank 0's GP-EI advisor proposes ``world_size`` knob sets -> RCCL broadcast (packed fp64);
  2. each rank builds its VGG-small trial on the gfx950 kernel engine, captures the train step
     into a hipGraph, and trains on a synthetic on-device dataset (no network: random-init weights,
     class-conditional synthetic images of the real shape);
  3. W untimed warmup steps, then K timed steps bracketed by barrier + synchronize;
  4. per-rank elapsed -> all-reduce MAX; per-rank (loss, acc) -> all_gather -> advisor feedback.

``python bench.py`` defaults to 1 GPU and finishes in well under a minute.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# multi-process GPU work on this host needs dmabuf IPC (RCCL peer buffers); set before HIP initialises
os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch', type=int, default=256, help='per-trial (per-GPU) batch size')
    ap.add_argument('--dataset-size', type=int, default=50000)
    ap.add_argument('--trial-epochs', type=float, default=10.0)
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--dtype', default=os.environ.get('RAFIKI_DTYPE', 'fp32'), choices=('fp32', 'bf16'),
                    help='compute dtype (fp32 = the reference precision; bf16 is opt-in)')
    return ap.parse_args()


def main():
    args = parse()
    from rafiki_amd.advisor.advisor import GpAdvisor
    from rafiki_amd.engine.convnet import ConvNetEngine
    from rafiki_amd.model.dataset import synthetic_images
    from rafiki_amd.model.knob import FixedKnob, FloatKnob
    from rafiki_amd.ops import autotune
    from rafiki_amd.ops import f32 as S
    from rafiki_amd.ops import functional as F
    from rafiki_amd.parallel import dist as D

    info = D.init_distributed()
    world = info.world_size
    # one GPU per rank; with the gloo rehearsal backend on a smaller box ranks wrap onto the GPUs present
    gpu = info.local_rank if info.backend == 'nccl' else info.local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device('cuda', gpu)

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
    imgs, labels = synthetic_images(args.dataset_size, size=32, channels=3, classes=10,
                                    seed=args.seed + info.rank)
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
    elapsed = time.perf_counter() - t0
    elapsed = D.all_reduce_max(info, elapsed)

    seen = max(1, int(eng.seen.item()))
    loss = float(eng.loss_sum.item()) / seen
    acc = float(eng.correct.item()) / seen
    table = D.gather_floats(info, [loss, acc])
    if info.is_main:
        for r in range(world):  # training accuracy over the timed window as the trial signal
            advisor.feedback(proposals[r], float(table[r, 1]))

    ms = elapsed * 1000.0 / args.steps
    ips_trial = B * args.steps / elapsed
    ips_total = ips_trial * world
    trial_images = args.trial_epochs * args.dataset_size
    trials_per_hour = world * 3600.0 / (trial_images / ips_trial)
    tflops = eng.flops_per_image() * 3 * ips_total / 1e12
    if info.is_main:
        out = {
            'metric': 'images/sec aggregate over concurrent VGG-small 32x32x3 HPO trials (1 trial/GPU)',
            'value': round(ips_total, 1),
            'unit': 'images/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': eng.dtype,
            'data': 'synthetic (class-conditional 32x32x3 images, random-init weights)',
            'config': {'model': 'VGG-small 32x32x3 (8 conv3x3+BN+ReLU, 4 maxpool, FC512, FC10)',
                       'global_batch': B * world, 'per_trial_batch': B, 'seq_len': None,
                       'parallelism': 'trial-parallel x{} (1 trial/GPU, knobs over RCCL)'.format(world),
                       'optimizer': 'SGD nesterov momentum + wd (fused flat-arena kernel)',
                       'hipgraph': use_graph},
            'images_per_sec_per_trial': round(ips_trial, 1),
            'trials_per_hour': round(trials_per_hour, 2),
            'trial_definition': '{} epochs x {} images per trial'.format(args.trial_epochs, args.dataset_size),
            'model_tflops': round(tflops, 2),
            'autotune': dict(autotune.stats),
            'train_loss': round(loss, 4),
            'train_acc': round(acc, 4),
            'knobs_rank0': proposals[0],
        }
        print(json.dumps(out), flush=True)
    D.destroy(info)


if __name__ == '__main__':
    main()
