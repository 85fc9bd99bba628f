"""PG-GAN training throughput on one MI355X (BASELINE config #5: pg_gans.py train trial).

Runs the reference architecture (fmap_base 8192, fmap_max 512, latent 512, MNIST-shaped 32x32x1)
with WGAN-GP + mbstd + Gs EMA at a fixed level of detail and reports images/s through the D step
(3 D forwards + double backward) and the G step, per LOD:
  lod 3 = 4x4 (the only LOD the reference's default schedule, total_kimg=2, ever reaches),
  lod 0 = 32x32 (full network, conv-transpose Conv0_up layers active).
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lods', default='3,0')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--minibatch', type=int, default=0, help='0: reference schedule minibatch for the LOD')
    ap.add_argument('--no-graph', action='store_true', help='eager rounds (no hipGraph replay)')
    ap.add_argument('--dtype', default='fp32', choices=('fp32', 'bf16'))
    ap.add_argument('--force-allreduce', action='store_true',
                    help='the data-parallel round on a 1-rank RCCL group: gradients (graph) -> bucketed '
                         'all-reduce (eager) -> mean + Adam + EMA (graph), as PgGan.train runs it at N > 1')
    a = ap.parse_args()
    if a.force_allreduce:
        import socket
        import torch.distributed as dist
        with socket.socket() as so:
            so.bind(('127.0.0.1', 0))
            port = so.getsockname()[1]
        dist.init_process_group('nccl', init_method='tcp://127.0.0.1:{}'.format(port), rank=0, world_size=1,
                                device_id=torch.device('cuda', 0))
    from rafiki_amd.engine.flat import FlatAdam
    from rafiki_amd.models.pg_gan import PgGan, TrainingSchedule
    from rafiki_amd.ops import _lib
    _lib.lib()
    dev = torch.device('cuda', 0)
    m = PgGan(D_repeats=1, minibatch_base=16, G_lrate=1e-3, D_lrate=1e-3, dtype=a.dtype)
    m.device = dev
    m._build([1, 32, 32], 0)
    nets = m.nets
    G_opt = FlatAdam(nets.G, 1e-3, betas=(0.0, 0.99))
    D_opt = FlatAdam(nets.D, 1e-3, betas=(0.0, 0.99))
    for o in (G_opt, D_opt):
        o.skip_flag = torch.zeros(1, dtype=torch.int32, device=dev)
    from rafiki_amd.models.pg_gan import GraphedRounds, TrialRng
    from rafiki_amd.parallel.grad_bucket import FlatGradAllReduce
    rng = TrialRng(dev, 0)
    g_ar = d_ar = None
    if a.force_allreduce:
        g_ar = FlatGradAllReduce(nets.G.grad, nets.G.param_ranges(), list(nets.g_params.values()), 1, force=True)
        d_ar = FlatGradAllReduce(nets.D.grad, nets.D.param_ranges(), list(nets.d_params.values()), 1, force=True)
    acc = torch.zeros(6, device=dev)
    res = {'metric': 'PG-GAN train throughput (images/s through D+G steps), 1 GPU', 'params_G': nets.G.num_params(),
           'params_D': nets.D.num_params(), 'dtype': nets.dtype, 'data': 'synthetic uint8 32x32x1, random-init weights',
           'lods': {}}
    for lod in [float(x) for x in a.lods.split(',')]:
        r = 2 ** (5 - int(lod))
        sched = TrainingSchedule(0, 5, minibatch_base=16)
        mb = a.minibatch or TrainingSchedule.MINIBATCH_DICTS[16].get(r, 16)
        level = torch.randint(0, 256, (4096, 1, r, r), dtype=torch.uint8, device=dev)
        labels = torch.zeros((4096, 0), device=dev)

        graphs = GraphedRounds(not a.no_graph)
        m.set_lod_live(lod)

        def step():
            if a.force_allreduce:
                graphs.run_segments(lod, m.round_segments(lod, mb, level, labels, rng, G_opt, D_opt, acc,
                                                          d_ar=d_ar, g_ar=g_ar, tag=lod))
            else:
                graphs.run(lod, lambda: m.train_round(lod, mb, level, labels, rng, G_opt, D_opt, acc))
        for _ in range(max(2, a.warmup)):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        res['lods'][str(lod)] = {'resolution': r, 'minibatch': mb, 'ms_per_DG_step': round(dt * 1e3, 3),
                                 'images_per_sec': round(mb / dt, 1), 'hipgraph': not a.no_graph,
                                 'dp_segmented_allreduce': a.force_allreduce}
    print(json.dumps(res))
    if a.force_allreduce:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
