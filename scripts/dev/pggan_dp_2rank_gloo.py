"""Two-process rehearsal of the data-parallel PG-GAN round on ONE GPU (both ranks on cuda:0, gloo standing in
for RCCL, which refuses two ranks on one device).

Each rank draws the global minibatch with the same Philox counters and keeps its shard (PgGan._shard);
the round runs as GraphedRounds segments — gradients (graph) -> bucketed all-reduce (eager, between
replays) -> mean + finite guard + Adam + Gs EMA (graph) — exactly as PgGan.train runs it at N > 1.
Checks that after the timed rounds the G, D and Gs weights are bit-identical on both ranks (the
all-reduced gradients keep the replicas in lock step) and that the losses are finite.  Rank 0 prints
one JSON line.  Not a throughput number: both ranks share one GPU.

usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
         scripts/dev/pggan_dp_2rank_gloo.py --lods 3,0 --rounds 6
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lods', default='3,0')
    ap.add_argument('--rounds', type=int, default=6)
    a = ap.parse_args()
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    from rafiki_amd.engine.flat import FlatAdam
    from rafiki_amd.models.pg_gan import GraphedRounds, PgGan, TrainingSchedule, TrialRng
    from rafiki_amd.ops import _lib
    from rafiki_amd.parallel.grad_bucket import FlatGradAllReduce
    _lib.lib()
    dev = torch.device('cuda', 0)
    m = PgGan(D_repeats=1, minibatch_base=16, G_lrate=1e-3, D_lrate=1e-3)
    m.device = dev
    m.world, m.rank = world, rank
    m._build([1, 32, 32], 0)
    nets = m.nets
    G_opt = FlatAdam(nets.G, 1e-3, betas=(0.0, 0.99))
    D_opt = FlatAdam(nets.D, 1e-3, betas=(0.0, 0.99))
    for o in (G_opt, D_opt):
        o.skip_flag = torch.zeros(1, dtype=torch.int32, device=dev)
    g_ar = FlatGradAllReduce(nets.G.grad, nets.G.param_ranges(), list(nets.g_params.values()), world)
    d_ar = FlatGradAllReduce(nets.D.grad, nets.D.param_ranges(), list(nets.d_params.values()), world)
    rng = TrialRng(dev, 0)   # same seed on every rank: the same global draws, then each rank's shard
    acc = torch.zeros(6, device=dev)
    out = {'world': world, 'backend': 'gloo', 'device': 'cuda:0 shared by both ranks', 'lods': {}}
    for lod in [float(x) for x in a.lods.split(',')]:
        r = 2 ** (5 - int(lod))
        mb_global = TrainingSchedule.MINIBATCH_DICTS[16].get(r, 16)
        mb = mb_global // world
        gen = torch.Generator().manual_seed(123)   # identical dataset on every rank
        level = torch.randint(0, 256, (4096, 1, r, r), dtype=torch.uint8, generator=gen).to(dev)
        labels = torch.zeros((4096, 0), device=dev)
        graphs = GraphedRounds(True)
        m.set_lod_live(lod)   # as PgGan.train / utils.benchmarks.pg_gan_rounds run a level of detail

        def rnd():
            graphs.run_segments(lod, m.round_segments(lod, mb, level, labels, rng, G_opt, D_opt, acc, d_ar=d_ar,
                                                      g_ar=g_ar, tag=lod))
        for _ in range(3):
            rnd()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.rounds):
            rnd()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.rounds
        sums = torch.stack([nets.G.master.double().sum(), nets.D.master.double().sum(), nets.Gs_master.double().sum(),
                            nets.G.master.double().square().sum(), nets.D.master.double().square().sum()]).cpu()
        allsums = [torch.zeros_like(sums) for _ in range(world)]
        dist.all_gather(allsums, sums)
        same = all(torch.equal(allsums[0], s) for s in allsums[1:])
        finite = bool(torch.isfinite(acc).all().item())
        out['lods'][str(lod)] = {'global_minibatch': mb_global, 'per_rank_minibatch': mb, 'graph_segments_captured':
                                 graphs.captures, 'ms_per_round_shared_gpu': round(dt * 1e3, 3),
                                 'replicas_bit_identical': same, 'losses_finite': finite}
        if not (same and finite):
            out['ok'] = False
    out.setdefault('ok', True)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if out['ok'] else 1)


if __name__ == '__main__':
    main()
