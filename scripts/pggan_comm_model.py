"""Communication model of the data-parallel PG-GAN round (docs/architecture.md, "Comm model").

Traces, on the CPU, which gradient buckets a D step and a G step touch at lod 3 (4x4, the reference's
total_kimg=2 schedule) and lod 0 (32x32, whole network) and in which order the backward completes them
(FlatGradAllReduce.traced, the plan the overlapped rounds run), for several bucket sizes.  Then, per
rank count N = 2 / 4 / 8, it models one round:

  compute   the MEASURED 1-GPU round at the per-rank minibatch mb / N (scripts/bench_pg_gan.py --minibatch,
            profiles/pg_gan_dp_rank_shapes_r6.jsonl: lod 3 at mb 512 / 256 / 128 / 64 = 3.70 / 2.72 / 2.01 /
            1.67 ms, lod 0 at mb 64 / 32 / 16 / 8 = 37.0 / 21.8 / 13.2 / 8.8 ms — far from linear in mb:
            small per-rank batches leave the GPU underused); the D step is ~70 % of a round, its backward
            ~60 % of the step, likewise for G;
  buckets   bucket i completes at a point of its step's backward proportional to the position of its
            last gradient contribution in the traced order;
  reduce    a ring all-reduce moves 2 (N-1)/N of the bucket over one xGMI link per hop: ~100 GB/s
            effective of 153 GB/s peak, plus a per-call latency (--latency-us, 25);
  overlap   bucket i's reduce starts when it completes and the previous reduce has ended (one RCCL
            stream); what is left after the step's backward is EXPOSED (the optimizer waits for it).
            Serialised = every reduce after the backward (the round-5 design).

Prints one JSON document: exposed comm ms and its share of the per-rank round, and the round's speedup over one
GPU, per LOD, N and bucket size.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def trace(bucket_mb):
    from rafiki_amd.engine.flat import FlatAdam
    from rafiki_amd.models.pg_gan import PgGan, TrialRng
    from rafiki_amd.parallel.context import TrialContext, use_context
    from rafiki_amd.parallel.grad_bucket import FlatGradAllReduce
    out = {}
    with use_context(TrialContext(device=torch.device('cpu'))):
        m = PgGan(D_repeats=1, minibatch_base=16)
        m._build([1, 32, 32], 0)
        nets = m.nets
        G_opt = FlatAdam(nets.G, 1e-3, betas=(0.0, 0.99))
        D_opt = FlatAdam(nets.D, 1e-3, betas=(0.0, 0.99))
        for o in (G_opt, D_opt):
            o.skip_flag = torch.zeros(1, dtype=torch.int32)
        ars = {'G': FlatGradAllReduce(nets.G.grad, nets.G.param_ranges(), list(nets.g_params.values()), 1,
                                      force=True, bucket_mb=bucket_mb),
               'D': FlatGradAllReduce(nets.D.grad, nets.D.param_ranges(), list(nets.d_params.values()), 1,
                                      force=True, bucket_mb=bucket_mb)}
        out['params'] = {'G': nets.G.num_params(), 'D': nets.D.num_params()}
        rng = TrialRng(torch.device('cpu'), 0)
        acc = torch.zeros(6)
        for lod in (3.0, 0.0):
            r = 2 ** (5 - int(lod))
            level = torch.randint(0, 256, (64, 1, r, r), dtype=torch.uint8)
            labels = torch.zeros((64, 0))
            m.set_lod_live(lod)
            segs = m.round_segments(lod, 8, level, labels, rng, G_opt, D_opt, acc, d_ar=ars['D'], g_ar=ars['G'],
                                    tag=lod)
            for kind, fn in segs:
                if kind != 'e':
                    fn()    # the tracing run (a 1-rank group: no collective is issued without a reduce call)
            res = {}
            for name, ar in ars.items():
                plan = [p for t, p in ar._plans.items() if t[0] == lod][0]
                res[name] = [{'mib': 4 * (ar.buckets[b][1] - ar.buckets[b][0]) / 2 ** 20, 'at': plan['at'][b]}
                             for b in plan['order']]
            out['lod{}'.format(int(lod))] = res
        for ar in ars.values():
            ar.remove()
    return out


def model(buckets, t_bwd, t_after, n, bw_gbs, lat_us):
    """(exposed ms, serialised ms) of one step's reduces: buckets complete at ``at`` * t_bwd ms."""
    end = 0.0
    serial = 0.0
    for b in buckets:
        t = lat_us * 1e-3 + 2 * (n - 1) / n * b['mib'] * 2 ** 20 / (bw_gbs * 1e9) * 1e3
        end = max(end, b['at'] * t_bwd) + t
        serial += t
    return max(0.0, end - t_bwd - t_after), serial


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--buckets', default='4,8,16,32')
    ap.add_argument('--t-lod3', default='3.70,2.717,2.012,1.666', help='measured rounds (ms) at mb 512/N, N=1,2,4,8')
    ap.add_argument('--t-lod0', default='37.0,21.75,13.203,8.834', help='measured rounds (ms) at mb 64/N, N=1,2,4,8')
    ap.add_argument('--bw-gbs', type=float, default=100.0)
    ap.add_argument('--latency-us', type=float, default=25.0)
    a = ap.parse_args()
    rt = {lod: dict(zip((1, 2, 4, 8), [float(x) for x in v.split(',')])) for lod, v in (('lod3', a.t_lod3),
                                                                                       ('lod0', a.t_lod0))}
    out = {'assumptions': {'per_rank_round_ms': rt, 'ring_bw_gbs': a.bw_gbs, 'latency_us': a.latency_us,
                           'D_share_of_round': 0.7, 'backward_share_of_step': 0.6}, 'bucket_mb': {}}
    for bmb in [float(x) for x in a.buckets.split(',')]:
        tr = trace(bmb)
        out['params'] = tr['params']
        per = {}
        for lod in ('lod3', 'lod0'):
            rows = {'live_buckets': {k: len(v) for k, v in tr[lod].items()},
                    'live_mib': {k: round(sum(b['mib'] for b in v), 1) for k, v in tr[lod].items()}}
            for n in (2, 4, 8):
                rnd = rt[lod][n]
                exp = ser = 0.0
                for name, share in (('D', 0.7), ('G', 0.3)):
                    step = rnd * share
                    e, s = model(tr[lod][name], 0.6 * step, 0.0, n, a.bw_gbs, a.latency_us)
                    exp += e
                    ser += s
                rows['N{}'.format(n)] = {'per_rank_round_ms': round(rnd, 3), 'exposed_ms': round(exp, 3),
                                         'exposed_share': round(exp / (rnd + exp), 3), 'serialised_ms': round(ser, 3),
                                         'serialised_share': round(ser / (rnd + ser), 3),
                                         'speedup_vs_1gpu': round(rt[lod][1] / (rnd + exp), 2)}
            per[lod] = rows
        out['bucket_mb'][str(bmb)] = per
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
