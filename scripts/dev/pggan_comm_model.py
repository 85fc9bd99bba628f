"""Communication model of the data-parallel PG-GAN round (docs/architecture.md): parameter bytes of G
and D at the reference configuration (fmap_base 8192, fmap_max 512, latent 512, 32x32x1), their
all-reduce buckets, and which buckets a round at lod 3 (4x4) / lod 0 (32x32) actually touches —
traced on the CPU through FlatGradAllReduce.traced — then the ring all-reduce time per round at
N = 2, 4, 8 over xGMI."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
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
        g_ar = FlatGradAllReduce(nets.G.grad, nets.G.param_ranges(), list(nets.g_params.values()), 1, force=True)
        d_ar = FlatGradAllReduce(nets.D.grad, nets.D.param_ranges(), list(nets.d_params.values()), 1, force=True)
        out['G_params'], out['D_params'] = nets.G.num_params(), nets.D.num_params()
        out['bucket_mb'] = g_ar.bucket_mb
        out['G_buckets_mib'] = [round(4 * (e - a) / 2 ** 20, 2) for a, e in g_ar.buckets]
        out['D_buckets_mib'] = [round(4 * (e - a) / 2 ** 20, 2) for a, e in d_ar.buckets]
        rng = TrialRng(torch.device('cpu'), 0)
        acc = torch.zeros(6)
        for lod in (3.0, 0.0):
            r = 2 ** (5 - int(lod))
            level = torch.randint(0, 256, (64, 1, r, r), dtype=torch.uint8)
            labels = torch.zeros((64, 0))
            segs = m.round_segments(lod, 8, level, labels, rng, G_opt, D_opt, acc, d_ar=d_ar, g_ar=g_ar, tag=lod)
            for kind, fn in segs:
                if kind == 'g':
                    fn()
            res = {}
            for name, ar in (('D', d_ar), ('G', g_ar)):
                plan = [p for t, p in ar._plans.items() if t[0] == lod][0]
                live = sorted(plan['last'])
                res[name + '_live_buckets'] = len(live)
                res[name + '_live_mib'] = round(sum(4 * (ar.buckets[b][1] - ar.buckets[b][0]) for b in live) / 2 ** 20,
                                                2)
            out['lod{}'.format(int(lod))] = res
    # ring all-reduce: each rank sends and receives 2 (N-1)/N of the bytes over one link per hop;
    # effective RCCL ring bandwidth per link on MI355X xGMI taken as ~100 GB/s of the 153 GB/s peak,
    # plus ~15 us per bucket launch / latency
    for lod in ('lod3', 'lod0'):
        mib = out[lod]['D_live_mib'] + out[lod]['G_live_mib']
        nb = out[lod]['D_live_buckets'] + out[lod]['G_live_buckets']
        full = 4 * (out['G_params'] + out['D_params']) / 2 ** 20
        out[lod]['ms_per_round'] = {}
        for n in (2, 4, 8):
            t = lambda b: 2 * (n - 1) / n * b * 2 ** 20 / 100e9 * 1e3 + nb * 0.015
            out[lod]['ms_per_round'][n] = {'live_buckets': round(t(mib), 3), 'whole_arena': round(t(full), 3)}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
