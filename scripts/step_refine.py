"""Step-level refinement of the tune database (run on the GPU box).

``--workload pggan --lod L``: the same re-ranking on the captured PG-GAN D+G round at LOD L (mb from the
reference schedule) instead of the VGG-small step.

The autotuner times each candidate in isolation (a captured graph of back-to-back launches of one op);
inside the training step the same kernel runs between other kernels, with other L2 / Infinity-Cache
contents and clocks, and the isolated ranking of near-tied candidates does not always carry over
(profiles/tune_db_ab_r4.txt: two cold captures of the same sources differ by 2% end to end).  This
script re-ranks the near-tied candidates of every tuned op of the VGG-small step by the STEP time:

  1. a cold in-process tune of the step with RAFIKI_AUTOTUNE_LOG (every candidate's isolated time);
  2. the shipped picks restored; baseline step time (captured graph, min of repeats);
  3. greedy coordinate descent over the step's keys (largest op first): each candidate within ``--within``
     of the key's best isolated time is swapped in, the step re-built and re-timed, kept if the step is
     faster by more than ``--gain``;
  4. the refined database written as JSON (ship with scripts/ship_tune_db.py after an A/B).

usage: python scripts/step_refine.py --out gpurun_out/refine [--within 1.25] [--gain 0.003]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def build_and_time(dev, data, y_all, idx, steps, reps):
    from rafiki_amd.engine.convnet import ConvNetEngine
    eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=32, device=dev, seed=0, lr=0.05, momentum=0.9,
                        weight_decay=5e-4, dtype='fp32')
    B = idx.shape[1]
    eng.capture_scheduled(data, y_all, idx.shape[0], B)
    eng.set_schedule(idx)
    for _ in range(5):
        eng.replay()
    torch.cuda.synchronize()
    best = float('inf')
    for _ in range(reps):
        eng.set_schedule(idx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / steps * 1e3)
    del eng
    torch.cuda.empty_cache()
    return best


class _PgRound:
    """build_and_time's PG-GAN counterpart: one model, a fresh GraphedRounds per evaluation (first round
    eager, second captured, then timed replays)."""

    def __init__(self, dev, lod):
        from rafiki_amd.engine.flat import FlatAdam
        from rafiki_amd.models.pg_gan import PgGan, TrainingSchedule, TrialRng
        self.m = PgGan(D_repeats=1, minibatch_base=16, G_lrate=1e-3, D_lrate=1e-3)
        self.m.device = dev
        self.m._build([1, 32, 32], 0)
        nets = self.m.nets
        self.G_opt = FlatAdam(nets.G, 1e-3, betas=(0.0, 0.99))
        self.D_opt = FlatAdam(nets.D, 1e-3, betas=(0.0, 0.99))
        for o in (self.G_opt, self.D_opt):
            o.skip_flag = torch.zeros(1, dtype=torch.int32, device=dev)
        self.rng = TrialRng(dev, 0)
        self.acc = torch.zeros(6, device=dev)
        self.lod = lod
        self.m.set_lod_live(lod)
        r = 2 ** (5 - int(lod))
        self.mb = TrainingSchedule.MINIBATCH_DICTS[16].get(r, 16)
        self.level = torch.randint(0, 256, (4096, 1, r, r), dtype=torch.uint8, device=dev)
        self.labels = torch.zeros((4096, 0), device=dev)

    def __call__(self, steps, reps):
        from rafiki_amd.models.pg_gan import GraphedRounds
        g = GraphedRounds(True)

        def rnd():
            g.run(self.lod, lambda: self.m.train_round(self.lod, self.mb, self.level, self.labels, self.rng,
                                                       self.G_opt, self.D_opt, self.acc))
        for _ in range(3):
            rnd()
        torch.cuda.synchronize()
        best = float('inf')
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                rnd()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / steps * 1e3)
        del g
        torch.cuda.empty_cache()
        return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='vgg', choices=('vgg', 'pggan'))
    ap.add_argument('--lod', type=float, default=3.0)
    ap.add_argument('--out', default='gpurun_out/refine')
    ap.add_argument('--within', type=float, default=1.25)
    ap.add_argument('--gain', type=float, default=0.003)
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--max-alts', type=int, default=3)
    ap.add_argument('--start', default='', help='start from this database JSON instead of the shipped one')
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    log_path = os.path.join(a.out, 'cold_tune.jsonl')
    if os.path.exists(log_path):
        os.remove(log_path)
    os.environ['RAFIKI_AUTOTUNE_LOG'] = log_path
    os.environ['RAFIKI_TUNE_CACHE'] = 'off'
    from rafiki_amd.model.dataset import synthetic_images
    from rafiki_amd.ops import _lib, autotune
    from rafiki_amd.ops import f32 as S
    _lib.lib()
    dev = torch.device('cuda', 0)
    imgs, labels = synthetic_images(8192, size=32, channels=3, classes=10, seed=0)
    x_u8 = torch.from_numpy(imgs).permute(0, 3, 1, 2).contiguous().to(dev)
    data = S.pack_nhwc(x_u8, 8, 1.0 / 127.5, -1.0)
    y_all = torch.from_numpy(labels).to(dev, torch.int32)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    idx = torch.randint(0, 8192, (64, 256), device=dev, generator=gen)
    if a.workload == 'pggan':
        pg = _PgRound(dev, a.lod)

        def measure():
            return pg(a.steps, a.reps)
    else:
        def measure():
            return build_and_time(dev, data, y_all, idx, a.steps, a.reps)

    shipped = autotune._read(a.start or os.path.join(autotune.SHIPPED_DIR, autotune.db_name()))
    # 1. cold tune (nothing loaded), recording which keys the step looks up
    autotune._loaded = True
    autotune.clear()
    used = []
    orig_lookup = autotune.lookup

    def rec(key):
        if key not in used:
            used.append(key)
        return orig_lookup(key)
    autotune.lookup = rec
    cold_ms = measure()
    autotune.lookup = orig_lookup
    times = {}
    with open(log_path) as f:
        for line in f:
            d = json.loads(line)
            times[json.dumps(d['key'])] = {tuple(json.loads(c)): t for c, t in d['all'].items()}
    # 2. the shipped picks
    autotune.clear()
    autotune._cache.update(shipped)
    base = measure()
    print(json.dumps({'cold_tuned_ms': round(cold_ms, 4), 'shipped_ms': round(base, 4), 'keys': len(used)}),
          flush=True)
    cur = dict(autotune._cache)
    # 3. greedy refinement, biggest ops first
    order = []
    for key in used:
        k = json.dumps([str(x) for x in key])
        cand = times.get(k)
        if not cand or key not in cur:
            continue
        best_t = min(cand.values())
        alts = sorted((t, c) for c, t in cand.items() if t <= best_t * a.within and c != tuple(cur[key]))
        if alts:
            order.append((best_t, key, [c for _, c in alts[:a.max_alts]]))
    order.sort(key=lambda r: -r[0])
    best_ms = base
    changes = []
    for best_t, key, alts in order:
        for c in alts:
            prev = cur[key]
            autotune._cache[key] = c
            ms = measure()
            keep = ms < best_ms * (1.0 - a.gain)
            print(json.dumps({'key': [str(x) for x in key], 'op_us': round(best_t, 1), 'from': list(prev),
                              'to': list(c), 'step_ms': round(ms, 4), 'best_ms': round(best_ms, 4), 'kept': keep}),
                  flush=True)
            if keep:
                best_ms = ms
                cur[key] = c
                changes.append((key, prev, c))
            else:
                autotune._cache[key] = prev
    final = measure()
    out = {json.dumps(list(k)): list(v) for k, v in autotune._cache.items()}
    for k, v in shipped.items():   # keys the step does not use (trials / serving shapes) stay as shipped
        out.setdefault(json.dumps(list(k)), list(v))
    with open(os.path.join(a.out, 'refined_db.json'), 'w') as f:
        json.dump(out, f)
    print(json.dumps({'shipped_ms': round(base, 4), 'refined_ms': round(final, 4), 'changes': len(changes)}),
          flush=True)


if __name__ == '__main__':
    main()
