"""Which PyTorch (at::native) kernels does one PG-GAN D+G round still launch, and from where?

Runs the bench_pg_gan.py configuration eagerly (after warm-up rounds that settle the tuner) under a
TorchDispatchMode that records every aten op producing a CUDA tensor (metadata-only ops excluded) with
its shapes, the autograd node running it (backward ops) and the innermost rafiki_amd frame.  Prints one
JSON line per LOD: the ops grouped by (op, origin) with counts, most frequent first.
"""
import argparse
import collections
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from torch.utils._python_dispatch import TorchDispatchMode

_META = {'view', '_unsafe_view', 'as_strided', 't', 'transpose', 'permute', 'detach', 'alias', 'expand', 'slice',
         'select', 'unsqueeze', 'squeeze', 'split', 'unbind', '_reshape_alias', 'empty', 'empty_strided',
         'empty_like', 'new_empty', 'new_empty_strided', 'lift_fresh', 'split_with_sizes', 'chunk', 'narrow',
         'is_nonzero', '_local_scalar_dense', 'reshape', 'contiguous', 'view_as', 'expand_as', 'numpy_T'}


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.overloadpacket.__name__
        if name in _META:
            return out
        outs = out if isinstance(out, (tuple, list)) else (out,)
        if not any(isinstance(o, torch.Tensor) and o.is_cuda for o in outs):
            return out
        node = torch._C._current_autograd_node()
        where = 'fwd'
        for fr in reversed(traceback.extract_stack()[:-1]):
            if 'rafiki_amd' in fr.filename:
                where = '%s:%d %s' % (os.path.basename(fr.filename), fr.lineno, fr.name)
                break
        shapes = [tuple(a.shape) for a in args if isinstance(a, torch.Tensor)][:3]
        self.rows[(name, node.name() if node is not None else '-', where, str(shapes))] += 1
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lods', default='3,0')
    a = ap.parse_args()
    from rafiki_amd.engine.flat import FlatAdam
    from rafiki_amd.models.pg_gan import PgGan, TrainingSchedule, TrialRng
    from rafiki_amd.ops import _lib
    _lib.lib()
    dev = torch.device('cuda', 0)
    m = PgGan(D_repeats=1, minibatch_base=16, G_lrate=1e-3, D_lrate=1e-3)
    m.device = dev
    m._build([1, 32, 32], 0)
    G_opt = FlatAdam(m.nets.G, 1e-3, betas=(0.0, 0.99))
    D_opt = FlatAdam(m.nets.D, 1e-3, betas=(0.0, 0.99))
    for o in (G_opt, D_opt):
        o.skip_flag = torch.zeros(1, dtype=torch.int32, device=dev)
    rng = TrialRng(dev, 0)
    acc = torch.zeros(6, device=dev)
    for lod in [float(x) for x in a.lods.split(',')]:
        r = 2 ** (5 - int(lod))
        mb = TrainingSchedule.MINIBATCH_DICTS[16].get(r, 16)
        level = torch.randint(0, 256, (4096, 1, r, r), dtype=torch.uint8, device=dev)
        labels = torch.zeros((4096, 0), device=dev)
        for _ in range(2):
            m.train_round(lod, mb, level, labels, rng, G_opt, D_opt, acc)
        torch.cuda.synchronize()
        c = Census()
        with c:
            m.train_round(lod, mb, level, labels, rng, G_opt, D_opt, acc)
        torch.cuda.synchronize()
        rows = [{'n': n, 'op': k[0], 'node': k[1], 'where': k[2], 'shapes': k[3]} for k, n in c.rows.most_common()]
        print(json.dumps({'lod': lod, 'minibatch': mb, 'aten_launching_ops': sum(c.rows.values()), 'rows': rows}),
              flush=True)


if __name__ == '__main__':
    main()
