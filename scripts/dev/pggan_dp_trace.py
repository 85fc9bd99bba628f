"""One-GPU rehearsal of the segmented data-parallel PG-GAN round for a kernel trace.

A 1-rank RCCL group with the bucketed all-reduce forced on (force_grad_allreduce), small buckets
(RAFIKI_GRAD_BUCKET_MB, default here 2 MiB) so the D / G arenas split into several buckets: the
segmented rounds capture each bucket's completion event and reduce it from a side stream while the
replay continues.  Run under ``rocprofv3 --kernel-trace`` and summarise with
``scripts/dev/dp_overlap_summary.py``."""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

os.environ.setdefault('RAFIKI_GRAD_BUCKET_MB', '2')

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from rafiki_amd.models.pg_gan import PgGan
    from rafiki_amd.parallel.context import TrialContext, use_context
    from rafiki_amd.parallel.dist import DistInfo
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:{}".format(port), rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))
    kimg = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
    try:
        knobs = dict(D_repeats=1, minibatch_base=32, G_lrate=1e-3, D_lrate=1e-3, lod_initial_resolution=4,
                     total_kimg=kimg, lod_training_kimg=100, lod_transition_kimg=100, fmap_base=2048, fmap_max=256,
                     minibatch_repeats=4, seed=3, force_grad_allreduce=True)
        data = "synthetic://image?n=512&size=32&channels=3&classes=0&seed=0"
        ctx = TrialContext(device=torch.device('cuda'), dist=DistInfo(0, 1, 0, "nccl"), data_parallel=True)
        with use_context(ctx):
            m = PgGan(**knobs)
            m.train(data)
        torch.cuda.synchronize()
        print('captures', m.graphs.captures, 'segmented', m.segmented)
    finally:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
