"""PG-GAN training throughput (BASELINE config #5: pg_gans.py train trial) — stand-alone form of the
phase bench.py runs (rafiki_amd/utils/benchmarks.py ``pg_gan_rounds``).  Prints one JSON line.

  python scripts/bench_pg_gan.py [--lods 3,0] [--steps 10] [--force-allreduce]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_pg_gan.py
      (data parallel over RCCL: the global minibatch split across the ranks, bucketed all-reduce
       overlapped with the graphed backward)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lods', default='3,0')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--minibatch', type=int, default=0, help='0: reference schedule (global) minibatch')
    ap.add_argument('--no-graph', action='store_true', help='eager rounds (no hipGraph replay)')
    ap.add_argument('--dtype', default='fp32', choices=('fp32', 'bf16'))
    ap.add_argument('--bucket-mb', type=float, default=None)
    ap.add_argument('--force-allreduce', action='store_true',
                    help='one rank: the data-parallel round on a 1-rank RCCL group (collectives issued)')
    a = ap.parse_args()
    from rafiki_amd.parallel import dist as D
    from rafiki_amd.utils.benchmarks import pg_gan_rounds
    info = None
    if int(os.environ.get('WORLD_SIZE', '1')) > 1:
        info = D.init_distributed()
    elif a.force_allreduce:
        os.environ.update(RANK='0', WORLD_SIZE='1', MASTER_ADDR='127.0.0.1')
        from rafiki_amd.parallel.launch import free_port
        import torch.distributed as dist
        os.environ['MASTER_PORT'] = str(free_port())
        dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
        info = D.DistInfo(0, 1, 0, 'nccl')
    # one GPU per rank over RCCL; a gloo group (the one-box rehearsal of the data-parallel path) may put
    # several ranks on one GPU
    local = info.local_rank % max(1, torch.cuda.device_count()) if info is not None else 0
    torch.cuda.set_device(local)
    res = pg_gan_rounds(torch.device('cuda', local), lods=[float(x) for x in a.lods.split(',')], steps=a.steps,
                        warmup=a.warmup, minibatch=a.minibatch, graph=not a.no_graph, dtype=a.dtype,
                        force_allreduce=a.force_allreduce, info=info, bucket_mb=a.bucket_mb)
    if info is None or info.is_main:
        print(json.dumps(res), flush=True)
    if info is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
