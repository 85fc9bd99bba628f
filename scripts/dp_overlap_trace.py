"""Host-side call order of the captured data-parallel PG-GAN round, from a rocprofv3 HIP API trace.

Run (one GPU, a 1-rank RCCL group with the bucketed all-reduce forced on):
  rocprofv3 --kernel-trace --hip-trace --output-format csv -d <dir> -o run -- \\
      python3 scripts/bench_pg_gan.py --lods 3 --steps 4 --warmup 2 --force-allreduce
  python3 scripts/dp_overlap_trace.py <dir>

Prints, for the last timed round, the sequence of graph launches (G) and of the stream-ordering calls
ProcessGroupNCCL makes around each bucket all-reduce: the RCCL stream waiting on the compute stream (the
bucket's gradients are done: ``hipStreamWaitEvent`` after an ``hipEventRecord`` on the compute stream) and,
in the reduce segment, the compute stream waiting on each bucket's end event before the optimizer graph.
With the overlapped rounds the D and G gradient passes are several graphs each and a bucket's reduce is
enqueued between two of them — i.e. it is ordered only after the graph that finished its bucket and runs
beside the next one; the round-5 design showed every wait after the last gradient graph.  (A 1-rank group
moves no data, so RCCL launches no kernel here: the evidence is the enqueue order, which is what the
multi-rank run executes.)
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--rounds', type=int, default=1)
    a = ap.parse_args()
    api = sorted(glob.glob(os.path.join(a.dir, '**', '*hip_api_trace.csv'), recursive=True))
    if not api:
        raise SystemExit('no hip_api_trace.csv under ' + a.dir)
    calls = []
    with open(api[0]) as f:
        for r in csv.DictReader(f):
            fn = r.get('Function') or r.get('Operation') or ''
            if fn in ('hipGraphLaunch', 'hipStreamWaitEvent', 'hipEventRecord', 'hipEventRecordWithFlags'):
                calls.append((int(r['Start_Timestamp']), fn, r.get('Thread_Id', '')))
    calls.sort()
    code = {'hipGraphLaunch': 'G', 'hipStreamWaitEvent': 'W', 'hipEventRecord': 'E', 'hipEventRecordWithFlags': 'E'}
    seq = ''.join(code[c[1]] for c in calls)
    # a round ends with the G step's optimizer graph; rounds are separated by the longest runs of G-only
    # activity only loosely, so report the tail: the last round = from the (k+1)-th last 'WG' optimizer join
    # back to the previous one
    joins = [i for i in range(len(seq) - 1) if seq[i] == 'W' and seq[i + 1] == 'G']
    print('calls traced: {} graph launches, {} stream waits, {} event records'.format(
        seq.count('G'), seq.count('W'), seq.count('E')))
    tail = seq[-400:]
    print('last calls (G = graph launch, E = event record, W = stream wait):')
    for i in range(0, len(tail), 100):
        print('  ' + tail[i:i + 100])
    # graph launches between the first and the last wait of each reduce: G's that follow a bucket's
    # enqueue (E W) inside one gradient segment = replays overlapping an in-flight reduce
    overl = 0
    i = 0
    while i < len(seq) - 2:
        if seq[i] == 'G' and seq[i + 1:i + 3] == 'EW':
            j = i + 3
            while j < len(seq) and seq[j] in 'EW':
                j += 1
            if j < len(seq) and seq[j] == 'G':
                overl += 1
        i += 1
    print('graph launches enqueued after a bucket all-reduce was issued and before its wait: {}'.format(overl))
    print('optimizer joins (W then G): {}'.format(len(joins)))


if __name__ == '__main__':
    main()
