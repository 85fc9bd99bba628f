"""PG-GAN (IMAGE_GENERATION) on CPU: TFRecord format, schedule, WGAN-GP training, DP over gloo.

Parity notes: the reference's pg_gans.py needs TensorFlow 1.12 (not importable here), so the
schedule is checked against values derived by hand from pg_gans.py:1227-1274 and the TFRecord
bytes against the format spec (length/CRC framing + tf.train.Example wire encoding).
"""
import os
import socket
import tempfile
from contextlib import closing

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from rafiki_amd.model import tfrecord as T

TINY = dict(D_repeats=1, minibatch_base=4, G_lrate=1e-3, D_lrate=1e-3, lod_initial_resolution=4, total_kimg=0.3,
            lod_training_kimg=0.1, lod_transition_kimg=0.1, fmap_base=128, fmap_max=32, eval_images=128,
            minibatch_repeats=1)
DATA = 'synthetic://image?n=256&size=16&channels=1&classes=4&seed=0'


def test_crc32c_known_vector():
    assert T.crc32c(b'123456789') == 0xE3069283
    assert T.masked_crc(b'') == ((((0 >> 15) | (0 << 17)) + 0xA282EAD8) & 0xFFFFFFFF)


def test_example_roundtrip():
    payload = T.encode_example({'shape': [3, 8, 8], 'data': bytes(range(192)), 'f': [0.5, 1.5]})
    ex = T.decode_example(payload)
    assert ex['shape'] == [3, 8, 8] and ex['data'][0] == bytes(range(192)) and ex['f'] == [0.5, 1.5]


def test_tfrecord_dataset_roundtrip(tmp_path):
    rng = np.random.RandomState(0)
    imgs = rng.randint(0, 256, (40, 3, 16, 16)).astype(np.uint8)
    d = str(tmp_path / 'cifar')
    T.write_tfrecord_dataset(d, imgs, labels=np.arange(40) % 5)
    names = sorted(os.listdir(d))
    assert names == ['cifar-r02.tfrecords', 'cifar-r03.tfrecords', 'cifar-r04.tfrecords', 'cifar-rxx.labels']
    for n in names[:-1]:
        assert sum(1 for _ in T.iter_records(os.path.join(d, n), verify=True)) == 40
    ds = T.TFRecordImageDataset(d)
    order = np.arange(40)
    np.random.RandomState(123).shuffle(order)
    assert ds.shape == [3, 16, 16] and ds.label_size == 5 and ds.resolution_log2 == 4
    assert (ds.images[0] == imgs[order]).all()
    lod1 = np.rint(T.downscale_images(imgs[order].astype(np.float32))).clip(0, 255).astype(np.uint8)
    assert (ds.images[1] == lod1).all()
    assert (ds.labels.argmax(1) == (order % 5)).all()


def test_tfrecord_python_fallback_matches_native(tmp_path, monkeypatch):
    from rafiki_amd import runtime
    if not runtime.available():
        pytest.skip('native runtime not built')
    imgs = np.random.RandomState(1).randint(0, 256, (10, 1, 8, 8)).astype(np.uint8)
    d = str(tmp_path / 'm')
    T.write_tfrecord_dataset(d, imgs, shuffle=False)
    native = T._read_images(os.path.join(d, 'm-r03.tfrecords'))
    monkeypatch.setattr(runtime, 'lib', lambda: None)
    py = T._read_images(os.path.join(d, 'm-r03.tfrecords'))
    assert (native == py).all() and (py == imgs).all()


def test_training_schedule():
    from rafiki_amd.models.pg_gan import TrainingSchedule as S
    s = S(0, 5, minibatch_base=16)
    assert s.lod == 3.0 and s.resolution == 4 and s.minibatch == 512
    s = S(900_000, 5, minibatch_base=4)  # halfway through the first transition
    assert abs(s.lod - 2.5) < 1e-9 and s.resolution == 8 and s.minibatch == 128
    s = S(1_200_000, 5, minibatch_base=8, num_gpus=3)
    assert s.lod == 2.0 and s.minibatch == 255  # 256 - 256 % 3
    s = S(10_000_000, 5, minibatch_base=32)
    assert s.lod == 0.0 and s.resolution == 32 and s.minibatch == 64


def test_pg_gan_train_eval_predict_cpu(tmp_path, monkeypatch):
    monkeypatch.setenv('RAFIKI_OUTPUT_DIR', str(tmp_path))
    from rafiki_amd.models.pg_gan import PgGan
    m = PgGan(**TINY)
    m.train(DATA)
    assert m.lod == 1.0  # 0.3 kimg with 0.1/0.1 phases reaches the 8x8 -> 16x16 level
    assert all(np.isfinite(v) for v in m.stats.values())
    score = m.evaluate('synthetic://image?n=128&size=16&channels=1&classes=4&seed=1')
    assert isinstance(score, float) and 1.0 <= score <= 4.0 + 1e-6
    params = m.dump_parameters()
    m2 = PgGan(**TINY)
    m2.load_parameters(params)
    a = m.generate(4, seed=3)
    b = m2.generate(4, seed=3)
    assert a.shape == (4, 16, 16, 1) and (a == b).all()
    paths = m2.predict([2, 2, 2])
    assert len(paths) == 2 and all(os.path.exists(p) and p.endswith('.jpeg') for p in paths)


def test_pg_gan_tfrecord_input_and_labels(tmp_path):
    from rafiki_amd.model.dataset import synthetic_images
    from rafiki_amd.models.pg_gan import PgGan
    imgs, labels = synthetic_images(64, size=8, channels=3, classes=3, seed=0)
    d = str(tmp_path / 'cond')
    T.write_tfrecord_dataset(d, imgs.transpose(0, 3, 1, 2), labels=labels)
    m = PgGan(**dict(TINY, total_kimg=0.1))
    m.train(d)
    assert m.nets.label_size == 3 and m.nets.num_channels == 3  # AC-GAN label penalty path
    assert all(np.isfinite(v) for v in m.stats.values())


def test_gradient_penalty_double_backward_cpu():
    """The D-side ops are twice differentiable: d/dw ||dD/dx|| matches finite differences."""
    from rafiki_amd.models.pg_gan import PgNetworks
    torch.manual_seed(0)
    nets = PgNetworks(num_channels=1, resolution=8, fmap_base=64, fmap_max=16, device='cpu', seed=0)
    P = nets.src_D()
    x = torch.randn(4, 8, 8, nets.cpad)
    x[..., 1:] = 0

    def gp():
        xi = x.clone().requires_grad_(True)
        s, _ = nets.discriminator(P, xi, 0.0)
        (g,) = torch.autograd.grad(s.sum(), xi, create_graph=True)
        return g.square().sum()

    name = '8x8/Conv0/weight'
    p = nets.d_params[name]
    p.grad.zero_()
    gp().backward()
    ana = p.grad.flatten()[:5].clone()
    eps = 1e-3
    num = []
    flat = p.detach().view(-1)  # aliases the parameter storage
    for i in range(5):
        o = flat[i].item()
        flat[i] = o + eps
        up = gp().item()
        flat[i] = o - eps
        dn = gp().item()
        flat[i] = o
        num.append((up - dn) / (2 * eps))
    num = torch.tensor(num)
    assert torch.allclose(ana, num, rtol=2e-2, atol=1e-4 * max(1.0, num.abs().max().item())), (ana, num)


# ------------------------------------------------------------------------------ DP over gloo
def _free_port():
    with closing(socket.socket(socket.AF_INET, socket.SOCK_STREAM)) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _env(rank, world, port):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'RAFIKI_CPU_ONLY': '1'})


def _bucket_worker(rank, world, port, out_dir):
    _env(rank, world, port)
    import torch.distributed as dist
    from rafiki_amd.engine.flat import FlatParams, init_const
    from rafiki_amd.parallel.grad_bucket import FlatGradAllReduce
    dist.init_process_group('gloo', rank=rank, world_size=world)
    flat = FlatParams('cpu')
    for i in range(6):
        flat.add('p{}'.format(i), (100 + 37 * i,), init_const(1.0))
    flat.build()
    params = []
    for s in flat.specs:
        p = torch.nn.Parameter(flat.w(s.name))
        p.grad = flat.g(s.name)
        params.append(p)
    ar = FlatGradAllReduce(flat.grad, flat.param_ranges(), params, world, bucket_mb=0.001)
    assert len(ar.buckets) > 1
    ar.begin()
    loss = sum((p * (rank + 1) * (i + 1)).sum() for i, p in enumerate(params[:4]))  # p4, p5 unused
    loss.backward()
    ar.finish()
    torch.save(flat.grad.clone(), os.path.join(out_dir, 'g{}.pt'.format(rank)))
    dist.destroy_process_group()


def test_flat_grad_allreduce_gloo():
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_bucket_worker, args=(2, port, d), nprocs=2, join=True)
        g0 = torch.load(os.path.join(d, 'g0.pt'), weights_only=True)
        g1 = torch.load(os.path.join(d, 'g1.pt'), weights_only=True)
    assert torch.equal(g0, g1)
    from rafiki_amd.engine.flat import FlatParams, init_const
    flat = FlatParams('cpu')
    for i in range(6):
        flat.add('p{}'.format(i), (100 + 37 * i,), init_const(1.0))
    flat.build()
    for i, s in enumerate(flat.specs):
        v = g0[s.offset:s.offset + s.numel]
        expect = (1 + 2) / 2 * (i + 1) if i < 4 else 0.0
        assert torch.allclose(v, torch.full_like(v, expect)), (i, v[:3])


def _dp_worker(rank, world, port, out_dir):
    _env(rank, world, port)
    from rafiki_amd.models.pg_gan import PgGan
    from rafiki_amd.parallel import dist as D
    from rafiki_amd.parallel.context import TrialContext, use_context
    info = D.init_distributed(backend='gloo')
    with use_context(TrialContext(device=torch.device('cpu'), dist=info, data_parallel=True)):
        m = PgGan(**dict(TINY, total_kimg=0.2))
        m.train(DATA)
        torch.save({'G': m.nets.G.master.clone(), 'D': m.nets.D.master.clone(), 'Gs': m.nets.Gs_master.clone(),
                    'stats': torch.tensor([m.stats['D_loss'], m.stats['G_loss']])},
                   os.path.join(out_dir, 'r{}.pt'.format(rank)))
    D.destroy(info)


def test_pg_gan_data_parallel_gloo():
    """2-rank DP: replicas stay bit-identical (same averaged grads, same Adam), shards differ."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_worker, args=(2, port, d), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, 'r0.pt'), weights_only=True)
        r1 = torch.load(os.path.join(d, 'r1.pt'), weights_only=True)
    for k in ('G', 'D', 'Gs'):
        assert torch.equal(r0[k], r1[k]), k
    assert not torch.equal(r0['stats'], r1['stats'])  # each rank saw its own minibatch shard


def _dp_equiv_worker(rank, world, port, out_dir):
    _env(rank, world, port)
    from rafiki_amd.models.pg_gan import PgGan
    from rafiki_amd.parallel import dist as D
    from rafiki_amd.parallel.context import TrialContext, use_context
    info = D.init_distributed(backend='gloo')
    with use_context(TrialContext(device=torch.device('cpu'), dist=info, data_parallel=True)):
        m = PgGan(**EQUIV)
        m.train(DATA)
        torch.save({'G': m.nets.G.master.clone(), 'D': m.nets.D.master.clone(), 'Gs': m.nets.Gs_master.clone()},
                   os.path.join(out_dir, 'r{}.pt'.format(rank)))
    D.destroy(info)


# 8 rounds of 128 (2 ranks x 64: 16 minibatch-stddev groups each) through a 4x4 -> 8x8 LOD fade
EQUIV = dict(TINY, minibatch_base=8, total_kimg=1.0, lod_training_kimg=0.3, lod_transition_kimg=0.3)


def test_pg_gan_dp_two_half_batches_equal_one_full_batch():
    """2 ranks x half minibatch == 1 rank x full minibatch (same shared RNG stream, strided shards,
    averaged bucketed all-reduce), up to fp32 summation order — a wrong averaging scale, a shard
    that double-counts samples or per-rank data streams all fail this."""
    from rafiki_amd.models.pg_gan import PgGan
    from rafiki_amd.parallel.context import TrialContext, use_context
    with use_context(TrialContext(device=torch.device('cpu'))):
        m = PgGan(**EQUIV)
        m.train(DATA)
        ref = {'G': m.nets.G.master.clone(), 'D': m.nets.D.master.clone(), 'Gs': m.nets.Gs_master.clone()}
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_equiv_worker, args=(2, port, d), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, 'r0.pt'), weights_only=True)
        r1 = torch.load(os.path.join(d, 'r1.pt'), weights_only=True)
    for k in ('G', 'D', 'Gs'):
        assert torch.equal(r0[k], r1[k]), k
        err = ((r0[k] - ref[k]).norm() / ref[k].norm()).item()
        moved = ((ref[k] - PgGan_init(k)).norm() / ref[k].norm()).item()
        print('dp-equivalence', k, 'rel err', err, 'moved', moved)
        assert moved > 1e-5 and err < 1e-5 + 1e-3 * moved, (k, err, moved)


def PgGan_init(k):
    from rafiki_amd.models.pg_gan import PgGan
    from rafiki_amd.parallel.context import TrialContext, use_context
    with use_context(TrialContext(device=torch.device('cpu'))):
        m = PgGan(**EQUIV)
        from rafiki_amd.models.pg_gan import load_gan_dataset
        m._build(load_gan_dataset(DATA).shape, 0)
        return {'G': m.nets.G.master, 'D': m.nets.D.master, 'Gs': m.nets.Gs_master}[k].clone()


def test_pg_gan_crash_resume_matches_uninterrupted(tmp_path, monkeypatch):
    """Checkpoint every tick, crash after tick 2, resume in a fresh model: the final G / D / Gs equal
    the uninterrupted run's exactly (weights, both Adam states, RNG position and schedule restored)."""
    from rafiki_amd.models.pg_gan import PgGan
    from rafiki_amd.parallel.context import TrialContext, use_context
    from rafiki_amd.utils import faults
    from rafiki_amd.utils.checkpoint import TrialCheckpoint
    knobs = dict(TINY, total_kimg=0.5, checkpoint_secs=0)   # 4 ticks of 128 images
    with use_context(TrialContext(device=torch.device('cpu'))):
        a = PgGan(**knobs)
        a.train(DATA)
    ck = TrialCheckpoint(str(tmp_path), 'trial1')
    monkeypatch.setenv('RAFIKI_FAULT_INJECT', 'crash:tick=2')
    faults.reset()
    with use_context(TrialContext(device=torch.device('cpu'), checkpoint=ck)):
        with pytest.raises(faults.WorkerCrash):
            PgGan(**knobs).train(DATA)
        assert ck.exists()
        monkeypatch.setenv('RAFIKI_FAULT_INJECT', '')
        faults.reset()
        b = PgGan(**knobs)
        b.train(DATA)
    assert ck.resumed_from == 2
    for x, y in ((a.nets.G.master, b.nets.G.master), (a.nets.D.master, b.nets.D.master),
                 (a.nets.Gs_master, b.nets.Gs_master)):
        assert torch.equal(x, y)
    assert a.stats == b.stats and a.lod == b.lod


def _gen_worker(rank, world, port, out_dir):
    _env(rank, world, port)
    from rafiki_amd.models.pg_gan import PgGan, load_gan_dataset
    from rafiki_amd.parallel import dist as D
    from rafiki_amd.parallel.context import TrialContext, use_context
    info = D.init_distributed(backend='gloo')
    with use_context(TrialContext(device=torch.device('cpu'), dist=info, data_parallel=True)):
        m = PgGan(**TINY)
        m._build(load_gan_dataset(DATA).shape, 0)
        m.lod = 1.0
        np.save(os.path.join(out_dir, 'g{}.npy'.format(rank)), m.generate(11, seed=5, batch=7))
    D.destroy(info)


def test_pg_gan_generation_split_over_ranks():
    """Data-parallel generate(): each of 2 ranks renders half of every batch (odd sizes included) and
    the all-gathered images equal a single-rank run."""
    from rafiki_amd.models.pg_gan import PgGan, load_gan_dataset
    m = PgGan(**TINY)
    m._build(load_gan_dataset(DATA).shape, 0)
    m.lod = 1.0
    ref = m.generate(11, seed=5, batch=7)
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gen_worker, args=(2, port, d), nprocs=2, join=True)
        g0, g1 = np.load(os.path.join(d, 'g0.npy')), np.load(os.path.join(d, 'g1.npy'))
    assert g0.shape == ref.shape == (11, 16, 16, 1)
    assert (g0 == g1).all()
    assert np.abs(g0.astype(int) - ref.astype(int)).max() <= 1


def _dp_seg_worker(rank, world, port, out_dir):
    _env(rank, world, port)
    from rafiki_amd.models.pg_gan import PgGan
    from rafiki_amd.parallel import dist as D
    from rafiki_amd.parallel.context import TrialContext, use_context
    info = D.init_distributed(backend='gloo')
    out = {}
    for seg in (True, False):
        with use_context(TrialContext(device=torch.device('cpu'), dist=info, data_parallel=True)):
            m = PgGan(**dict(EQUIV, dp_segmented=seg))
            m.train(DATA)
            assert m.segmented == seg
            for k, v in (('G', m.nets.G.master), ('D', m.nets.D.master), ('Gs', m.nets.Gs_master)):
                out['{}{}'.format(k, int(seg))] = v.clone()
    torch.save(out, os.path.join(out_dir, 'r{}.pt'.format(rank)))
    D.destroy(info)


def test_pg_gan_dp_traced_segments_match_unsegmented_gloo():
    """2 ranks: the segmented round (bucket all-reduces from FlatGradAllReduce.traced — traced
    gradient contributions, untouched buckets skipped) gives bit-identical weights to the unsegmented
    round (hook-launched buckets over the whole arena), through a LOD fade."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_seg_worker, args=(2, port, d), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, 'r0.pt'), weights_only=True)
        r1 = torch.load(os.path.join(d, 'r1.pt'), weights_only=True)
    for k in ('G', 'D', 'Gs'):
        assert torch.equal(r0[k + '1'], r0[k + '0']), k
        assert torch.equal(r0[k + '1'], r1[k + '1']), k


def test_flat_grad_allreduce_traces_and_skips_untouched_buckets():
    """traced(): the trace records each bucket's last contribution; buckets with none are never
    reduced (their gradients are zero on every rank).  After the tracing run, each bucket's all-reduce
    starts INSIDE the backward, at the first contribution after the bucket's last one (the overlap the
    captured rounds get by cutting their graphs there), in backward-completion order."""
    from rafiki_amd.engine.flat import FlatParams, init_const
    from rafiki_amd.parallel.grad_bucket import FlatGradAllReduce
    flat = FlatParams('cpu')
    for i in range(6):
        flat.add('p{}'.format(i), (100 + 37 * i,), init_const(1.0))
    flat.build()
    params = []
    for s in flat.specs:
        p = torch.nn.Parameter(flat.w(s.name))
        p.grad = flat.g(s.name)
        params.append(p)
    ar = FlatGradAllReduce(flat.grad, flat.param_ranges(), params, 1, bucket_mb=0.001, force=True)
    calls = []
    state = {'bwd': False}
    import torch.distributed as dist
    orig = dist.all_reduce
    dist.all_reduce = lambda t, **kw: calls.append((t.data_ptr(), state['bwd'])) or _Done()

    def grads():
        state['bwd'] = True
        # params 0, 1 and 3 receive gradients (in the order autograd accumulates them); 2, 4, 5 do not
        sum((p * (i + 1)).sum() for i, p in ((0, params[0]), (1, params[1]), (3, params[3]))).backward()
        state['bwd'] = False
    try:
        gr, red = ar.traced(grads, ('k', 0))
        first = []
        for _ in range(gr.TRACES):   # tracing runs: the reduce segment launches everything
            gr()
            red()
            first.append(list(calls))
            calls.clear()
        gr()          # planned run: launches from inside the backward
        red()
    finally:
        dist.all_reduce = orig
        ar.remove()
    plan = ar._plans[('k', 0)]
    touched = {ar.bucket_of[0], ar.bucket_of[1], ar.bucket_of[3]}
    assert set(plan['order']) == touched and plan['ready']
    assert all(v == 1 for v in plan['count'].values())
    for f in first:
        assert len(f) == len(touched) < len(ar.buckets)
        assert not any(inside for _, inside in f)                  # tracing runs: reduce segment only
    assert sorted(p for p, _ in calls) == sorted(p for p, _ in first[0])   # the same buckets
    # backward accumulates param 3 first (bucket order ascending = reverse arena order): each bucket starts
    # at the next contribution once it and every lower bucket are complete; the last one after the backward
    assert sum(inside for _, inside in calls) >= 1 and not calls[-1][1]


class _Done:
    def wait(self):
        return True


def test_pg_gan_live_ranges_bit_identical():
    """Zeroing, the finite check and Adam over the LOD's live arena ranges only (PgGan.set_lod_live) give
    bit-identical G / D / Gs to the whole-arena round, through a 4x4 -> 8x8 fade and the stable 8x8 LOD."""
    from rafiki_amd.models.pg_gan import PgGan
    from rafiki_amd.parallel.context import TrialContext, use_context
    out = []
    for live in (True, False):
        with use_context(TrialContext(device=torch.device('cpu'))):
            m = PgGan(**dict(EQUIV, live_ranges=live))
            m.train(DATA)
            out.append((m.nets.G.master.clone(), m.nets.D.master.clone(), m.nets.Gs_master.clone(), m._live))
    (g1, d1, s1, l1), (g0, d0, s0, l0) = out
    assert l1 is not None and l0 is None
    assert torch.equal(g1, g0) and torch.equal(d1, d0) and torch.equal(s1, s0)


def test_pg_gan_live_names_cover_the_lod():
    from rafiki_amd.models.pg_gan import PgGan, load_gan_dataset
    from rafiki_amd.parallel.context import TrialContext, use_context
    with use_context(TrialContext(device=torch.device('cpu'))):
        m = PgGan(**EQUIV)
        m._build(load_gan_dataset(DATA).shape, 0)
    nets = m.nets
    g3, d3 = nets.live_names(float(nets.L - 2))     # 4x4 only
    gall, dall = nets.live_names(0.0)
    assert set(g3) < set(nets.G.names()) and set(d3) < set(nets.D.names())
    # the layers live at 4x4 stay live at full resolution, except the 4x4 RGB adapters
    assert {n for n in g3 if 'RGB' not in n} <= set(gall) and {n for n in d3 if 'RGB' not in n} <= set(dall)
    assert all(n in nets.G.names() for n in gall) and all(n in nets.D.names() for n in dall)
    # at full resolution every conv / dense layer is live; only the coarser RGB adapters are not
    assert all('RGB' in n for n in set(nets.G.names()) - set(gall))
    assert all('RGB' in n for n in set(nets.D.names()) - set(dall))


def _rounds_worker(rank, world, port, out_dir):
    _env(rank, world, port)
    from rafiki_amd.parallel import dist as D
    from rafiki_amd.utils.benchmarks import pg_gan_rounds
    info = D.init_distributed(backend='gloo')
    res = pg_gan_rounds(torch.device('cpu'), lods=(3.0,), steps=1, warmup=2, minibatch=16, info=info)
    if rank == 0:
        import json as _json
        with open(os.path.join(out_dir, 'res.json'), 'w') as f:
            _json.dump(res, f)
    D.destroy(info)


def test_bench_pg_gan_rounds_data_parallel_gloo():
    """bench.py's PG-GAN phase at N > 1 (BASELINE #5 data parallel): 2 ranks split the global minibatch,
    the overlapped bucketed all-reduce round runs, and rank 0 reports the global rate."""
    import json as _json
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rounds_worker, args=(2, port, d), nprocs=2, join=True)
        with open(os.path.join(d, 'res.json')) as f:
            res = _json.load(f)
    r = res['lods']['3.0']
    assert res['world_size'] == 2 and r['global_minibatch'] == 16 and r['minibatch_per_rank'] == 8
    assert r['images_per_sec'] > 0 and 'data parallel x2' in res['parallelism']
