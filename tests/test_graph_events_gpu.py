"""External events recorded inside a captured hipGraph order another stream's later work behind the
graph's work before the event (ops.graphs.external_events_ok) — the mechanism of the overlapped
per-bucket all-reduce (parallel/grad_bucket.py FlatGradAllReduce.overlapped)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_external_events_order_side_stream_after_replay():
    from rafiki_amd.ops.graphs import external_events_ok
    assert external_events_ok(torch.device('cuda', 0))


def test_overlapped_plan_records_events_in_capture():
    """A captured gradient segment records one event per touched bucket (in completion order), and the
    reduce of a 1-rank forced group waits on them without error."""
    from rafiki_amd.ops import graphs
    from rafiki_amd.parallel.grad_bucket import FlatGradAllReduce, prepare_events
    dev = torch.device('cuda', 0)
    assert prepare_events(dev)
    n = [4096, 8192, 4096, 16384]
    grad = torch.zeros(sum(n), device=dev)
    w = torch.randn(sum(n), device=dev)
    params, ranges, off = [], [], 0
    for k in n:
        p = torch.nn.Parameter(w[off:off + k].clone())
        p.grad = grad[off:off + k]
        params.append(p)
        ranges.append((off, k))
        off += k
    ar = FlatGradAllReduce(grad, ranges, params, 1, bucket_mb=8192 * 4 / 2 ** 20, force=True)
    x = torch.randn(16, device=dev)

    def grads():
        loss = sum((p[:16] * x).sum() * (i + 1) for i, p in enumerate(params[:3]))
        loss.backward()
    gr, red = ar.overlapped(grads, ('t', 0))
    gr()                                    # eager trace
    plan = ar._plans[('t', 0)]
    assert plan['events'] is None and len(plan['last']) >= 2
    torch.cuda.synchronize()
    ar.remove()
    assert graphs.external_events_ok(dev)
