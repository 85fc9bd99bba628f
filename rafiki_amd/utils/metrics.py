"""Prometheus-style service metrics (the reference has none).

Each Flask app gets ``GET /metrics`` in the Prometheus text format with a per-route request
counter and latency histogram; the admin adds gauges of job/trial states read from the store, the
predictor its batching counters.  Each app owns a private ``CollectorRegistry`` (several apps can
live in one test process).
"""
from __future__ import annotations

import time

from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, Counter, Gauge, Histogram, generate_latest


def instrument(app, service: str, extra=None):
    """extra(registry) -> callable run before every scrape to refresh gauges."""
    from flask import Response, request
    reg = CollectorRegistry()
    reqs = Counter('rafiki_http_requests', 'HTTP requests', ['service', 'route', 'method', 'status'], registry=reg)
    lat = Histogram('rafiki_http_request_seconds', 'HTTP request latency', ['service', 'route'], registry=reg,
                    buckets=(0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10))
    refresh = extra(reg) if extra else None

    @app.before_request
    def _t0():
        request._rk_t0 = time.perf_counter()

    @app.after_request
    def _count(resp):
        rule = request.url_rule.rule if request.url_rule is not None else 'unmatched'
        if rule != '/metrics':
            reqs.labels(service, rule, request.method, str(resp.status_code)).inc()
            t0 = getattr(request, '_rk_t0', None)
            if t0 is not None:
                lat.labels(service, rule).observe(time.perf_counter() - t0)
        return resp

    @app.route('/metrics')
    def metrics():
        if refresh:
            try:
                refresh()
            except Exception:
                pass
        return Response(generate_latest(reg), mimetype=CONTENT_TYPE_LATEST)

    return reg


def admin_gauges(get_db):
    def setup(reg):
        g_jobs = Gauge('rafiki_train_jobs', 'Train jobs by status', ['status'], registry=reg)
        g_inf = Gauge('rafiki_inference_jobs', 'Inference jobs by status', ['status'], registry=reg)
        g_trials = Gauge('rafiki_trials', 'Trials by status', ['status'], registry=reg)

        def refresh():
            db = get_db()
            conn = db._conn()
            for table, g in (('train_job', g_jobs), ('inference_job', g_inf), ('trial', g_trials)):
                for status, n in conn.execute('SELECT status, COUNT(*) FROM {} GROUP BY status'.format(table)):
                    g.labels(status).set(n)
        return refresh
    return setup


def predictor_gauges(predictor):
    def setup(reg):
        g = Gauge('rafiki_predictor', 'Predictor counters', ['kind'], registry=reg)
        g_models = Gauge('rafiki_predictor_models', 'Models in the ensemble', registry=reg)
        g_bytes = Gauge('rafiki_predictor_resident_bytes', 'Model bytes resident in HBM', registry=reg)

        def refresh():
            for k, v in predictor.stats.items():
                g.labels(k).set(v)
            g_models.set(len(predictor.models))
            g_bytes.set(predictor.cache.used)
        return refresh
    return setup
