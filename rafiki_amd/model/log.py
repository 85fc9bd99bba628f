"""Structured trial logging: messages, metrics and plot definitions as JSON lines.

Schema identical to the reference (rafiki/model/log.py:107-158): every line is
``{"type": PLOT|METRICS|MESSAGE, "time": "%Y-%m-%dT%H:%M:%S", ...}`` so the admin's
``GET /trials/<id>/logs`` and the web UI parse them the same way.  Extension: ``log_phase``
records per-trial phase timers as ordinary METRICS lines.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from datetime import datetime

MODEL_LOG_DATETIME_FORMAT = '%Y-%m-%dT%H:%M:%S'


class LogType:
    PLOT = 'PLOT'
    METRICS = 'METRICS'
    MESSAGE = 'MESSAGE'


class ModelLogger:
    """Models log through the global ``logger`` of ``rafiki_amd.model``; workers inject a handler."""

    def __init__(self):
        lg = logging.getLogger('rafiki_amd.model.log')
        lg.setLevel(logging.INFO)
        lg.propagate = False
        if not any(isinstance(h, ModelLoggerDebugHandler) for h in lg.handlers):
            lg.addHandler(ModelLoggerDebugHandler())
        self._default = lg
        self._tls = threading.local()  # workers inject per-thread loggers (several trials per process)

    @property
    def _logger(self):
        return getattr(self._tls, 'logger', None) or self._default

    def define_loss_plot(self):
        self.define_plot('Loss Over Epochs', ['loss'], x_axis='epoch')

    def log_loss(self, loss, epoch):
        self.log(loss=loss, epoch=epoch)

    def define_plot(self, title, metrics, x_axis=None):
        self._log(LogType.PLOT, {'title': title, 'metrics': list(metrics), 'x_axis': x_axis})

    def log(self, msg='', **metrics):
        if msg:
            self._log(LogType.MESSAGE, {'message': msg})
        if metrics:
            self._log(LogType.METRICS, dict(metrics))

    def log_phase(self, phase, seconds, **extra):
        self._log(LogType.METRICS, {'phase': phase, 'phase_seconds': float(seconds), **extra})

    class _Timer:
        def __init__(self, lg, phase):
            self.lg, self.phase = lg, phase

        def __enter__(self):
            self.cuda = _cuda_in_use()
            if self.cuda is not None:
                # allocator accounting is host-side: no synchronize (one would be refused while another
                # thread of the process — in-process worker, predictor — captures a hipGraph)
                self.cuda.reset_peak_memory_stats()
            self.t0 = time.perf_counter()
            return self

        def __exit__(self, *exc):
            extra = {}
            if self.cuda is not None:
                # GPU telemetry: HBM peak of the phase
                extra = {'hbm_peak_bytes': int(self.cuda.max_memory_allocated()),
                         'hbm_reserved_bytes': int(self.cuda.memory_reserved())}
            self.lg.log_phase(self.phase, time.perf_counter() - self.t0, **extra)
            return False

    def phase(self, name):
        return ModelLogger._Timer(self, name)

    def set_logger(self, logger):
        """Route this thread's model logs to ``logger`` (None restores the stdout debug logger)."""
        self._tls.logger = None if logger is self._default else logger

    def get_logger(self):
        return self._logger

    def _log(self, log_type, log_dict):
        d = dict(log_dict)
        d['type'] = log_type
        d['time'] = datetime.now().strftime(MODEL_LOG_DATETIME_FORMAT)
        self._logger.info(json.dumps(d, default=_json_default))

    @staticmethod
    def parse_log_line(log_line):
        try:
            d = json.loads(log_line)
            if isinstance(d, dict):
                return d
        except (ValueError, TypeError):
            pass
        return {'type': LogType.MESSAGE, 'message': log_line}

    @staticmethod
    def parse_logs(log_lines):
        """-> (messages, metrics, plots), each a list of dicts."""
        messages, metrics, plots = [], [], []
        for line in log_lines:
            d = ModelLogger.parse_log_line(line)
            t = d.pop('type', None)
            if t == LogType.MESSAGE:
                messages.append({'time': d.get('time'), 'message': d.get('message')})
            elif t == LogType.METRICS:
                metrics.append({'time': d.get('time'), **d})
            elif t == LogType.PLOT:
                plots.append(dict(d))
        return messages, metrics, plots


def _json_default(o):
    try:
        return float(o)
    except Exception:
        return str(o)


class ModelLoggerDebugHandler(logging.Handler):
    """Prints model logs to stdout when running outside a worker (local ``test_model_class``)."""

    def emit(self, record):
        d = ModelLogger.parse_log_line(record.getMessage())
        t = d.get('type')
        if t == LogType.PLOT:
            msg = 'Plot `{}` of {} against {} will be registered when this model is being trained'.format(
                d.get('title'), ', '.join(d.get('metrics') or []), d.get('x_axis') or 'time')
        elif t == LogType.METRICS:
            msg = 'Metric(s) logged: ' + ', '.join('{}={}'.format(k, v) for k, v in d.items())
        elif t == LogType.MESSAGE:
            msg = d.get('message')
        else:
            msg = record.getMessage()
        print('[rafiki_amd.model]', msg)


logger = ModelLogger()


def _cuda_in_use():
    """torch.cuda if this process already initialised a GPU (never initialises one itself)."""
    import sys
    torch = sys.modules.get('torch')
    if torch is None:
        return None
    try:
        return torch.cuda if torch.cuda.is_initialized() else None
    except Exception:
        return None
