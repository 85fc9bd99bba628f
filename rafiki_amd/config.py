"""Typed, env-driven configuration.

Tier 1 (deployment env, reference .env.sh:1-55), tier 2 (python constants, reference
rafiki/config.py:1-18) and a node section for one MI355X node.  Defaults match the reference.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field


def _env(name, default, cast=str):
    v = os.environ.get(name)
    if v is None or v == '':
        return default
    if cast is bool:
        return v.lower() in ('1', 'true', 'yes', 'on')
    return cast(v)


# ---- tier 2: reference rafiki/config.py ----------------------------------------------------
APP_SECRET = _env('APP_SECRET', 'rafiki')
SUPERADMIN_EMAIL = 'superadmin@rafiki'
SUPERADMIN_PASSWORD = _env('SUPERADMIN_PASSWORD', 'rafiki')
SERVICE_STATUS_WAIT = 1
INFERENCE_WORKER_REPLICAS_PER_TRIAL = _env('INFERENCE_WORKER_REPLICAS_PER_TRIAL', 2, int)
INFERENCE_MAX_BEST_TRIALS = _env('INFERENCE_MAX_BEST_TRIALS', 2, int)
PREDICTOR_PREDICT_SLEEP = 0.25
INFERENCE_WORKER_SLEEP = 0.25
INFERENCE_WORKER_PREDICT_BATCH_SIZE = 32
DEFAULT_MODEL_TRIAL_COUNT = 5
PREDICTOR_TIMEOUT_S = _env('PREDICTOR_TIMEOUT_S', 30.0, float)  # fixes reference bug (g): no timeout


@dataclass
class NodeConfig:
    """Single-node MI355X layout (replaces the Docker-Swarm node labels of the reference)."""
    gpus_per_node: int = field(default_factory=lambda: _env('RAFIKI_GPUS_PER_NODE', 8, int))
    hbm_gb_per_gpu: int = 288
    param_cache_gb: float = field(default_factory=lambda: _env('RAFIKI_PARAM_CACHE_GB', 32.0, float))
    grad_bucket_mb: float = field(default_factory=lambda: _env('RAFIKI_GRAD_BUCKET_MB', 32.0, float))
    dist_backend: str = field(default_factory=lambda: _env('RAFIKI_DIST_BACKEND', 'nccl'))


@dataclass
class AppConfig:
    workdir: str = field(default_factory=lambda: _env('WORKDIR_PATH', os.path.join(os.getcwd(), 'rafiki_workdir')))
    data_dir: str = field(default_factory=lambda: _env('DATA_DIR_PATH', 'data'))
    logs_dir: str = field(default_factory=lambda: _env('LOGS_DIR_PATH', 'logs'))
    params_dir: str = field(default_factory=lambda: _env('PARAMS_DIR_PATH', 'params'))
    db_path: str = field(default_factory=lambda: _env('RAFIKI_DB_PATH', ''))
    admin_host: str = field(default_factory=lambda: _env('ADMIN_HOST', '127.0.0.1'))
    admin_port: int = field(default_factory=lambda: _env('ADMIN_PORT', 3000, int))
    advisor_host: str = field(default_factory=lambda: _env('ADVISOR_HOST', '127.0.0.1'))
    advisor_port: int = field(default_factory=lambda: _env('ADVISOR_PORT', 3002, int))
    predictor_port: int = field(default_factory=lambda: _env('PREDICTOR_PORT', 3003, int))
    app_mode: str = field(default_factory=lambda: _env('APP_MODE', 'DEV'))
    node: NodeConfig = field(default_factory=NodeConfig)

    def path(self, *parts):
        return os.path.join(self.workdir, *parts)

    @property
    def resolved_db_path(self):
        return self.db_path or self.path('rafiki.sqlite3')


def get_config() -> AppConfig:
    return AppConfig()
