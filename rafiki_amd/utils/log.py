"""Per-process log file under ``<workdir>/logs`` (reference rafiki/utils/log.py:11-16)."""
import logging
import os


def configure_logging(process_name):
    from ..config import get_config
    cfg = get_config()
    logs_dir = os.path.join(cfg.workdir, cfg.logs_dir)
    os.makedirs(logs_dir, exist_ok=True)
    root = logging.getLogger()
    path = os.path.join(logs_dir, '{}.log'.format(process_name))
    if any(isinstance(h, logging.FileHandler) and getattr(h, 'baseFilename', '') == path for h in root.handlers):
        return path
    fh = logging.FileHandler(path)
    fh.setFormatter(logging.Formatter('%(asctime)s %(name)s %(levelname)s %(message)s'))
    root.addHandler(fh)
    root.setLevel(logging.INFO)
    return path
