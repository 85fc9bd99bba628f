"""Admin process entry: ``python -m rafiki_amd.admin`` (reference scripts/start_admin.py:1-18):
seed the superadmin, then serve the REST API (threaded) on ADMIN_PORT."""
import sys


def main():
    from ..config import get_config
    from ..utils.log import configure_logging
    from .admin import Admin
    from .app import create_app
    cfg = get_config()
    configure_logging('admin')
    admin = Admin()
    admin.seed()
    create_app(admin).run(host='0.0.0.0', port=cfg.admin_port, threaded=True)
    return 0


if __name__ == '__main__':
    sys.exit(main())
