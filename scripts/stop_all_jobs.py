"""Stop every running train and inference job through the admin API as superadmin
(reference scripts/stop_all_jobs.py:1-15)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rafiki_amd.client import Client  # noqa: E402
from rafiki_amd.config import SUPERADMIN_EMAIL, SUPERADMIN_PASSWORD, get_config  # noqa: E402

if __name__ == '__main__':
    cfg = get_config()
    c = Client(admin_host=os.environ.get('ADMIN_HOST', cfg.admin_host), admin_port=cfg.admin_port)
    c.login(email=SUPERADMIN_EMAIL, password=SUPERADMIN_PASSWORD)
    print(c.stop_all_jobs())
