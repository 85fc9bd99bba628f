"""Start the admin REST server (reference scripts/start_admin.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rafiki_amd.admin.__main__ import main  # noqa: E402

if __name__ == '__main__':
    sys.exit(main())
