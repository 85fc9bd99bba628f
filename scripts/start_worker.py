"""Start a worker service process (reference scripts/start_worker.py); normally launched by the
admin's LocalProcessManager with RAFIKI_SERVICE_ID / RAFIKI_SERVICE_TYPE and torchrun-style env."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rafiki_amd.worker.__main__ import main  # noqa: E402

if __name__ == '__main__':
    sys.exit(main())
