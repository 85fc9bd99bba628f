"""Start a predictor service process (reference scripts/start_predictor.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rafiki_amd.predictor.server import main  # noqa: E402

if __name__ == '__main__':
    sys.exit(main())
