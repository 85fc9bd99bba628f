"""Predictor process entry: ``python -m rafiki_amd.predictor`` (reference scripts/start_predictor.py)."""
import sys

from .server import main

if __name__ == '__main__':
    sys.exit(main())
