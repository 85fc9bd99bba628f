#!/usr/bin/env bash
# Run the test suite (reference scripts/test.sh): CPU tests here, add `-m gpu` on an MI355X.
set -euo pipefail
cd "$(dirname "$0")/.."
python -m rafiki_amd._build
python -m pytest tests/ -q -m "${1:-not gpu}"
