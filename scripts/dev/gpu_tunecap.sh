# Capture the node-wide autotune database of a full default bench.py run (phase 1 step, HPO trials, probe
# trials, serving) for shipping (scripts/ship_tune_db.py); prints the bench line of that cold run
set -o pipefail
O=gpurun_out/tunecap
mkdir -p $O
RAFIKI_TUNE_CACHE=$PWD/$O/tune_db.json timeout -k 10 900 python -u bench.py --gpus 1 --steps 50 --warmup 10 \
  > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
python3 -c "import json; print(len(json.load(open('$O/tune_db.json'))), 'entries')"
