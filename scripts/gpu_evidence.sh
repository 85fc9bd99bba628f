# Secondary-benchmark evidence in one call: BiLSTM / tagger step (+ its kernel list), PG-GAN eager vs
# graphed rounds at LOD 3 and 0, predictor QPS with 1 and 2 replicas.  Outputs under gpurun_out/ev/.
#   bash scripts/gpu_evidence.sh [lstm] [pggan] [serve]   (default: all three)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ev
mkdir -p $O
WHAT="${*:-lstm pggan serve}"
for w in $WHAT; do
  case $w in
    lstm)
      timeout -k 10 300 python3 -u scripts/dev/bench_lstm.py --reps 20 > $O/lstm.json 2> $O/lstm.err || exit 1
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lstm_prof -o run -- \
        python3 scripts/dev/bench_lstm.py --reps 5 --only-tagger > $O/lstm_prof.log 2>&1 || exit 1
      python3 scripts/dev/kernel_summary.py $(find $O/lstm_prof -name '*kernel_trace.csv' | head -1) > $O/lstm_kernels.txt
      rm -rf $O/lstm_prof
      cat $O/lstm.json; head -30 $O/lstm_kernels.txt ;;
    pggan)
      timeout -k 10 600 python3 -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 > $O/pggan_graph.log 2>&1 || exit 1
      timeout -k 10 600 python3 -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --no-graph > $O/pggan_eager.log 2>&1 || exit 1
      tail -1 $O/pggan_graph.log | cut -c1-600; tail -1 $O/pggan_eager.log | cut -c1-600 ;;
    serve)
      timeout -k 10 400 python3 -u scripts/bench_predictor.py --replicas 1 --out $O/qps_1rep.json > $O/qps1.log 2>&1 || exit 1
      timeout -k 10 400 python3 -u scripts/bench_predictor.py --replicas 2 --skip-http-asyncio --out $O/qps_2rep.json > $O/qps2.log 2>&1 || exit 1
      cut -c1-1500 $O/qps_1rep.json; cut -c1-1500 $O/qps_2rep.json ;;
  esac
done
echo evidence-done
