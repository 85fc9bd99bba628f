"""Per-layer table of an autotune log (RAFIKI_AUTOTUNE_LOG jsonl): best config, time and achieved TFLOP/s
of each fp32 GEMM shape, so per-layer efficiency can be read against the MFMA ceiling.

usage: python scripts/dev/tune_log_table.py <tune.jsonl>
Keys (rafiki_amd/ops/f32.py): sf conv fwd / sd conv dgrad (M, N, K, ...), sw weight grad (M, N, K, ...),
sl dense, sx dense dX, sdw dense dW (M, N, K), sfg / slg grouped (groups, M, N, K, ...).
"""
import json
import sys


def flops(key):
    kind = key[0]
    v = [int(x) for x in key[1:5] if x.lstrip('-').isdigit()]
    if kind in ('sfg', 'slg'):
        g, M, N, K = v[:4]
        return 2.0 * g * M * N * K
    M, N, K = v[:3]
    return 2.0 * M * N * K


def main():
    rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
    print('{:<5} {:>8} {:>6} {:>6} {:>12} {:>9} {:>8}'.format('op', 'M', 'N', 'K', 'best cfg', 'us', 'TFLOP/s'))
    for r in rows:
        k = r['key']
        f = flops(k)
        dims = k[1:4] if k[0] not in ('sfg', 'slg') else k[2:5]
        print('{:<5} {:>8} {:>6} {:>6} {:>12} {:>9.2f} {:>8.1f}'.format(
            k[0], *dims, str(tuple(r['best'])), r['us'], f / (r['us'] * 1e-6) / 1e12))


if __name__ == '__main__':
    main()
