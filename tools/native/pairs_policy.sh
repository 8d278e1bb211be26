#!/bin/bash
# /Sum under native threads (tools/native/pair_bench) for each serving policy (0 GPU batches, 1 lone
# requests on the host, 2 every request on the host) at 1, 8 and 64 callers: host CPU per call by
# phase, latency, throughput. usage (repo root): tools/native/pairs_policy.sh [calls_per_thread]
cd "$(dirname "$0")/../.." || exit 1
M=$(python3 -c "import json;print(int(json.load(open('tests/golden/keys.json'))['paillier2048_committed']['nsquare'],16))")
for p in 0 1 2; do
  for t in 1 8 64; do
    echo "== policy=$p threads=$t"
    DDSHE_PAIR_POLICY=$p timeout -k 5 120 tools/native/pair_bench "$M" "$t" "${1:-200}" | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d.pop('samples'); print(json.dumps(d))" || exit 1
  done
done
