#!/bin/bash
# /Sum under native threads (tools/native/pair_bench): sweep of the waiters' spin time, the batches in
# flight per modulus and the caller count
cd /root/repo
M=$(python3 -c "import json;print(int(json.load(open('tests/golden/keys.json'))['paillier2048_committed']['nsquare'],16))")
IFS="|" read -ra SW <<< "${PAIR_SWEEP:-100 2 64|0 2 64|20 2 64|20 4 64|0 4 64|100 4 64|20 8 64}"
for v in "${SW[@]}"; do
  set -- $v
  echo "== spin_us=$1 inflight=$2 threads=$3"
  DDSHE_PAIR_SPIN_US=$1 DDSHE_PAIR_INFLIGHT=$2 timeout -k 5 120 tools/native/pair_bench "$M" "$3" 200 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d.pop('samples'); print(json.dumps(d))" || exit 1
done
