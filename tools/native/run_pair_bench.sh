#!/bin/bash
# tools/native/run_pair_bench.sh THREADS CALLS: pair_bench under the committed key's n^2 (tests/golden/keys.json)
cd "$(dirname "$0")/../.." || exit 1
M=$(python -c 'import json; print(int(json.load(open("tests/golden/keys.json"))["paillier2048_committed"]["nsquare"], 16))')
exec tools/native/pair_bench "$M" "${1:-64}" "${2:-200}"
