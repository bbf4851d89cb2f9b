#!/usr/bin/env bash
# round 6 GPU job r: long verified runs (every frame checked bit for bit against a second,
# whole-frame renderer in the same process: bench.py --verify), final build
set -uo pipefail
O=gpurun_out/r06ri; mkdir -p $O
run() {  # config steps
  timeout -k 10 300 python3 -u bench.py --config $1 --steps $2 --warmup 8 --verify --no-cpu-baseline > $O/verify_$1.json 2> $O/verify_$1.err || return $?
  python3 -c "import json; d=json.loads(open('$O/verify_$1.json').read().strip().splitlines()[-1]); v=d.get('verify') or {}; print('$1', d['steps'], v.get('frames_checked'), v.get('mismatched'), v.get('diag'))"
}
run d 400 && run b 2000 && run c 400 && run a 3000 && run e 40 && run p 200
