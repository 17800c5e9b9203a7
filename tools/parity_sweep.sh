#!/bin/bash
# A large parity sample at the bench geometries (GPU box via gpurun): every
# config's bench line with --parity-streams N (whole streams re-encoded by the
# CPU oracle and compared channel-block by channel-block).  PAR2/PAR3/PAR4: the
# stream counts for configs[2]/[3]/[4].  Lines under gpurun_out/parity_*.json.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
set -o pipefail
run() { local name=$1; shift; timeout -k 10 900 python3 bench.py --steps 2 --warmup 1 "$@" > gpurun_out/parity_$name.json 2> gpurun_out/parity_$name.err || { echo "parity $name failed"; tail -5 gpurun_out/parity_$name.err; exit 1; }; echo "parity $name: $(grep -o '"checked_channel_blocks": [0-9]*, "mismatching": [0-9]*' gpurun_out/parity_$name.json | head -1)"; }
[ -n "$PAR2" ] && { run config2 --config 2 --parity-streams $PAR2 || exit 1; }
[ -n "$PAR3" ] && { run config3 --config 3 --parity-streams $PAR3 || exit 1; }
[ -n "$PAR4" ] && { run config4 --config 4 --parity-streams $PAR4 || exit 1; }
echo PARITY_DONE
