#!/bin/bash
# Round-4 final measurement of the shipped library: kernel trace, the six PMC passes and the
# default bench (tools/tools_round_profile.sh), then a two-run A/B (tools/r04_ab.sh RUNS).
set -o pipefail
bash tools/tools_round_profile.sh --steps 20 --warmup 5 || exit 1
NOTEST=1 bash tools/r04_ab.sh
