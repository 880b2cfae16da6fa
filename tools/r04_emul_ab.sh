#!/bin/bash
# Per-rank emulation of an 8-GPU job (tools/r04_emul.sh), then a short A/B (tools/r04_ab.sh RUNS).
set -o pipefail
bash tools/r04_emul.sh || exit 1
NOTEST=1 bash tools/r04_ab.sh
