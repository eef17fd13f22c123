set -eo pipefail
export TMPDIR=/tmp
# round-6 profiling, phase 2: per-row set + the final default bench line (tools/profile_round.sh)
bash tools/profile_round.sh r6 rows
