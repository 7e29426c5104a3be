# dwconv + RESID output-byte microbenchmarks first (short), then the GPU suite / fp8 breakdown / default bench
set -u
export TMPDIR=/tmp
bash scripts/r04_dwconv.sh || exit $?
bash scripts/r04_resid_bytes.sh || exit $?
bash scripts/r04_iter2.sh
