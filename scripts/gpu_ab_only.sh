# A/B of in-tree library variants only (no tests): bench.py per lib, interleaved by the caller's order
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_ab.sh "$@"
