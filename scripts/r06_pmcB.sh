set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/pmc.sh --candidates rs124 rs173 lrcenc || exit $?
