set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/pmc.sh --candidates rs124 rs173 lrcenc || exit $?
bash scripts/pmc.sh --candidates rs173_blocked rs124_blocked rs173_pitchrecommended rs124_pitchrecommended || exit $?
bash scripts/pmc.sh rs173_blocked rs124_blocked rs173_pitchrecommended rs124_pitchrecommended clay104_sub1048576 || exit $?
