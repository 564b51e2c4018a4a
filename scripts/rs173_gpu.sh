set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python scripts/rs173_knobs.py --set xcd --rounds 2 > $O/rs173_xcd_pad0.jsonl 2> $O/rs173_xcd.err || exit $?
timeout -k 10 300 python scripts/rs173_knobs.py --set xcd --rounds 2 --pad 64 > $O/rs173_xcd_pad64.jsonl 2>> $O/rs173_xcd.err || exit $?
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  for PAD in 0 64; do
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_rs173_${C}_$PAD -o run -- python3 $GRAFT_REPO_ROOT/scripts/rs173_knobs.py --set default --rounds 1 --reps 1 --pad $PAD) > $O/pmc_rs173_${C}_$PAD.log 2>&1 || exit $?
  done
done
cat $O/rs173_xcd_pad0.jsonl $O/rs173_xcd_pad64.jsonl
