set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/r06_rss_n1.json 2>/dev/null; rc=$?; echo "n1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --pool 1024 --stripes-per-step 4096 > gpurun_out/r06_rss_n1_small.json 2>/dev/null; rc=$?; echo "n1 small rc=$rc"; exit $rc
