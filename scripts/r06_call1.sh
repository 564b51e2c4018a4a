set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_first.json 2> gpurun_out/r06_bench_first.err; rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r06_bench_first.json; [ $rc -ne 0 ] && exit $rc
ECX_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --pool 1024 --stripes-per-step 4096 --steps 4 --warmup 1 --cpu-seconds 0 --no-probes > gpurun_out/r06_bench_gloo8.json 2> gpurun_out/r06_bench_gloo8.err; rc=$?; echo "gloo8 rc=$rc"; tail -c 400 gpurun_out/r06_bench_gloo8.json; [ $rc -ne 0 ] && exit $rc
bash scripts/clay104_ab.sh
