set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ECX_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --pool 1024 --stripes-per-step 4096 --steps 4 --warmup 1 --cpu-seconds 0 --no-probes > gpurun_out/r06_bench_gloo8.json 2> gpurun_out/r06_bench_gloo8.err; rc=$?; echo "gloo8 rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r06_bench_gloo8.err; exit $rc; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 4 --warmup 1 --cpu-seconds 0 > gpurun_out/r06_bench_rccl1.json 2> gpurun_out/r06_bench_rccl1.err; rc=$?; echo "rccl1 rc=$rc"; exit $rc
