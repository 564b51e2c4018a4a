#!/bin/bash
# Resident-workgroup caps over ten RS layouts (one process) and the rs173 / rs124 bench lines.
timeout -k 10 600 python scripts/occ_bench.py --sets "occ_lds=0;occ_lds=-1;occ_lds=32768;occ_lds=53248;block_threads=64,occ_lds=0;block_threads=64,occ_lds=10240;block_threads=64,occ_lds=8192" > gpurun_out/occ_bench.jsonl 2> gpurun_out/occ_bench.err || exit $?
for W in rs173 rs124; do timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/b_$W.log 2>&1 || exit $?; done
