#!/bin/bash
# Clay(10,4) plane-group kernel: non-temporal load policies (ecx_tune rtc_nt) against cached loads,
# two interleaved sweeps (scripts/clay104_diag.py) and bench lines.
set -u
J1='[{"rtc_nt": 0}, {"rtc_nt": 1}, {"rtc_nt": 5}, {"rtc_nt": 1, "rtc_xcd": 3}, {"rtc_nt": 5, "rtc_xcd": 3}, {"rtc_nt": 1, "rtc_xcd": 4}, {"rtc_nt": 5, "rtc_xcd": 4}, {"rtc_nt": 1, "rtc_sched": 1, "rtc_waves": 4, "rtc_lookahead": 0}, {"rtc_nt": 5, "rtc_sched": 1, "rtc_waves": 4, "rtc_lookahead": 0, "rtc_xcd": 3}, {"rtc_nt": 5, "rtc_sched": 0}, {"rtc_nt": 5, "rtc_lookahead": 8}]'
timeout -k 10 400 python scripts/clay104_diag.py --json "$J1" --rounds 4 > gpurun_out/nt2_a.jsonl 2> gpurun_out/nt2_a.err || exit $?
timeout -k 10 300 python bench.py --workload clay104 --steps 3 --warmup 1 --cpu-seconds 0 --tune rtc_nt=5 --tune rtc_xcd=3 > gpurun_out/b104_nt5x3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload clay104 --steps 3 --warmup 1 --cpu-seconds 0 --tune rtc_nt=0 > gpurun_out/b104_nt0.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload clay104 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/b104_def.log 2>&1 || exit $?
timeout -k 10 400 python scripts/clay104_diag.py --json "$J1" --rounds 4 > gpurun_out/nt2_b.jsonl 2> gpurun_out/nt2_b.err || exit $?
