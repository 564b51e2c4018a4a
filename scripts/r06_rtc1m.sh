set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
line() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], r['frac'], r['avg_launch_ms'])" "$1"; }
for rep in 1 2; do for T in "rtc_xcd=2" "rtc_xcd=0" "rtc_xcd=1" "rtc_xcd=3" "rtc_nt=1" "rtc_nt=0" "rtc_sched=1"; do
  tag=$(echo $T | tr '=' '_'); timeout -k 10 300 python bench.py --workload clay104 --sub-bytes 1048576 --steps 3 --warmup 1 --cpu-seconds 0 --e2e-seconds 0 --no-probes --tune $T > gpurun_out/r06_rtc1m_${tag}_$rep.json 2>/dev/null; rc=$?; echo "$T rep$rep rc=$rc $(line gpurun_out/r06_rtc1m_${tag}_$rep.json)"; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
