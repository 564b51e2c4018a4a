set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_jni_runtime.py -x -v --timeout 300 --timeout-method thread -m gpu -k "layout_select or two_streams or host_buffer" > $O/t5_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/t5_pytest.log; exit 1; }
tail -12 $O/t5_pytest.log
timeout -k 10 400 python -u scripts/layout_sweep.py --set select > $O/lsweep_select.jsonl 2> $O/lsweep_select.err || { echo sweep failed; tail $O/lsweep_select.err; exit 1; }
cat $O/lsweep_select.jsonl
