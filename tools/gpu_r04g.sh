set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu "tests/test_gpu_api.py::test_wgrad_variants_match" "tests/test_gpu_api.py::test_order_only_knobs_bitwise" "tests/test_gpu_api.py::test_stgcn_autograd_matches_oracle" "tests/test_gpu_api.py::test_stgcn_forward_matches_reference" "tests/test_gpu_parity.py::test_gcnconv_dropin_matches_oracle" "tests/test_gpu_accuracy.py::test_bf16x6_special_values" > gpurun_out/r04g_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04g_pytest.log; grep -E "FAILED|Error" gpurun_out/r04g_pytest.log | head -5
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u tools/ab_run.py gpurun_out/r04g_ab.log 1 ws=libsmaml.so wsoff=libsmaml.so:SMAML_OPTIONS=wgrad_ws=0 remap=libsmaml.so:SMAML_OPTIONS=wgrad_ws=0,bwdd_remap=1 || exit 1
BA="--steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing --adapt-epochs 0 --cfg5-share-tasks 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex "k_wgrad" -f csv -d gpurun_out/r04g_pmc_ws -o run -- python bench.py $BA > gpurun_out/r04g_pmc_ws.log 2>&1
r=$?; echo "pmc rc=$r"; [ $r -eq 0 ] || exit $r
for v in off:bwdd_remap=0 on:bwdd_remap=1; do
  n=${v%%:*}; o=${v#*:}
  SMAML_OPTIONS=wgrad_ws=0,$o timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_lstm_bwd_dual" -f csv -d gpurun_out/r04g_fetch_$n -o run -- python bench.py $BA > gpurun_out/r04g_fetch_$n.log 2>&1
  r=$?; echo "fetch $n rc=$r"; [ $r -eq 0 ] || exit $r
done
exit $rc
