set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/ab_run.py gpurun_out/r04e_ab.log 1 ws8=libsmaml.so wsp0=libsmaml_wsp0.so wsp2=libsmaml_wsp2.so wsoff=libsmaml.so:SMAML_OPTIONS=wgrad_ws=0 bwdd2=libsmaml_bwdd2.so:SMAML_OPTIONS=wgrad_ws=0 || exit 1
BA="--steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing --adapt-epochs 0 --cfg5-share-tasks 0"
for v in ws:wgrad_ws=1 off:wgrad_ws=0; do
  n=${v%%:*}; o=${v#*:}
  SMAML_OPTIONS=$o timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex "k_wgrad" -f csv -d gpurun_out/r04e_pmc_$n -o run -- python bench.py $BA > gpurun_out/r04e_pmc_$n.log 2>&1
  echo "pmc $n rc=$?"
  SMAML_OPTIONS=$o timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "k_wgrad" -f csv -d gpurun_out/r04e_pmc2_$n -o run -- python bench.py $BA > gpurun_out/r04e_pmc2_$n.log 2>&1
  echo "pmc2 $n rc=$?"
done
