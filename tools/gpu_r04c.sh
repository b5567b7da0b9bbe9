set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in nobar:grid_barrier=0 bar:grid_barrier=1; do
  n=${v%%:*}; o=${v#*:}
  SMAML_OPTIONS=$o SMAML_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --tasks 4 --steps 1 --warmup 1 --adapt-epochs 0 --cfg5-share-tasks 0 > gpurun_out/r04c_gloo_$n.log 2> gpurun_out/r04c_gloo_$n.err || { tail -5 gpurun_out/r04c_gloo_$n.err; exit 1; }
  python -c "
import json,sys
l=[x for x in open('gpurun_out/r04c_gloo_$n.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$n', j['ms_per_step'], j.get('collective'), {k:round(v['ms_per_step'],1) for k,v in j['kernels'].items()})"
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu "tests/test_gpu_api.py::test_wgrad_variants_match" > gpurun_out/r04c_pytest.log 2>&1 || { tail -30 gpurun_out/r04c_pytest.log; exit 1; }
tail -1 gpurun_out/r04c_pytest.log
timeout -k 10 900 python -u tools/ab_run.py gpurun_out/r04c_ab.log 2 ws8=libsmaml.so ws4=libsmaml_ws4.so wsoff=libsmaml.so:SMAML_OPTIONS=wgrad_ws=0 || exit 1
