set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu "tests/test_gpu_api.py::test_wgrad_variants_match" "tests/test_gpu_so_depth.py::test_second_order_k10_cfg5" > gpurun_out/r04d_pytest.log 2>&1 || { tail -30 gpurun_out/r04d_pytest.log; exit 1; }
tail -1 gpurun_out/r04d_pytest.log
SMAML_LIB=weatherforecast_stgcn_maml_amd/libsmaml_ws4.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu "tests/test_gpu_api.py::test_wgrad_variants_match" > gpurun_out/r04d_pytest4.log 2>&1 || { tail -30 gpurun_out/r04d_pytest4.log; exit 1; }
tail -1 gpurun_out/r04d_pytest4.log
timeout -k 10 900 python -u tools/ab_run.py gpurun_out/r04d_ab.log 2 ws8=libsmaml.so ws4=libsmaml_ws4.so wsoff=libsmaml.so:SMAML_OPTIONS=wgrad_ws=0 || exit 1
