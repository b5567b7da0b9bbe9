set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "tests/test_gpu_api.py::test_wgrad_variants_match" tests/test_gpu_so_depth.py "tests/test_gpu_parity.py" -k "wgrad or so_depth or second_order or k5 or k10 or bench_configuration or config5" > gpurun_out/r04b_pytest.log 2>&1 || { tail -30 gpurun_out/r04b_pytest.log; exit 1; }
tail -2 gpurun_out/r04b_pytest.log
timeout -k 10 900 python -u tools/ab_run.py gpurun_out/r04b_ab.log 2 base=libsmaml.so wsoff=libsmaml.so:SMAML_OPTIONS=wgrad_ws=0 ntb=libsmaml_ntb.so || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r04b_bench.log 2> gpurun_out/r04b_bench.err || { tail -5 gpurun_out/r04b_bench.err; exit 1; }
tail -1 gpurun_out/r04b_bench.log | cut -c1-300
SMAML_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --adapt-epochs 0 --cfg5-share-tasks 0 > gpurun_out/r04b_gloo2.log 2> gpurun_out/r04b_gloo2.err || { tail -5 gpurun_out/r04b_gloo2.err; exit 1; }
tail -1 gpurun_out/r04b_gloo2.log | cut -c1-300
