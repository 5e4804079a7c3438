set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_host_pipeline.py "tests/test_gpu_parity.py::test_product_full_size_parity" "tests/test_gpu_parity.py::test_ragged_batch_sizes" "tests/test_gpu_parity.py::test_debug_switches_do_not_change_results" > gpurun_out/r06a/pytest.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --host --steps 20 --warmup 3 --cpu-sample 65536 > gpurun_out/r06a/bench_host.json 2> gpurun_out/r06a/bench_host.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err
rc=$?
tail -15 gpurun_out/r06a/pytest.txt; cat gpurun_out/r06a/bench_host.json gpurun_out/r06a/bench.json; exit $rc
