set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pipeline.py tests/test_abi_consumer.py tests/test_reference_headers.py tests/test_output_stream.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02_pipe_tests.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r02_pipe_tests.txt; exit 1; }
tail -3 gpurun_out/r02_pipe_tests.txt
timeout -k 10 400 python -u tools/e2e_write.py > gpurun_out/r02_e2e_write.jsonl 2>&1 || { echo "e2e_write failed"; tail -20 gpurun_out/r02_e2e_write.jsonl; exit 1; }
cat gpurun_out/r02_e2e_write.jsonl
