set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_packet_stream.py tests/test_gpu_segments.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02_dense_tests.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r02_dense_tests.txt; exit 1; }
tail -2 gpurun_out/r02_dense_tests.txt
timeout -k 10 300 python tools/compute_layout_probe.py > gpurun_out/r02_compute_layout_dense.jsonl 2>&1 && cat gpurun_out/r02_compute_layout_dense.jsonl
