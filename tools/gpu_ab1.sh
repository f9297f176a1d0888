set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "variant" > gpurun_out/r02_variant_tests.txt 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/r02_variant_tests.txt; exit 1; }
tail -2 gpurun_out/r02_variant_tests.txt
timeout -k 10 240 python tools/ab.py --variants 0,60,61 --bpc 512,1024 --rounds 9 --reps 48 > gpurun_out/r02_ab_block_barriered.jsonl && cat gpurun_out/r02_ab_block_barriered.jsonl
timeout -k 10 240 python tools/ab.py --variants 0,60,61 --bpc 512 --rounds 9 --reps 48 --overlap > gpurun_out/r02_ab_block_overlap.jsonl && cat gpurun_out/r02_ab_block_overlap.jsonl
timeout -k 10 240 python tools/ab.py --variants 0,60 --bpc 512 --rounds 9 --reps 48 --mode compute > gpurun_out/r02_ab_block_compute.jsonl && cat gpurun_out/r02_ab_block_compute.jsonl
