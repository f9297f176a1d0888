set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "variant and 82" > gpurun_out/r02_v82_tests.txt 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/r02_v82_tests.txt; exit 1; }
tail -2 gpurun_out/r02_v82_tests.txt
timeout -k 10 240 python tools/ab.py --variants 44,78,82 --bpc 512 --rounds 15 --reps 64 --overlap > gpurun_out/r02_ab_solohalf_overlap.jsonl && cat gpurun_out/r02_ab_solohalf_overlap.jsonl
timeout -k 10 240 python tools/ab.py --variants 44,78,82 --bpc 512 --rounds 9 --reps 48 > gpurun_out/r02_ab_solohalf_barriered.jsonl && cat gpurun_out/r02_ab_solohalf_barriered.jsonl
