set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "variant and (74 or 75)" > gpurun_out/r02_v74_tests.txt 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/r02_v74_tests.txt; exit 1; }
tail -2 gpurun_out/r02_v74_tests.txt
timeout -k 10 240 python tools/ab.py --variants 0,74,75 --bpc 512 --rounds 9 --reps 48 > gpurun_out/r02_ab_wave2_barriered.jsonl && cat gpurun_out/r02_ab_wave2_barriered.jsonl
timeout -k 10 240 python tools/ab.py --variants 0,74,75 --bpc 512 --rounds 9 --reps 48 --overlap > gpurun_out/r02_ab_wave2_overlap.jsonl && cat gpurun_out/r02_ab_wave2_overlap.jsonl
timeout -k 10 240 python tools/ab.py --variants 0,74,75 --bpc 512 --rounds 5 --reps 24 --block-mib 1024 --blocks 2 > gpurun_out/r02_ab_wave2_1g.jsonl && cat gpurun_out/r02_ab_wave2_1g.jsonl
