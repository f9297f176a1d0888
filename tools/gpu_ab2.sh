set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "variant and (84 or 85 or 86)" > gpurun_out/r02_v84_tests.txt 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/r02_v84_tests.txt; exit 1; }
tail -2 gpurun_out/r02_v84_tests.txt
timeout -k 10 240 python tools/ab.py --variants 0,84,85,86 --bpc 512 --rounds 5 --reps 24 --block-mib 1024 --blocks 2 > gpurun_out/r02_ab_steal_1g.jsonl && cat gpurun_out/r02_ab_steal_1g.jsonl
timeout -k 10 240 python tools/ab.py --variants 0,84,85,86 --bpc 512 --rounds 9 --reps 48 > gpurun_out/r02_ab_steal_barriered.jsonl && cat gpurun_out/r02_ab_steal_barriered.jsonl
timeout -k 10 240 python tools/ab.py --variants 0,84,85,86 --bpc 512 --rounds 9 --reps 48 --overlap > gpurun_out/r02_ab_steal_overlap.jsonl && cat gpurun_out/r02_ab_steal_overlap.jsonl
