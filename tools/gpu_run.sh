#!/bin/bash
# One GPU-box pass made of named steps, each under its own time limit; the first failure ends the
# call (nothing more runs on the GPU after a failed, aborted or timed-out step). Outputs go to
# gpurun_out/<tag>_<step>.* and are merged back by gpurun.
#
#   gpurun --timeout 1100 -- bash tools/gpu_run.sh <tag> <step> [<step> ...]
#
# steps:
#   tests            the whole -m gpu suite
#   tests:<expr>     the -m gpu tests selected by -k <expr> (+ for spaces: tests:bench_json+or+scaling)
#   file:<path>      the -m gpu tests of one test file
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (the default line: K = 2000)
#   bench_k20        the driver's command: python3 bench.py --gpus 1 --steps 20 --warmup 5
#   prof             rocprofv3 --kernel-trace --stats of the driver's command (PMC and CPU legs off)
#   tool:<script>    python tools/<script> (extra args after '@': tool:ab.py@--variants@0,154@--overlap)
#   rprof:<script>   the same under rocprofv3 --kernel-trace --stats (csv in gpurun_out/<tag>_<script>_<i>/)
#   pmc[:args]       tools/pmc.sh counter passes over tools/pmc_driver.py (args after '@', e.g. pmc:--overlap)
set -o pipefail
TAG=${1:?tag}
shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"

run() {  # run <seconds> <outfile> <cmd...>
    local secs=$1 out=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "$out" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then
        echo "STEP FAILED rc=$rc: $*"
        tail -40 "$out"
        exit 1
    fi
}

i=0
for step in "$@"; do
    i=$((i + 1))
    echo "== $step ($(date +%T))"
    case "$step" in
    tests) run 900 gpurun_out/${TAG}_gpu_tests.txt $PYT tests; tail -3 gpurun_out/${TAG}_gpu_tests.txt ;;
    tests:*) k=${step#tests:}; k=${k//+/ }
             run 900 gpurun_out/${TAG}_gpu_tests_k.txt $PYT tests -k "$k"; tail -3 gpurun_out/${TAG}_gpu_tests_k.txt ;;
    file:*) f=${step#file:}; n=$(basename "$f" .py)
            run 900 gpurun_out/${TAG}_${n}.txt $PYT "$f"; tail -3 gpurun_out/${TAG}_${n}.txt ;;
    smoke) run 120 gpurun_out/${TAG}_smoke.txt python -c "import __graft_entry__ as g; g.smoke()"; cat gpurun_out/${TAG}_smoke.txt ;;
    bench) run 400 gpurun_out/${TAG}_bench.err python -u bench.py --out-json gpurun_out/${TAG}_bench.json
           cat gpurun_out/${TAG}_bench.json ;;
    bench_k20) run 400 gpurun_out/${TAG}_bench_k20.err python3 -u bench.py --gpus 1 --steps 20 --warmup 5 \
                   --out-json gpurun_out/${TAG}_bench_k20.json
               cat gpurun_out/${TAG}_bench_k20.json ;;
    prof) run 400 gpurun_out/${TAG}_prof.err rocprofv3 --kernel-trace --stats --output-format csv \
              -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline \
              --out-json gpurun_out/${TAG}_prof_bench.json
          cat gpurun_out/${TAG}_prof_bench.json ;;
    tool:*) t=${step#tool:}; IFS=@ read -r -a parts <<< "$t"; n=$(basename "${parts[0]}" .py)_$i
            run 600 gpurun_out/${TAG}_${n}.jsonl python -u tools/"${parts[0]}" "${parts[@]:1}"; tail -30 gpurun_out/${TAG}_${n}.jsonl ;;
    rprof:*) t=${step#rprof:}; IFS=@ read -r -a parts <<< "$t"; n=$(basename "${parts[0]}" .py)_$i
              run 600 gpurun_out/${TAG}_${n}.txt rocprofv3 --kernel-trace --stats --output-format csv \
                  -d gpurun_out/${TAG}_${n} -o run -- python3 -u tools/"${parts[0]}" "${parts[@]:1}"
              tail -5 gpurun_out/${TAG}_${n}.txt ;;
    pmc|pmc:*) t=${step#pmc}; t=${t#:}; IFS=@ read -r -a parts <<< "$t"
               run 900 gpurun_out/${TAG}_pmc_$i.txt bash tools/pmc.sh gpurun_out/${TAG}_pmc_$i "${parts[@]}"
               python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_$i | tail -40 ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "== done ($(date +%T))"
