#!/bin/bash
# Config 5 after the pool's least-recent-first shedding and the opt-in NUMA binding: the reader and
# pool GPU tests (also once with HDFS3_NUMA=1), then e2e_read default vs an uncapped pool, twice.
set -o pipefail
TAG=${1:-r3e2e_fix}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_input_readahead.py tests/test_input_stream.py tests/test_block_reader.py tests/test_local_reader.py tests/test_multigpu.py tests/test_numa.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
HDFS3_NUMA=1 timeout -k 10 400 python -u -m pytest $T -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests_numa1.txt 2>&1
rc=$?; echo "tests numa1 rc=$rc"; tail -2 gpurun_out/${TAG}_tests_numa1.txt; [ $rc -eq 0 ] || exit $rc
run() { # name env...
    local n=$1; shift
    env "$@" timeout -k 10 300 python -u tools/e2e_read.py --reps 2 --readahead 1,2,3,7 > gpurun_out/${TAG}_$n.jsonl 2> gpurun_out/${TAG}_$n.err \
        || { echo "e2e $n failed"; tail -20 gpurun_out/${TAG}_$n.err; exit 1; }
    echo "== $n"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['mode'], j.get('verify',''), j.get('streams',''), j.get('readahead_blocks',''), j['gib_s'])" gpurun_out/${TAG}_$n.jsonl
}
for rep in 1 2; do
run default_$rep HDFS3_E2E=1 || exit 1
run bigcap_$rep HDFS3_POOL_PINNED_MAX=16G || exit 1
done
