#!/bin/bash
# Config 5 read lines at pool caps of 512 MiB (default), 1 GiB and 2 GiB, interleaved twice.
set -o pipefail
TAG=${1:-r3e2e_caps}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() { # name env...
    local n=$1; shift
    env "$@" timeout -k 10 300 python -u tools/e2e_read.py --reps 2 --readahead 1,2,3,7 > gpurun_out/${TAG}_$n.jsonl 2> gpurun_out/${TAG}_$n.err \
        || { echo "e2e $n failed"; tail -20 gpurun_out/${TAG}_$n.err; exit 1; }
    echo "== $n"; python3 -c "
import json,sys
r=[]
for l in open(sys.argv[1]):
    j=json.loads(l)
    if j['mode'] in ('hdfsRead','parallel_pread','hdfsRead_readahead','local_read'): r.append('%s%s%s=%.1f' % (j['mode'][:8], '' if j.get('verify', True) else '-off', j.get('readahead_blocks', j.get('streams','')), j['gib_s']))
print(' '.join(r))" gpurun_out/${TAG}_$n.jsonl
}
for rep in 1 2; do
run cap512_$rep HDFS3_POOL_PINNED_MAX=512M || exit 1
run cap1g_$rep HDFS3_POOL_PINNED_MAX=1G || exit 1
run cap2g_$rep HDFS3_POOL_PINNED_MAX=2G || exit 1
done
