#!/bin/bash
# kernel timeline of the overlapped chain (C3), rocprofv3 kernel trace
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
KS_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_tl -o run -- python3 $GRAFT_REPO_ROOT/tests/dev/ab_resolvers.py --noprof chunk > $GRAFT_REPO_ROOT/gpurun_out/r4_tl.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 profiles/timeline.py $(find gpurun_out/prof_tl -name "*.db" | head -1)
